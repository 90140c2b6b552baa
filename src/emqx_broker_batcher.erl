%% emqx_broker_batcher -- publish micro-batching for emqx_broker's route lookup.
%%
%% The reference looks up the routes of each publish on its own, in the
%% publisher's process (emqx_broker.erl:293-298):
%%     do_publish(#message{topic = Topic} = Msg) ->
%%         ...
%%         Routes = aggre(emqx_router:match_routes(Topic)),
%% With the match on the GPU, one call per message would cost one device round
%% trip per publish (~0.1 ms, bounded by the dirty schedulers).  Instead the
%% publisher hands its topic to the batcher of its scheduler, which takes every
%% request already in its mailbox (up to ?MAX_BATCH), matches them with ONE
%% emqx_router_gpu:match_routes_batch/1 call, and replies to each publisher
%% with its own routes.  There is no timer: an idle batcher serves a lone
%% publish at once, and under load the batch is whatever arrived while the
%% previous one was on the GPU -- it grows with the publish rate.  aggre/1 (:408-424) and dispatch stay
%% per message in the publisher; a topic with a '+'/'#' level fails only its
%% own publisher with badarg (emqx_trie_search.erl:374-375), as before.
%%
%% One batcher per scheduler (registered emqx_broker_batcher_<N>), started by
%% the broker supervisor; a publisher reaches the one of its current scheduler
%% so the collection stays NUMA-local.  The batcher runs the NIF on a dirty I/O
%% scheduler (emqx_tmatch_nif), so its own scheduler keeps serving publishers.
%%
%% The change in emqx_broker:do_publish/1 is one line:
%%     Routes = aggre(emqx_broker_batcher:match_routes(Topic)),
%%
%% Not built in this image (no OTP, SURVEY.md 8c); emqx_amd/broker.py is the
%% Python mirror of the same collector and what the tests run.
-module(emqx_broker_batcher).

-behaviour(gen_server).

-export([start_link/1, match_routes/1, name/1]).
-export([init/1, handle_call/3, handle_cast/2, handle_info/2]).

-define(MAX_BATCH, 4096).
-define(CALL_TIMEOUT, 5000).

-record(st, {id :: pos_integer(), batches = 0 :: non_neg_integer()}).

name(Id) ->
    list_to_atom("emqx_broker_batcher_" ++ integer_to_list(Id)).

start_link(Id) ->
    gen_server:start_link({local, name(Id)}, ?MODULE, Id, []).

%% The publisher's side: routes of Topic, as emqx_router:match_routes/1 gives them.
-spec match_routes(emqx_types:topic()) -> [emqx_types:route()].
match_routes(Topic) ->
    Batcher = name(erlang:system_info(scheduler_id)),
    case whereis(Batcher) of
        undefined ->
            emqx_router_gpu:match_routes(Topic);
        Pid ->
            %% The reply goes to a process alias tied to the monitor
            %% (reply_demonitor: the reply deactivates both), so a reply that
            %% arrives after the timeout below -- the alias deactivated by the
            %% demonitor -- is dropped by the runtime instead of landing in the
            %% publisher's (connection process's) mailbox (VERDICT r3).  A
            %% 'DOWN' the batcher's death queued after its reply is flushed
            %% with the monitor, as gen:do_call does (ADVICE r4).
            Alias = erlang:monitor(process, Pid, [{alias, reply_demonitor}]),
            Pid ! {match, Alias, Topic},
            receive
                {Alias, {error, Reason}} ->
                    erlang:demonitor(Alias, [flush]),
                    error(Reason);
                {Alias, Routes} ->
                    erlang:demonitor(Alias, [flush]),
                    Routes;
                {'DOWN', Alias, process, _, _} ->
                    %% the batcher died with our request: ask the router directly
                    emqx_router_gpu:match_routes(Topic)
            after ?CALL_TIMEOUT ->
                erlang:demonitor(Alias, [flush]),
                %% a reply sent before the alias went inactive may already be queued
                receive
                    {Alias, _} -> ok
                after 0 -> ok
                end,
                emqx_router_gpu:match_routes(Topic)
            end
    end.

init(Id) ->
    {ok, #st{id = Id}}.

handle_call(_Req, _From, St) ->
    {reply, ignored, St}.

handle_cast(_Msg, St) ->
    {noreply, St}.

handle_info({match, Alias, Topic}, St = #st{batches = B}) ->
    %% this request plus every one already queued behind it
    Reqs = [{Alias, Topic} | drain(?MAX_BATCH - 1, [])],
    Results =
        try
            emqx_router_gpu:match_routes_batch([T || {_, T} <- Reqs])
        catch
            %% a batch the device failed ({error, device}): every publisher of
            %% the batch gets the error, none a badarg
            error:{tmatch, {error, Reason}} -> [{error, Reason} || _ <- Reqs]
        end,
    lists:foreach(fun({{A, _}, Res}) -> A ! {A, Res} end, lists:zip(Reqs, Results)),
    {noreply, St#st{batches = B + 1}};
handle_info(_Info, St) ->
    {noreply, St}.

drain(0, Acc) ->
    lists:reverse(Acc);
drain(K, Acc) ->
    receive
        {match, Alias, Topic} -> drain(K - 1, [{Alias, Topic} | Acc])
    after 0 ->
        lists:reverse(Acc)
    end.
