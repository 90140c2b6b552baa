%% emqx_router_gpu -- emqx_router's v2 read path (apps/emqx/src/emqx_router.erl)
%% with the filter match on the MI355X (emqx_topic_index_gpu over the NIF).
%%
%% The reference's match_routes/1 (:205-212) dispatches on the schema version
%% and, for v2 (the default, emqx_schema.erl:1303-1310), is
%%     match_routes_v2(Topic) ->
%%         lookup_route_tab(Topic) ++ [match_to_route(M) || M <- match_filters(Topic)].
%% (:511-516): the exact-topic bag ?ROUTE_TAB first, in insertion order, then
%% the filter table's matches in matches/3 order.  This module keeps that
%% composition and the same #route{} records; only match_filters/1 runs on the
%% device, and match_routes_batch/1 does it for a whole broker micro-batch in
%% one NIF call (emqx_broker_batcher).  Writes keep going through emqx_router
%% (mria); the device mirror of ?ROUTE_TAB_FILTERS is fed by
%% emqx_topic_index_gpu:apply_batch/2 (router syncer batches) and
%% table_event/2 (replicated writes, SURVEY.md 3.2).
%%
%% The mirror handle lives in persistent_term (set once at boot by
%% attach/1, read lock-free by every publisher, as the reference reads its
%% schema version from persistent_term at :660-661).
%%
%% Not built in this image (no OTP, SURVEY.md 8c); the Python mirror
%% emqx_amd/router.py implements the same composition and is what the tests run.
-module(emqx_router_gpu).

-include_lib("emqx/include/emqx.hrl").
-include_lib("emqx/include/emqx_router.hrl").

-behaviour(gen_server).

-export([attach/1, detach/0, mirror/0]).
-export([match_routes/1, match_routes_batch/1]).
-export([start_link/1, init/1, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(PT_KEY, {?MODULE, mirror}).
-define(BOOT_BATCH, 100000).
-define(MAX_EVENTS, 10000).

%% Boot: mirror the existing ?ROUTE_TAB_FILTERS (emqx_router.erl:148-160) on the
%% given devices and publish the handle.  Called from emqx_router_sup after
%% emqx_router:create_tables/0 (emqx_router_sup.erl:25-33), as the child
%% start_link(Devices): the process subscribes to the table's events FIRST,
%% then loads the table, so no write is lost between the two (a write seen
%% both ways is an idempotent delta).
-spec attach([integer()]) -> ok.
attach(Devices) ->
    G = emqx_topic_index_gpu:attach(?ROUTE_TAB_FILTERS, ?BOOT_BATCH, Devices),
    persistent_term:put(?PT_KEY, G),
    ok.

-spec detach() -> ok.
detach() ->
    _ = persistent_term:erase(?PT_KEY),
    ok.

%% The mirror's event process: every write to ?ROUTE_TAB_FILTERS on this node
%% -- local router writes, mria-replicated ones and the match_delete of a
%% node-down cleanup_routes/1 (emqx_router.erl:535-550) alike -- reaches the
%% device as table events, drained from the mailbox and shipped as one delta
%% batch per drain (the router never writes the mria-managed table behind
%% mria's back; VERDICT r3).
start_link(Devices) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Devices, []).

init(Devices) ->
    {ok, _} = mnesia:subscribe({table, ?ROUTE_TAB_FILTERS, detailed}),
    ok = attach(Devices),
    {ok, mirror()}.

handle_call(_Req, _From, G) ->
    {reply, ignored, G}.

handle_cast(_Msg, G) ->
    {noreply, G}.

handle_info({mnesia_table_event, E}, G) ->
    ok = emqx_topic_index_gpu:table_events([E | drain_events(?MAX_EVENTS - 1, [])], G),
    {noreply, G};
handle_info(_Info, G) ->
    {noreply, G}.

terminate(_Reason, _G) ->
    _ = mnesia:unsubscribe({table, ?ROUTE_TAB_FILTERS, detailed}),
    detach().

drain_events(0, Acc) ->
    lists:reverse(Acc);
drain_events(K, Acc) ->
    receive
        {mnesia_table_event, E} -> drain_events(K - 1, [E | Acc])
    after 0 ->
        lists:reverse(Acc)
    end.

-spec mirror() -> emqx_topic_index_gpu:gtab() | undefined.
mirror() ->
    persistent_term:get(?PT_KEY, undefined).

%% match_routes/1 (emqx_router.erl:205-212, v2 :511-516).
-spec match_routes(emqx_types:topic()) -> [emqx_types:route()].
match_routes(Topic) when is_binary(Topic) ->
    case match_routes_batch([Topic]) of
        [{error, Reason}] -> error(Reason);
        [Routes] -> Routes
    end.

%% One broker micro-batch: per topic, lookup_route_tab(Topic) ++ the filter
%% routes, or {error, badarg} for a topic with a '+'/'#' level (only that
%% message fails, as each publisher's own call fails in the reference).
-spec match_routes_batch([emqx_types:topic()]) -> [[emqx_types:route()] | {error, atom()}].
match_routes_batch(Topics) ->
    case mirror() of
        undefined ->
            %% no device mirror on this node: the reference's own path
            [
                try
                    emqx_router:match_routes(T)
                catch
                    error:badarg -> {error, badarg}
                end
             || T <- Topics
            ];
        G ->
            Matches = emqx_topic_index_gpu:matches_batch(Topics, G, [return_errors]),
            lists:zipwith(fun compose/2, Topics, Matches)
    end.

compose(_Topic, {error, _} = Err) ->
    Err;
compose(Topic, Keys) ->
    ets:lookup(?ROUTE_TAB, Topic) ++ [match_to_route(K) || K <- Keys].

%% emqx_router.erl:648-649
match_to_route(M) ->
    #route{topic = emqx_topic_index:get_topic(M), dest = emqx_topic_index:get_id(M)}.
