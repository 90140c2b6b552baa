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
%% (mria); the device mirror of ?ROUTE_TAB_FILTERS is fed synchronously by
%% the router's hook (filters_written/1, batch_written/1: the mirror has a
%% route before do_add_route/2 returns) and asynchronously by the table's
%% mnesia events (replicated writes, node-down cleanups, SURVEY.md 3.2); both
%% reconcile each key against the table (emqx_topic_index_gpu:mirror_batch/2).
%% The bag ?ROUTE_TAB stays in ETS: its rows come back in insertion order from
%% ets:lookup (the Python mirror emqx_amd/router.py keeps it the same way).
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
-export([filters_written/1, batch_written/1]).
-export([match_routes/1, match_routes_batch/1]).
-export([start_link/1, init/1, handle_continue/2, handle_call/3, handle_cast/2, handle_info/2, terminate/2]).

-define(PT_KEY, {?MODULE, mirror}).
-define(BOOT_BATCH, 100000).
%% copies of the route tables per device: the router's mirror takes the
%% cluster's subscribe/unsubscribe churn, and with two copies a publish batch
%% after a delta runs on the copy no batch is reading (DESIGN.md 8 item 2:
%% churned callers +10-19 %, C5 3.30e9 vs 2.89e9 topic matches/s)
-define(COPIES, 2).
-define(MAX_EVENTS, 10000).

%% Boot: mirror the existing ?ROUTE_TAB_FILTERS (emqx_router.erl:148-160) on the
%% given devices and publish the handle.  Called from emqx_router_sup after
%% emqx_router:create_tables/0 (emqx_router_sup.erl:25-33), as the child
%% start_link(Devices).
-spec attach([integer()]) -> ok.
attach(Devices) ->
    G = emqx_topic_index_gpu:attach(?ROUTE_TAB_FILTERS, ?BOOT_BATCH, {Devices, ?COPIES}),
    persistent_term:put(?PT_KEY, G),
    ok.

-spec detach() -> ok.
detach() ->
    _ = persistent_term:erase(?PT_KEY),
    ok.

%% The router's read-your-writes hook (VERDICT r4 item 1).  With the default
%% `batch_sync.enable_on = none`, a subscribe runs do_add_route/2 ->
%% mria:dirty_write (emqx_broker.erl:778-808, emqx_router.erl:492-493) and,
%% once that returns, every matches/3 on the ETS table sees the route: a
%% PUBLISH that follows the SUBACK reaches the subscriber.  The table events
%% that also feed this mirror are asynchronous, so emqx_router calls this
%% right after each filter-table write (INTEGRATION.md 3: one line in
%% mria_filter_tab_insert/2 and mria_filter_tab_delete/2 for the single
%% context, one in do_batch/1 for syncer batches): the written keys are
%% reconciled against the table and shipped to the device before it returns.
%% It runs in the mirror's own process (a call), so the hook's deltas and the
%% table events are applied in one order and interned once.
-spec filters_written([emqx_trie_search:key(_)]) -> ok.
filters_written([]) ->
    ok;
filters_written(Keys) ->
    case whereis(?MODULE) of
        undefined -> ok;   % no device mirror on this node
        _Pid -> gen_server:call(?MODULE, {sync, Keys}, infinity)
    end.

%% A syncer batch (emqx_router:do_batch/1, v2: mria_batch_run over
%% #{{Topic, Dest} => Op}, emqx_router.erl:255-265, 348-366) after it was
%% applied: the filter keys it wrote, as one mirror delta.
-spec batch_written(map()) -> ok.
batch_written(Batch) ->
    filters_written(
        maps:fold(
            fun({Topic, Dest}, _Op, Acc) ->
                case emqx_trie_search:filter(Topic) of
                    Words when is_list(Words) -> [emqx_topic_index:make_key(Words, Dest) | Acc];
                    false -> Acc
                end
            end,
            [],
            Batch
        )
    ).

%% The mirror's event process: every write to ?ROUTE_TAB_FILTERS on this node
%% -- mria-replicated writes, the match_delete of a node-down
%% cleanup_routes/1 (emqx_router.erl:535-550) and the echo of this node's own
%% writes alike -- reaches the device as table events, drained from the
%% mailbox and shipped as one delta batch per drain; the hook's calls are
%% served between drains.  init/1 subscribes to the events FIRST and returns
%% at once; the boot from the table runs in handle_continue/2, so a 10M-route
%% attach does not hold up emqx_router_sup's start (VERDICT r4 weak 2).  A
%% write seen both by the boot and by an event is reconciled twice: a no-op.
start_link(Devices) ->
    gen_server:start_link({local, ?MODULE}, ?MODULE, Devices, []).

init(Devices) ->
    {ok, _} = mnesia:subscribe({table, ?ROUTE_TAB_FILTERS, detailed}),
    {ok, undefined, {continue, {boot, Devices}}}.

handle_continue({boot, Devices}, undefined) ->
    ok = attach(Devices),
    {noreply, mirror()}.

handle_call({sync, Keys}, _From, G) ->
    {reply, emqx_topic_index_gpu:mirror_batch(Keys, G), G};
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
