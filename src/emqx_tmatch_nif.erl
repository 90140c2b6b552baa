%% emqx_tmatch_nif -- Erlang stubs of c_src/emqx_tmatch_nif.c (libtmatch.so,
%% include/tmatch.h).  Not built in this image (no OTP, SURVEY.md 8c).
-module(emqx_tmatch_nif).

-export([new/1, apply/2, commit/2, match_batch/3, first_batch/2, read_begin/1, read_end/2, epoch/1, stats/1]).
%% apply/2 is the NIF's name (c_src/emqx_tmatch_nif.c); callers always qualify it
-compile({no_auto_import, [apply/2]}).
-on_load(init/0).

-type ref() :: reference().
-type u32() :: 0..4294967295.
%% Op: 1 insert, 0 delete.  Kind: 0 binary key, 1 word list, 2 the word list [],
%% 5 an escaped word list (include/tmatch.h TM_KEY_WORDS | TM_KEY_ESCAPED).
-type delta() :: {0 | 1, binary(), u32(), 0 | 1 | 2 | 5}.
-type order() :: traversal | sorted | unique.
-type ticket() :: reference().
-export_type([ref/0, u32/0, delta/0, order/0, ticket/0]).

init() ->
    Priv =
        case code:priv_dir(emqx) of
            {error, _} -> "priv";
            Dir -> Dir
        end,
    erlang:load_nif(filename:join(Priv, "emqx_tmatch_nif"), 0).

%% A list of devices: one host image with a replica on each (tm_create_replicas);
%% {Devices, Copies}: Copies copies of the tables per device (tm_options.copies);
%% {Devices, Copies, VramInputs}: VramInputs false keeps batch inputs in pinned
%% host memory (default true: device memory the host writes, where the device's
%% memory is mapped for the host).
-spec new(integer() | [integer()] | {integer() | [integer()], 1..4} | {integer() | [integer()], 1..4, boolean()}) ->
    {ok, ref()} | {error, integer()}.
new(_Device) -> erlang:nif_error(nif_not_loaded).

%% {ok, Epoch}: the delta epoch the batch made current (include/tmatch.h "Reader epochs").
-spec apply(ref(), [delta()]) -> {ok, non_neg_integer()} | {error, integer()}.
apply(_Ref, _Deltas) -> erlang:nif_error(nif_not_loaded).

%% apply/2 through tm_commit: returns once every later batch reads a table copy
%% holding the deltas, and no batch waits on the GPU for them (the route
%% mirror's group commit).
-spec commit(ref(), [delta()]) -> {ok, non_neg_integer()} | {error, integer()}.
commit(_Ref, _Deltas) -> erlang:nif_error(nif_not_loaded).

%% {error, device}: the GPU failed the batch (never a per-topic badarg).
-spec match_batch(ref(), [binary()], order()) -> [[u32()] | badarg | system_limit] | {error, device | integer()}.
match_batch(_Ref, _Topics, _Order) -> erlang:nif_error(nif_not_loaded).

-spec first_batch(ref(), [binary()]) -> [{ok, u32()} | false | badarg | system_limit] | {error, integer()}.
first_batch(_Ref, _Topics) -> erlang:nif_error(nif_not_loaded).

%% A reader registers before its batch and unregisters after decoding it.  The
%% ticket is a resource: a reader killed before read_end ends its read when
%% the ticket is garbage collected, so the safe epoch never stays pinned.
-spec read_begin(ref()) -> {ok, ticket()}.
read_begin(_Ref) -> erlang:nif_error(nif_not_loaded).

-spec read_end(ref(), ticket()) -> ok.
read_end(_Ref, _Ticket) -> erlang:nif_error(nif_not_loaded).

%% {Current, Safe}: a kid released at epoch E may be reused once Safe >= E.
-spec epoch(ref()) -> {non_neg_integer(), non_neg_integer()}.
epoch(_Ref) -> erlang:nif_error(nif_not_loaded).

-spec stats(ref()) -> #{atom() => non_neg_integer()}.
stats(_Ref) -> erlang:nif_error(nif_not_loaded).
