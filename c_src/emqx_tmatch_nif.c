/*
 * emqx_tmatch_nif.c -- Erlang NIF over libtmatch.so (include/tmatch.h).
 *
 * The binding a maintainer adds to EMQX so that emqx_topic_index (and the
 * router's filter table, emqx_router.erl:511-516) matches on the MI355X.
 * Erlang side: src/emqx_tmatch_nif.erl, src/emqx_topic_index_gpu.erl.  Not
 * built in this image (no OTP, no erl_nif.h -- SURVEY.md 8c); build line in
 * INTEGRATION.md.  Everything that does not touch ERTS -- buffer pool, packing,
 * the TM_ECAP retry, result rows -- is in tmatch_nif_core.c, which the CPU
 * tests compile and run (tests/test_nif_core_cpu.py); this file only converts
 * terms.
 *
 * Concurrency follows the reference's read path: every publishing process
 * calls emqx_topic_index:matches/3 on its own, lock-free, against a
 * read_concurrency ETS table (emqx_topic_index.erl:41-48).  Here:
 *   - tm_match_batch_ex / tm_first_batch / tm_apply_deltas_ex are thread safe
 *     (include/tmatch.h): each host batch runs on its own stream and the
 *     library never holds its index lock across a GPU wait;
 *   - a dirty scheduler takes a pinned buffer set from the pool (a few
 *     instructions under the pool mutex), runs its batch with no lock held,
 *     and gives the set back;
 *   - readers register with the library's reader epochs (read_begin/read_end)
 *     around the batch and the decoding of its u32s, and the writer reuses a
 *     deleted key's u32 only once epoch/1's safe epoch has passed the delete's
 *     epoch (src/emqx_topic_index_gpu.erl), so no reader decodes a stale u32
 *     into a newer key.
 *
 * Functions:
 *   new(Device | [Device])                -> {ok, Ref} | {error, Code}   (a list: one replica per device)
 *   apply(Ref, [{Op, Filter, U32, Kind}]) -> {ok, Epoch} | {error, Code}
 *                                            Op 1 insert, 0 delete; Kind 0 binary, 1 words, 2 []
 *   match_batch(Ref, [Topic], Order)      -> [[U32] | badarg | system_limit] | {error, device | Code}
 *                                            Order: traversal | sorted | unique; {error, device}: the
 *                                            GPU failed the batch (never a per-topic badarg)
 *   first_batch(Ref, [Topic])             -> [{ok, U32} | false | badarg | system_limit] | {error, Code}
 *   read_begin(Ref)                       -> {ok, Ticket}   (a resource: collected unended -> the read ends)
 *   read_end(Ref, Ticket)                 -> ok
 *   epoch(Ref)                            -> {Current, Safe}
 *   stats(Ref)                            -> #{n_keys => ..., ...}
 */
#include <erl_nif.h>
#include <string.h>

#include "tmatch.h"
#include "tmatch_nif_core.h"

typedef struct {
    tm_index *h;
    tmn_pool pool;
} idx_res;

/* A reader's ticket (read_begin/1): a resource, so a reader that dies between
   read_begin and read_end -- killed, brutal_kill at shutdown -- still ends its
   read when its term is garbage collected (the destructor), and the safe epoch
   moves on; a bare integer left in the library's reader set forever would pin
   every deleted key's u32 in quarantine.  It holds a reference to
   the index resource, so the index outlives its open readers. */
typedef struct {
    idx_res *idx;
    tmn_ticket t;   /* tmatch_nif_core.c: ended exactly once */
} ticket_res;

static ErlNifResourceType *IDX_RT, *TICKET_RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_FALSE, A_TRUE, A_BADARG, A_SYSTEM_LIMIT, A_TRAVERSAL, A_SORTED, A_UNIQUE, A_DEVICE;

static void idx_dtor(ErlNifEnv *env, void *obj) {
    idx_res *r = obj;
    (void)env;
    if (!r->h) return;
    tmn_pool_destroy(&r->pool);
    tm_destroy(r->h);
}

static void ticket_dtor(ErlNifEnv *env, void *obj) {
    ticket_res *t = obj;
    (void)env;
    if (!t->idx) return;
    tmn_ticket_destroy(&t->t);
    enif_release_resource(t->idx);
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv; (void)info;
    IDX_RT = enif_open_resource_type(env, NULL, "tm_index", idx_dtor, ERL_NIF_RT_CREATE, NULL);
    TICKET_RT = enif_open_resource_type(env, NULL, "tm_read_ticket", ticket_dtor, ERL_NIF_RT_CREATE, NULL);
    A_OK = enif_make_atom(env, "ok");
    A_ERROR = enif_make_atom(env, "error");
    A_FALSE = enif_make_atom(env, "false");
    A_TRUE = enif_make_atom(env, "true");
    A_BADARG = enif_make_atom(env, "badarg");
    A_SYSTEM_LIMIT = enif_make_atom(env, "system_limit");
    A_TRAVERSAL = enif_make_atom(env, "traversal");
    A_SORTED = enif_make_atom(env, "sorted");
    A_UNIQUE = enif_make_atom(env, "unique");
    A_DEVICE = enif_make_atom(env, "device");
    return IDX_RT && TICKET_RT ? 0 : 1;
}

/* {error, device} when the GPU failed the call (TM_EDEVICE: e.g. a batch
   whose look-back failed twice, include/tmatch.h err flag 4) -- the caller
   logs it and may fall back to the ETS walk; never badarg, which the
   reference raises only for a '+'/'#' topic level (emqx_trie_search.erl:374-375);
   {error, Code} for the other library codes */
static ERL_NIF_TERM err_term(ErlNifEnv *env, int rc) {
    return enif_make_tuple2(env, A_ERROR, rc == TM_EDEVICE ? A_DEVICE : enif_make_int(env, rc));
}

/* new(Device | [Device] | {Device | [Device], Copies} | {Device | [Device], Copies, VramInputs})
       -> {ok, Ref} | {error, Code}
   A list: one host image with a replica on each device (tm_create_replicas).
   Copies: copies of the tables per device (tm_options.copies, 1..4): a batch
   after a delta runs on a copy no batch is reading instead of waiting.
   VramInputs (default true): pack batch inputs into device memory the host
   writes through the BAR (tm_host_alloc_ex TM_ALLOC_VRAM); false keeps them in
   pinned host memory. */
static ERL_NIF_TERM nif_new(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    int dev = -1, devs[8], copies = 1, arity = 0, vram = 1;
    unsigned nd = 0;
    const ERL_NIF_TERM *tup;
    ERL_NIF_TERM spec = argv[0];
    (void)argc;
    if (enif_get_tuple(env, argv[0], &arity, &tup)) {
        if ((arity != 2 && arity != 3) || !enif_get_int(env, tup[1], &copies) || copies < 1 || copies > 4)
            return enif_make_badarg(env);
        if (arity == 3) {
            if (enif_is_identical(tup[2], A_FALSE)) vram = 0;
            else if (!enif_is_identical(tup[2], A_TRUE)) return enif_make_badarg(env);
        }
        spec = tup[0];
    }
    if (enif_get_list_length(env, spec, &nd)) {
        ERL_NIF_TERM l = spec, h;
        if (nd == 0 || nd > 8) return enif_make_badarg(env);
        for (unsigned i = 0; enif_get_list_cell(env, l, &h, &l); i++)
            if (!enif_get_int(env, h, &devs[i])) return enif_make_badarg(env);
    } else if (!enif_get_int(env, spec, &dev)) {
        return enif_make_badarg(env);
    }
    idx_res *r = enif_alloc_resource(IDX_RT, sizeof *r);
    memset(r, 0, sizeof *r);
    tm_options o = {dev, (uint32_t)copies, 0};
    int rc = nd ? tm_create_replicas(&o, devs, nd, &r->h) : tm_create(&o, &r->h);
    if (rc != TM_OK) { r->h = NULL; enif_release_resource(r); return err_term(env, rc); }
    tmn_pool_init(&r->pool, r->h);
    /* batch inputs in HBM the host writes through the BAR, so the in-place
       kernel reads no host memory.  Asked of every index (a one-element device
       list is a one-device index too): tm_host_alloc_ex refuses it
       for an index spanning several devices or a device whose memory the host
       cannot map (no large BAR) -- a set then falls back to pinned host
       memory (tmn_get_ex) and stops asking */
    r->pool.in_flags = vram ? TM_ALLOC_VRAM : 0;
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, A_OK, t);
}

/* apply(Ref, [{Op, FilterBin, U32, Kind}]) -> {ok, Epoch} | {error, Code}
   One router-syncer batch (emqx_router_syncer.erl:297-356) = one call.
   commit(Ref, Deltas): the same through tm_commit -- published on a table copy
   no publish batch is reading (the route mirror's group commit,
   src/emqx_router_gpu.erl) */
static ERL_NIF_TERM apply_deltas(ErlNifEnv *env, const ERL_NIF_TERM argv[], int commit) {
    idx_res *r;
    unsigned n;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &n))
        return enif_make_badarg(env);
    uint64_t epoch = 0;
    if (n == 0) {
        tm_epoch(r->h, &epoch, NULL);
        return enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch));
    }
    uint8_t *ops = enif_alloc(n), *kinds = enif_alloc(n);
    uint32_t *vals = enif_alloc(4ull * n);
    uint64_t *offs = enif_alloc(8ull * (n + 1));
    ErlNifBinary *bins = enif_alloc(sizeof(ErlNifBinary) * n);
    uint8_t *blob = NULL;
    ERL_NIF_TERM l = argv[1], h, res;
    uint64_t tot = 0;
    for (unsigned i = 0; enif_get_list_cell(env, l, &h, &l); i++) {
        const ERL_NIF_TERM *e;
        int ar;
        unsigned op, v, k;
        if (!enif_get_tuple(env, h, &ar, &e) || ar != 4 || !enif_get_uint(env, e[0], &op) || op > 1 ||
            !enif_inspect_binary(env, e[1], &bins[i]) || !enif_get_uint(env, e[2], &v) ||
            !enif_get_uint(env, e[3], &k) || (k > 2 && k != (TM_KEY_WORDS | TM_KEY_ESCAPED))) {
            res = enif_make_badarg(env);
            goto out;
        }
        ops[i] = (uint8_t)op; vals[i] = v; kinds[i] = (uint8_t)k; offs[i] = tot; tot += bins[i].size;
    }
    offs[n] = tot;
    blob = enif_alloc(tot + 1);
    for (unsigned i = 0; i < n; i++) memcpy(blob + offs[i], bins[i].data, bins[i].size);
    int rc = commit ? tm_commit(r->h, n, ops, blob, offs, vals, kinds, &epoch)   /* thread safe, no NIF lock */
                    : tm_apply_deltas_ex(r->h, n, ops, blob, offs, vals, kinds, &epoch);
    res = rc == TM_OK ? enif_make_tuple2(env, A_OK, enif_make_uint64(env, epoch)) : err_term(env, rc);
out:
    enif_free(ops); enif_free(kinds); enif_free(vals); enif_free(offs); enif_free(bins);
    if (blob) enif_free(blob);
    return res;
}

static ERL_NIF_TERM nif_apply(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return apply_deltas(env, argv, 0);
}

static ERL_NIF_TERM nif_commit(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    (void)argc;
    return apply_deltas(env, argv, 1);
}

/* the topic list's binaries (views into the caller's terms, valid during the call) */
static int topic_views(ErlNifEnv *env, ERL_NIF_TERM list, unsigned n, const uint8_t ***ps, uint64_t **ls) {
    const uint8_t **p = enif_alloc(sizeof *p * (n + 1));
    uint64_t *len = enif_alloc(sizeof *len * (n + 1));
    ERL_NIF_TERM l = list, h;
    ErlNifBinary b;
    for (unsigned i = 0; enif_get_list_cell(env, l, &h, &l); i++) {
        if (!enif_inspect_binary(env, h, &b)) { enif_free(p); enif_free(len); return 0; }
        p[i] = b.data;
        len[i] = b.size;
    }
    *ps = p;
    *ls = len;
    return 1;
}

/* match_batch(Ref, [TopicBin], Order) -> [[U32] | badarg | system_limit]
   matches/3 for each topic of a broker micro-batch (emqx_trie_search.erl:182-226):
   traversal = ascending term order of the keys (the NIF caller reverses it, as
   match_add/2 prepends); sorted / unique = ascending u32 (unique: no repeats). */
static ERL_NIF_TERM nif_match_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    unsigned n;
    uint32_t order;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &n))
        return enif_make_badarg(env);
    if (enif_is_identical(argv[2], A_TRAVERSAL)) order = TM_ORDER_TRAVERSAL;
    else if (enif_is_identical(argv[2], A_SORTED)) order = TM_ORDER_SORTED;
    else if (enif_is_identical(argv[2], A_UNIQUE)) order = TM_ORDER_UNIQUE;
    else return enif_make_badarg(env);
    if (n == 0) return enif_make_list(env, 0);
    const uint8_t **tp;
    uint64_t *tl;
    if (!topic_views(env, argv[1], n, &tp, &tl)) return enif_make_badarg(env);
    tmn_set *s = tmn_take(&r->pool);
    int rc = s ? tmn_pack(s, r->h, n, tp, tl) : TM_ENOMEM;
    enif_free(tp); enif_free(tl);
    if (rc == TM_OK) rc = tmn_match(s, r->h, n, order);
    ERL_NIF_TERM out = enif_make_list(env, 0);
    const uint32_t *vals = s ? tmn_vals(s) : NULL;
    for (unsigned i = n; rc == TM_OK && i-- > 0;) {
        uint64_t b, e;
        const int err = tmn_row(s, n, order, i, &b, &e);
        ERL_NIF_TERM row;
        if (err == TMN_ERR_DEVICE) {   /* (tmn_match already returned TM_EDEVICE for such a batch) */
            rc = TM_EDEVICE;
            break;
        } else if (err) {
            row = err == TMN_ERR_TOO_DEEP ? A_SYSTEM_LIMIT : A_BADARG;
        } else {
            row = enif_make_list(env, 0);
            for (uint64_t k = e; k-- > b;) row = enif_make_list_cell(env, enif_make_uint(env, vals[k]), row);
        }
        out = enif_make_list_cell(env, row, out);
    }
    tmn_give(&r->pool, s);
    return rc == TM_OK ? out : err_term(env, rc);
}

/* first_batch(Ref, [TopicBin]) -> [{ok, U32} | false | badarg | system_limit]
   match/2 (emqx_trie_search.erl:171-178): the first key in traversal order. */
static ERL_NIF_TERM nif_first_batch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    unsigned n;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &n))
        return enif_make_badarg(env);
    if (n == 0) return enif_make_list(env, 0);
    const uint8_t **tp;
    uint64_t *tl;
    if (!topic_views(env, argv[1], n, &tp, &tl)) return enif_make_badarg(env);
    tmn_set *s = tmn_take(&r->pool);
    int rc = s ? tmn_pack(s, r->h, n, tp, tl) : TM_ENOMEM;
    enif_free(tp); enif_free(tl);
    if (rc == TM_OK) rc = tmn_first(s, r->h, n);
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (unsigned i = n; rc == TM_OK && i-- > 0;) {
        uint32_t v;
        const int f = tmn_first_row(s, i, &v);
        ERL_NIF_TERM row = f == 1 ? enif_make_tuple2(env, A_OK, enif_make_uint(env, v))
                         : f == 2 ? A_BADARG : f == 3 ? A_SYSTEM_LIMIT : A_FALSE;
        out = enif_make_list_cell(env, row, out);
    }
    tmn_give(&r->pool, s);
    return rc == TM_OK ? out : err_term(env, rc);
}

/* read_begin(Ref) -> {ok, Ticket}: a reader registers before its batch; the
   ticket is a resource (ticket_res) that ends the read if it is collected
   before read_end */
static ERL_NIF_TERM nif_read_begin(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r)) return enif_make_badarg(env);
    ticket_res *tk = enif_alloc_resource(TICKET_RT, sizeof *tk);
    tk->idx = NULL;
    int rc = tmn_ticket_begin(&tk->t, r->h);
    if (rc != TM_OK) {
        enif_release_resource(tk);   /* idx NULL: the destructor does nothing */
        return err_term(env, rc);
    }
    enif_keep_resource(r);
    tk->idx = r;
    ERL_NIF_TERM term = enif_make_resource(env, tk);
    enif_release_resource(tk);
    return enif_make_tuple2(env, A_OK, term);
}

/* read_end(Ref, Ticket) -> ok: after the reader has decoded its results
   (idempotent: a second call, or the ticket's later collection, does nothing) */
static ERL_NIF_TERM nif_read_end(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    ticket_res *tk;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r) ||
        !enif_get_resource(env, argv[1], TICKET_RT, (void **)&tk) || tk->idx != r)
        return enif_make_badarg(env);
    tmn_ticket_end(&tk->t);
    return A_OK;
}

/* epoch(Ref) -> {Current, Safe} (include/tmatch.h "Reader epochs") */
static ERL_NIF_TERM nif_epoch(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    uint64_t cur, safe;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r)) return enif_make_badarg(env);
    int rc = tm_epoch(r->h, &cur, &safe);
    return rc == TM_OK ? enif_make_tuple2(env, enif_make_uint64(env, cur), enif_make_uint64(env, safe))
                       : err_term(env, rc);
}

/* stats(Ref) -> map (emqx_router:stats/1's n_routes part, emqx_router.erl:632-635) */
static ERL_NIF_TERM nif_stats(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    tm_stats_t st;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r)) return enif_make_badarg(env);
    int rc = tm_stats(r->h, &st);
    if (rc != TM_OK) return err_term(env, rc);
    const char *k[] = {"n_keys", "n_wild_keys", "n_exact_keys", "n_dead_keys", "n_nodes",
                       "n_edges", "n_words", "device_bytes", "uploads", "patch_bytes"};
    const uint64_t v[] = {st.n_keys, st.n_wild_keys, st.n_exact_keys, st.n_dead_keys, st.n_nodes,
                          st.n_edges, st.n_words, st.device_bytes, st.uploads, st.patch_bytes};
    ERL_NIF_TERM keys[10], values[10], m;
    for (int i = 0; i < 10; i++) { keys[i] = enif_make_atom(env, k[i]); values[i] = enif_make_uint64(env, v[i]); }
    if (!enif_make_map_from_arrays(env, keys, values, 10, &m)) return enif_make_badarg(env);
    return m;
}

static ErlNifFunc funcs[] = {
    {"new", 1, nif_new, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"apply", 2, nif_apply, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"commit", 2, nif_commit, ERL_NIF_DIRTY_JOB_IO_BOUND},   /* (may wait for a table copy to drain) */
    {"match_batch", 3, nif_match_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"first_batch", 2, nif_first_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"read_begin", 1, nif_read_begin, 0},
    {"read_end", 2, nif_read_end, 0},
    {"epoch", 1, nif_epoch, 0},
    {"stats", 1, nif_stats, 0},
};

ERL_NIF_INIT(emqx_tmatch_nif, funcs, load, NULL, NULL, NULL)
