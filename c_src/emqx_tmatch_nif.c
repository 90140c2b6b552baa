/*
 * emqx_tmatch_nif.c -- Erlang NIF over libtmatch.so (include/tmatch.h).
 *
 * The binding a maintainer adds to EMQX so that emqx_topic_index (and the
 * router's filter table, emqx_router.erl:511-516) matches on the MI355X.
 * Erlang side: src/emqx_topic_index_gpu.erl.  Not built in this image (no
 * OTP, no erl_nif.h -- SURVEY.md 8c); build line in INTEGRATION.md.
 *
 * Concurrency follows the reference's read path: every publishing process
 * calls emqx_topic_index:matches/3 on its own, lock-free, against a
 * read_concurrency ETS table (emqx_topic_index.erl:41-48).  Here:
 *   - tm_match_batch_ex / tm_first_batch / tm_apply_deltas are thread safe
 *     (include/tmatch.h): each host batch runs on its own stream and the
 *     library never holds its index lock across a GPU wait;
 *   - the NIF keeps a pool of pinned batch-buffer sets (tm_host_alloc, so a
 *     batch of <= 64k topics runs in place with no staging copies).  A dirty
 *     scheduler takes a set from the pool under `pool_mu` for a few
 *     instructions, runs its batch with no lock held, and returns the set.
 *     Nothing is locked while the GPU works.
 *
 * Functions (all on dirty schedulers; a 4k-topic batch takes ~0.1 ms):
 *   new(Device)                         -> {ok, Ref} | {error, Code}
 *   apply(Ref, [{Op, Filter, U32, Kind}]) -> ok      Op 1 insert, 0 delete;
 *                                                   Kind 0 binary, 1 words, 2 []
 *   match_batch(Ref, [Topic], Order)    -> [[U32] | badarg | system_limit]
 *                                          Order: traversal | sorted | unique
 *   first_batch(Ref, [Topic])           -> [{ok, U32} | false | badarg | system_limit]
 *   stats(Ref)                          -> #{n_keys => ..., ...}
 */
#include <erl_nif.h>
#include <string.h>

#include "tmatch.h"

#define POOL_MAX 64      /* buffer sets kept; more concurrent callers allocate and free their own */

typedef struct { void *p; uint64_t cap; } pbuf;

typedef struct bufset {
    pbuf blob, offs, hit, vals, err, uniq;
    struct bufset *next;
} bufset;

typedef struct {
    tm_index *h;
    ErlNifMutex *pool_mu;   /* guards `pool` and `npool` only */
    bufset *pool;
    int npool;
} idx_res;

static ErlNifResourceType *IDX_RT;
static ERL_NIF_TERM A_OK, A_ERROR, A_FALSE, A_BADARG, A_SYSTEM_LIMIT, A_TRAVERSAL, A_SORTED, A_UNIQUE;

/* grow-only pinned buffer (contents are not kept across a grow) */
static void *pget(tm_index *h, pbuf *b, uint64_t need) {
    if (need <= b->cap) return b->p;
    if (b->p) tm_host_free(h, b->p);
    b->cap = need + need / 2 + 4096;
    if (tm_host_alloc(h, b->cap, &b->p) != TM_OK) { b->p = NULL; b->cap = 0; }
    return b->p;
}

static void set_free(tm_index *h, bufset *s) {
    pbuf *all[] = {&s->blob, &s->offs, &s->hit, &s->vals, &s->err, &s->uniq};
    for (unsigned i = 0; i < sizeof all / sizeof all[0]; i++)
        if (all[i]->p) tm_host_free(h, all[i]->p);
    enif_free(s);
}

static bufset *set_take(idx_res *r) {
    enif_mutex_lock(r->pool_mu);
    bufset *s = r->pool;
    if (s) { r->pool = s->next; r->npool--; }
    enif_mutex_unlock(r->pool_mu);
    if (!s) {
        s = enif_alloc(sizeof *s);
        if (s) memset(s, 0, sizeof *s);
    }
    return s;
}

static void set_give(idx_res *r, bufset *s) {
    enif_mutex_lock(r->pool_mu);
    if (r->npool < POOL_MAX) { s->next = r->pool; r->pool = s; r->npool++; s = NULL; }
    enif_mutex_unlock(r->pool_mu);
    if (s) set_free(r->h, s);
}

static void idx_dtor(ErlNifEnv *env, void *obj) {
    idx_res *r = obj;
    (void)env;
    while (r->pool) { bufset *s = r->pool; r->pool = s->next; set_free(r->h, s); }
    if (r->h) tm_destroy(r->h);
    if (r->pool_mu) enif_mutex_destroy(r->pool_mu);
}

static int load(ErlNifEnv *env, void **priv, ERL_NIF_TERM info) {
    (void)priv; (void)info;
    IDX_RT = enif_open_resource_type(env, NULL, "tm_index", idx_dtor, ERL_NIF_RT_CREATE, NULL);
    A_OK = enif_make_atom(env, "ok");
    A_ERROR = enif_make_atom(env, "error");
    A_FALSE = enif_make_atom(env, "false");
    A_BADARG = enif_make_atom(env, "badarg");
    A_SYSTEM_LIMIT = enif_make_atom(env, "system_limit");
    A_TRAVERSAL = enif_make_atom(env, "traversal");
    A_SORTED = enif_make_atom(env, "sorted");
    A_UNIQUE = enif_make_atom(env, "unique");
    return IDX_RT ? 0 : 1;
}

static ERL_NIF_TERM err_term(ErlNifEnv *env, int rc) {
    return enif_make_tuple2(env, A_ERROR, enif_make_int(env, rc));
}

/* new(Device) -> {ok, Ref} | {error, Code} */
static ERL_NIF_TERM nif_new(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    int dev;
    (void)argc;
    if (!enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
    idx_res *r = enif_alloc_resource(IDX_RT, sizeof *r);
    memset(r, 0, sizeof *r);
    r->pool_mu = enif_mutex_create("tm_index_pool");
    tm_options o = {dev, 0, 0};
    int rc = tm_create(&o, &r->h);
    if (rc != TM_OK) { r->h = NULL; enif_release_resource(r); return err_term(env, rc); }
    ERL_NIF_TERM t = enif_make_resource(env, r);
    enif_release_resource(r);
    return enif_make_tuple2(env, A_OK, t);
}

/* apply(Ref, [{Op, FilterBin, U32, Kind}]) -> ok | {error, Code}
   One router-syncer batch (emqx_router_syncer.erl:297-356) = one call. */
static ERL_NIF_TERM nif_apply(ErlNifEnv *env, int argc, const ERL_NIF_TERM argv[]) {
    idx_res *r;
    unsigned n;
    (void)argc;
    if (!enif_get_resource(env, argv[0], IDX_RT, (void **)&r) || !enif_get_list_length(env, argv[1], &n))
        return enif_make_badarg(env);
    if (n == 0) return A_OK;
    uint8_t *ops = enif_alloc(n), *kinds = enif_alloc(n);
    uint32_t *vals = enif_alloc(4ull * n);
    uint64_t *offs = enif_alloc(8ull * (n + 1));
    ErlNifBinary *bins = enif_alloc(sizeof(ErlNifBinary) * n);
    uint8_t *blob = NULL;
    ERL_NIF_TERM l = argv[1], h, res = A_OK;
    uint64_t tot = 0;
    for (unsigned i = 0; enif_get_list_cell(env, l, &h, &l); i++) {
        const ERL_NIF_TERM *e;
        int ar;
        unsigned op, v, k;
        if (!enif_get_tuple(env, h, &ar, &e) || ar != 4 || !enif_get_uint(env, e[0], &op) || op > 1 ||
            !enif_inspect_binary(env, e[1], &bins[i]) || !enif_get_uint(env, e[2], &v) ||
            !enif_get_uint(env, e[3], &k) || k > 2) {
            res = enif_make_badarg(env);
            goto out;
        }
        ops[i] = (uint8_t)op; vals[i] = v; kinds[i] = (uint8_t)k; offs[i] = tot; tot += bins[i].size;
    }
    offs[n] = tot;
    blob = enif_alloc(tot + 1);
    for (unsigned i = 0; i < n; i++) memcpy(blob + offs[i], bins[i].data, bins[i].size);
    int rc = tm_apply_deltas(r->h, n, ops, blob, offs, vals, kinds);   /* thread safe, no NIF lock */
    if (rc != TM_OK) res = err_term(env, rc);
out:
    enif_free(ops); enif_free(kinds); enif_free(vals); enif_free(offs); enif_free(bins);
    if (blob) enif_free(blob);
    return res;
}

/* pack a topic list into the set's pinned blob/offs; n = list length */
static int pack_topics(ErlNifEnv *env, idx_res *r, bufset *s, ERL_NIF_TERM list, unsigned n,
                       uint8_t **blob_out, uint64_t **offs_out) {
    ERL_NIF_TERM l = list, h;
    uint64_t tot = 0;
    ErlNifBinary b;
    while (enif_get_list_cell(env, l, &h, &l)) {
        if (!enif_inspect_binary(env, h, &b)) return TM_EINVAL;
        tot += b.size;
    }
    uint8_t *blob = pget(r->h, &s->blob, tot + 16);
    uint64_t *offs = pget(r->h, &s->offs, 8ull * (n + 1));
    if (!blob || !offs) return TM_ENOMEM;
    tot = 0;
    l = list;
    for (unsigned i = 0; enif_get_list_cell(env, l, &h, &l); i++) {
        enif_inspect_binary(env, h, &b);
        offs[i] = tot;
        memcpy(blob + tot, b.data, b.size);
        tot += b.size;
    }
    offs[n] = tot;
    *blob_out = blob;
    *offs_out = offs;
    return TM_OK;
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
    bufset *s = set_take(r);
    if (!s) return err_term(env, TM_ENOMEM);
    uint8_t *blob;
    uint64_t *offs;
    int rc = pack_topics(env, r, s, argv[1], n, &blob, &offs);
    if (rc == TM_EINVAL) { set_give(r, s); return enif_make_badarg(env); }
    uint64_t *hit = pget(r->h, &s->hit, 8ull * (n + 1));
    uint8_t *err = pget(r->h, &s->err, (uint64_t)n + 1);
    uint32_t *uniq = order == TM_ORDER_UNIQUE ? pget(r->h, &s->uniq, 4ull * n) : NULL;
    /* capacity: what the set already holds, at least 16 ids per topic */
    uint64_t cap = s->vals.cap / 4 > 16ull * n ? s->vals.cap / 4 : 16ull * n + 1024;
    uint32_t *vals = pget(r->h, &s->vals, 4 * cap);
    if (rc == TM_OK && (!hit || !err || !vals || (order == TM_ORDER_UNIQUE && !uniq))) rc = TM_ENOMEM;
    if (rc == TM_OK) {
        rc = tm_match_batch_ex(r->h, n, blob, offs, hit, vals, cap, err, order, uniq);
        if (rc == TM_ECAP) {   /* offsets are valid: rerun with room for every id */
            cap = hit[n];
            vals = pget(r->h, &s->vals, 4 * cap);
            rc = vals ? tm_match_batch_ex(r->h, n, blob, offs, hit, vals, cap, err, order, uniq) : TM_ENOMEM;
        }
    }
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (unsigned i = n; rc == TM_OK && i-- > 0;) {
        ERL_NIF_TERM row;
        if (err[i]) {
            row = err[i] == 2 ? A_SYSTEM_LIMIT : A_BADARG;   /* 2: > 65536 levels */
        } else {
            const uint64_t b = hit[i], e = order == TM_ORDER_UNIQUE ? hit[i] + uniq[i] : hit[i + 1];
            row = enif_make_list(env, 0);
            for (uint64_t k = e; k-- > b;) row = enif_make_list_cell(env, enif_make_uint(env, vals[k]), row);
        }
        out = enif_make_list_cell(env, row, out);
    }
    set_give(r, s);
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
    bufset *s = set_take(r);
    if (!s) return err_term(env, TM_ENOMEM);
    uint8_t *blob;
    uint64_t *offs;
    int rc = pack_topics(env, r, s, argv[1], n, &blob, &offs);
    if (rc == TM_EINVAL) { set_give(r, s); return enif_make_badarg(env); }
    uint32_t *val = pget(r->h, &s->vals, 4ull * n);
    uint8_t *found = pget(r->h, &s->err, n);
    if (rc == TM_OK && (!val || !found)) rc = TM_ENOMEM;
    if (rc == TM_OK) rc = tm_first_batch(r->h, n, blob, offs, val, found);
    ERL_NIF_TERM out = enif_make_list(env, 0);
    for (unsigned i = n; rc == TM_OK && i-- > 0;) {
        ERL_NIF_TERM row = found[i] == 1 ? enif_make_tuple2(env, A_OK, enif_make_uint(env, val[i]))
                         : found[i] == 2 ? A_BADARG : found[i] == 3 ? A_SYSTEM_LIMIT : A_FALSE;
        out = enif_make_list_cell(env, row, out);
    }
    set_give(r, s);
    return rc == TM_OK ? out : err_term(env, rc);
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
    {"match_batch", 3, nif_match_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"first_batch", 2, nif_first_batch, ERL_NIF_DIRTY_JOB_IO_BOUND},
    {"stats", 1, nif_stats, 0},
};

ERL_NIF_INIT(emqx_tmatch_nif, funcs, load, NULL, NULL, NULL)
