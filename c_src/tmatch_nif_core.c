/*
 * tmatch_nif_core.c -- ERTS-free half of the NIF (see tmatch_nif_core.h).
 */
#include "tmatch_nif_core.h"

#include <stdlib.h>
#include <string.h>

void tmn_pool_init(tmn_pool *p, tm_index *h) {
    memset(p, 0, sizeof *p);
    p->h = h;
    pthread_mutex_init(&p->mu, NULL);
}

static void set_free(tm_index *h, tmn_set *s) {
    tmn_buf *all[] = {&s->blob, &s->offs, &s->hit, &s->vals, &s->err, &s->uniq, &s->offs64};
    for (unsigned i = 0; i < sizeof all / sizeof all[0]; i++)
        if (all[i]->p) tm_host_free(h, all[i]->p);
    free(s);
}

void tmn_pool_destroy(tmn_pool *p) {
    while (p->pool) {
        tmn_set *s = p->pool;
        p->pool = s->next;
        set_free(p->h, s);
    }
    p->npool = 0;
    pthread_mutex_destroy(&p->mu);
}

tmn_set *tmn_take(tmn_pool *p) {
    pthread_mutex_lock(&p->mu);
    tmn_set *s = p->pool;
    if (s) { p->pool = s->next; p->npool--; }
    pthread_mutex_unlock(&p->mu);
    if (!s && (s = calloc(1, sizeof *s))) s->in_flags = p->in_flags;   /* (a pooled set keeps its own: 0 after a failed device allocation) */
    if (s) s->next = NULL;
    return s;
}

void tmn_give(tmn_pool *p, tmn_set *s) {
    if (!s) return;
    pthread_mutex_lock(&p->mu);
    if (p->npool < TMN_POOL_MAX) { s->next = p->pool; p->pool = s; p->npool++; s = NULL; }
    pthread_mutex_unlock(&p->mu);
    if (s) set_free(p->h, s);
}

void *tmn_get_ex(tm_index *h, tmn_buf *b, uint64_t need, uint32_t flags) {
    if (need <= b->cap && b->p && b->flags == flags) return b->p;
    if (b->p) tm_host_free(h, b->p);
    b->p = NULL;
    b->cap = need + need / 2 + 4096;
    b->flags = flags;
    if (flags && tm_host_alloc_ex(h, b->cap, flags, &b->p) != TM_OK) { b->p = NULL; b->flags = 0; }
    if (!b->p && tm_host_alloc(h, b->cap, &b->p) != TM_OK) { b->p = NULL; b->cap = 0; }
    return b->p;
}

void *tmn_get(tm_index *h, tmn_buf *b, uint64_t need) { return tmn_get_ex(h, b, need, 0); }

int tmn_pack(tmn_set *s, tm_index *h, uint32_t n, const uint8_t *const *topics, const uint64_t *lens) {
    uint64_t tot = 0;
    for (uint32_t i = 0; i < n; i++) tot += lens[i];
    if (tot > 0xFFFFFFFFull) return TM_EINVAL;
    uint8_t *blob = tmn_get_ex(h, &s->blob, tot + 16, s->in_flags);
    uint32_t *offs = tmn_get_ex(h, &s->offs, 4ull * (n + 1), s->in_flags);
    if (!blob || !offs) return TM_ENOMEM;
    /* a device allocation that failed is not retried batch after batch (each
       retry would free a host buffer, which waits for the index's batches) */
    if (s->in_flags && (s->blob.flags != s->in_flags || s->offs.flags != s->in_flags)) s->in_flags = 0;
    if (s->offs.flags) {
        /* device memory: written once, in order, never read back (each host
           read would be a PCIe round trip); the u64 offsets tm_first_batch
           takes are kept on the host beside them */
        uint64_t *o64 = tmn_get(h, &s->offs64, 8ull * (n + 1));
        if (!o64) return TM_ENOMEM;
        tot = 0;
        for (uint32_t i = 0; i < n; i++) {
            o64[i] = tot;
            if (lens[i]) memcpy(blob + tot, topics[i], lens[i]);
            tot += lens[i];
        }
        o64[n] = tot;
        for (uint32_t i = 0; i <= n; i++) offs[i] = (uint32_t)o64[i];
        return TM_OK;
    }
    tot = 0;
    for (uint32_t i = 0; i < n; i++) {
        offs[i] = (uint32_t)tot;
        if (lens[i]) memcpy(blob + tot, topics[i], lens[i]);
        tot += lens[i];
    }
    offs[n] = (uint32_t)tot;
    return TM_OK;
}

int tmn_match(tmn_set *s, tm_index *h, uint32_t n, uint32_t order) {
    /* traversal order: (offset, count) pairs (tm_match_batch32_pairs), the
       launches' blocks never wait for each other; sorted / unique: the CSR */
    const int pairs = order == TM_ORDER_TRAVERSAL;
    uint32_t *hit = tmn_get(h, &s->hit, pairs ? 4ull * (2ull * n + 1) : 4ull * (n + 1));
    uint8_t *err = tmn_get(h, &s->err, (uint64_t)n + 1);
    uint32_t *uniq = order == TM_ORDER_UNIQUE ? tmn_get(h, &s->uniq, 4ull * n + 4) : NULL;
    /* capacity: what the set already holds, at least TMN_IDS_PER_TOPIC ids per topic */
    const uint64_t want = (uint64_t)TMN_IDS_PER_TOPIC * n + 1024;
    uint64_t cap = s->vals.cap / 4 > want ? s->vals.cap / 4 : want;
    uint32_t *vals = tmn_get(h, &s->vals, 4 * cap);
    if (!hit || !err || !vals || (order == TM_ORDER_UNIQUE && !uniq)) return TM_ENOMEM;
    cap = s->vals.cap / 4;
    int rc = pairs ? tm_match_batch32_pairs(h, n, s->blob.p, s->offs.p, hit, vals, cap, err)
                   : tm_match_batch32_ex(h, n, s->blob.p, s->offs.p, hit, vals, cap, err, order, uniq);
    /* TM_ECAP: the offsets are valid, so rerun with room for every id (again
       if concurrent inserts grew the total in between; a few times at most) */
    for (int tries = 0; rc == TM_ECAP && tries < 4; tries++) {
        s->reruns++;
        vals = tmn_get(h, &s->vals, 4ull * (pairs ? hit[2ull * n] : hit[n]));
        rc = !vals ? TM_ENOMEM
             : pairs ? tm_match_batch32_pairs(h, n, s->blob.p, s->offs.p, hit, vals, s->vals.cap / 4, err)
                     : tm_match_batch32_ex(h, n, s->blob.p, s->offs.p, hit, vals, s->vals.cap / 4, err, order, uniq);
    }
    /* err flag 4 (a batch the device failed; the library runs it again and
       returns TM_EDEVICE instead -- checked here all the same): the whole
       call fails as a device error, never as a client badarg */
    for (uint32_t i = 0; rc == TM_OK && i < n; i++)
        if (err[i] > TMN_ERR_TOO_DEEP) rc = TM_EDEVICE;
    return rc;
}

int tmn_first(tmn_set *s, tm_index *h, uint32_t n) {
    uint32_t *val = tmn_get(h, &s->vals, 4ull * n + 4);
    uint8_t *found = tmn_get(h, &s->err, (uint64_t)n + 1);
    uint64_t *o64 = tmn_get(h, &s->offs64, 8ull * (n + 1));
    if (!val || !found || !o64) return TM_ENOMEM;
    if (!s->offs.flags) {   /* (device-memory offsets: tmn_pack filled o64 already) */
        const uint32_t *o32 = s->offs.p;
        for (uint32_t i = 0; i <= n; i++) o64[i] = o32[i];   /* tm_first_batch takes u64 offsets */
    }
    return tm_first_batch(h, n, s->blob.p, o64, val, found);
}

int tmn_row(const tmn_set *s, uint32_t n, uint32_t order, uint32_t i, uint64_t *b, uint64_t *e) {
    const uint32_t *hit = s->hit.p;
    const uint8_t *err = s->err.p;
    (void)n;
    *b = *e = 0;
    if (err[i]) return err[i] <= TMN_ERR_TOO_DEEP ? err[i] : TMN_ERR_DEVICE;
    if (order == TM_ORDER_TRAVERSAL) {   /* (offset, count) pairs */
        *b = hit[2ull * i];
        *e = *b + hit[2ull * i + 1];
        return 0;
    }
    *b = hit[i];
    *e = order == TM_ORDER_UNIQUE ? hit[i] + ((const uint32_t *)s->uniq.p)[i] : hit[i + 1];
    return 0;
}

int tmn_first_row(const tmn_set *s, uint32_t i, uint32_t *v) {
    *v = ((const uint32_t *)s->vals.p)[i];
    return ((const uint8_t *)s->err.p)[i];
}

int tmn_ticket_begin(tmn_ticket *t, tm_index *h) {
    memset(t, 0, sizeof *t);
    t->h = h;
    if (pthread_mutex_init(&t->mu, NULL)) return TM_ENOMEM;
    int rc = tm_read_begin(h, &t->ticket);
    t->open = rc == TM_OK;
    if (rc != TM_OK) pthread_mutex_destroy(&t->mu);   /* a failed begin leaves nothing to end or destroy */
    return rc;
}

void tmn_ticket_end(tmn_ticket *t) {
    pthread_mutex_lock(&t->mu);
    if (t->open) {
        t->open = 0;
        (void)tm_read_end(t->h, t->ticket);
    }
    pthread_mutex_unlock(&t->mu);
}

void tmn_ticket_destroy(tmn_ticket *t) {
    tmn_ticket_end(t);
    pthread_mutex_destroy(&t->mu);
}
