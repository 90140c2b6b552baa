/*
 * fake_tmatch.c -- TEST INFRASTRUCTURE: a stand-in for libtmatch's C ABI
 * (include/tmatch.h) with no device, so c_src/tmatch_nif_core.c can be
 * exercised on the CPU (tests/test_nif_core_cpu.py).  Topic i "matches" one
 * value per byte: values 1000 * i + k; a topic whose first byte is '+' is
 * badarg; one whose first byte is '!' gets err flag 4 (a batch the device
 * failed, as a library that did not retry would leave it) and one whose first
 * byte is '~' makes the call return TM_EDEVICE.  Counts host allocations and
 * batch calls.
 */
#include <stdlib.h>
#include <string.h>

#include "tmatch.h"
#include "tmatch_nif_core.h"

static long n_alloc, n_free, n_match, n_first;

int tm_host_alloc(tm_index *h, uint64_t bytes, void **out) {
    (void)h;
    *out = malloc(bytes ? bytes : 1);
    if (!*out) return TM_ENOMEM;
    n_alloc++;
    return TM_OK;
}

/* TM_ALLOC_VRAM: host memory here, counted apart; fake_vram_fail(1) makes
   such allocations fail (the NIF core then falls back to tm_host_alloc) */
static long n_vram;
static int vram_fail;
int tm_host_alloc_ex(tm_index *h, uint64_t bytes, uint32_t flags, void **out) {
    if (!flags) return tm_host_alloc(h, bytes, out);
    if (vram_fail) { *out = NULL; return TM_ENOMEM; }
    int rc = tm_host_alloc(h, bytes, out);
    if (rc == TM_OK) n_vram++;
    return rc;
}
long fake_vram_count(void) { return n_vram; }
void fake_vram_fail(int f) { vram_fail = f; }
void fake_pool_set_inputs(tmn_pool *p, uint32_t flags) { p->in_flags = flags; }

int tm_host_free(tm_index *h, void *p) {
    (void)h;
    free(p);
    n_free++;
    return TM_OK;
}

int tm_match_batch_ex(tm_index *h, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t *hit,
                      uint32_t *vals, uint64_t cap, uint8_t *err, uint32_t order, uint32_t *uniq) {
    (void)h;
    n_match++;
    hit[0] = 0;
    for (uint64_t i = 0; i < n; i++)
        if (to[i + 1] > to[i] && tb[to[i]] == '~') return TM_EDEVICE;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t len = to[i + 1] - to[i];
        err[i] = len && tb[to[i]] == '+' ? 1 : len && tb[to[i]] == '!' ? 4 : 0;
        const uint64_t c = err[i] ? 0 : len;
        for (uint64_t k = 0; k < c; k++) {
            const uint64_t pos = hit[i] + k;
            /* unique: distinct values first (here: every other one), padded */
            uint32_t v = (uint32_t)(1000 * i + k);
            if (order == TM_ORDER_UNIQUE) v = k < (c + 1) / 2 ? (uint32_t)(1000 * i + k) : 0xFFFFFFFFu;
            if (pos < cap) vals[pos] = v;
        }
        if (uniq) uniq[i] = (uint32_t)((c + 1) / 2);
        hit[i + 1] = hit[i] + c;
    }
    return hit[n] > cap ? TM_ECAP : TM_OK;
}

int tm_match_batch32_ex(tm_index *h, uint64_t n, const uint8_t *tb, const uint32_t *to, uint32_t *hit,
                        uint32_t *vals, uint64_t cap, uint8_t *err, uint32_t order, uint32_t *uniq) {
    uint64_t *o64 = malloc(8 * (n + 1)), *h64 = malloc(8 * (n + 1));
    for (uint64_t i = 0; i <= n; i++) o64[i] = to[i];
    const int rc = tm_match_batch_ex(h, n, tb, o64, h64, vals, cap, err, order, uniq);
    for (uint64_t i = 0; i <= n; i++) hit[i] = (uint32_t)h64[i];
    free(o64); free(h64);
    return rc;
}

/* pairs: the CSR's rows laid out in REVERSE topic order (the library's
   spans are disjoint but in no particular order) */
int tm_match_batch32_pairs(tm_index *h, uint64_t n, const uint8_t *tb, const uint32_t *to, uint32_t *pairs,
                           uint32_t *vals, uint64_t cap, uint8_t *err) {
    uint32_t *hit = malloc(4 * (n + 1));
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total += to[i + 1] > to[i] ? to[i + 1] - to[i] : 0;
    uint32_t *tmp = malloc(4 * (total + 1));
    int rc = tm_match_batch32_ex(h, n, tb, to, hit, tmp, total + 1, err, TM_ORDER_TRAVERSAL, NULL);
    if (rc != TM_OK) { free(hit); free(tmp); return rc; }
    uint64_t pos = 0;
    for (uint64_t j = n; j-- > 0;) {
        const uint32_t c = hit[j + 1] - hit[j];
        pairs[2 * j] = (uint32_t)pos;
        pairs[2 * j + 1] = c;
        for (uint32_t k = 0; k < c; k++, pos++)
            if (pos < cap) vals[pos] = tmp[hit[j] + k];
    }
    pairs[2 * n] = (uint32_t)pos;
    free(hit); free(tmp);
    return pos > cap ? TM_ECAP : TM_OK;
}

int tm_first_batch(tm_index *h, uint64_t n, const uint8_t *tb, const uint64_t *to, uint32_t *val, uint8_t *found) {
    (void)h;
    n_first++;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t len = to[i + 1] - to[i];
        found[i] = len && tb[to[i]] == '+' ? 2 : len ? 1 : 0;
        val[i] = found[i] == 1 ? (uint32_t)(1000 * i) : 0;
    }
    return TM_OK;
}

static long n_readers, n_read_end;
static uint64_t next_ticket = 1;

int tm_read_begin(tm_index *h, uint64_t *ticket) {
    (void)h;
    *ticket = next_ticket++;
    n_readers++;
    return TM_OK;
}

int tm_read_end(tm_index *h, uint64_t ticket) {
    (void)h; (void)ticket;
    n_readers--;
    n_read_end++;
    return TM_OK;
}

long fake_count(int what) {
    return what == 0 ? n_alloc : what == 1 ? n_free : what == 2 ? n_match : what == 3 ? n_first
         : what == 4 ? n_readers : n_read_end;
}

/* a ticket on the heap, as the NIF's resource holds one */
tmn_ticket *fake_ticket_new(void) {
    tmn_ticket *t = malloc(sizeof *t);
    if (t && tmn_ticket_begin(t, (tm_index *)0x1) != TM_OK) { free(t); t = NULL; }
    return t;
}
void fake_ticket_free(tmn_ticket *t) { tmn_ticket_destroy(t); free(t); }

/* pool / set handles for ctypes */
tmn_pool *fake_pool_new(void) {
    tmn_pool *p = malloc(sizeof *p);
    tmn_pool_init(p, (tm_index *)0x1);
    return p;
}
void fake_pool_free(tmn_pool *p) { tmn_pool_destroy(p); free(p); }
int fake_pool_size(tmn_pool *p) { return p->npool; }
uint64_t fake_set_vals_cap(tmn_set *s) { return s->vals.cap; }
uint64_t fake_set_reruns(tmn_set *s) { return s->reruns; }
const uint32_t *fake_set_vals(tmn_set *s) { return tmn_vals(s); }
