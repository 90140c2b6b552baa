/*
 * tmatch_nif_core.h -- the ERTS-free half of the NIF (c_src/emqx_tmatch_nif.c):
 * pooled pinned batch buffers, topic packing, the capacity retry of a match
 * batch and the per-topic result rows.  Plain C over libtmatch's C ABI
 * (include/tmatch.h) and pthreads, so it compiles and is tested without OTP
 * (tests/test_nif_core_cpu.py links it against a stand-in libtmatch).
 *
 * The reference's readers call emqx_topic_index:matches/3 one topic at a time
 * from every client process (emqx_broker.erl:293-298 -> emqx_router.erl:511-516);
 * the NIF gets a micro-batch of them per call and runs it with no lock held
 * while the GPU works: a dirty scheduler takes a buffer set from the pool,
 * packs the topics into it, matches, builds the rows and gives the set back.
 */
#ifndef TMATCH_NIF_CORE_H
#define TMATCH_NIF_CORE_H

#include <pthread.h>
#include <stdint.h>

#include "tmatch.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TMN_POOL_MAX 64          /* sets kept; more concurrent callers allocate and free their own */
#define TMN_IDS_PER_TOPIC 16     /* first capacity guess: values per topic */

typedef struct { void *p; uint64_t cap; uint32_t flags; } tmn_buf;   /* flags: what p is (TM_ALLOC_VRAM or 0) */

typedef struct tmn_set {         /* one caller's batch buffers (tm_host_alloc: the batch runs in place) */
    tmn_buf blob, offs, hit, vals, err, uniq;   /* offs, hit: u32 (tm_match_batch32_ex) */
    tmn_buf offs64;                              /* tm_first_batch's u64 offsets */
    uint32_t in_flags;           /* the pool's input placement (tmn_pool.in_flags) */
    uint64_t reruns;             /* batches rerun after TM_ECAP (diagnostics) */
    struct tmn_set *next;
} tmn_set;

typedef struct {
    tm_index *h;
    pthread_mutex_t mu;          /* guards pool / npool only: held for a few instructions */
    tmn_set *pool;
    int npool;
    /* TM_ALLOC_VRAM: pack the topics and offsets into device memory the host
       writes through the BAR (tm_host_alloc_ex), so the in-place kernel reads
       HBM; never read back by the host.  0: pinned host memory.  Set once,
       before the first tmn_take (the NIF: for a one-device index). */
    uint32_t in_flags;
} tmn_pool;

void tmn_pool_init(tmn_pool *p, tm_index *h);
void tmn_pool_destroy(tmn_pool *p);      /* frees every pooled set (not the index) */
tmn_set *tmn_take(tmn_pool *p);          /* NULL: out of memory */
void tmn_give(tmn_pool *p, tmn_set *s);  /* back to the pool, or freed beyond TMN_POOL_MAX */

/* grow-only pinned buffer (contents are not kept across a grow); NULL on failure */
void *tmn_get(tm_index *h, tmn_buf *b, uint64_t need);
/* the same in memory of kind `flags` (TM_ALLOC_VRAM), or pinned host memory if
   that allocation fails (b->flags says which it got) */
void *tmn_get_ex(tm_index *h, tmn_buf *b, uint64_t need, uint32_t flags);

/* Topic i is topics[i][0 .. lens[i]).  Packs them into the set's pinned blob
 * (16-byte aligned, as the in-place path needs) and u32 offsets (TM_EINVAL if
 * the topics exceed 2^32 bytes: never for a broker micro-batch). */
int tmn_pack(tmn_set *s, tm_index *h, uint32_t n, const uint8_t *const *topics, const uint64_t *lens);

/* matches/3 for the packed batch in `order` (TM_ORDER_*): traversal order
 * through tm_match_batch32_pairs (per-topic (offset, count) pairs: the launch's
 * blocks never wait for each other), sorted / unique through
 * tm_match_batch32_ex -- u32 offsets in and out, half the offset bytes of the
 * in-place batch over PCIe each way: sizes the value
 * buffer from what the set already holds (>= TMN_IDS_PER_TOPIC per topic), and
 * on TM_ECAP (offsets valid, values truncated) grows it to the exact total
 * and runs the batch again.  TM_EDEVICE: the device failed the batch (the
 * library's retry included, or a topic flagged err 4) -- a device error for
 * the whole call, never a per-topic badarg. */
int tmn_match(tmn_set *s, tm_index *h, uint32_t n, uint32_t order);

/* match/2 for the packed batch: value and found flag per topic (tm_first_batch) */
int tmn_first(tmn_set *s, tm_index *h, uint32_t n);

/* Row i of a tmn_match result: 0 and its values vals()[*b .. *e), or the
 * topic's err flag with no values: TMN_ERR_BADARG (a '+'/'#' level),
 * TMN_ERR_TOO_DEEP (more than 65536 levels), TMN_ERR_DEVICE (the batch failed
 * on the device -- tmn_match returns TM_EDEVICE for such a batch, so a caller
 * that checked its result never sees it). */
enum { TMN_ERR_BADARG = 1, TMN_ERR_TOO_DEEP = 2, TMN_ERR_DEVICE = 4 };
int tmn_row(const tmn_set *s, uint32_t n, uint32_t order, uint32_t i, uint64_t *b, uint64_t *e);
static inline const uint32_t *tmn_vals(const tmn_set *s) { return (const uint32_t *)s->vals.p; }

/* Row i of a tmn_first result: 1 and *v found, 0 none, 2 badarg, 3 too deep */
int tmn_first_row(const tmn_set *s, uint32_t i, uint32_t *v);

/* A reader's ticket (tm_read_begin / tm_read_end), held in an Erlang resource
 * by the NIF: ended exactly once -- by read_end/2, or by the resource's
 * destructor when a reader died before ending it (its term collected), so a
 * killed reader never pins the safe epoch. */
typedef struct {
    tm_index *h;
    uint64_t ticket;
    int open;
    pthread_mutex_t mu;
} tmn_ticket;

int tmn_ticket_begin(tmn_ticket *t, tm_index *h);   /* TM_OK: registered, open; else nothing to end or destroy */
void tmn_ticket_end(tmn_ticket *t);                 /* idempotent */
void tmn_ticket_destroy(tmn_ticket *t);             /* ends it if still open */

#ifdef __cplusplus
}
#endif
#endif /* TMATCH_NIF_CORE_H */
