/*
 * tmatch.h -- C ABI of the MI355X topic-match engine (libtmatch.so).
 *
 * Drop-in boundary for EMQX's publish-routing match path.  Plain C types only:
 * pointers, sizes, status codes; no exceptions cross this boundary.  What each
 * entry point replaces in the reference (paths relative to the reference root):
 *
 *   tm_create / tm_create_replicas / tm_destroy
 *       emqx_topic_index:new/0,1          apps/emqx/src/emqx_topic_index.erl:40-48
 *       (replicas: the node-wide replicated route table, emqx_router.erl:133-162)
 *       (the ETS ordered_set stays the source of truth on the Erlang side; this
 *        handle is its HBM mirror -- SURVEY.md 8b "Ownership")
 *   tm_apply_deltas
 *       emqx_topic_index:insert/4, delete/3 apps/emqx/src/emqx_topic_index.erl:53-62
 *       via emqx_trie_search:make_key/2     apps/emqx/src/emqx_trie_search.erl:115-128
 *       and the router's batched writes     apps/emqx/src/emqx_router.erl:255-273,483-509
 *   tm_match_batch / tm_match_batch_dev
 *       emqx_topic_index:matches/3          apps/emqx/src/emqx_topic_index.erl:76-78
 *       = emqx_trie_search:matches/3        apps/emqx/src/emqx_trie_search.erl:182-226,381-389
 *       called per publish by emqx_router:match_routes/1 (emqx_router.erl:205-212,511-516)
 *   tm_first_batch
 *       emqx_topic_index:match/2            apps/emqx/src/emqx_topic_index.erl:70-72
 *       (first key in traversal order; emqx_trie_search.erl:171-178,350-356)
 *   tm_apply_deltas_ex, tm_read_begin / tm_read_end / tm_epoch
 *       safe reuse of u32 values under lock-free readers (see "Reader epochs";
 *       emqx_topic_index.erl:41-48 is the read_concurrency contract kept)
 *   tm_stats
 *       emqx_router:stats/1 n_routes part    apps/emqx/src/emqx_router.erl:632-635
 *   tm_merge_shards
 *       no reference counterpart: the reference holds every route on every
 *       node (mria-replicated emqx_route_filters, emqx_router.erl:105-108);
 *       filter sets beyond one GPU are split into shards and the
 *       shards' hit lists, allgathered over RCCL, are merged by this call so
 *       the result equals emqx_topic_index:matches/3 over the whole set
 *
 * Keys.  An index entry is the pair (filter, value).  `value` is a caller-chosen
 * u32 (the NIF interns the Erlang {ID} term, or the whole key, to a u32).
 * Key form follows make_key/2: a binary filter with a '+'/'#' level is a word
 * list; a binary without one is a binary key; TM_KEY_WORDS forces the
 * word-list form (make_key(Words, ID) with a list); TM_KEY_EMPTY_LIST is the
 * word list [] (which has no byte form).  TM_KEY_WORDS | TM_KEY_ESCAPED is
 * a word list whose binary words may hold any bytes: words are separated by
 * '/', and inside a word "\/" stands for a '/' byte and "\\" for a '\';
 * a word written "\+" or "\#" is the binary word <<"+">> / <<"#">>, where
 * a bare "+" / "#" is the wildcard ('+' / '#' atoms).  A key with such a
 * word can never match a publish topic (a topic level is never "+" or "#",
 * never holds a '/'), but it is one of the table's keys for matches_filter/3
 * (tm_matches_filter), where it takes its place in Erlang term order.
 * Inserting an existing key and deleting a missing key are no-ops (ETS set
 * semantics, emqx_topic_index.erl:58-62).
 *
 * Output.  For each topic the matching values are written in TRAVERSAL order:
 * ascending Erlang term order of the keys {Filter, {Value}} -- word-list keys
 * (by word: '#' < '+' < binary words, shorter first), then binary keys, and
 * ascending value inside one filter.  This is exactly the order in which the
 * reference's walk visits them; its matches/3 list is the reverse
 * (match_add/2 prepends, emqx_trie_search.erl:353-354).
 * A topic with a level equal to "+" or "#" is badarg (emqx_trie_search.erl:374-375):
 * its err flag is 1 and it has no hits.
 * A topic of more than 65536 levels (longer than MQTT's 65535-byte maximum,
 * emqx_mqtt.hrl:44, so never seen from a client) is not matched: err flag 2,
 * no hits.  Err flag 4 marks a topic whose batch failed inside the device
 * (the bounded wait of a one-launch batch's look-back scan expired -- never
 * expected: a block waits only for blocks already running); its offsets and
 * values are undefined.  It is never a client error (the reference raises
 * badarg only for a '+'/'#' level): the host API (tm_match_batch*) runs such
 * a batch again once and returns TM_EDEVICE if it fails again, so its callers
 * never see err 4; a device-API caller (tm_match_batch_dev*, asynchronous)
 * finds the flags in d_out_err and submits the batch again.
 *
 * Forward progress (k_walk_small's look-back).  A block of a
 * one-launch batch waits only for blocks of its own launch (segment) that
 * come before it.  In dispatch order (TM_DEBUG_SMALL_TICKET 0), "before" is
 * blockIdx: the command processor hands a launch's workgroups to the 8 XCDs
 * round robin and each XCD starts its share in index order, so within ONE
 * launch the lowest unfinished block never waits for an unstarted one once
 * the blocks below it have left their XCD -- but the XCDs start their shares
 * independently, and with several look-back launches in flight (concurrent
 * callers, the combiner's leaders) every slot of one XCD can be held by
 * waiting blocks of one launch while the predecessor they wait for sits
 * unstarted behind another launch's waiting blocks on another XCD.  So
 * dispatch order alone does not guarantee progress on gfx950; the bounded
 * wait turns such a stall into err 4 (a rerun, then TM_EDEVICE), never a
 * wrong result.  With a start-order ticket (TM_DEBUG_SMALL_TICKET 1, the
 * default since round 6: measured free) a block
 * takes its index from an atomic counter when it starts, so every block it
 * waits for has started and runs to its publication without waiting for a
 * later one: progress by construction.
 */
#ifndef TMATCH_H
#define TMATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tm_index tm_index;

enum {
    TM_OK = 0,
    TM_EINVAL = -1,   /* bad argument (null pointer, bad op code)            */
    TM_ENOMEM = -2,   /* host or device allocation failed                    */
    TM_EDEVICE = -3,  /* HIP runtime error                                   */
    TM_ECAP = -4      /* output capacity too small: offsets are valid, ids   */
                      /* were truncated to `cap`; retry with cap >= total    */
};

enum { TM_OP_DELETE = 0, TM_OP_INSERT = 1 };
enum { TM_KEY_BINARY = 0, TM_KEY_WORDS = 1, TM_KEY_EMPTY_LIST = 2, TM_KEY_ESCAPED = 4 };

typedef struct {
    int32_t device;          /* HIP device ordinal; -1 = current device        */
    uint32_t copies;         /* copies of the tables per device (0 = 1; <= 4):
                                with 2 or more a batch after a delta runs on a
                                copy no batch is reading, which takes the delta
                                at once, instead of waiting for the batches in
                                flight on a single copy (churn, C5); without
                                deltas every batch reads the first copy       */
    uint64_t hint_keys;      /* expected number of keys (sizes tables up front) */
} tm_options;

typedef struct {
    uint64_t n_keys;         /* live keys (word-list + binary + never-matching) */
    uint64_t n_wild_keys;    /* word-list keys (trie terminals)                 */
    uint64_t n_exact_keys;   /* binary keys                                     */
    uint64_t n_dead_keys;    /* keys that can never match ('#' not last, [])     */
    uint64_t n_nodes, n_edges, n_words;
    uint64_t device_bytes;   /* HBM held by the mirror                          */
    uint64_t uploads;        /* full + patch uploads performed                   */
    uint64_t patch_bytes;    /* bytes moved by incremental patches              */
} tm_stats_t;

/* Create an empty index on a device.  opts may be NULL. */
int tm_create(const tm_options *opts, tm_index **out);
int tm_destroy(tm_index *h);

/* One host image, n device replicas (1 <= n <= 8; a device may repeat):
 * the topic-sharded mode of SURVEY.md 8e in one process, as one EMQX node
 * (one BEAM VM) drives all its GPUs.  The reference keeps one replicated route
 * table per node (emqx_router.erl:133-162); here the host key set, its
 * compiler and tm_apply_deltas run once, and every patch's staged runs are
 * copied to every replica (one pinned buffer, one H2D copy + one patch kernel
 * per device), lazily: a replica takes the patches logged since its last batch
 * when a batch is about to run there.  Each device entry holds opts->copies
 * copies (replica r is copy r % copies of device entry r / copies).  Host-API
 * batches go to the device entry with the fewest batches in flight (round
 * robin among equals); device-API calls use the entry of the calling thread's
 * current HIP device (the first one there); within an entry a batch reads its
 * first up-to-date copy, else a copy no batch is reading, else the least
 * recently used one.  opts->device is ignored; matches_filter runs on replica
 * 0.  tm_stats().device_bytes is per replica. */
int tm_create_replicas(const tm_options *opts, const int32_t *devices, uint32_t n, tm_index **out);

/* Batches (host and device API) replica r has served so far, and its device. */
int tm_replica_stats(tm_index *h, uint32_t r, uint64_t *batches, int32_t *device);

/* Apply n deltas in order (a later op on the same key wins).  Host buffers:
 * filter i is filter_bytes[filter_offsets[i] .. filter_offsets[i+1]).
 * key_flags may be NULL (all TM_KEY_BINARY).  Device upload is deferred to the
 * next match / tm_sync on the stream given there (patches are applied in
 * stream order, so a batch sees exactly the deltas applied before it). */
int tm_apply_deltas(tm_index *h, uint64_t n, const uint8_t *ops, const uint8_t *filter_bytes,
                    const uint64_t *filter_offsets, const uint32_t *values, const uint8_t *key_flags);

/* tm_apply_deltas, also returning the delta epoch the batch made current
 * (*out_epoch, may be NULL): every call with n > 0 advances the index's epoch
 * by one (see "Reader epochs" below). */
int tm_apply_deltas_ex(tm_index *h, uint64_t n, const uint8_t *ops, const uint8_t *filter_bytes,
                       const uint64_t *filter_offsets, const uint32_t *values, const uint8_t *key_flags,
                       uint64_t *out_epoch);

/* tm_apply_deltas_ex for a writer that must not slow the readers: the route
 * mirror's group commit (src/emqx_router_gpu.erl, the read-your-writes hook
 * of emqx_router.erl:483-509 under the broker pool's concurrent route writes,
 * emqx_broker.erl:778-808).  The deltas are applied to the host image, the
 * resulting patch is shipped to a copy of the tables (tm_options.copies) that
 * no batch is reading, and only then published: it returns once every batch
 * queued afterwards reads a copy holding these deltas (as tm_apply_deltas
 * does), but no batch waits on the GPU for the patch -- with tm_apply_deltas
 * every batch after a delta first waits for the batches still reading the
 * copy it patches.  While every copy has readers, tm_commit waits for one to
 * drain (bounded; past the bound, or with copies = 1, it publishes as
 * tm_apply_deltas does).  Batches do not collect these deltas before
 * tm_commit publishes them (they were queued before it returned); a
 * tm_apply_deltas running meanwhile is published with them. */
int tm_commit(tm_index *h, uint64_t n, const uint8_t *ops, const uint8_t *filter_bytes, const uint64_t *filter_offsets,
              const uint32_t *values, const uint8_t *key_flags, uint64_t *out_epoch);

/* Reader epochs: when may a caller hand a value freed by a delete to a new key?
 * The reference's readers walk a read_concurrency ETS table and decode keys
 * from it lock-free (emqx_topic_index.erl:41-48): a concurrent delete can hide
 * a key, but a reader never sees a key that does not match.  Here a reader gets
 * u32 values back and turns them into keys afterwards, so a value must not be
 * reused while a reader that may still return it is running:
 *   tm_read_begin   registers a reader at the current epoch (before it queues
 *                   its batches); *ticket identifies it;
 *   tm_read_end     unregisters it (after it has decoded its results);
 *   tm_epoch        *current = the index's epoch, *safe = the smallest epoch
 *                   of a registered reader (= *current when there is none).
 * A value freed by a delete that tm_apply_deltas_ex reported as epoch E may be
 * reused once *safe >= E: every reader still running began after the delete,
 * and its batches cannot see the old key.  No reference counterpart (ETS
 * keys are their own identity).  Thread safe; never blocks on the GPU. */
int tm_read_begin(tm_index *h, uint64_t *ticket);
int tm_read_end(tm_index *h, uint64_t ticket);
int tm_epoch(tm_index *h, uint64_t *current, uint64_t *safe);

/* Upload pending patches on `stream` (hipStream_t; NULL = the default stream). */
int tm_sync(tm_index *h, void *stream);

/* Host buffers in, host buffers out (pinned staging inside).  Blocks until the
 * hit lists are in host memory.  out_hit_offsets has n+1 entries;
 * out_err has n entries (may be NULL).
 * Thread safety: any number of threads may call tm_match_batch,
 * tm_first_batch and tm_apply_deltas on one index at once (the reference's
 * readers run concurrently on a read_concurrency ETS table,
 * emqx_topic_index.erl:41-48).  Each host-API batch runs on its own stream
 * with its own scratch (up to 16 in flight; more callers wait for one), and
 * the index lock is held only while pending deltas are shipped and the
 * kernels are queued, never while waiting for the GPU.  A batch sees every
 * delta applied before it was queued. */
int tm_match_batch(tm_index *h, uint64_t n, const uint8_t *topic_bytes, const uint64_t *topic_offsets,
                   uint64_t *out_hit_offsets, uint32_t *out_values, uint64_t cap, uint8_t *out_err);

/* Output order of a topic's hit list:
 *   TM_ORDER_TRAVERSAL  the reference's traversal order (see "Output" above)
 *   TM_ORDER_SORTED     ascending u32
 *   TM_ORDER_UNIQUE     ascending u32 without repeats -- matches/3 with
 *                       [unique] (emqx_trie_search.erl:201-211) when the NIF
 *                       interns IDs (not whole keys) to u32: the distinct
 *                       values come first in the topic's segment, the rest of
 *                       the segment is 0xFFFFFFFF, and out_unique[i] (n
 *                       entries, may be NULL) is topic i's distinct count.
 * Offsets are the same in every order. */
enum { TM_ORDER_TRAVERSAL = 0, TM_ORDER_SORTED = 1, TM_ORDER_UNIQUE = 2 };

int tm_match_batch_ex(tm_index *h, uint64_t n, const uint8_t *topic_bytes, const uint64_t *topic_offsets,
                      uint64_t *out_hit_offsets, uint32_t *out_values, uint64_t cap, uint8_t *out_err,
                      uint32_t order, uint32_t *out_unique);

/* tm_match_batch_ex with 32-bit offsets: topic_offsets[n+1] and
 * out_hit_offsets[n+1] are u32 (a batch's topic bytes and its values must each
 * stay below 2^32 -- a NIF micro-batch always does).  An in-place batch of up
 * to 65536 topics (see tm_host_alloc) in TM_ORDER_TRAVERSAL then moves half
 * the offset bytes over PCIe in each direction; any other batch is widened to
 * tm_match_batch_ex on the host.  cap is clamped to 2^32 - 1; TM_EINVAL if the
 * values exceed that.  (No reference counterpart: the NIF's own buffers.) */
int tm_match_batch32_ex(tm_index *h, uint64_t n, const uint8_t *topic_bytes, const uint32_t *topic_offsets,
                        uint32_t *out_hit_offsets, uint32_t *out_values, uint64_t cap, uint8_t *out_err,
                        uint32_t order, uint32_t *out_unique);

/* tm_match_batch32_ex in TM_ORDER_TRAVERSAL with the hit lists as per-topic
 * (first position, count) pairs instead of a CSR: out_pairs[2 i] is topic i's
 * first value in out_values, out_pairs[2 i + 1] its count, out_pairs[2 n] the
 * values' total (TM_ECAP when it exceeds cap: the pairs are valid, values past
 * cap dropped).  A topic's values are contiguous and in traversal order, as
 * in the CSR; the topics' spans are disjoint but NOT in topic order.  What
 * the NIF binds (c_src/tmatch_nif_core.c tmn_row): an in-place batch (every
 * buffer from tm_host_alloc / TM_ALLOC_VRAM) of up to 65536 topics runs in
 * one launch whose blocks each reserve their values' span with one atomic
 * and never wait for another block (no cross-block scan: a finished block
 * frees its slot at once for concurrent callers' launches, and forward
 * progress needs no argument); any other batch takes tm_match_batch32_ex and
 * is converted.  out_err is required (n entries).  (No reference counterpart:
 * the NIF builds each topic's list from its span.) */
int tm_match_batch32_pairs(tm_index *h, uint64_t n, const uint8_t *topic_bytes, const uint32_t *topic_offsets,
                           uint32_t *out_pairs, uint32_t *out_values, uint64_t cap, uint8_t *out_err);

/* tm_match_batch_dev with 32-bit offsets (traversal order): a batch of up to
 * 65536 topics reads and writes them as they are; a larger one is widened
 * into the stream's scratch, matched and narrowed on the device (two small
 * copy kernels).  For host-fed pipelines: 4 B per topic less each way. */
int tm_match_batch32_dev(tm_index *h, uint64_t n, const uint8_t *d_topic_bytes, const uint32_t *d_topic_offsets,
                         uint32_t *d_out_hit_offsets, uint32_t *d_out_values, uint64_t cap, uint8_t *d_out_err,
                         void *stream);

/* Pinned host buffers, mapped into the index's device.  A NIF keeps its
 * per-scheduler batch buffers here: when every buffer given to tm_match_batch
 * (topic bytes -- 16-byte aligned --, offsets, hit offsets, values and err if
 * not NULL) lies in tm_host_alloc memory of the same index and n <= 65536, the
 * kernels read the topics and write the hit lists in place: no staging copy
 * in, no copy out.  The same holds for tm_first_batch (out_value, out_found).
 * Other batches take the staged path; results are the same.
 * tm_host_free waits for the index's batches to finish first. */
int tm_host_alloc(tm_index *h, uint64_t bytes, void **out);
int tm_host_free(tm_index *h, void *p);

/* tm_host_alloc with flags.  TM_ALLOC_VRAM: device memory of the index's GPU
 * (fine-grained HBM) mapped into the host's address space through the PCIe
 * BAR, for a batch's INPUTS (topic bytes, offsets): the host writes it with
 * ordinary stores (write-combined: ~37 GB/s for a 4k-topic batch's 140 KB,
 * tools/study/bar_probe.hip), and an in-place batch's kernel then reads HBM --
 * no PCIe read on its critical path.  Host READS of it are uncached PCIe reads
 * (~0.6 us each): write it, never read it back.  Outputs stay in tm_host_alloc
 * memory.  Only on an index with one device (TM_EINVAL for replicas); freed by
 * tm_host_free.  flags 0 = tm_host_alloc.  (No reference counterpart: the
 * NIF's own buffers.) */
#define TM_ALLOC_VRAM 1u
int tm_host_alloc_ex(tm_index *h, uint64_t bytes, uint32_t flags, void **out);

/* Device-resident batch: every pointer is device memory; asynchronous on
 * `stream` (hipStream_t; NULL = HIP's default stream, which PyTorch's default
 * stream handle 0 also names).  d_out_hit_offsets has
 * n+1 entries and d_out_hit_offsets[n] is the total; values beyond `cap` are
 * dropped (the caller compares the total with cap after synchronising).
 * The library keeps batch scratch for the 16 most recently used streams (an
 * older stream's is released after its batches finish). */
int tm_match_batch_dev(tm_index *h, uint64_t n, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                       uint64_t *d_out_hit_offsets, uint32_t *d_out_values, uint64_t cap,
                       uint8_t *d_out_err, void *stream);

int tm_match_batch_dev_ex(tm_index *h, uint64_t n, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                          uint64_t *d_out_hit_offsets, uint32_t *d_out_values, uint64_t cap,
                          uint8_t *d_out_err, uint32_t order, uint32_t *d_out_unique, void *stream);

/* tm_match_batch_dev (traversal order) with the hit lists as per-topic (first
 * position, count) pairs: d_out_pairs[2 i] / [2 i + 1] (u32; the array 8-byte
 * aligned, 2 n + 2 entries), d_out_pairs[2 n] the values' total and
 * d_out_pairs[2 n + 1] the extent -- the end of the highest position used
 * (both saturated at 2^32 - 1; cap is clamped to 2^32 - 1).  Each topic's
 * values are contiguous and in traversal order; the topics' spans are disjoint,
 * NOT in topic order, and may leave gaps: each walk block reserves its span
 * with one atomic in one of up to 64 regions of the output (together 7/8 of
 * cap; one region per 8192 topics) or, when its region is full, in the pool
 * above them, so no counter is hot.  extent > cap means values were dropped (a
 * topic whose first position + count exceeds cap lost those values: submit
 * the batch again with a larger cap).  With one region (batches below 16k
 * topics) none are when cap >= total + 64 x the most hits of one topic (a
 * region's last reservation that did not fit wastes its tail); a larger
 * batch needs cap >= total + 4096 x the most hits of one topic and every
 * region to receive at least 7/8 of an even share of the values (its ~128+
 * walk blocks' topics are interleaved with the other regions' 64 apart, so a
 * batch whose hits are not laid out in a period of 64 topics meets it); for
 * any layout, cap >= 8 x (total + 64 x the most hits of one topic) is enough
 * (the pool alone then holds every value).
 * Two launches per batch: the walk writes its own topics' values (no
 * cross-block scan, no range lists, no emit kernel), then one small kernel
 * finishes the topics deeper than the walk's level store and those with more
 * than 8 value runs.  For a consumer that builds one list per topic (the NIF, a
 * fan-out stage): the same lists as tm_match_batch_dev, fewer passes over HBM.
 * (No reference counterpart: emqx_topic_index:matches/3 per topic,
 * emqx_topic_index.erl:54-57.) */
int tm_match_batch_dev_pairs(tm_index *h, uint64_t n, const uint8_t *d_topic_bytes, const uint64_t *d_topic_offsets,
                             uint32_t *d_out_pairs, uint32_t *d_out_values, uint64_t cap, uint8_t *d_out_err,
                             void *stream);

/* Sort each segment of a device CSR (n segments, d_hit_offsets[n+1]) in
 * place in TM_ORDER_SORTED / TM_ORDER_UNIQUE order (d_out_unique as above),
 * asynchronously on `stream`: e.g. the merged lists of tm_merge_shards, which
 * then equal one index's sorted lists exactly.  Segments past `cap` values are
 * left alone. */
int tm_sort_segments(tm_index *h, uint64_t n, const uint64_t *d_hit_offsets, uint32_t *d_values, uint64_t cap,
                     uint32_t order, uint32_t *d_out_unique, void *stream);

/* Release the batch scratch kept for `stream` (after its batches finish);
 * a caller that retires a stream calls this.  No reference counterpart. */
int tm_stream_release(tm_index *h, void *stream);

/* match/2: first hit per topic in traversal order.  out_found[i] = 1 and
 * out_value[i] = value if topic i has a match, 0 otherwise (2 = badarg,
 * 3 = more than 65536 levels). */
int tm_first_batch(tm_index *h, uint64_t n, const uint8_t *topic_bytes, const uint64_t *topic_offsets,
                   uint32_t *out_value, uint8_t *out_found);

/* emqx_topic_index:matches_filter/3 (emqx_topic_index.erl:82-84 ->
 * emqx_trie_search.erl:186-189, filter clauses :291-300): for each of n
 * subscription filters, the values of the word-list keys the reference's
 * ordered search returns, in traversal order (the reference's list is the
 * reverse).  Runs on the device over the keys in Erlang term order (rebuilt
 * after key changes; seconds at 10M keys -- a control-plane call).  Host
 * buffers; out_hit_offsets[n+1] always written; TM_ECAP when the values do
 * not fit `cap` (the first `cap` are written).  out_err[i] = 1 if filter i's
 * walk exceeded its step bound (never for a valid filter). */
int tm_matches_filter(tm_index *h, uint64_t n, const uint8_t *filter_bytes, const uint64_t *filter_offsets,
                      uint64_t *out_hit_offsets, uint32_t *out_values, uint64_t cap, uint8_t *out_err);
/* The same with a flags byte per filter (may be NULL: all plain):
 * TM_KEY_ESCAPED marks a filter given as an escaped word list (the key form
 * above) -- matches_filter(Words, Tab, Opts) with binary words that hold a
 * '/' or equal "+" / "#". */
int tm_matches_filter_ex(tm_index *h, uint64_t n, const uint8_t *filter_bytes, const uint64_t *filter_offsets,
                         const uint8_t *filter_flags, uint64_t *out_hit_offsets, uint32_t *out_values, uint64_t cap,
                         uint8_t *out_err);

int tm_stats(tm_index *h, tm_stats_t *out);

/* Filter-sharded merge (device buffers, asynchronous on `stream`; runs on the
 * current HIP device).  `world` shards matched the same n topics;
 * d_shard_hit_offsets is [world][n+1] (each shard's CSR offsets, starting at
 * 0), d_shard_values is [world][stride] (shard r's values at r*stride).  Writes
 * the merged CSR: d_out_hit_offsets[n+1] and, up to `cap`, d_out_values --
 * topic t's values of shard 0, then shard 1, ..., each in that shard's
 * traversal order (the same value set as one index holding all the keys). */
int tm_merge_shards(uint32_t world, uint64_t n, const uint64_t *d_shard_hit_offsets, const uint32_t *d_shard_values,
                    uint64_t stride, uint64_t *d_out_hit_offsets, uint32_t *d_out_values, uint64_t cap,
                    void *stream);

/* Diagnostics.  While enabled, every match batch records HIP events on its
 * stream around the main walk kernel (k_walk_small for a one-launch batch,
 * k_walk_fast for a two-phase one) and around the whole batch;
 * tm_profile_read() resolves them and returns the accumulated device times
 * (milliseconds) and the number of batches since the last reset. */
int tm_profile_enable(tm_index *h, int enable);
int tm_profile_read(tm_index *h, double *walk_ms, double *batch_ms, uint64_t *batches, int reset);

/* Test hooks (no reference counterpart; tests/test_gpu_parity.py):
 *   TM_DEBUG_LB_SPINS       the look-back wait bound (polls of one word) of the
 *   TM_DEBUG_LB_FAIL_BLOCK  next TM_DEBUG_LB_LAUNCHES one-launch batches, and
 *   TM_DEBUG_LB_LAUNCHES    the block that fails as if its wait expired
 *                           (>= 2^32: none)
 *   TM_DEBUG_PHASES         1: batches of <= 65536 topics take the two-phase
 *                           path too (walk, tails, scan, emit); 0 (default):
 *                           one launch where the index allows it
 *   TM_DEBUG_SMALL_KERNEL   the one-launch kernel of small batches: 0 the
 *                           default; 1 k_walk_small with 16
 *                           lanes per topic; 3 with 8 lanes per topic (2 named
 *                           round 5's one-lane-per-topic kernel, removed:
 *                           TM_EINVAL)
 *   TM_DEBUG_COMBINE        concurrent combined launches of small 32-bit
 *                           in-place host batches (tm_match_batch32_ex): 0 =
 *                           every batch its own launch (default 4)
 *   TM_DEBUG_CMB_GATHER     (study) microseconds a new combined launch waits
 *                           for the callers between two batches to queue
 *                           theirs (0 = none, the default)
 *   TM_DEBUG_SMALL_TICKET   1 (default): k_walk_small's blocks take a
 *                           start-order ticket (see "Forward progress"); 0:
 *                           dispatch order
 *   TM_DEBUG_PATCH_ZC       1 (default): patches up to 64 KiB are read by the
 *                           patch kernel from mapped pinned memory; 0: copied
 *                           to the device first
 *   TM_DEBUG_CMB_SPIN       microseconds a caller waiting in the combiner spins
 *                           before it sleeps (0: sleeps at once)
 *   TM_DEBUG_CMB_LAND       retired (round 6: the combined launch's outputs
 *                           landed from HBM by a copy kernel, measured slower
 *                           and removed): 0 only, TM_EINVAL otherwise
 * tm_debug_get: those settings; TM_DEBUG_COMMITS / _COMMIT_WAITS / _COMMIT_FORCED:
 * tm_commit patches, those that waited for a copy to drain, and those
 * published without an idle copy; TM_DEBUG_FAILED_BATCHES (one-launch batches whose look-back
 * failed, host API), TM_DEBUG_RETRIED_BATCHES (of those, run again) and the
 * match launches per kernel path: TM_DEBUG_PATH_PHASES (walk, tails, scan,
 * emit), TM_DEBUG_PATH_SMALL (k_walk_small), TM_DEBUG_PATH_LANE (retired:
 * always 0), TM_DEBUG_COMBINED_LAUNCHES / _BATCHES: the combiner's
 * launches and the host batches they carried, and TM_DEBUG_WIDE_NODES /
 * TM_DEBUG_DENSE_WIDE: trie nodes with a child bitmap, and those of them
 * dense enough that the walk probes their child table without it.  (Keys
 * 9-11 named the round-4 one-pass kernel's hooks; 9 and 10 now name these,
 * 11 is retired.) */
enum { TM_DEBUG_LB_SPINS = 1, TM_DEBUG_LB_FAIL_BLOCK = 2, TM_DEBUG_LB_LAUNCHES = 3, TM_DEBUG_PHASES = 4,
       TM_DEBUG_FAILED_BATCHES = 5, TM_DEBUG_RETRIED_BATCHES = 6, TM_DEBUG_PATH_PHASES = 7,
       TM_DEBUG_PATH_SMALL = 8, TM_DEBUG_PATH_LANE = 9, TM_DEBUG_SMALL_KERNEL = 10,
       TM_DEBUG_COMBINE = 12, TM_DEBUG_COMBINED_LAUNCHES = 13, TM_DEBUG_COMBINED_BATCHES = 14,
       TM_DEBUG_WIDE_NODES = 15, TM_DEBUG_DENSE_WIDE = 16, TM_DEBUG_CMB_GATHER = 17, TM_DEBUG_CMB_LAND = 18,
       TM_DEBUG_COMMITS = 19, TM_DEBUG_COMMIT_WAITS = 20, TM_DEBUG_COMMIT_FORCED = 21, TM_DEBUG_SMALL_TICKET = 22,
       TM_DEBUG_CMB_SPIN = 23, TM_DEBUG_PATCH_ZC = 24 };
int tm_debug_set(tm_index *h, uint32_t key, uint64_t value);
int tm_debug_get(tm_index *h, uint32_t key, uint64_t *value);

/* Last error text of the calling thread (h is ignored; kept for the ABI). */
const char *tm_last_error(tm_index *h);

/* ABI version: (major << 16) | minor. */
uint32_t tm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TMATCH_H */
