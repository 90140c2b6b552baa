// tm_dev.h -- what the host side hands to the gfx950 kernels (tm_kernels.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "tm_layout.h"

namespace tmx {

// Read-only view of the HBM-resident index (one snapshot per batch; patches
// are applied in stream order before the batch's kernels run).
struct DevIndex {
    const VocabEntry *vocab; uint32_t vmask;
    const uint8_t *wpool;
    const Node *nodes;
    const CSlot *ctab;
    const uint32_t *vals;
    const ExactEntry *exact; uint32_t xmask;
    const uint16_t *xfp;
    const uint32_t *wseq;
    const uint32_t *wbits; uint32_t wcap;   // wide nodes' child bitmaps, bits per bitmap (tm_layout.h WIDE_LIT)
    // A walk needs a topic's level words only down to the trie's depth (no node
    // deeper than `depth` exists), unless a binary key of the topic's length
    // exists (xlen_mask bit L for L < 64, L <= xlen_max beyond): need_levels().
    uint32_t depth, xlen_max;
    uint64_t xlen_mask;
    uint32_t hdesc;   // keys with a '#' that is not last are stored (NLIT_HDESC nodes exist)
};

constexpr int FAST_L = 8;        // levels handled by the main walk kernel (LDS frontier)

// levels of an L-level topic whose words a walk must resolve (see DevIndex)
__host__ __device__ __forceinline__ uint32_t need_levels(const DevIndex &ix, uint32_t L) {
    const bool exact = L < 64 ? ((ix.xlen_mask >> L) & 1u) != 0 : L <= ix.xlen_max;
    return exact || L < ix.depth ? L : ix.depth;
}
constexpr int MID_L = 32;        // levels handled by the list kernels with an LDS frontier
constexpr int MAX_LEVELS = 65536;// MQTT topics are <= 65535 bytes
constexpr int RCAP = 8;          // terminal ranges kept per topic before the re-walk path
constexpr int DEEP_LANES = 64;   // lanes of the global-scratch (deep / overflow) kernels

enum { L_MID = 0, L_DEEP = 1, L_OVF_MID = 2, L_OVF_DEEP = 3, L_COUNT = 4 };

// Per-batch device scratch (grow-only, owned by the index).
// The one-launch kernel's (k_walk_small) look-back word of a
// block: launch tag (19 bits), state (LB_AGG: its own hit total; LB_INCL: the
// total of it and every block before it; LB_FAIL: its wait expired, or a
// predecessor's did -- every later block fails too) and the value (42 bits)
// in ONE 64-bit word, so a reader gets state and value from one coherent load
// (no acquire / release: those write back and invalidate the whole L2 of the
// XCD, under every kernel running there)
enum : uint32_t { LB_AGG = 1, LB_INCL = 2, LB_FAIL = 3 };
constexpr uint32_t LB_TAG_BITS = 19, LB_TAG_MASK = (1u << LB_TAG_BITS) - 1;
constexpr uint64_t LB_VAL_MASK = (1ull << 42) - 1;
__host__ __device__ constexpr uint64_t lb_word(uint32_t tag, uint32_t st, uint64_t v) {
    return (uint64_t)tag << 45 | (uint64_t)st << 42 | (v & LB_VAL_MASK);
}
__host__ __device__ constexpr uint32_t lb_tag(uint64_t w) { return (uint32_t)(w >> 45); }
__host__ __device__ constexpr uint32_t lb_state(uint64_t w) { return (uint32_t)(w >> 42) & 7u; }

// The look-back's bounded wait.  A block waits only for blocks that started
// before it (so they are running and publish soon); the bound keeps a lost
// publication (e.g. a predecessor's waves preempted for long) from leaving a
// spinning grid behind: past it the block and every later one flag their
// topics err 4 and raise the workspace's fail word, and the host API runs the
// batch again (tm_host.cpp retry_or_fail).
constexpr uint32_t LB_SPINS = 1u << 22;   // polls of one predecessor word (LB_SLEEP apart: >= 0.1 s)
constexpr uint32_t LB_SLEEP = 1;          // s_sleep between polls of a word not yet published (x 64 clocks)
constexpr uint32_t LB_STRIDE = 1;         // 8-B words between consecutive blocks' look-back words
struct LbCtl {
    uint32_t spins;        // the bound (LB_SPINS; tm_debug_set can lower it)
    uint32_t fail_block;   // test hook: this block acts as if its wait expired (NONE: off)
    uint32_t ticket;       // 1: k_walk_small's blocks take a start-order ticket (TM_DEBUG_SMALL_TICKET)
};

constexpr int SMALL_SEGS = 16;   // host batches one combined small launch can carry (SmallSegs)

struct Workspace {
    uint32_t *cnt;        // [n] hits per topic
    uint32_t *nr;         // [n] ranges per topic (RCAP+1 = overflow)
    uint2 *rng;           // [n * RCAP] (value offset, count)
    uint32_t *lists;      // [(L_COUNT + 1) * n] topic lists (the last one: long segments to sort)
    uint32_t *list_n;     // [L_COUNT] list lengths, [L_COUNT] reset ticket, [L_COUNT + 1] scan ticket,
                          // [L_COUNT + 2] long-segment count, [L_COUNT + 3] its reset ticket,
                          // [SM_TICK + k] k_walk_small's start-order ticket of segment k (zero between launches)
    uint64_t *blk;        // [n / TILE + 4] tile hit totals (zero between batches)
    uint64_t *sup;        // [n / (TILE * SUP) + 4] superblock hit totals (zero between batches; in blk's allocation)
    uint32_t *deep_wid;   // [DEEP_LANES * MAX_LEVELS]
    uint2 *deep_stk;      // [DEEP_LANES * (MAX_LEVELS + 1)]
    uint8_t *deep_plus;   // [DEEP_LANES * MAX_LEVELS] '+' levels of each deep lane's path
    uint64_t *look;       // [(n / SM_TOPICS + 4) * LB_STRIDE] one-launch kernels: per block, one look-back word (lb_word)
    uint32_t *pairs;      // [2 * SMALL_SEGS] pairs launches: per segment, its values counter and block ticket (zero between launches)
    uint64_t *vres;       // [VRES_WORDS] a device pairs batch's value reservations (zero between batches):
                          // region k's fill at [k * VRES_STRIDE], its failed attempts at [+1]; the pool at [VRES_POOL]
    // list lengths of the last count-mode batch that finished here ([0, L_COUNT))
    // and its topic count ([L_COUNT]; 0: none yet), written by the device into
    // mapped host memory: the next batch sizes its tail grids from them;
    // [HINT_FAIL]: set by a one-launch kernel whose look-back failed (the host
    // clears it)
    uint32_t *hint_h, *hint_d;
    uint64_t cap_n;
};

constexpr int TILE = 256;    // topics per walk block = per scan tile = per emit block
constexpr int SUP = 64;      // tiles per superblock (Workspace::sup)
constexpr int SM_TICK = L_COUNT + 4;     // Workspace::list_n words: k_walk_small's tickets, one per segment
constexpr int LIST_SLOTS = SM_TICK + SMALL_SEGS;   // Workspace::list_n entries
constexpr int HINT_FAIL = L_COUNT + 1;    // Workspace::hint_* word of the fail flag
constexpr int HINT_WORDS = L_COUNT + 2;
// A device pairs batch reserves its values' spans in VRES_K regions of the
// output (a walk block takes region blockIdx % VRES_K, each region's counter on
// a line of its own) and, when its region is full, in the pool at the top: one
// hot counter took 15.6k same-address device-scope atomics per 1M-topic batch,
// +80 us on a 250 us walk
constexpr int VRES_K = 64;
constexpr int VRES_STRIDE = 16;                      // u64 words between counters (128 B)
constexpr int VRES_POOL = VRES_K * VRES_STRIDE;
constexpr int VRES_WORDS = VRES_POOL + VRES_STRIDE;
constexpr int SM_TOPICS = 16;             // topics per block of the one-launch small-batch path
constexpr int SM_TB = 256;                // topic bytes it stages in LDS (longer topics: the lane walk)
constexpr int SM_VSTAGE = 1024;           // values of a block it stages in LDS before one contiguous write


// Pipeline entry points (tm_kernels.hip).  All asynchronous on `s`.
// phase 1: tokenise + walk + tile totals (hit_offs[n] = total becomes valid)
// phase 2: finish the scan (hit_offs[0..n)), emit the values, re-walk
//          overflowing topics, reset the device-side list counters
// ev_walk0/ev_walk1 (may be null): recorded right before / after the main walk kernel
hipError_t launch_match_phase1(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                               const uint64_t *offs, uint64_t *hit_offs, uint8_t *err, hipStream_t s,
                               hipEvent_t ev_walk0 = nullptr, hipEvent_t ev_walk1 = nullptr);
hipError_t launch_match_phase2(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                               const uint64_t *offs, uint64_t *hit_offs, uint32_t *out, uint64_t cap,
                               hipStream_t s);
// A batch with its hit lists as per-topic (first position, count) pairs
// (pairs[2 t], pairs[2 t + 1]; pairs[2 n] = the values' total, saturated at
// 2^32 - 1): k_walk_pairs writes every value itself, k_tail_pairs finishes the
// deep and overflowed topics -- two launches, no scan and no k_emit
hipError_t launch_match_pairs(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                              const uint64_t *offs, uint8_t *err, uint32_t *pairs, uint32_t *out, uint64_t cap,
                              hipStream_t s, hipEvent_t ev_walk0 = nullptr, hipEvent_t ev_walk1 = nullptr);
// The whole batch in ONE launch when the index allows it: up to SMALL_TOPICS
// topics (small_path_ok: the fallback store of k_walk_small holds the index's
// depth) on k_walk_small (16 or 8 lanes per topic); the two phases otherwise
// (or when `phases` forces them: tests of that path).  `tag` must differ
// between consecutive launches on one workspace (the one-launch look-back scan
// tells its own blocks' words from older ones by it).  A one-launch batch whose
// look-back failed flags its topics err 4 and sets ws.hint_h[HINT_FAIL].
bool small_path_ok(const DevIndex &ix, uint64_t n);
bool one_launch_ok(const DevIndex &ix);
bool lite_path_ok(const DevIndex &ix);   // k_walk_small<8>'s LITE fallback store holds every topic
// which one-launch kernel (small_kind): the default, k_walk_small with 16 / 8
// lanes per topic.  (2 named round 5's k_walk_lane, removed in round 6.)
enum { SMALL_AUTO = 0, SMALL_WAVE = 1, SMALL_WAVE8 = 3 };
enum { PATH_PHASES = 0, PATH_SMALL = 1, PATH_LANE = 2, PATH_COUNT = 3 };   // *path of launch_match (PATH_LANE: retired, 0)
hipError_t launch_match(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                        const uint64_t *offs, uint64_t *hit_offs, uint8_t *err, uint32_t *out, uint64_t cap,
                        uint32_t tag, LbCtl lb, bool phases, int small_kind, hipStream_t s,
                        hipEvent_t ev_walk0 = nullptr, hipEvent_t ev_walk1 = nullptr, int *path = nullptr);
// Several host batches in ONE one-launch small kernel (the host's combiner,
// tm_host.cpp small_combined): segment k owns the launch's blocks
// [block0, next block0), its own inputs and outputs and its own look-back
// region; a launch holds at most SMALL_SEGS
// segments of at most SMALL_TOPICS topics together.  Offsets are uint64_t or
// uint32_t for the whole launch.
struct SmallSeg {
    const uint8_t *blob; const void *offs; void *hit; uint8_t *err; uint32_t *out;
    uint64_t cap; uint32_t n, block0;
};
// pairs: the launch writes per-topic (first position, count) pairs instead of
// a CSR (hit[2 t], hit[2 t + 1]; hit[2 n] = the values' total; u32 offsets
// only): tm_match_batch32_pairs
struct SmallSegs { uint32_t count, pairs; SmallSeg s[SMALL_SEGS]; };
hipError_t launch_small_segs(const DevIndex &ix, const Workspace &ws, const SmallSegs &sg, bool u32, uint32_t tag,
                             LbCtl lb, int small_kind, hipStream_t s, int *path = nullptr);
// The one-launch small batch with 32-bit offsets in and out (hipErrorInvalidValue
// if small_path_ok refuses the batch), and the 32 <-> 64-bit offset copies
hipError_t launch_match32(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                          const uint32_t *offs, uint32_t *hit_offs, uint8_t *err, uint32_t *out, uint64_t cap,
                          uint32_t tag, LbCtl lb, int small_kind, hipStream_t s, int *path = nullptr);
hipError_t launch_offs_widen(const uint32_t *in, uint64_t *out, uint64_t m, hipStream_t s);
hipError_t launch_offs_narrow(const uint64_t *in, uint32_t *out, uint64_t m, hipStream_t s);
hipError_t launch_first(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                        const uint64_t *offs, uint32_t *out_value, uint8_t *out_found, hipStream_t s);
// filter-sharded merge of allgathered per-shard CSR hit lists (k_merge_shards)
hipError_t launch_merge_shards(uint32_t world, uint64_t n, const uint64_t *shard_hit, const uint32_t *shard_vals,
                               uint64_t stride, uint64_t *out_hit, uint32_t *out, uint64_t cap, hipStream_t s);
// sort each topic's segment of a CSR in place (ascending u32); unique: distinct
// values first, padded with 0xFFFFFFFF, distinct count in ucnt (may be null)
hipError_t launch_sort_segments(const Workspace &ws, uint64_t n, const uint64_t *hit_offs, uint32_t *out, uint64_t cap,
                                int unique, uint32_t *ucnt, hipStream_t s);
// out[0 .. min(hit[n], cap)) = src[...] (device -> device or mapped host memory)
hipError_t launch_copy_values(const uint64_t *hit_offs, uint64_t n, const uint32_t *src, uint32_t *dst, uint64_t cap,
                              hipStream_t s);
// delta upload: run i copies runs[i].n u32 words from data + runs[i].src to
// word (dst & PATCH_OFF) of table (dst >> 48), whose device address on the
// replica being patched is bases.b[table] (the same runs patch every replica)
constexpr int N_TABLES = 9;   // vocab, wpool, nodes, ctab, vals, exact, xfp, wseq, wbits
constexpr uint64_t PATCH_OFF = (1ull << 48) - 1;
struct PatchRun { uint64_t dst; uint32_t src, n; };
struct PatchBases { uint64_t b[N_TABLES]; };
hipError_t launch_patch(const PatchRun *d_runs, const uint32_t *d_data, uint64_t n_runs, PatchBases bases,
                        hipStream_t s);
// matches_filter/3 over the term-ordered word-list keys (pass 1: hit == null, per-query counts; pass 2: values)
hipError_t launch_matches_filter(uint64_t n, const uint32_t *qoff, const uint32_t *qr, const uint32_t *qbase,
                                 const uint32_t *pool, const uint64_t *koff, const uint32_t *kval, uint64_t K,
                                 uint32_t *cnt, const uint64_t *hit, uint32_t *out, uint64_t cap, uint8_t *err,
                                 hipStream_t s);

}  // namespace tmx
