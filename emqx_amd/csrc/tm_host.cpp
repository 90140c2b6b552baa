// tm_host.cpp -- host side of libtmatch: the index compiler, the delta applier
// that keeps an HBM mirror of it current, and the C ABI of include/tmatch.h.
//
// The reference stores one ETS ordered_set key per (filter, ID)
// (apps/emqx/src/emqx_topic_index.erl:50-62, key construction
// apps/emqx/src/emqx_trie_search.erl:115-140).  Here every insert/delete is
// applied to host copies of the flat tables described in tm_layout.h; each
// table records which of its 4-byte words changed, and tm_sync() ships exactly
// those words to HBM with one pinned H2D copy + one scatter kernel, in stream
// order before the next batch.  Tables that grow or
// rehash are re-uploaded whole.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <map>
#include <unordered_map>
#include <unordered_set>
#include <set>
#include <vector>

#include "../../include/tmatch.h"
#include "tm_dev.h"
#include "tm_layout.h"

using namespace tmx;

namespace {

thread_local std::string g_last_error;

// ------------------------------------------------------------ dirty words

struct Dirty {
    std::vector<std::pair<uint64_t, uint64_t>> r;   // [lo, hi) in 4-byte words
    bool all = true;
    void add(uint64_t lo, uint64_t hi) {
        if (all || lo >= hi) return;
        if (!r.empty() && lo >= r.back().first && lo <= r.back().second) {
            r.back().second = std::max(r.back().second, hi);
            return;
        }
        r.push_back({lo, hi});
    }
    void set_all() { all = true; r.clear(); }
    void clear() { all = false; r.clear(); }
};

constexpr int MAX_REPLICAS = 16;  // device copies of one host image (tm_create_replicas: devices x copies)

// host vector + its HBM copy on every replica
template <class T>
struct Mirror {
    std::vector<T> h;
    T *d[MAX_REPLICAS] = {};
    uint64_t dcap = 0;   // elements allocated on each replica's device
    Dirty dirty;
    void touch(uint64_t i, uint64_t n = 1) {
        uint64_t lo = i * sizeof(T), hi = (i + n) * sizeof(T);
        dirty.add(lo / 4, (hi + 3) / 4);
    }
    uint64_t bytes() const { return h.size() * sizeof(T); }
};

struct NodeAux {
    uint32_t parent = NONE, wid = NONE, hash_cap = 0, exact_cap = 0;
    uint32_t depth = 0;                       // words on the path from the root
    uint32_t hash_roff = 0, exact_roff = 0;   // the runs' offsets in vals (the line may hold an inline value)
    uint8_t is_plus = 0;
    uint32_t bm = NONE;                       // word offset of its child bitmap in wbits (wide nodes)
    uint32_t hdesc = 0;                       // keys P/#/... ('#' not last) ending their walk here (NLIT_HDESC)
};

struct WordRef { const uint8_t *p; uint32_t n; int kind; };   // kind: 0 binary, 1 '+', 2 '#'

// literal children of a node (its nlit word also carries NLIT_HDESC)
inline uint32_t nlit_of(const Node &n) { return n.nlit & NLIT_MASK; }

}  // namespace

// Per-caller execution context.  Host-API callers (tm_match_batch /
// tm_first_batch) check one out of a pool, so concurrent callers -- every
// client process calls matches/3 at once in the reference, on a shared
// read_concurrency table (emqx_topic_index.erl:41-48) -- run their batches on
// their own streams with their own scratch and staging buffers, and wait for
// the GPU without holding the index lock.  Device-API callers
// (tm_match_batch_dev) get one per stream they pass, in a bounded LRU pool.
struct Lane {
    int r = 0;                // the replica whose tables this lane's batches read
    hipStream_t s = nullptr;
    bool owned = false;       // stream created by the library (host-API lane)
    bool busy = false;        // checked out by a host-API caller
    bool used = false;        // `done` has been recorded
    bool drained = false;     // `done` was seen complete since it was last recorded (no API call needed)
    hipEvent_t done = nullptr;   // after the lane's last batch: later patches wait for it
    uint64_t tick = 0;        // last use (LRU of device-API lanes)
    uint32_t tag = 0;         // launches on this workspace (the one-launch path's look-back tag)
    uint64_t waited = 0;      // the replica's patch (seq) this lane's stream last waited for
    Workspace w{};
    // host-API staging: mapped pinned buffers (*_dev = their device
    // addresses) and the HBM copies used for batches above ZC_TOPICS
    uint8_t *pin_in = nullptr, *pin_in_dev = nullptr; uint64_t pin_in_cap = 0;
    uint8_t *pin_out = nullptr, *pin_out_dev = nullptr; uint64_t pin_out_cap = 0;
    uint8_t *d_in = nullptr; uint64_t d_in_cap = 0;
    uint8_t *d_res = nullptr; uint64_t d_res_cap = 0;
    uint32_t *pin_vals = nullptr, *pin_vals_dev = nullptr; uint64_t pin_vals_cap = 0;
    uint32_t *d_vals = nullptr; uint64_t d_vals_cap = 0;   // sorted output: values sorted in HBM first
    uint64_t *d_o64 = nullptr, *d_h64 = nullptr; uint64_t d_o64_cap = 0, d_h64_cap = 0;   // 32-bit device API: widened offsets
};

// Patch log: a ring of the last PATCH_RING patches (numbered 1, 2, ... in the
// order they were collected).  A patch is one pinned [PatchRun x runs | u32
// data] buffer shared by every replica (one host image: collected once), and
// reaches each replica lazily -- when a batch is about to run there -- so a
// replica no batch is reading can take a patch at once while the others are
// still busy with theirs (tm_options.copies).  A slot is reused only once
// every replica has applied the patch it holds (a lagging replica is brought
// up on its patch stream then).
// 128 slots: a slot is reused only once every copy has taken its patch, and a
// copy no batch reads lags the others; with 16 slots and a route mirror's
// group commits (~12k/s on 3 copies) the reuse brought a lagging copy up and
// waited for it under the index lock, 25 us per commit (TM_HOST_TIMING)
constexpr int PATCH_RING = 128;
constexpr uint64_t PATCH_ZC_MAX = 64 << 10;   // patches up to this size are read in place by the patch kernel
struct PatchSlot {
    uint8_t *pin = nullptr; uint64_t pin_cap = 0;
    uint8_t *pin_dev = nullptr;               // its device address (mapped: small patches are read in place)
    uint64_t bytes = 0, nr = 0, seq = 0;      // the patch held: size, runs, number (0: none)
};

// One device copy of the tables.  Patches reach it on the stream of the batch
// that is about to read it, or on the replica's patch stream.  Replicas of one
// entry of tm_create_replicas' device list form a group (tm_options.copies
// copies of the tables on that device).
struct Replica {
    int device = 0, group = 0;
    hipStream_t ps = nullptr;                 // patch stream (a lagging replica brought up out of band)
    hipEvent_t last_patch = nullptr;          // event of its latest patch (every batch waits for it)
    uint8_t *pdev[PATCH_RING] = {}; uint64_t pdev_cap[PATCH_RING] = {};
    hipEvent_t pdone[PATCH_RING] = {}; bool ppending[PATCH_RING] = {};
    uint64_t applied = 0;                     // patches applied (== tm_index::patch_seq: up to date)
    uint64_t last_use = 0;                    // tick of its latest batch
    uint64_t batches = 0;                     // host-API batches served (tm_replica_stats)
};


constexpr int MAX_HOST_LANES = 16;   // concurrent host-API batches in flight, per replica
constexpr int MAX_DEV_LANES = 16;    // device-API streams with a workspace kept

// concurrent combined launches of small host batches (tm_index::cmb_leaders)
constexpr int CMB_LEADERS = 4;   // (2 / 3 / 6 measured: profiles/r4/combiner/; round 5: 2 / 3, profiles/r5/conc/leaders_*)

struct tm_index {
    // Two locks (order: mu, then img).  `mu` covers the device side: lanes,
    // the patch log, the replicas, pinned buffers, profiling.  `img` covers
    // the host image: the tables' host vectors and dirty sets, the key maps,
    // matches_filter's log.  tm_apply_deltas takes only `img`, so compiling a
    // syncer batch never blocks a match batch that has no delta to pick up: a
    // batch takes `img` only to collect deltas applied since the last one
    // (`img_dirty`), and otherwise launches on the device view cached then.
    std::mutex mu;
    std::mutex img;
    std::atomic<bool> img_dirty{true};
    bool view_ok = false;
    std::condition_variable cv;      // a host lane was released
    int nrep = 1, ngroups = 1;
    Replica rep[MAX_REPLICAS];
    uint64_t rr = 0;                 // round-robin among equally loaded replicas

    // vocab: live words, next fresh wid, per-wid reference count (trie edges +
    // exact-key levels) and slot, wids freed for reuse; a word nothing refers
    // to any more is erased, so churn through unique levels (client ids, UUIDs)
    // does not grow the tables
    Mirror<VocabEntry> vocab; uint64_t vcount = 0; uint32_t wid_next = 0;
    std::vector<uint32_t> wref, wslot, free_wids;
    Mirror<uint8_t> wpool; uint64_t wpool_dead = 0;   // bytes of erased long words (compacted later)
    Mirror<Node> nodes; std::vector<NodeAux> aux; std::vector<uint32_t> free_nodes; uint64_t live_nodes = 0;
    Mirror<CSlot> ctab; std::vector<uint32_t> free_ctab[33]; uint64_t nlinks = 0, ntables = 0;
    Mirror<uint32_t> vals; std::vector<uint32_t> free_blocks[33];
    Mirror<ExactEntry> exact; std::vector<uint32_t> xcap, xroff; uint64_t xcount = 0;
    Mirror<uint16_t> xfp;   // exact-table fingerprints, slot for slot (0 = empty)
    Mirror<uint32_t> wseq; uint64_t wseq_dead = 0;   // words of erased long exact keys
    Mirror<uint32_t> wbits; uint32_t wb_words = 0;   // wide nodes' child bitmaps, wb_words words each
    std::vector<uint32_t> free_wbits; std::set<uint32_t> wide;
    // literal edges per (level, wid) and distinct edge words per level: a wide
    // node whose children cover most of its level's words probes its child
    // table directly (its line's bitmap pointer NONE, wide_dense)
    std::unordered_map<uint64_t, uint32_t> lvl_edges;
    std::vector<uint32_t> lvl_distinct;
    bool dense_dirty = false;

    // levels a walk must resolve (DevIndex::depth / xlen_*): live nodes per
    // depth and live exact keys per level count
    std::vector<uint64_t> depth_cnt, xlen_cnt;

    std::unordered_set<std::string> dead;
    // matches_filter/3 (tm_matches_filter) keeps its own copy of the word-list
    // keys, in term order on the device.  It is built from a fuzzy snapshot
    // of the trie taken in short slices under `mu` plus the log of every
    // word-list key op since the snapshot began (replayed afterwards), and
    // follows the log from then on, so the index lock is held only for
    // slices of a few hundred microseconds and to swap the log -- never for a
    // sort, an upload or a GPU wait (matches_filter stalled every
    // match batch for a second at 10M keys).
    struct MfState {
        std::mutex mu;                        // one matches_filter call at a time (never taken by matching)
        bool log_on = false, log_lost = false;   // (under ix->img) ops logged since the snapshot / log dropped
        std::vector<std::pair<bool, std::string>> log;   // (insert?, key) -- under ix->img
        std::unordered_set<std::string> keys; // kind | value | filter of every word-list key (under mu)
        bool have_keys = false, dev_stale = true;
        std::atomic<size_t> nkeys{0};         // keys.size(), for the log bound (read under ix->img)
        std::vector<std::string> words;       // distinct binary words, byte order
        uint32_t *pool = nullptr, *val = nullptr; uint64_t *koff = nullptr, K = 0;
        uint64_t pcap = 0, vcap = 0, kcap = 0;
        uint32_t *q = nullptr; uint64_t qcap = 0;   // staging: query offsets, ranks, bases, counts
        uint8_t *err = nullptr; uint64_t *hit = nullptr; uint32_t *out = nullptr;
        uint64_t ecap = 0, ocap = 0, hcap = 0;
        hipStream_t s = nullptr;
        uint64_t snapshots = 0, slices = 0;   // diagnostics
    } mf;
    uint64_t n_wild = 0, n_exact = 0;
    uint64_t n_hdesc_keys = 0;       // '#'-not-last keys stored (DevIndex::hdesc)
    uint64_t uploads = 0, patch_bytes = 0;

    PatchSlot patch[PATCH_RING]; uint64_t patch_seq = 0;   // patches collected so far
    // Patches every batch queued from now on must see (<= patch_seq): a
    // collect by a batch publishes what it collects at once; tm_commit
    // publishes its patch only once a copy no batch is reading holds it.
    uint64_t pub_seq = 0;
    int serving[MAX_REPLICAS];       // per group: the copy tm_commit last published on (-1: none)
    // tm_commit's image changes not yet published: batches do not collect
    // them meanwhile (they were not applied before those batches were queued)
    std::atomic<int> img_hold{0};
    std::atomic<uint64_t> commits{0}, commit_waits{0}, commit_forced{0};
    DevIndex view[MAX_REPLICAS];     // each replica's device view as of the last collect_patch

    std::vector<std::unique_ptr<Lane>> lanes;
    uint64_t tick = 0;

    // caller buffers from tm_host_alloc (host address -> size, device address;
    // vram: TM_ALLOC_VRAM device memory, the same address on both sides)
    struct Pinned { uint8_t *host, *dev; uint64_t size; bool vram; };
    std::vector<Pinned> pinned;

    // reader epochs (tm_read_begin / tm_read_end / tm_epoch): the epoch
    // advances after each delta batch is applied; registered readers' epochs
    std::atomic<uint64_t> epoch{1};
    std::mutex ep_mu;
    uint64_t next_ticket = 1;
    std::map<uint64_t, uint64_t> readers;     // ticket -> epoch at tm_read_begin
    std::multiset<uint64_t> reader_epochs;

    // diagnostics (tm_profile_*)
    bool prof = false;
    struct ProfEv { hipEvent_t b0, w0, w1, b1; int device; };
    std::vector<ProfEv> prof_pending, prof_free;
    double prof_walk_ms = 0, prof_batch_ms = 0;
    uint64_t prof_batches = 0;

    // test hooks (tm_debug_set, under mu): the look-back control of the next
    // dbg_lb_launches one-launch batches, and the two-phase path forced for
    // large batches
    LbCtl dbg_lb{LB_SPINS, NONE, 0};
    // TM_DEBUG_SMALL_TICKET: k_walk_small's blocks take start-order tickets
    // (the default since round 6: forward progress by construction, measured
    // free -- a lone 4k batch 0.038 vs 0.040 ms, concurrent CSR callers
    // 3.6-3.7 vs 3.3e8, profiles/r6/ticket/)
    uint32_t small_ticket = 1;
    bool patch_zc = true;           // TM_DEBUG_PATCH_ZC: small patches read in place from pinned memory
    uint64_t dbg_lb_launches = 0;
    bool dbg_phases = false;        // TM_DEBUG_PHASES: small batches on the two-phase path too (tests)
    int small_kind = SMALL_AUTO;    // TM_DEBUG_SMALL_KERNEL: which one-launch kernel takes small batches
    std::atomic<uint64_t> failed_batches{0}, retried_batches{0};   // one-launch look-back failures seen / retried
    std::atomic<uint64_t> path_batches[PATH_COUNT] = {};             // match launches per kernel path
    // The host-batch combiner (small_combined): small in-place 32-bit batches
    // of concurrent callers queue here; up to cmb_leaders callers at a time
    // each take what is queued and run it as ONE k_walk_small launch
    // (TM_DEBUG_COMBINE: 0 = every batch its own launch)
    std::mutex cmb_mu;
    std::condition_variable cmb_gcv;  // a gathering leader waits here for more batches
    std::deque<struct SmallReq *> cmb_q;
    int cmb_running = 0;              // launches being prepared or in flight (at most cmb_leaders)
    int cmb_inflight = 0;             // host batches those launches carry
    int cmb_gathering = 0;            // leaders waiting in the gather window
    int cmb_hw = 0;                   // recent high-water mark of queued + in-flight batches
    uint64_t cmb_hw_ns = 0;           // when it was last reached
    std::atomic<int> cmb_leaders{CMB_LEADERS};
    std::atomic<int> cmb_gather_us{0};   // TM_DEBUG_CMB_GATHER
    std::atomic<int> cmb_spin_us{0};     // TM_DEBUG_CMB_SPIN: a waiting caller spins this long before it sleeps
    std::atomic<uint64_t> cmb_launches{0}, cmb_batches{0};
};

namespace {

// errors are kept per calling thread (tm_last_error): concurrent callers of
// one index each see their own
int fail(tm_index *, int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIPCHK(h, x)                                                                    \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess)                                                           \
            return fail(h, TM_EDEVICE, std::string(#x ": ") + hipGetErrorString(e_));   \
    } while (0)

// ---------------------------------------------------------------- hashing

void pack8(const uint8_t *p, uint32_t n, uint32_t &b0, uint32_t &b1);

uint64_t word_hash(const uint8_t *p, uint32_t n) {
    if (n <= VINL) {
        uint32_t b0, b1;
        pack8(p, n, b0, b1);
        return word_hash_short(b0, b1, n);
    }
    uint64_t x = FNV_OFF;
    for (uint32_t i = 0; i < n; i++) x = (x ^ p[i]) * FNV_PRIME;
    return word_hash_finish(x, n);
}

uint32_t pow2_at_least(uint64_t x) {
    uint64_t c = 16;
    while (c < x) c <<= 1;
    return (uint32_t)c;
}

// ------------------------------------------------------------------ vocab

void pack8(const uint8_t *p, uint32_t n, uint32_t &b0, uint32_t &b1) {
    b0 = b1 = 0;
    for (uint32_t i = 0; i < n && i < 8; i++) (i < 4 ? b0 : b1) |= (uint32_t)p[i] << (8 * (i % 4));
}

bool vocab_eq(tm_index *ix, const VocabEntry &e, uint64_t h, const uint8_t *p, uint32_t n) {
    if (e.tag != vocab_tag(h, n)) return false;
    if (n <= VINL) {
        uint32_t b0, b1;
        pack8(p, n, b0, b1);
        return e.b0 == b0 && e.b1 == b1;
    }
    return e.b1 == n && !memcmp(ix->wpool.h.data() + e.b0, p, n);
}

uint32_t vocab_find(tm_index *ix, const uint8_t *p, uint32_t n) {
    const uint64_t h = word_hash(p, n);
    const uint32_t mask = (uint32_t)ix->vocab.h.size() - 1;
    for (uint32_t s = (uint32_t)h & mask;; s = (s + 1) & mask) {
        const VocabEntry &e = ix->vocab.h[s];
        if (e.wid == NONE) return NONE;
        if (vocab_eq(ix, e, h, p, n)) return e.wid;
    }
}

VocabEntry empty_vocab() { VocabEntry e; memset(&e, 0, sizeof e); e.wid = NONE; return e; }

// the word bytes of an entry (for rehashing)
void vocab_bytes(tm_index *ix, const VocabEntry &e, std::string &out) {
    uint32_t n = e.tag & 0xFF;
    if (n < VINL + 1) {
        out.resize(n);
        for (uint32_t i = 0; i < n; i++) out[i] = (char)(((i < 4 ? e.b0 : e.b1) >> (8 * (i % 4))) & 0xFF);
    } else {
        out.assign(reinterpret_cast<const char *>(ix->wpool.h.data() + e.b0), e.b1);
    }
}

constexpr uint32_t VOCAB_LOAD_SHIFT = 2;   // vocab load <= 1/4
uint64_t vocab_entry_hash(tm_index *ix, const VocabEntry &e) {
    std::string w;
    vocab_bytes(ix, e, w);
    return word_hash(reinterpret_cast<const uint8_t *>(w.data()), (uint32_t)w.size());
}

void vocab_rehash(tm_index *ix, uint64_t cap) {
    std::vector<VocabEntry> nt(cap, empty_vocab());
    const uint32_t mask = (uint32_t)nt.size() - 1;
    for (const VocabEntry &e : ix->vocab.h) {
        if (e.wid == NONE) continue;
        const uint64_t h = vocab_entry_hash(ix, e);
        for (uint32_t s = (uint32_t)h & mask;; s = (s + 1) & mask)
            if (nt[s].wid == NONE) { nt[s] = e; ix->wslot[e.wid] = s; break; }
    }
    ix->vocab.h.swap(nt);
    ix->vocab.dirty.set_all();
}

void wide_cover(tm_index *ix);

void vocab_grow(tm_index *ix, uint64_t need) {
    // load <= 1/4: the walk's deferred probes resolve on the first slot
    // almost always (one round trip per topic for all its levels)
    if ((need << VOCAB_LOAD_SHIFT) <= ix->vocab.h.size()) return;
    vocab_rehash(ix, pow2_at_least(need << VOCAB_LOAD_SHIFT));
}

uint32_t vocab_intern(tm_index *ix, const uint8_t *p, uint32_t n) {
    uint32_t w = vocab_find(ix, p, n);
    if (w != NONE) return w;
    vocab_grow(ix, ix->vcount + 1);
    VocabEntry e = empty_vocab();
    const uint64_t h = word_hash(p, n);
    e.tag = vocab_tag(h, n);
    if (!ix->free_wids.empty()) { e.wid = ix->free_wids.back(); ix->free_wids.pop_back(); }
    else {
        e.wid = ix->wid_next++;
        ix->wref.push_back(0);
        ix->wslot.push_back(NONE);
        wide_cover(ix);
    }
    if (n <= VINL) {
        pack8(p, n, e.b0, e.b1);
    } else {
        uint64_t off = ix->wpool.h.size();
        ix->wpool.h.resize(off + ((n + 3) & ~3u), 0);
        memcpy(ix->wpool.h.data() + off, p, n);
        ix->wpool.touch(off, (n + 3) & ~3u);
        e.b0 = (uint32_t)off;
        e.b1 = n;
    }
    const uint32_t mask = (uint32_t)ix->vocab.h.size() - 1;
    for (uint32_t s = (uint32_t)h & mask;; s = (s + 1) & mask)
        if (ix->vocab.h[s].wid == NONE) { ix->vocab.h[s] = e; ix->vocab.touch(s); ix->wslot[e.wid] = s; break; }
    ix->vcount++;
    return e.wid;
}

// the last trie edge / exact key using word `wid` is gone: erase it
// (backward-shift deletion, as ctab_erase) and free its wid and wpool bytes
void vocab_erase(tm_index *ix, uint32_t wid) {
    auto &t = ix->vocab.h;
    const uint32_t mask = (uint32_t)t.size() - 1;
    uint32_t i = ix->wslot[wid];
    if (t[i].wid != wid) return;   // never: wslot tracks every move
    if ((t[i].tag & 0xFF) > VINL) ix->wpool_dead += (t[i].b1 + 3) & ~3u;
    for (uint32_t j = (i + 1) & mask; t[j].wid != NONE; j = (j + 1) & mask) {
        const uint32_t k = (uint32_t)vocab_entry_hash(ix, t[j]) & mask;
        const bool stays = (i <= j) ? (i < k && k <= j) : (i < k || k <= j);
        if (!stays) { t[i] = t[j]; ix->wslot[t[i].wid] = i; ix->vocab.touch(i); i = j; }
    }
    t[i] = empty_vocab();
    ix->vocab.touch(i);
    ix->wslot[wid] = NONE;
    ix->free_wids.push_back(wid);
    ix->vcount--;
}

void word_ref(tm_index *ix, uint32_t wid) { ix->wref[wid]++; }
void word_unref(tm_index *ix, uint32_t wid) {
    if (--ix->wref[wid] == 0) vocab_erase(ix, wid);
}

// ------------------------------------------------- private child tables

uint32_t cls_of(uint32_t cap);

uint32_t ctab_alloc(tm_index *ix, uint32_t cap) {
    auto &fl = ix->free_ctab[cls_of(cap)];
    uint32_t o;
    if (!fl.empty()) { o = fl.back(); fl.pop_back(); }
    else { o = (uint32_t)ix->ctab.h.size(); ix->ctab.h.resize(o + cap); }
    for (uint32_t i = 0; i < cap; i++) ix->ctab.h[o + i] = CSlot{NONE, NONE, 0, 0};
    ix->ctab.touch(o, cap);
    ix->ntables++;
    return o;
}

void ctab_free(tm_index *ix, uint32_t off, uint32_t cap) {
    ix->free_ctab[cls_of(cap)].push_back(off);
    ix->ntables--;
}

void ctab_put(tm_index *ix, uint32_t off, uint32_t mask, uint32_t wid, uint32_t child, uint64_t sum) {
    for (uint32_t s = child_hash(wid) & mask;; s = (s + 1) & mask)
        if (ix->ctab.h[off + s].wid == NONE) {
            ix->ctab.h[off + s] = CSlot{wid, child, (uint32_t)sum, (uint32_t)(sum >> 32)};
            ix->ctab.touch(off + s);
            return;
        }
}

uint32_t ctab_find(tm_index *ix, uint32_t off, uint32_t mask, uint32_t wid) {
    for (uint32_t s = child_hash(wid) & mask;; s = (s + 1) & mask) {
        const CSlot &c = ix->ctab.h[off + s];
        if (c.wid == NONE) return NONE;
        if (c.wid == wid) return s;
    }
}

// backward-shift deletion inside one private table
void ctab_erase(tm_index *ix, uint32_t off, uint32_t mask, uint32_t wid) {
    uint32_t i = ctab_find(ix, off, mask, wid);
    if (i == NONE) return;
    CSlot *t = ix->ctab.h.data() + off;
    for (uint32_t j = (i + 1) & mask; t[j].wid != NONE; j = (j + 1) & mask) {
        uint32_t k = child_hash(t[j].wid) & mask;
        bool stays = (i <= j) ? (i < k && k <= j) : (i < k || k <= j);
        if (!stays) { t[i] = t[j]; ix->ctab.touch(off + i); i = j; }
    }
    t[i] = CSlot{NONE, NONE, 0, 0};
    ix->ctab.touch(off + i);
}

// ------------------------------------------------------------- value runs

uint32_t cls_of(uint32_t cap) { uint32_t c = 0; while ((1u << c) < cap) c++; return c; }

uint32_t val_alloc(tm_index *ix, uint32_t cap) {
    auto &fl = ix->free_blocks[cls_of(cap)];
    if (!fl.empty()) { uint32_t o = fl.back(); fl.pop_back(); return o; }
    uint64_t o = ix->vals.h.size();
    ix->vals.h.resize(o + cap, 0);
    return (uint32_t)o;
}

void val_free(tm_index *ix, uint32_t off, uint32_t cap) {
    if (cap) ix->free_blocks[cls_of(cap)].push_back(off);
}

// insert v into the sorted run (off, cnt) of capacity cap; false if present
bool run_insert(tm_index *ix, uint32_t &off, uint32_t &cnt, uint32_t &cap, uint32_t v) {
    uint32_t *b = ix->vals.h.data() + off;
    uint32_t pos = (uint32_t)(std::lower_bound(b, b + cnt, v) - b);
    if (pos < cnt && b[pos] == v) return false;
    if (cnt == cap) {
        uint32_t ncap = cap ? cap * 2 : 1;
        uint32_t noff = val_alloc(ix, ncap);
        memmove(ix->vals.h.data() + noff, ix->vals.h.data() + off, sizeof(uint32_t) * cnt);
        val_free(ix, off, cap);
        off = noff; cap = ncap;
        ix->vals.touch(off, cnt);
    }
    uint32_t *r = ix->vals.h.data() + off;
    memmove(r + pos + 1, r + pos, sizeof(uint32_t) * (cnt - pos));
    r[pos] = v;
    cnt++;
    ix->vals.touch(off + pos, cnt - pos);
    return true;
}

bool run_erase(tm_index *ix, uint32_t &off, uint32_t &cnt, uint32_t &cap, uint32_t v) {
    uint32_t *b = ix->vals.h.data() + off;
    uint32_t pos = (uint32_t)(std::lower_bound(b, b + cnt, v) - b);
    if (pos >= cnt || b[pos] != v) return false;
    memmove(b + pos, b + pos + 1, sizeof(uint32_t) * (cnt - pos - 1));
    cnt--;
    if (pos < cnt) ix->vals.touch(off + pos, cnt - pos);
    if (!cnt) { val_free(ix, off, cap); off = 0; cap = 0; }
    return true;
}

// Insert or erase v in a run kept at host offset roff (capacity cap), then
// write the run's device encoding into (doff, dcnt): a single value inline.
bool run_op(tm_index *ix, bool ins, uint32_t &roff, uint32_t &cap, uint32_t &doff, uint32_t &dcnt, uint32_t v) {
    uint32_t off = roff, cnt = dcnt & RUN_CNT;
    const bool changed = ins ? run_insert(ix, off, cnt, cap, v) : run_erase(ix, off, cnt, cap, v);
    roff = off;
    if (cnt == 1) { doff = ix->vals.h[off]; dcnt = 1u | RUN_INLINE; }
    else { doff = off; dcnt = cnt; }
    return changed;
}

// ------------------------------------------------------------------ nodes

uint32_t node_new(tm_index *ix, uint32_t parent, uint32_t wid, bool is_plus) {
    uint32_t id;
    if (!ix->free_nodes.empty()) { id = ix->free_nodes.back(); ix->free_nodes.pop_back(); }
    else { id = (uint32_t)ix->nodes.h.size(); ix->nodes.h.emplace_back(); ix->aux.emplace_back(); }
    Node nd; memset(&nd, 0, sizeof nd); nd.plus = NONE;
    for (uint32_t k = 0; k < KINL; k++) { nd.kw[k] = NONE; nd.kc[k] = NONE; }
    ix->nodes.h[id] = nd;
    ix->nodes.touch(id);
    NodeAux a; a.parent = parent; a.wid = wid; a.is_plus = is_plus;
    a.depth = parent == NONE ? 0 : ix->aux[parent].depth + 1;
    ix->aux[id] = a;
    ix->live_nodes++;
    if (ix->depth_cnt.size() <= a.depth) ix->depth_cnt.resize(a.depth + 1, 0);
    ix->depth_cnt[a.depth]++;
    if (!is_plus && wid != NONE) word_ref(ix, wid);   // the edge parent -> id uses the word
    return id;
}

// literal child of `node` for word `wid`
uint32_t child_find(tm_index *ix, uint32_t node, uint32_t wid) {
    const Node &n = ix->nodes.h[node];
    if (nlit_of(n) <= KINL) {
        for (uint32_t k = 0; k < KINL; k++) if (n.kw[k] == wid) return n.kc[k];
        return NONE;
    }
    uint32_t s = ctab_find(ix, n.kw[0], n.kw[1], wid);
    return s == NONE ? NONE : ix->ctab.h[n.kw[0] + s].child;
}

void set_bloom(Node &n, uint32_t wid) {
    const uint32_t b = child_bit(child_hash(wid));
    bloom_word(n, b >> 5) |= 1u << (b & 31);
}

// ---- wide nodes' exact child bitmaps (tm_layout.h WIDE_LIT)

void wide_bit(tm_index *ix, uint32_t node, uint32_t wid, bool on) {
    const uint32_t bm = ix->aux[node].bm;
    if (bm == NONE) return;
    uint32_t &w = ix->wbits.h[bm + (wid >> 5)];
    if (on) w |= 1u << (wid & 31); else w &= ~(1u << (wid & 31));
    ix->wbits.touch(bm + (wid >> 5));
}

// (re)write node's bitmap from its child table and point the line at it
void wide_fill(tm_index *ix, uint32_t node) {
    const uint32_t bm = ix->aux[node].bm;
    std::fill(ix->wbits.h.begin() + bm, ix->wbits.h.begin() + bm + ix->wb_words, 0u);
    Node &n = ix->nodes.h[node];
    for (uint32_t i = 0; i <= n.kw[1]; i++) {
        const uint32_t w = ix->ctab.h[n.kw[0] + i].wid;
        if (w != NONE) ix->wbits.h[bm + (w >> 5)] |= 1u << (w & 31);
    }
    ix->wbits.touch(bm, ix->wb_words);
    n.kw[2] = bm;   // (wide_dense may point a dense node's line away from it again)
    ix->nodes.touch(node);
    ix->dense_dirty = true;
}

uint32_t wide_alloc(tm_index *ix) {
    if (!ix->free_wbits.empty()) { uint32_t o = ix->free_wbits.back(); ix->free_wbits.pop_back(); return o; }
    const uint32_t o = (uint32_t)ix->wbits.h.size();
    ix->wbits.h.resize(o + ix->wb_words, 0u);
    return o;
}

// bitmaps cover every wid handed out so far: grow them all (rare: the vocab
// doubles) before a new wid could be looked up in one
void wide_cover(tm_index *ix) {
    if (ix->wide.empty() || (uint64_t)ix->wb_words * 32 >= ix->wid_next) return;
    uint32_t words = std::max<uint32_t>(ix->wb_words, 1024);
    while ((uint64_t)words * 32 < ix->wid_next) words *= 2;
    ix->wb_words = words;
    ix->wbits.h.clear();
    ix->free_wbits.clear();
    for (uint32_t node : ix->wide) {
        ix->aux[node].bm = wide_alloc(ix);
        wide_fill(ix, node);
    }
    ix->wbits.dirty.set_all();
}

void to_wide(tm_index *ix, uint32_t node) {
    if (ix->wide.empty()) ix->wb_words = 0;
    ix->wide.insert(node);
    if ((uint64_t)ix->wb_words * 32 < ix->wid_next) {
        ix->aux[node].bm = NONE;
        wide_cover(ix);   // sizes the bitmaps and fills this node's too
        return;
    }
    ix->aux[node].bm = wide_alloc(ix);
    wide_fill(ix, node);
}

void from_wide(tm_index *ix, uint32_t node) {
    ix->free_wbits.push_back(ix->aux[node].bm);
    ix->aux[node].bm = NONE;
    ix->wide.erase(node);
    Node &n = ix->nodes.h[node];
    for (uint32_t j = 0; j < 6; j++) bloom_word(n, j) = 0;
    for (uint32_t i = 0; i <= n.kw[1]; i++) {
        const uint32_t w = ix->ctab.h[n.kw[0] + i].wid;
        if (w != NONE) set_bloom(n, w);
    }
    ix->nodes.touch(node);
}

// literal-children Bloom of node q (PSUM_BLOOM bits), all ones past PSUM_BLOOM children
uint64_t lit_bloom(tm_index *ix, uint32_t q) {
    const Node &n = ix->nodes.h[q];
    uint64_t m = 0;
    auto add = [&](uint32_t wid) { m |= 1ull << psum_bit(child_hash(wid)); };
    if (nlit_of(n) <= KINL) {
        for (uint32_t k = 0; k < KINL; k++) if (n.kw[k] != NONE) add(n.kw[k]);
    } else if (nlit_of(n) > PSUM_BLOOM) {
        m = (1ull << PSUM_BLOOM) - 1;
    } else {
        for (uint32_t i = 0; i <= n.kw[1]; i++) if (ix->ctab.h[n.kw[0] + i].wid != NONE) add(ix->ctab.h[n.kw[0] + i].wid);
    }
    return m;
}

uint64_t node_flags(const Node &n) {
    return (n.hash_cnt ? PSUM_HASH : 0) | (n.exact_cnt ? PSUM_EXACT : 0) | (n.plus != NONE ? PSUM_PLUS : 0) |
           ((n.nlit & NLIT_HDESC) ? PSUM_HDESC : 0);
}

// summary of node q as its parent keeps it (tm_layout.h PSUM_*)
uint64_t node_psum(tm_index *ix, uint32_t q) {
    const Node &n = ix->nodes.h[q];
    uint64_t m = node_flags(n) | lit_bloom(ix, q) << PSUM_BQ;
    if (n.plus != NONE) m |= node_flags(ix->nodes.h[n.plus]) << PSUM_QQ | lit_bloom(ix, n.plus) << PSUM_BQQ;
    return m;
}

// node x changed: refresh its parent's summary of it -- the parent line's psum
// for a '+' child, the child-table slot for a literal child of a table-mode
// parent (inline-mode parents keep no per-child summary)
void summary_refresh1(tm_index *ix, uint32_t x);
void summary_refresh(tm_index *ix, uint32_t x) {
    // x's summary sits in its parent; the parent's own summary (in the
    // grandparent) covers x too when x is the parent's '+' child
    summary_refresh1(ix, x);
    if (x != ROOT && ix->aux[x].is_plus) summary_refresh1(ix, ix->aux[x].parent);
}

void summary_refresh1(tm_index *ix, uint32_t x) {
    if (x == ROOT) return;
    const NodeAux &a = ix->aux[x];
    const uint32_t p = a.parent;
    Node &pn = ix->nodes.h[p];
    if (a.is_plus) {
        if (pn.plus != x) return;
        const uint64_t m = node_psum(ix, x);
        if (pn.psum_lo != (uint32_t)m || pn.psum_hi != (uint32_t)(m >> 32)) {
            pn.psum_lo = (uint32_t)m; pn.psum_hi = (uint32_t)(m >> 32);
            ix->nodes.touch(p);
        }
        return;
    }
    if (nlit_of(pn) <= KINL) return;
    const uint32_t sl = ctab_find(ix, pn.kw[0], pn.kw[1], a.wid);
    if (sl == NONE) return;
    CSlot &c = ix->ctab.h[pn.kw[0] + sl];
    if (c.child != x) return;
    const uint64_t m = node_psum(ix, x);
    if (c.sum_lo != (uint32_t)m || c.sum_hi != (uint32_t)(m >> 32)) {
        c.sum_lo = (uint32_t)m; c.sum_hi = (uint32_t)(m >> 32);
        ix->ctab.touch(pn.kw[0] + sl);
    }
}

// move a node's children into a private table of `cap` slots (cap = pow2)
void to_table(tm_index *ix, uint32_t node, uint32_t cap) {
    Node &n = ix->nodes.h[node];
    std::vector<CSlot> kids;
    if (nlit_of(n) <= KINL) {
        for (uint32_t k = 0; k < KINL; k++)
            if (n.kw[k] != NONE) {
                const uint64_t m = node_psum(ix, n.kc[k]);
                kids.push_back({n.kw[k], n.kc[k], (uint32_t)m, (uint32_t)(m >> 32)});
            }
    } else {
        for (uint32_t i = 0; i <= n.kw[1]; i++) if (ix->ctab.h[n.kw[0] + i].wid != NONE) kids.push_back(ix->ctab.h[n.kw[0] + i]);
        ctab_free(ix, n.kw[0], n.kw[1] + 1);
    }
    uint32_t off = ctab_alloc(ix, cap);
    Node &m = ix->nodes.h[node];
    for (uint32_t j = 0; j < 6; j++) bloom_word(m, j) = 0;
    for (auto &c : kids) {
        ctab_put(ix, off, cap - 1, c.wid, c.child, (uint64_t)c.sum_hi << 32 | c.sum_lo);
        set_bloom(m, c.wid);
    }
    m.kw[0] = off; m.kw[1] = cap - 1;
    if (ix->aux[node].bm != NONE) {   // wide: the bitmap, not the Bloom (wide_dense decides again)
        m.kw[2] = ix->aux[node].bm;
        ix->dense_dirty = true;
    }
}

// A literal edge with word `wid` appears at / leaves level `lvl`.
void lvl_edge(tm_index *ix, uint32_t lvl, uint32_t wid, bool add) {
    const uint64_t k = (uint64_t)lvl << 32 | wid;
    if (ix->lvl_distinct.size() <= lvl) ix->lvl_distinct.resize(lvl + 1, 0);
    if (add) {
        if (ix->lvl_edges[k]++ == 0) { ix->lvl_distinct[lvl]++; ix->dense_dirty |= !ix->wide.empty(); }
    } else {
        auto it = ix->lvl_edges.find(k);
        if (it != ix->lvl_edges.end() && --it->second == 0) {
            ix->lvl_edges.erase(it);
            ix->lvl_distinct[lvl]--;
            ix->dense_dirty |= !ix->wide.empty();
        }
    }
}

// Dense wide nodes.  A wide node's bitmap line answers "may w be a child?"
// before its child table is probed: one more L2 request in the chain of every
// visit, worth it only where the answer is often no.  C3's level-1 nodes and
// the root's '+' child have (nearly) every word of their level as a child, so
// their bitmap is pure overhead on almost every topic; there the line's
// bitmap pointer is NONE and the walk probes the table at once.  Dense: the
// node's children are at least DENSE_NUM/DENSE_DEN of the distinct words
// that appear as literal edges at its children's level anywhere in the trie
// (the words a topic reaching it is likely to carry there).  Re-evaluated for
// every wide node when an edge count changed, before the next patch.
constexpr uint64_t DENSE_NUM = 3, DENSE_DEN = 5;
void wide_dense(tm_index *ix) {
    if (!ix->dense_dirty) return;
    ix->dense_dirty = false;
    for (uint32_t node : ix->wide) {
        Node &n = ix->nodes.h[node];
        const uint32_t lvl = ix->aux[node].depth;
        const uint64_t distinct = lvl < ix->lvl_distinct.size() ? ix->lvl_distinct[lvl] : 0;
        const bool dense = (uint64_t)nlit_of(n) * DENSE_DEN >= distinct * DENSE_NUM;
        const uint32_t want = dense ? NONE : ix->aux[node].bm;
        if (n.kw[2] != want) { n.kw[2] = want; ix->nodes.touch(node); }
    }
}

void child_add(tm_index *ix, uint32_t node, uint32_t wid, uint32_t child) {
    ix->nlinks++;
    lvl_edge(ix, ix->aux[node].depth, wid, true);
    if (ix->aux[node].bm != NONE) ix->dense_dirty = true;
    Node *n = &ix->nodes.h[node];
    if (nlit_of(*n) < KINL) {
        for (uint32_t k = 0; k < KINL; k++)
            if (n->kw[k] == NONE) { n->kw[k] = wid; n->kc[k] = child; break; }
    } else {
        if (nlit_of(*n) == KINL) to_table(ix, node, 16);
        else if ((nlit_of(*n) + 1) * 2 > n->kw[1] + 1) to_table(ix, node, (n->kw[1] + 1) * 2);
        n = &ix->nodes.h[node];
        ctab_put(ix, n->kw[0], n->kw[1], wid, child, node_psum(ix, child));
        if (ix->aux[node].bm != NONE) wide_bit(ix, node, wid, true);
        else set_bloom(*n, wid);
    }
    n->nlit++;
    if (nlit_of(*n) == WIDE_LIT && ix->aux[node].bm == NONE) { to_wide(ix, node); n = &ix->nodes.h[node]; }
    ix->nodes.touch(node);
    summary_refresh(ix, node);
}

void child_remove(tm_index *ix, uint32_t node, uint32_t wid) {
    ix->nlinks--;
    lvl_edge(ix, ix->aux[node].depth, wid, false);
    if (ix->aux[node].bm != NONE) ix->dense_dirty = true;
    Node &n = ix->nodes.h[node];
    if (nlit_of(n) <= KINL) {
        for (uint32_t k = 0; k < KINL; k++)
            if (n.kw[k] == wid) { n.kw[k] = NONE; n.kc[k] = NONE; break; }
        n.nlit--;
    } else {
        ctab_erase(ix, n.kw[0], n.kw[1], wid);
        wide_bit(ix, node, wid, false);
        n.nlit--;
        if (ix->aux[node].bm != NONE && nlit_of(n) < WIDE_LIT) from_wide(ix, node);
        if (nlit_of(n) == KINL) {   // back to inline mode
            std::vector<CSlot> kids;
            for (uint32_t i = 0; i <= n.kw[1]; i++) if (ix->ctab.h[n.kw[0] + i].wid != NONE) kids.push_back(ix->ctab.h[n.kw[0] + i]);
            ctab_free(ix, n.kw[0], n.kw[1] + 1);
            for (uint32_t k = 0; k < KINL; k++) { n.kw[k] = kids[k].wid; n.kc[k] = kids[k].child; }
        }
    }
    ix->nodes.touch(node);
    summary_refresh(ix, node);
}

bool node_empty(tm_index *ix, uint32_t id) {
    const Node &n = ix->nodes.h[id];
    return n.plus == NONE && n.nlit == 0 && n.hash_cnt == 0 && n.exact_cnt == 0 && ix->aux[id].hdesc == 0;
}

void node_prune(tm_index *ix, uint32_t id) {
    while (id != ROOT && node_empty(ix, id)) {
        NodeAux a = ix->aux[id];
        if (a.is_plus) {
            Node &pn = ix->nodes.h[a.parent];
            pn.plus = NONE; pn.psum_lo = pn.psum_hi = 0;
            ix->nodes.touch(a.parent);
            summary_refresh(ix, a.parent);
        } else {
            child_remove(ix, a.parent, a.wid);
            word_unref(ix, a.wid);
        }
        ix->free_nodes.push_back(id);
        ix->live_nodes--;
        ix->depth_cnt[a.depth]--;
        id = a.parent;
    }
}

// ------------------------------------------------------------ exact table

ExactEntry empty_exact() { ExactEntry e; memset(&e, 0, sizeof e); e.nlev = NONE; return e; }

uint64_t seq_hash(const std::vector<uint32_t> &w) {
    uint64_t x = FNV_OFF;
    for (uint32_t v : w) x = seq_hash_step(x, v);
    return seq_hash_finish(x, (uint32_t)w.size());
}

bool exact_eq(tm_index *ix, const ExactEntry &e, uint64_t h, const std::vector<uint32_t> &w) {
    if (e.h_lo != (uint32_t)h || e.h_hi != (uint32_t)(h >> 32) || e.nlev != w.size()) return false;
    const uint32_t *s = w.size() <= XINL ? e.wids : ix->wseq.h.data() + e.seq_off;
    return !memcmp(s, w.data(), sizeof(uint32_t) * w.size());
}

uint32_t exact_find_slot(tm_index *ix, uint64_t h, const std::vector<uint32_t> &w) {
    const uint32_t mask = (uint32_t)ix->exact.h.size() - 1;
    for (uint32_t s = (uint32_t)h & mask;; s = (s + 1) & mask) {
        const ExactEntry &e = ix->exact.h[s];
        if (e.nlev == NONE) return NONE;
        if (exact_eq(ix, e, h, w)) return s;
    }
}

void exact_rehash(tm_index *ix, uint32_t ncap);
void exact_grow(tm_index *ix, uint64_t need) {
    if (need * 2 <= ix->exact.h.size()) return;
    exact_rehash(ix, pow2_at_least(need * 2));
}

void exact_rehash(tm_index *ix, uint32_t ncap) {
    std::vector<ExactEntry> nt(ncap, empty_exact());
    std::vector<uint32_t> nc(ncap, 0), nr(ncap, 0);
    std::vector<uint16_t> nf(ncap, 0);
    const uint32_t mask = ncap - 1;
    for (size_t i = 0; i < ix->exact.h.size(); i++) {
        const ExactEntry &e = ix->exact.h[i];
        if (e.nlev == NONE) continue;
        for (uint32_t s = e.h_lo & mask;; s = (s + 1) & mask)
            if (nt[s].nlev == NONE) { nt[s] = e; nc[s] = ix->xcap[i]; nr[s] = ix->xroff[i]; nf[s] = ix->xfp.h[i]; break; }
    }
    ix->exact.h.swap(nt);
    ix->xcap.swap(nc);
    ix->xroff.swap(nr);
    ix->xfp.h.swap(nf);
    ix->exact.dirty.set_all();
    ix->xfp.dirty.set_all();
}

void exact_erase_slot(tm_index *ix, uint32_t i) {
    auto &t = ix->exact.h;
    const uint32_t mask = (uint32_t)t.size() - 1;
    {   // the key's levels no longer use their words
        const uint32_t nl = t[i].nlev;
        const uint32_t *ws = nl <= XINL ? t[i].wids : ix->wseq.h.data() + t[i].seq_off;
        std::vector<uint32_t> used(ws, ws + nl);
        if (nl > XINL) ix->wseq_dead += nl;
        for (uint32_t w : used) word_unref(ix, w);
        ix->xlen_cnt[nl]--;
    }
    for (uint32_t j = (i + 1) & mask; t[j].nlev != NONE; j = (j + 1) & mask) {
        uint32_t k = t[j].h_lo & mask;
        bool stays = (i <= j) ? (i < k && k <= j) : (i < k || k <= j);
        if (!stays) {
            t[i] = t[j]; ix->xcap[i] = ix->xcap[j]; ix->xroff[i] = ix->xroff[j]; ix->xfp.h[i] = ix->xfp.h[j];
            ix->exact.touch(i); ix->xfp.touch(i);
            i = j;
        }
    }
    t[i] = empty_exact();
    ix->xcap[i] = 0;
    ix->xroff[i] = 0;
    ix->xfp.h[i] = 0;
    ix->exact.touch(i);
    ix->xfp.touch(i);
    ix->xcount--;
}

// Reclaim what deletes left behind (end of every delta batch): long words'
// bytes in wpool and long exact keys' wid runs in wseq are compacted once half
// of the pool is dead; the vocab and exact tables shrink back when their load
// falls below 1/16 and 1/8 (they double at 1/4 and 1/2).  Each of these
// rewrites whole tables, so the next sync re-uploads them.
void reclaim(tm_index *ix) {
    if (ix->wpool_dead * 2 > ix->wpool.h.size() && ix->wpool.h.size() >= (64u << 10)) {
        std::vector<uint8_t> np;
        np.reserve(ix->wpool.h.size() - ix->wpool_dead);
        for (VocabEntry &e : ix->vocab.h) {
            if (e.wid == NONE || (e.tag & 0xFF) <= VINL) continue;
            const uint64_t off = np.size(), padded = (e.b1 + 3) & ~3u;
            np.insert(np.end(), ix->wpool.h.begin() + e.b0, ix->wpool.h.begin() + e.b0 + padded);
            e.b0 = (uint32_t)off;
        }
        ix->wpool.h.swap(np);
        ix->wpool_dead = 0;
        ix->wpool.dirty.set_all();
        ix->vocab.dirty.set_all();
    }
    if (ix->wseq_dead * 2 > ix->wseq.h.size() && ix->wseq.h.size() >= (16u << 10)) {
        std::vector<uint32_t> nq;
        nq.reserve(ix->wseq.h.size() - ix->wseq_dead);
        for (ExactEntry &e : ix->exact.h) {
            if (e.nlev == NONE || e.nlev <= XINL) continue;
            const uint64_t off = nq.size();
            nq.insert(nq.end(), ix->wseq.h.begin() + e.seq_off, ix->wseq.h.begin() + e.seq_off + e.nlev);
            e.seq_off = (uint32_t)off;
        }
        ix->wseq.h.swap(nq);
        ix->wseq_dead = 0;
        ix->wseq.dirty.set_all();
        ix->exact.dirty.set_all();
    }
    const uint64_t vmin = 1024;
    if (ix->vocab.h.size() > vmin && (ix->vcount << (VOCAB_LOAD_SHIFT + 2)) < ix->vocab.h.size())
        vocab_rehash(ix, std::max<uint64_t>(vmin, pow2_at_least(std::max<uint64_t>(ix->vcount, 1) << VOCAB_LOAD_SHIFT)));
    if (ix->exact.h.size() > 1024 && ix->xcount * 8 < ix->exact.h.size())
        exact_rehash(ix, std::max<uint32_t>(1024, pow2_at_least(ix->xcount * 2)));
}

// --------------------------------------------------------------- key ops

void split_words(const uint8_t *f, uint32_t len, std::vector<WordRef> &out) {
    out.clear();
    uint32_t s = 0;
    for (uint32_t i = 0; i <= len; i++) {
        if (i == len || f[i] == '/') {
            uint32_t n = i - s;
            int kind = (n == 1 && f[s] == '+') ? 1 : (n == 1 && f[s] == '#') ? 2 : 0;
            out.push_back({f + s, n, kind});
            s = i + 1;
        }
    }
}

std::string dead_key(const uint8_t *f, uint32_t len, uint32_t v, uint8_t flags) {
    std::string k;
    k.reserve(len + 5);
    k.push_back((char)flags);
    k.append(reinterpret_cast<const char *>(&v), 4);
    k.append(reinterpret_cast<const char *>(f), len);
    return k;
}

// matches_filter's log of word-list key ops (tm_index::MfState; caller holds
// ix->mu).  Unbounded growth between calls is cut: past a bound the log is
// dropped and the next call takes a new snapshot.
void mf_log(tm_index *ix, bool ins, const std::string &key) {
    auto &m = ix->mf;
    if (!m.log_on) return;
    if (m.log.size() >= std::max<size_t>(size_t(1) << 22, 2 * m.nkeys.load(std::memory_order_relaxed))) {
        m.log_on = false; m.log_lost = true;
        std::vector<std::pair<bool, std::string>>().swap(m.log);
        return;
    }
    m.log.emplace_back(ins, key);
}

// one insert (ins = true) or delete of the key make_key(Filter, V)
// An escaped word list (TM_KEY_WORDS | TM_KEY_ESCAPED): words split on '/',
// "\x" = the byte x; a word written "\+" / "\#" is a binary word, a bare
// "+" / "#" the wildcard.  -> (word bytes, wildcard?) per word.
void esc_words(const uint8_t *f, uint32_t len, std::vector<std::pair<std::string, bool>> &out) {
    out.clear();
    std::string cur;
    bool esc_any = false;
    auto push = [&]() {
        const bool wild = !esc_any && cur.size() == 1 && (cur[0] == '+' || cur[0] == '#');
        out.emplace_back(cur, wild);
        cur.clear();
        esc_any = false;
    };
    for (uint32_t i = 0; i < len; i++) {
        if (f[i] == '\\' && i + 1 < len) { cur.push_back((char)f[++i]); esc_any = true; }
        else if (f[i] == '/') push();
        else cur.push_back((char)f[i]);
    }
    push();
}

// the canonical escaped form of a word list ('/' and '\' escaped, binary
// "+" / "#" as "\+" / "\#")
std::string esc_join(const std::vector<std::pair<std::string, bool>> &w) {
    std::string o;
    for (size_t i = 0; i < w.size(); i++) {
        if (i) o.push_back('/');
        if (w[i].second) { o += w[i].first; continue; }
        if (w[i].first == "+" || w[i].first == "#") { o.push_back('\\'); o += w[i].first; continue; }
        for (char c : w[i].first) {
            if (c == '/' || c == '\\') o.push_back('\\');
            o.push_back(c);
        }
    }
    return o;
}

// a binary word no topic level can equal: "+" / "#" (a level exactly that is
// badarg) or one holding a '/'
bool word_never(const std::pair<std::string, bool> &w) {
    return !w.second && (w.first == "+" || w.first == "#" || w.first.find('/') != std::string::npos);
}

void word_key_op(tm_index *ix, bool ins, const std::vector<WordRef> &w, uint32_t v, const std::string &dk,
                 bool dead_done);

void key_op(tm_index *ix, bool ins, const uint8_t *f, uint32_t len, uint32_t v, uint8_t flags,
            std::vector<WordRef> &w, std::vector<uint32_t> &wids) {
    if ((flags & TM_KEY_ESCAPED) && !(flags & TM_KEY_EMPTY_LIST)) {
        std::vector<std::pair<std::string, bool>> ew;
        esc_words(f, len, ew);
        bool never = false;
        for (auto &x : ew) never |= word_never(x);
        if (!never) {   // plain words after all: the TM_KEY_WORDS key of the joined bytes
            std::string plain;
            for (size_t i = 0; i < ew.size(); i++) { if (i) plain.push_back('/'); plain += ew[i].first; }
            key_op(ix, ins, reinterpret_cast<const uint8_t *>(plain.data()), (uint32_t)plain.size(), v,
                   TM_KEY_WORDS, w, wids);
            return;
        }
        // never matches a topic: a key of the table for matches_filter/3 only --
        // but a '#' atom before its last word still steers the ordered walk at
        // the node of the words before it, if those are plain (NLIT_HDESC)
        const std::string canon = esc_join(ew);
        const std::string dk = dead_key(reinterpret_cast<const uint8_t *>(canon.data()), (uint32_t)canon.size(), v,
                                        TM_KEY_WORDS | TM_KEY_ESCAPED);
        if (ix->mf.log_on) mf_log(ix, ins, dk);
        if (ins ? !ix->dead.insert(dk).second : !ix->dead.erase(dk)) return;   // present / absent: no-op
        size_t hpos = ew.size();
        for (size_t i = 0; i + 1 < ew.size(); i++)
            if (ew[i].second && ew[i].first == "#") { hpos = i; break; }
        bool plain_prefix = hpos < ew.size();
        for (size_t i = 0; i < hpos && plain_prefix; i++) plain_prefix = !word_never(ew[i]);
        if (!plain_prefix) return;
        std::vector<WordRef> pw;   // the prefix, the '#', and a stand-in for the rest (only the prefix is walked)
        for (size_t i = 0; i <= hpos; i++)
            pw.push_back({reinterpret_cast<const uint8_t *>(ew[i].first.data()), (uint32_t)ew[i].first.size(),
                          ew[i].second ? (ew[i].first == "+" ? 1 : 2) : 0});
        pw.push_back({nullptr, 0, 0});
        word_key_op(ix, ins, pw, v, dk, true);
        return;
    }
    if (flags & TM_KEY_EMPTY_LIST) {   // [] never matches a topic (topics have >= 1 level)
        auto k = dead_key(nullptr, 0, v, TM_KEY_EMPTY_LIST);
        if (ins) ix->dead.insert(k); else ix->dead.erase(k);
        mf_log(ix, ins, k);
        return;
    }
    split_words(f, len, w);
    bool wild = false;
    for (auto &x : w) wild |= x.kind != 0;
    if (!wild && !(flags & TM_KEY_WORDS)) {
        // binary key (emqx_trie_search.erl:121-125) -> exact table keyed by wid sequence
        wids.clear();
        if (ins) {
            for (auto &x : w) wids.push_back(vocab_intern(ix, x.p, x.n));
            exact_grow(ix, ix->xcount + 1);
        } else {
            for (auto &x : w) {
                uint32_t id = vocab_find(ix, x.p, x.n);
                if (id == NONE) return;
                wids.push_back(id);
            }
        }
        const uint64_t h = seq_hash(wids);
        uint32_t s = exact_find_slot(ix, h, wids);
        if (s == NONE) {
            if (!ins) return;
            ExactEntry e = empty_exact();
            e.h_lo = (uint32_t)h; e.h_hi = (uint32_t)(h >> 32); e.nlev = (uint32_t)wids.size();
            if (wids.size() <= XINL) {
                std::copy(wids.begin(), wids.end(), e.wids);
            } else {
                e.seq_off = (uint32_t)ix->wseq.h.size();
                ix->wseq.h.insert(ix->wseq.h.end(), wids.begin(), wids.end());
                ix->wseq.touch(e.seq_off, wids.size());
            }
            const uint32_t mask = (uint32_t)ix->exact.h.size() - 1;
            for (s = (uint32_t)h & mask; ix->exact.h[s].nlev != NONE; s = (s + 1) & mask) {}
            ix->exact.h[s] = e;
            ix->xcap[s] = 0;
            ix->xroff[s] = 0;
            ix->xfp.h[s] = exact_fp(h);
            ix->xfp.touch(s);
            ix->xcount++;
            for (uint32_t wd : wids) word_ref(ix, wd);
            if (ix->xlen_cnt.size() <= wids.size()) ix->xlen_cnt.resize(wids.size() + 1, 0);
            ix->xlen_cnt[wids.size()]++;
        }
        ExactEntry &e = ix->exact.h[s];
        if (ins) { if (run_op(ix, true, ix->xroff[s], ix->xcap[s], e.val_off, e.val_cnt, v)) ix->n_exact++; }
        else if (run_op(ix, false, ix->xroff[s], ix->xcap[s], e.val_off, e.val_cnt, v)) {
            ix->n_exact--;
            if (!(e.val_cnt & RUN_CNT)) { exact_erase_slot(ix, s); return; }
        }
        ix->exact.touch(s);
        return;
    }
    word_key_op(ix, ins, w, v, dead_key(f, len, v, TM_KEY_WORDS), false);
}

// A word-list key (its words w; dk: its dead-key string, the identity
// matches_filter/3 and the never-matching set know it by; dead_done: the
// caller already logged it and entered it in that set).
void word_key_op(tm_index *ix, bool ins, const std::vector<WordRef> &w, uint32_t v, const std::string &dk,
                 bool dead_done) {
    if (ix->mf.log_on && !dead_done) mf_log(ix, ins, dk);
    // word-list key.  '#' anywhere but last never matches (compare/3 has no
    // clause for it, emqx_trie_search.erl:282-290 vs :341-348; emqx_topic.erl:110),
    // but the key still steers the reference's walk at the node P of its
    // prefix before that '#' (tm_layout.h NLIT_HDESC): P counts such keys
    size_t hpos = w.size();
    for (size_t i = 0; i + 1 < w.size(); i++)
        if (w[i].kind == 2) { hpos = i; break; }
    if (hpos < w.size() && !dead_done) {
        // (a wildcard filter is a word list whatever the flag: one key)
        if (ins ? !ix->dead.insert(dk).second : !ix->dead.erase(dk)) return;   // present / absent: no-op
    }
    const bool hash_term = hpos == w.size() && w.back().kind == 2;
    const size_t end = hpos < w.size() ? hpos : hash_term ? w.size() - 1 : w.size();
    uint32_t node = ROOT;
    for (size_t i = 0; i < end; i++) {
        if (w[i].kind == 1) {
            uint32_t c = ix->nodes.h[node].plus;
            if (c == NONE) {
                if (!ins) return;
                c = node_new(ix, node, NONE, true);
                ix->nodes.h[node].plus = c;
                ix->nodes.touch(node);
                summary_refresh(ix, node);   // node gained a '+' child
                summary_refresh(ix, c);
            }
            node = c;
        } else {
            uint32_t wid = ins ? vocab_intern(ix, w[i].p, w[i].n) : vocab_find(ix, w[i].p, w[i].n);
            if (wid == NONE) return;
            uint32_t c = child_find(ix, node, wid);
            if (c == NONE) {
                if (!ins) return;
                c = node_new(ix, node, wid, false);
                child_add(ix, node, wid, c);
            }
            node = c;
        }
    }
    Node &nd = ix->nodes.h[node];
    NodeAux &a = ix->aux[node];
    if (hpos < w.size()) {   // a '#'-not-last key: P's count (the path exists: the key was inserted)
        a.hdesc += ins ? 1 : -1;
        ix->n_hdesc_keys += ins ? 1 : -1;
        nd.nlit = nlit_of(nd) | (a.hdesc ? NLIT_HDESC : 0);
        ix->nodes.touch(node);
        summary_refresh(ix, node);
        if (!ins) node_prune(ix, node);
        return;
    }
    bool changed;
    changed = hash_term ? run_op(ix, ins, a.hash_roff, a.hash_cap, nd.hash_off, nd.hash_cnt, v)
                        : run_op(ix, ins, a.exact_roff, a.exact_cap, nd.exact_off, nd.exact_cnt, v);
    if (!changed) return;
    ix->nodes.touch(node);
    summary_refresh(ix, node);
    if (ins) ix->n_wild++;
    else { ix->n_wild--; node_prune(ix, node); }
}

// ------------------------------------------------------------- device side

constexpr uint64_t DEV_GUARD = 16;   // device elements kept allocated past the host size (see collect)

int bring_up(tm_index *ix, int r, uint64_t upto, hipStream_t st, bool idle = false);
int collect_patch_locked(tm_index *ix);

template <class T>
int upload_full(tm_index *ix, Mirror<T> &m) {
    // patches logged before this upload are older than it: every replica
    // takes them first (a lagging replica applying one later would write old
    // words over the new table)
    for (int r = 0; r < ix->nrep; r++)
        if (int rc = bring_up(ix, r, ix->patch_seq, ix->rep[r].ps)) return rc;
    uint64_t need = std::max<uint64_t>(m.h.size(), 1);
    const bool grow = need > m.dcap;
    const uint64_t cap = grow ? need + need / 2 + DEV_GUARD : m.dcap;
    // a failure part way leaves the device copies in doubt: dcap 0 makes the
    // next collect reallocate and ship the whole table again (its dirty set
    // is cleared only on success)
    auto ship = [&]() -> int {
        for (int r = 0; r < ix->nrep; r++) {
            // rare (first upload, growth, rehash): drain every stream that may
            // still read the old copy before touching it
            HIPCHK(ix, hipSetDevice(ix->rep[r].device));
            HIPCHK(ix, hipDeviceSynchronize());
            if (grow) {
                if (m.d[r]) HIPCHK(ix, hipFree(m.d[r]));
                m.d[r] = nullptr;
                HIPCHK(ix, hipMalloc(&m.d[r], cap * sizeof(T)));
            }
            if (m.bytes()) HIPCHK(ix, hipMemcpy(m.d[r], m.h.data(), m.bytes(), hipMemcpyHostToDevice));
        }
        return TM_OK;
    };
    if (int rc = ship()) {
        m.dcap = 0;
        return rc;
    }
    m.dcap = cap;
    if (getenv("TM_DEBUG_UPLOADS"))   // diagnostics: which table was shipped whole, and why
        fprintf(stderr, "tm upload_full: %zu-byte elements x %zu (%.1f MB), dcap %lu, %d replicas\n", sizeof(T),
                m.h.size(), m.bytes() / 1e6, (unsigned long)m.dcap, ix->nrep);
    m.dirty.clear();
    ix->uploads++;
    return TM_OK;
}

// One patch run: `n` (<= PATCH_RUN) consecutive 4-byte words copied from the
// patch data at `src` to word `dst & PATCH_OFF` of table `dst >> 48` (tm_dev.h
// PatchRun): the same runs serve every replica, each with its table bases.
constexpr uint32_t PATCH_RUN = 64;

template <class T>
int collect(tm_index *ix, Mirror<T> &m, uint32_t table, std::vector<PatchRun> &runs, std::vector<uint32_t> &data) {
    // the device copy keeps >= DEV_GUARD elements allocated past the host
    // size: k_emit's 16-B loads may overhang the last value run by 3 words
    // (with h.size() == dcap such a load would leave the allocation)
    if (m.h.size() + DEV_GUARD > m.dcap) m.dirty.set_all();
    if (!m.dirty.all) {
        uint64_t words = 0;
        for (auto &r : m.dirty.r) words += r.second - r.first;
        if (words * 4 > m.bytes() / 2) m.dirty.set_all();   // cheaper to ship the table
    }
    if (m.dirty.all) return upload_full(ix, m);
    const uint8_t *src = reinterpret_cast<const uint8_t *>(m.h.data());
    const uint64_t limit = (m.bytes() + 3) / 4;
    for (auto &r : m.dirty.r) {
        const uint64_t hi = std::min<uint64_t>(r.second, limit);
        for (uint64_t lo = r.first; lo < hi; lo += PATCH_RUN) {
            const uint32_t n = (uint32_t)std::min<uint64_t>(PATCH_RUN, hi - lo);
            const uint64_t at = data.size();
            runs.push_back(PatchRun{(uint64_t)table << 48 | lo, (uint32_t)at, n});
            data.resize(at + n, 0);
            memcpy(data.data() + at, src + 4 * lo, std::min<uint64_t>(4ull * n, m.bytes() - 4 * lo));
        }
    }
    m.dirty.clear();
    return TM_OK;
}

PatchBases patch_bases(tm_index *ix, int r) {
    PatchBases b;
    const void *t[N_TABLES] = {ix->vocab.d[r], ix->wpool.d[r], ix->nodes.d[r], ix->ctab.d[r], ix->vals.d[r],
                               ix->exact.d[r], ix->xfp.d[r], ix->wseq.d[r], ix->wbits.d[r]};
    for (int i = 0; i < N_TABLES; i++) b.b[i] = reinterpret_cast<uint64_t>(t[i]);
    return b;
}

// a fresh launch tag of the lane's workspace (1 .. LB_TAG_MASK); when the tags
// wrap, the look-back words are cleared first, on the launch's stream, so no
// word an earlier launch left can carry the new tag
int next_tag(tm_index *ix, Lane &ln, hipStream_t s, uint32_t &tag) {
    ln.tag = (ln.tag + 1) & LB_TAG_MASK;
    if (!ln.tag) {
        ln.tag = 1;
        HIPCHK(ix, hipMemsetAsync(ln.w.look, 0, (ln.w.cap_n / SM_TOPICS + 4) * 8 * LB_STRIDE, s));
    }
    tag = ln.tag;
    return TM_OK;
}

// the look-back control of the next launch (caller holds ix->mu): the
// default bound, or the test hook's for the next dbg_lb_launches launches
LbCtl next_lb(tm_index *ix) {
    LbCtl c{LB_SPINS, NONE, 0};
    if (ix->dbg_lb_launches) {
        ix->dbg_lb_launches--;
        c = ix->dbg_lb;
    }
    c.ticket = ix->small_ticket;
    return c;
}

// did the lane's last one-launch batch fail its look-back (err 4, the fail
// word raised by the device)?  Clears the word.  After the lane's stream
// has been synchronised.
bool batch_failed(tm_index *ix, Lane &ln) {
    volatile uint32_t *f = ln.w.hint_h + HINT_FAIL;
    if (!*f) return false;
    *f = 0;
    ix->failed_batches++;
    return true;
}

// the lane's batch is done with the index: later patches (on any stream) wait for it
int batch_done(tm_index *ix, Lane &ln) {
    HIPCHK(ix, hipEventRecord(ln.done, ln.s));
    ln.used = true;
    ln.drained = false;
    return TM_OK;
}

// Is a batch of the lane still running?  (caller holds ix->mu)  A lane seen
// drained stays so until its next batch: the copy pickers, the committer and
// the patches ask about every lane under the index lock, and with concurrent
// callers that was dozens of event queries (and stream waits) per launch and
// per commit, while most lanes were long idle
bool lane_busy(Lane &l) {
    if (!l.used || l.drained) return false;
    if (hipEventQuery(l.done) == hipErrorNotReady) return true;
    l.drained = true;
    return false;
}

// Apply logged patch q to replica r on stream st.  Patches rewrite the tables
// in place, so a patch first waits for every batch still reading the replica
// (each of its lanes' `done`) and for the replica's patch before it; every
// later batch there waits for this one (`last_patch`, ensure_ws): a batch
// sees exactly the deltas applied before it was queued (C5), whichever stream
// either ran on.
int apply_patch(tm_index *ix, int r, uint64_t q, hipStream_t st, bool wait_readers = true) {
    Replica &R = ix->rep[r];
    const uint32_t k = (uint32_t)((q - 1) % PATCH_RING);
    const PatchSlot &p = ix->patch[k];
    HIPCHK(ix, hipSetDevice(R.device));
    // a small patch (a route write's few runs) is read by the patch kernel
    // straight from the mapped pinned slot: one command on the stream instead
    // of a DMA copy and the kernel behind it (the slot is reused only after
    // pdone, recorded behind the kernel); larger ones are copied first, into a
    // device buffer of the slot allocated on first use
    const bool zc = ix->patch_zc && p.pin_dev && p.bytes <= PATCH_ZC_MAX;
    if (!zc && (p.bytes > R.pdev_cap[k] || !R.pdev[k])) {
        if (R.ppending[k]) { HIPCHK(ix, hipEventSynchronize(R.pdone[k])); R.ppending[k] = false; }
        if (R.pdev[k]) HIPCHK(ix, hipFree(R.pdev[k]));
        R.pdev[k] = nullptr;
        R.pdev_cap[k] = 0;
        // generous steps: a reallocation (hipHostFree / hipFree) synchronises
        // the device, a multi-millisecond stall inside a churn stream (C5)
        const uint64_t want = std::max<uint64_t>(p.bytes * 2, 1u << 20);
        uint8_t *np = nullptr;   // the capacity is recorded only once the buffer exists
        HIPCHK(ix, hipMalloc(&np, want));
        R.pdev[k] = np;
        R.pdev_cap[k] = want;
    }
    if (wait_readers)   // (not for a copy known to be idle, nor again behind a patch just queued on st)
        for (auto &l : ix->lanes)
            if (l->r == r && l->s != st && lane_busy(*l)) HIPCHK(ix, hipStreamWaitEvent(st, l->done, 0));
    if (R.last_patch) HIPCHK(ix, hipStreamWaitEvent(st, R.last_patch, 0));
    const uint8_t *src = R.pdev[k];
    if (zc) {
        src = p.pin_dev;
    } else {
        HIPCHK(ix, hipMemcpyAsync(R.pdev[k], p.pin, p.bytes, hipMemcpyHostToDevice, st));
    }
    HIPCHK(ix, launch_patch(reinterpret_cast<const PatchRun *>(src),
                            reinterpret_cast<const uint32_t *>(src + p.nr * sizeof(PatchRun)), p.nr,
                            patch_bases(ix, r), st));
    HIPCHK(ix, hipEventRecord(R.pdone[k], st));
    R.ppending[k] = true;
    R.last_patch = R.pdone[k];
    R.applied = q;
    return TM_OK;
}

// replica r takes every logged patch up to `upto`, in order, on stream st
int bring_up(tm_index *ix, int r, uint64_t upto, hipStream_t st, bool idle) {
    const uint64_t first = ix->rep[r].applied + 1;   // (readers waited for once, before the first patch)
    for (uint64_t q = first; q <= upto; q++)
        if (int rc = apply_patch(ix, r, q, st, !idle && q == first)) return rc;
    return TM_OK;
}

DevIndex dev_view_build(tm_index *ix, int r);

// Collect every dirty word into a new logged patch and refresh the replicas'
// cached device views (caller holds ix->mu; takes ix->img, and only when a
// delta was applied since the last call); nothing reaches a device here but
// whole-table uploads
int collect_patch(tm_index *ix, bool commit = false) {
    if (ix->view_ok && !commit &&
        (!ix->img_dirty.load(std::memory_order_acquire) || ix->img_hold.load(std::memory_order_acquire) > 0))
        return TM_OK;
    std::lock_guard<std::mutex> gi(ix->img);
    ix->img_dirty.store(false, std::memory_order_relaxed);   // (an apply from here on sets it again)
    int rc = collect_patch_locked(ix);
    for (int r = 0; r < ix->nrep; r++) ix->view[r] = dev_view_build(ix, r);
    ix->view_ok = rc == TM_OK;
    if (!commit) ix->pub_seq = ix->patch_seq;   // a batch's collect: published at once
    return rc;
}

int collect_patch_locked2(tm_index *ix);

// Every table's dirty words go into one patch.  collect() clears a table's
// dirty set as it takes its runs, so if anything fails after that (a pinned
// allocation, a lagging replica's bring-up) those runs would never reach a
// device: every table is then marked wholly dirty, and the next collect ships
// them whole.
int collect_patch_locked(tm_index *ix) {
    const int rc = collect_patch_locked2(ix);
    if (rc) {
        ix->vocab.dirty.set_all(); ix->wpool.dirty.set_all(); ix->nodes.dirty.set_all();
        ix->ctab.dirty.set_all(); ix->vals.dirty.set_all(); ix->exact.dirty.set_all();
        ix->xfp.dirty.set_all(); ix->wseq.dirty.set_all(); ix->wbits.dirty.set_all();
    }
    return rc;
}

// (TM_HOST_TIMING) collect_patch_locked2's parts: the tables' runs, the ring
// slot's reuse (a lagging replica brought up and waited for), the pinned copy
std::atomic<uint64_t> g_col_n{0}, g_col_runs_ns{0}, g_col_slot_ns{0}, g_col_copy_ns{0};
const bool g_col_timing = getenv("TM_HOST_TIMING") != nullptr;
uint64_t col_now() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

int collect_patch_locked2(tm_index *ix) {
    const uint64_t t0 = g_col_timing ? col_now() : 0;
    std::vector<PatchRun> runs;
    std::vector<uint32_t> data;
    int rc;
    if ((rc = collect(ix, ix->vocab, 0, runs, data))) return rc;
    if ((rc = collect(ix, ix->wpool, 1, runs, data))) return rc;
    if ((rc = collect(ix, ix->nodes, 2, runs, data))) return rc;
    if ((rc = collect(ix, ix->ctab, 3, runs, data))) return rc;
    if ((rc = collect(ix, ix->vals, 4, runs, data))) return rc;
    if ((rc = collect(ix, ix->exact, 5, runs, data))) return rc;
    if ((rc = collect(ix, ix->xfp, 6, runs, data))) return rc;
    if ((rc = collect(ix, ix->wseq, 7, runs, data))) return rc;
    if ((rc = collect(ix, ix->wbits, 8, runs, data))) return rc;
    const uint64_t nr = runs.size(), nw = data.size();
    if (!nr) return TM_OK;
    const uint64_t t1 = g_col_timing ? col_now() : 0;
    const uint64_t q = ix->patch_seq + 1;
    const uint32_t k = (uint32_t)((q - 1) % PATCH_RING);
    PatchSlot &p = ix->patch[k];
    if (p.seq) {   // the slot's patch must have reached every replica and left its pinned buffer
        for (int r = 0; r < ix->nrep; r++) {
            Replica &R = ix->rep[r];
            if (R.applied < p.seq && (rc = bring_up(ix, r, p.seq, R.ps))) return rc;
            if (R.ppending[k]) {
                HIPCHK(ix, hipSetDevice(R.device));
                HIPCHK(ix, hipEventSynchronize(R.pdone[k]));
                R.ppending[k] = false;
            }
        }
    }
    const uint64_t t2 = g_col_timing ? col_now() : 0;
    const uint64_t bytes = nr * sizeof(PatchRun) + nw * 4;
    if (bytes > p.pin_cap || !p.pin) {
        if (p.pin) HIPCHK(ix, hipHostFree(p.pin));
        p.pin = nullptr;
        p.pin_cap = 0;
        const uint64_t want = std::max<uint64_t>(bytes * 2, 64u << 10);
        uint8_t *np = nullptr;   // the capacity is recorded only once the buffer exists
        HIPCHK(ix, hipHostMalloc(&np, want, hipHostMallocPortable | hipHostMallocMapped));
        p.pin = np;
        p.pin_cap = want;
        void *dp = nullptr;
        p.pin_dev = hipHostGetDevicePointer(&dp, np, 0) == hipSuccess ? static_cast<uint8_t *>(dp) : nullptr;
    }
    memcpy(p.pin, runs.data(), nr * sizeof(PatchRun));
    memcpy(p.pin + nr * sizeof(PatchRun), data.data(), nw * 4);
    p.bytes = bytes; p.nr = nr; p.seq = q;
    if (g_col_timing) {
        g_col_n++;
        g_col_runs_ns += t1 - t0; g_col_slot_ns += t2 - t1; g_col_copy_ns += col_now() - t2;
    }
    ix->patch_seq = q;
    ix->patch_bytes += nw * 4;
    ix->uploads++;
    return TM_OK;
}

// Every delta applied so far, onto replica r0 before a batch runs there on
// stream s (caller holds ix->mu; the calling thread's device is r0's after)
int sync_locked(tm_index *ix, int r0, hipStream_t s) {
    int rc;
    if ((rc = collect_patch(ix))) return rc;
    if ((rc = bring_up(ix, r0, ix->pub_seq, s))) return rc;
    HIPCHK(ix, hipSetDevice(ix->rep[r0].device));
    return TM_OK;
}

// Which copy of group g a batch should read (caller holds ix->mu, pending
// deltas collected): the lowest-numbered copy that is up to date (so without
// churn one copy stays hot), else one no batch is reading (it takes the
// patch without waiting), else the least recently used one.  busy (host
// lanes per replica) excludes copies whose host lanes are all in use.
// A device-API batch names its stream s: then a copy whose unfinished
// readers all run on s counts as idle too (the patch is ordered behind them
// by the stream itself, no cross-stream wait), preferring the copy s read
// last, so with as many copies as streams each stream keeps to its own copy
// under churn.
int pick_copy(tm_index *ix, int g, const int *busy, hipStream_t s = nullptr, bool by_stream = false) {
    auto ok = [&](int r) { return ix->rep[r].group == g && (!busy || busy[r] < MAX_HOST_LANES); };
    const int sv = ix->serving[g];   // the copy tm_commit last published on: fresh, its readers' hot set
    if (sv >= 0 && ok(sv) && ix->rep[sv].applied >= ix->pub_seq) return sv;
    for (int r = 0; r < ix->nrep; r++)
        if (ok(r) && ix->rep[r].applied >= ix->pub_seq) return r;
    if (by_stream) {
        int pick = -1;
        uint64_t pick_tick = 0;
        for (int r = 0; r < ix->nrep; r++) {
            if (!ok(r)) continue;
            bool free_here = true;
            uint64_t mine = 0;   // when stream s last read copy r (0: never)
            for (auto &l : ix->lanes) {
                if (l->r != r || !l->used) continue;
                if (l->s == s) { mine = std::max<uint64_t>(mine, l->tick); continue; }
                if (lane_busy(*l)) { free_here = false; break; }
            }
            if (free_here && (pick < 0 || mine > pick_tick)) { pick = r; pick_tick = mine; }
        }
        if (pick >= 0) return pick;
    }
    for (int r = 0; r < ix->nrep; r++) {
        if (!ok(r)) continue;
        bool idle = true;
        for (auto &l : ix->lanes)
            if (l->r == r && lane_busy(*l)) { idle = false; break; }
        if (idle) return r;
    }
    int best = -1;
    for (int r = 0; r < ix->nrep; r++)
        if (ok(r) && (best < 0 || ix->rep[r].last_use < ix->rep[best].last_use)) best = r;
    return best;
}

// the device view of replica r as of the last collect_patch (caller holds ix->mu)
DevIndex dev_view(tm_index *ix, int r) { return ix->view[r]; }

// (caller holds ix->img)
DevIndex dev_view_build(tm_index *ix, int r) {
    DevIndex d;
    d.vocab = ix->vocab.d[r]; d.vmask = (uint32_t)ix->vocab.h.size() - 1;
    d.wpool = ix->wpool.d[r];
    d.nodes = ix->nodes.d[r];
    d.ctab = ix->ctab.d[r];
    d.vals = ix->vals.d[r];
    d.exact = ix->exact.d[r]; d.xmask = (uint32_t)ix->exact.h.size() - 1;
    d.xfp = ix->xfp.d[r];
    d.wseq = ix->wseq.d[r];
    d.wbits = ix->wbits.d[r]; d.wcap = ix->wide.empty() ? 0 : ix->wb_words * 32;
    // levels a walk must resolve: the deepest live node's depth (no node below
    // it has children), all of a topic's levels when a binary key has its length
    auto &dc = ix->depth_cnt, &xc = ix->xlen_cnt;
    while (dc.size() > 1 && dc.back() == 0) dc.pop_back();
    while (!xc.empty() && xc.back() == 0) xc.pop_back();
    d.depth = dc.empty() ? 0 : (uint32_t)dc.size() - 1;
    d.xlen_max = xc.empty() ? 0 : (uint32_t)xc.size() - 1;
    d.xlen_mask = 0;
    for (size_t k = 0; k < xc.size() && k < 64; k++) if (xc[k]) d.xlen_mask |= 1ull << k;
    d.hdesc = ix->n_hdesc_keys != 0;
    return d;
}

// ------------------------------------------------------------------ lanes

void free_workspace(Workspace &w) {
    void *wb[] = {w.cnt, w.nr, w.rng, w.lists, w.list_n, w.blk, w.deep_wid, w.deep_stk, w.deep_plus, w.look, w.pairs,
                  w.vres};
    for (void *p : wb) if (p) (void)hipFree(p);
    if (w.hint_h) (void)hipHostFree(w.hint_h);
    w = Workspace{};
}

void free_lane(Lane &l) {
    free_workspace(l.w);
    void *dv[] = {l.d_in, l.d_res, l.d_vals, l.d_o64, l.d_h64};
    for (void *p : dv) if (p) (void)hipFree(p);
    void *pins[] = {l.pin_in, l.pin_out, l.pin_vals};
    for (void *p : pins) if (p) (void)hipHostFree(p);
    if (l.done) (void)hipEventDestroy(l.done);
    if (l.owned && l.s) (void)hipStreamDestroy(l.s);
}

// a lane of replica r (the calling thread's device is r's)
int make_lane(tm_index *ix, int r, hipStream_t s, bool owned, Lane *&out) {
    auto l = std::make_unique<Lane>();
    l->r = r;
    l->owned = owned;
    if (owned) HIPCHK(ix, hipStreamCreateWithFlags(&l->s, hipStreamNonBlocking));
    else l->s = s;
    HIPCHK(ix, hipEventCreateWithFlags(&l->done, hipEventDisableTiming));
    out = l.get();
    ix->lanes.push_back(std::move(l));
    return TM_OK;
}

// A host-API lane for this caller: on the group (one entry of the device
// list) with the fewest batches in flight (round robin among equals), on the
// copy pick_copy chooses there; waiting while every copy has MAX_HOST_LANES in
// use.  Pending deltas are collected first (pick_copy must know which copies
// are up to date).  Leaves the calling thread on the lane's device.
int host_lane(tm_index *ix, std::unique_lock<std::mutex> &g, Lane *&out) {
    for (;;) {
        if (int rc = collect_patch(ix)) return rc;
        int busy[MAX_REPLICAS] = {}, gbusy[MAX_REPLICAS] = {};
        bool gfree[MAX_REPLICAS] = {};
        for (auto &l : ix->lanes)
            if (l->owned) busy[l->r] += l->busy;
        for (int r = 0; r < ix->nrep; r++) {
            gbusy[ix->rep[r].group] += busy[r];
            gfree[ix->rep[r].group] |= busy[r] < MAX_HOST_LANES;
        }
        int bg = -1;
        for (int k = 0; k < ix->ngroups; k++) {
            const int gi = (int)((ix->rr + k) % ix->ngroups);
            if (gfree[gi] && (bg < 0 || gbusy[gi] < gbusy[bg])) bg = gi;
        }
        if (bg >= 0) {
            ix->rr++;
            const int best = pick_copy(ix, bg, busy);
            ix->rep[best].last_use = ++ix->tick;
            HIPCHK(ix, hipSetDevice(ix->rep[best].device));
            for (auto &l : ix->lanes)
                if (l->owned && l->r == best && !l->busy) { l->busy = true; out = l.get(); return TM_OK; }
            int rc = make_lane(ix, best, nullptr, true, out);
            if (rc) return rc;
            out->busy = true;
            return TM_OK;
        }
        ix->cv.wait(g);
    }
}

// releases a checked-out host lane on every exit path (retaking the lock if
// the caller dropped it to wait for the GPU).  Round 6 measured releasing it
// without the lock (an atomic flag, waiters announced): the leader's 55-85 us
// wait for the lock after its GPU wait went, and 16 concurrent callers lost
// 10-15 % (4.0-4.1 vs 4.8-4.9e8 topics/s, profiles/r6/lane_release/) -- the
// lock paces the leaders; kept.
struct LaneLease {
    tm_index *ix;
    std::unique_lock<std::mutex> &g;
    Lane *ln = nullptr;
    ~LaneLease() {
        if (!ln) return;
        if (!g.owns_lock()) g.lock();
        ln->busy = false;
        ix->cv.notify_one();
    }
};

// the group of the calling thread's current HIP device (the first entry of
// the device list on it)
int dev_group(tm_index *ix, int &g) {
    int dev = 0;
    HIPCHK(ix, hipGetDevice(&dev));
    for (int r = 0; r < ix->nrep; r++)
        if (ix->rep[r].device == dev) { g = ix->rep[r].group; return TM_OK; }
    return fail(ix, TM_EINVAL, "device API: the current HIP device holds no replica of this index");
}

// the device-API lane of stream s on replica r; the least recently used one is
// retired (after its batches finish) when MAX_DEV_LANES (stream, replica)
// pairs hold a workspace
int dev_lane(tm_index *ix, hipStream_t s, int r, Lane *&out) {
    int n = 0;
    size_t lru = SIZE_MAX;
    for (size_t i = 0; i < ix->lanes.size(); i++) {
        Lane &l = *ix->lanes[i];
        if (l.owned) continue;
        if (l.s == s && l.r == r) { l.tick = ++ix->tick; out = &l; return TM_OK; }
        n++;
        if (lru == SIZE_MAX || l.tick < ix->lanes[lru]->tick) lru = i;
    }
    if (n >= MAX_DEV_LANES && lru != SIZE_MAX) {
        Lane &l = *ix->lanes[lru];
        HIPCHK(ix, hipSetDevice(ix->rep[l.r].device));
        if (l.used) HIPCHK(ix, hipEventSynchronize(l.done));
        free_lane(l);
        ix->lanes.erase(ix->lanes.begin() + lru);
    }
    HIPCHK(ix, hipSetDevice(ix->rep[r].device));
    int rc = make_lane(ix, r, s, false, out);
    if (rc) return rc;
    out->tick = ++ix->tick;
    return TM_OK;
}

template <class T>
int grow_dev(tm_index *ix, hipStream_t s, T *&p, uint64_t &cap, uint64_t need) {
    if (need <= cap && p) return TM_OK;
    HIPCHK(ix, hipStreamSynchronize(s));   // only this lane's stream uses its buffers
    if (p) HIPCHK(ix, hipFree(p));
    p = nullptr;
    cap = std::max<uint64_t>(need + need / 4, 64);
    HIPCHK(ix, hipMalloc(&p, cap * sizeof(T)));
    return TM_OK;
}

int ensure_ws(tm_index *ix, uint64_t n, Lane &ln) {
    Workspace &w = ln.w;
    if (!w.deep_wid) {
        HIPCHK(ix, hipMalloc(&w.deep_wid, (uint64_t)DEEP_LANES * MAX_LEVELS * 4));
        HIPCHK(ix, hipMalloc(&w.deep_stk, (uint64_t)DEEP_LANES * (MAX_LEVELS + 1) * 8));
        HIPCHK(ix, hipMalloc(&w.deep_plus, (uint64_t)DEEP_LANES * MAX_LEVELS));
        HIPCHK(ix, hipMalloc(&w.list_n, LIST_SLOTS * 4));
        HIPCHK(ix, hipMemsetAsync(w.list_n, 0, LIST_SLOTS * 4, ln.s));
        HIPCHK(ix, hipMalloc(&w.pairs, 2 * SMALL_SEGS * 4));
        HIPCHK(ix, hipMemsetAsync(w.pairs, 0, 2 * SMALL_SEGS * 4, ln.s));
        HIPCHK(ix, hipMalloc(&w.vres, VRES_WORDS * 8));
        HIPCHK(ix, hipMemsetAsync(w.vres, 0, VRES_WORDS * 8, ln.s));
        HIPCHK(ix, hipHostMalloc(&w.hint_h, HINT_WORDS * 4, hipHostMallocMapped));
        std::memset(w.hint_h, 0, HINT_WORDS * 4);
        HIPCHK(ix, hipHostGetDevicePointer(reinterpret_cast<void **>(&w.hint_d), w.hint_h, 0));
    }
    // the batch must see every patch shipped so far, whichever stream it went
    // on (once per patch: later batches on the lane's stream are behind it)
    if (ix->rep[ln.r].last_patch && ln.waited != ix->rep[ln.r].applied) {
        HIPCHK(ix, hipStreamWaitEvent(ln.s, ix->rep[ln.r].last_patch, 0));
        ln.waited = ix->rep[ln.r].applied;
    }
    if (n <= w.cap_n && w.cnt) return TM_OK;
    HIPCHK(ix, hipStreamSynchronize(ln.s));
    if (w.cnt) {
        void *old[] = {w.cnt, w.nr, w.rng, w.lists, w.blk, w.look};
        for (void *p : old) (void)hipFree(p);
    }
    uint64_t c = std::max<uint64_t>(n + n / 4, 1024);
    HIPCHK(ix, hipMalloc(&w.cnt, c * 4));
    HIPCHK(ix, hipMalloc(&w.nr, c * 4));
    HIPCHK(ix, hipMalloc(&w.rng, c * RCAP * 8));
    HIPCHK(ix, hipMalloc(&w.lists, c * (L_COUNT + 1) * 4));
    const uint64_t nblk = c / TILE + 4, nsup = c / ((uint64_t)TILE * SUP) + 4;
    HIPCHK(ix, hipMalloc(&w.blk, (nblk + nsup) * 8));
    HIPCHK(ix, hipMemsetAsync(w.blk, 0, (nblk + nsup) * 8, ln.s));   // zero between batches (k_rewalk_tail)
    w.sup = w.blk + nblk;
    HIPCHK(ix, hipMalloc(&w.look, (c / SM_TOPICS + 4) * 8 * LB_STRIDE));
    HIPCHK(ix, hipMemsetAsync(w.look, 0, (c / SM_TOPICS + 4) * 8 * LB_STRIDE, ln.s));   // no launch tag is 0
    w.cap_n = c;
    return TM_OK;
}

void init_tables(tm_index *ix, uint64_t hint) {
    // tables start small and double at load 1/2: their size follows the live
    // key set, so hot entries stay dense (vocab / top trie levels in L2)
    ix->vocab.h.assign(1024, empty_vocab());
    ix->exact.h.assign(1024, empty_exact());
    ix->xfp.h.assign(1024, 0);
    ix->xcap.assign(ix->exact.h.size(), 0);
    ix->xroff.assign(ix->exact.h.size(), 0);
    ix->nodes.h.reserve(hint / 2 + 1);
    ix->aux.reserve(hint / 2 + 1);
    node_new(ix, NONE, NONE, false);   // ROOT
    ix->vals.h.reserve(hint + 16);
    // a 16-B guard before the first run: k_emit's run-by-run copy loads whole
    // quads that may overhang a run by up to 3 words on either side (the
    // guard after the last run is the device copy's DEV_GUARD slack)
    ix->vals.h.assign(4, 0);
}

// NULL is HIP's default (null) stream -- the stream PyTorch's default stream
// handle (0) names, so device-API batches order with the caller's torch work
hipStream_t pick_stream(tm_index *, void *s) { return reinterpret_cast<hipStream_t>(s); }

// events of one profiled batch (null set when profiling is off)
int prof_begin(tm_index *ix, tm_index::ProfEv &ev, hipStream_t s) {
    ev = {nullptr, nullptr, nullptr, nullptr, 0};
    if (!ix->prof) return TM_OK;
    int dev = 0;
    HIPCHK(ix, hipGetDevice(&dev));
    for (size_t i = 0; i < ix->prof_free.size(); i++)   // events of this device
        if (ix->prof_free[i].device == dev) {
            ev = ix->prof_free[i];
            ix->prof_free.erase(ix->prof_free.begin() + i);
            break;
        }
    if (!ev.b0) {
        HIPCHK(ix, hipEventCreate(&ev.b0)); HIPCHK(ix, hipEventCreate(&ev.w0));
        HIPCHK(ix, hipEventCreate(&ev.w1)); HIPCHK(ix, hipEventCreate(&ev.b1));
        ev.device = dev;
    }
    HIPCHK(ix, hipEventRecord(ev.b0, s));
    return TM_OK;
}

int prof_end(tm_index *ix, tm_index::ProfEv &ev, hipStream_t s) {
    if (!ev.b0) return TM_OK;
    HIPCHK(ix, hipEventRecord(ev.b1, s));
    ix->prof_pending.push_back(ev);
    return TM_OK;
}

// wait for every batch of every lane (caller holds ix->mu)
int drain_lanes(tm_index *ix) {
    for (auto &l : ix->lanes)
        if (l->used) {
            HIPCHK(ix, hipSetDevice(ix->rep[l->r].device));
            HIPCHK(ix, hipEventSynchronize(l->done));
        }
    return TM_OK;
}

}  // namespace

// =================================================================== C ABI

extern "C" {

uint32_t tm_abi_version(void) { return (1u << 16) | 10u; }

const char *tm_last_error(tm_index *) { return g_last_error.c_str(); }

int tm_create_replicas(const tm_options *opts, const int32_t *devices, uint32_t n, tm_index **out) {
    if (!out) return fail(nullptr, TM_EINVAL, "tm_create: out is NULL");
    *out = nullptr;
    const uint32_t copies = opts && opts->copies ? opts->copies : 1;
    if (!devices || n == 0 || n > 8 || copies > 4 || n * copies > (uint32_t)MAX_REPLICAS)
        return fail(nullptr, TM_EINVAL, "tm_create_replicas: 1 to 8 devices, 1 to 4 copies, at most 16 replicas");
    tm_index *ix = new (std::nothrow) tm_index();
    if (!ix) return fail(nullptr, TM_ENOMEM, "tm_create: out of host memory");
    ix->nrep = (int)(n * copies);
    for (int g = 0; g < MAX_REPLICAS; g++) ix->serving[g] = -1;
    ix->ngroups = (int)n;
    hipError_t e = hipSuccess;
    for (uint32_t r = 0; r < n * copies && e == hipSuccess; r++) {
        Replica &R = ix->rep[r];
        R.device = devices[r / copies];
        R.group = (int)(r / copies);
        e = hipSetDevice(R.device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&R.ps, hipStreamNonBlocking);
        for (int i = 0; i < PATCH_RING && e == hipSuccess; i++)
            e = hipEventCreateWithFlags(&R.pdone[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        std::string m = std::string("tm_create: ") + hipGetErrorString(e);
        tm_destroy(ix);
        return fail(nullptr, TM_EDEVICE, m);
    }
    (void)hipSetDevice(ix->rep[0].device);
    init_tables(ix, opts ? opts->hint_keys : 0);
    *out = ix;
    return TM_OK;
}

int tm_create(const tm_options *opts, tm_index **out) {
    int32_t dev = opts ? opts->device : -1;
    if (dev < 0) {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) d = 0;
        dev = d;
    }
    return tm_create_replicas(opts, &dev, 1, out);
}

int tm_replica_stats(tm_index *ix, uint32_t r, uint64_t *batches, int32_t *device) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_replica_stats: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    if (r >= (uint32_t)ix->nrep) return fail(ix, TM_EINVAL, "tm_replica_stats: no such replica");
    if (batches) *batches = ix->rep[r].batches;
    if (device) *device = ix->rep[r].device;
    return TM_OK;
}

namespace { void mf_free_keys(tm_index::MfState &m); }

// TM_HOST_TIMING=1 (diagnostics): where a combined launch's host time goes,
// summed over the process and printed by tm_destroy
struct CmbTiming {
    std::atomic<uint64_t> groups{0}, reqs{0};
    std::atomic<uint64_t> lock_ns{0}, setup_ns{0}, launch_ns{0}, sync_ns{0}, release_ns{0}, done_ns{0}, req_ns{0};
};
static CmbTiming g_cmbt;
// (TM_HOST_TIMING) where tm_commit's time goes
struct CommitTiming {
    std::atomic<uint64_t> n{0}, apply_ns{0}, lock_ns{0}, collect_ns{0}, idle_ns{0}, ship_ns{0};
};
static CommitTiming g_cmt;
static const bool g_cmb_timing = getenv("TM_HOST_TIMING") != nullptr;
static inline uint64_t ns_now() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

int tm_destroy(tm_index *ix) {
    if (!ix) return TM_EINVAL;
    if (g_cmb_timing && g_cmbt.groups) {
        const double g = (double)g_cmbt.groups, us = 1e-3;
        fprintf(stderr, "tm combiner: %lu launches, %lu requests (%.2f per launch); per launch us: lock %.1f "
                        "setup %.1f launch %.1f sync %.1f lane-release %.1f mark-done %.1f; per request %.1f us\n",
                (unsigned long)g_cmbt.groups.load(), (unsigned long)g_cmbt.reqs.load(), g_cmbt.reqs / g,
                g_cmbt.lock_ns * us / g, g_cmbt.setup_ns * us / g, g_cmbt.launch_ns * us / g, g_cmbt.sync_ns * us / g,
                g_cmbt.release_ns * us / g, g_cmbt.done_ns * us / g,
                g_cmbt.req_ns * us / std::max<double>(1.0, (double)g_cmbt.reqs));
    }
    if (g_cmb_timing && g_col_n) {
        const double c = (double)g_col_n, us = 1e-3;
        fprintf(stderr, "tm collect: %lu patches; per patch us: runs %.1f slot-reuse %.1f pinned-copy %.1f\n",
                (unsigned long)g_col_n.load(), g_col_runs_ns * us / c, g_col_slot_ns * us / c, g_col_copy_ns * us / c);
    }
    if (g_cmb_timing && g_cmt.n) {
        const double c = (double)g_cmt.n, us = 1e-3;
        fprintf(stderr, "tm commit: %lu commits; per commit us: image %.1f lock %.1f collect %.1f wait-idle %.1f "
                        "ship %.1f\n", (unsigned long)g_cmt.n.load(), g_cmt.apply_ns * us / c, g_cmt.lock_ns * us / c,
                g_cmt.collect_ns * us / c, g_cmt.idle_ns * us / c, g_cmt.ship_ns * us / c);
    }
    for (int r = 0; r < ix->nrep; r++) {
        (void)hipSetDevice(ix->rep[r].device);
        (void)hipDeviceSynchronize();
    }
    for (auto &l : ix->lanes) {
        (void)hipSetDevice(ix->rep[l->r].device);
        free_lane(*l);
    }
    for (int r = 0; r < ix->nrep; r++) {
        Replica &R = ix->rep[r];
        (void)hipSetDevice(R.device);
        void *bufs[] = {ix->vocab.d[r], ix->wpool.d[r], ix->nodes.d[r], ix->ctab.d[r], ix->vals.d[r], ix->exact.d[r],
                        ix->xfp.d[r], ix->wseq.d[r], ix->wbits.d[r]};
        for (void *p : bufs) if (p) (void)hipFree(p);
        for (int i = 0; i < PATCH_RING; i++) {
            if (R.pdev[i]) (void)hipFree(R.pdev[i]);
            if (R.pdone[i]) (void)hipEventDestroy(R.pdone[i]);
        }
        if (R.ps) (void)hipStreamDestroy(R.ps);
    }
    (void)hipSetDevice(ix->rep[0].device);
    mf_free_keys(ix->mf);
    for (void *p : {(void *)ix->mf.q, (void *)ix->mf.err, (void *)ix->mf.hit, (void *)ix->mf.out}) if (p) (void)hipFree(p);
    if (ix->mf.s) (void)hipStreamDestroy(ix->mf.s);
    for (auto &p : ix->patch) if (p.pin) (void)hipHostFree(p.pin);
    for (auto &b : ix->pinned) (void)(b.vram ? hipFree(b.host) : hipHostFree(b.host));
    for (auto *v : {&ix->prof_pending, &ix->prof_free})
        for (auto &ev : *v) {
            (void)hipSetDevice(ev.device);
            for (hipEvent_t x : {ev.b0, ev.w0, ev.w1, ev.b1}) (void)hipEventDestroy(x);
        }
    delete ix;
    return TM_OK;
}

int tm_apply_deltas_ex(tm_index *ix, uint64_t n, const uint8_t *ops, const uint8_t *fb, const uint64_t *fo,
                       const uint32_t *values, const uint8_t *key_flags, uint64_t *out_epoch) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_apply_deltas: null handle");
    if (n && (!ops || !fo || !values || (!fb && fo[n] != fo[0])))
        return fail(ix, TM_EINVAL, "tm_apply_deltas: null buffer");
    for (uint64_t i = 0; i < n; i++)
        if (ops[i] > TM_OP_INSERT || fo[i + 1] < fo[i] || fo[i + 1] - fo[i] > 0xFFFFFFFFull)
            return fail(ix, TM_EINVAL, "tm_apply_deltas: bad op or offsets at " + std::to_string(i));
    std::lock_guard<std::mutex> g(ix->img);   // the host image only: batches without a delta to pick up go on
    std::vector<WordRef> w;
    std::vector<uint32_t> wids;
    try {
        for (uint64_t i = 0; i < n; i++)
            key_op(ix, ops[i] == TM_OP_INSERT, fb + fo[i], (uint32_t)(fo[i + 1] - fo[i]), values[i],
                   key_flags ? key_flags[i] : 0, w, wids);
        reclaim(ix);
        wide_dense(ix);
    } catch (const std::bad_alloc &) {
        return fail(ix, TM_ENOMEM, "tm_apply_deltas: out of host memory");
    }
    // the keys changed above are what every batch queued from now on sees:
    // a reader registered from now on begins at the new epoch
    if (n) ix->img_dirty.store(true, std::memory_order_release);
    const uint64_t e = n ? ix->epoch.fetch_add(1, std::memory_order_acq_rel) + 1 : ix->epoch.load();
    if (out_epoch) *out_epoch = e;
    return TM_OK;
}

int tm_apply_deltas(tm_index *ix, uint64_t n, const uint8_t *ops, const uint8_t *fb, const uint64_t *fo,
                    const uint32_t *values, const uint8_t *key_flags) {
    return tm_apply_deltas_ex(ix, n, ops, fb, fo, values, key_flags, nullptr);
}

// tm_commit (include/tmatch.h): the deltas reach the host image while
// batches are held off collecting them (img_hold), then -- under the device
// lock -- one patch is collected and applied to a copy of each group that no
// batch is reading, which becomes the group's serving copy, and only then is
// the patch published (pub_seq): batches queued afterwards read that copy,
// and no batch ever waits on the GPU for this patch.  While every copy of a
// group has readers the committer waits (the lock released) for one to
// drain, up to COMMIT_WAIT; past it -- or with one copy per group -- the
// patch is published as tm_apply_deltas' are (batches take it in stream
// order, behind the batches reading that copy).
constexpr auto COMMIT_WAIT = std::chrono::milliseconds(20);

int tm_commit(tm_index *ix, uint64_t n, const uint8_t *ops, const uint8_t *fb, const uint64_t *fo,
              const uint32_t *values, const uint8_t *key_flags, uint64_t *out_epoch) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_commit: null handle");
    ix->img_hold.fetch_add(1, std::memory_order_acq_rel);
    struct Unhold {
        tm_index *ix;
        ~Unhold() { ix->img_hold.fetch_sub(1, std::memory_order_acq_rel); }
    } unhold{ix};
    const uint64_t ta = g_cmb_timing ? ns_now() : 0;
    int rc = tm_apply_deltas_ex(ix, n, ops, fb, fo, values, key_flags, out_epoch);
    if (rc || !n) return rc;
    const uint64_t tb = g_cmb_timing ? ns_now() : 0;
    std::unique_lock<std::mutex> g(ix->mu);
    const uint64_t tc = g_cmb_timing ? ns_now() : 0;
    if ((rc = collect_patch(ix, true))) return rc;
    const uint64_t q = ix->patch_seq;
    if (ix->pub_seq >= q) return TM_OK;   // (nothing to ship: the deltas changed no device word)
    ix->commits++;
    const uint64_t td = g_cmb_timing ? ns_now() : 0;
    uint64_t t_idle = 0, t_ship = 0;
    const auto t0 = std::chrono::steady_clock::now();
    bool done[MAX_REPLICAS] = {}, waited = false;
    int left = ix->ngroups;
    for (;;) {
        const bool late = std::chrono::steady_clock::now() - t0 > COMMIT_WAIT;
        bool busy[MAX_REPLICAS] = {};   // copies with a batch still reading them (one event query per lane)
        for (auto &l : ix->lanes)
            if (!busy[l->r] && lane_busy(*l)) busy[l->r] = true;
        for (int gi = 0; gi < ix->ngroups; gi++) {
            if (done[gi]) continue;
            int pick = -1, copies = 0;
            for (int r = 0; r < ix->nrep; r++) {
                if (ix->rep[r].group != gi) continue;
                copies++;
                // the idle copy that lags most: every copy takes every patch in
                // turn, so none falls PATCH_RING behind (a ring slot's reuse
                // would otherwise bring a lagging copy up and wait for it
                // under the index lock)
                if (!busy[r] && (pick < 0 || ix->rep[r].applied < ix->rep[pick].applied)) pick = r;
            }
            if (pick < 0 && copies > 1 && !late) continue;   // wait for a copy to drain
            if (pick >= 0) {
                const uint64_t t0s = g_cmb_timing ? ns_now() : 0;
                if ((rc = bring_up(ix, pick, q, ix->rep[pick].ps, true))) return rc;
                if (g_cmb_timing) t_ship += ns_now() - t0s;
                ix->serving[gi] = pick;
            } else {
                ix->commit_forced++;   // published below; the group's batches take the patch themselves
            }
            done[gi] = true;
            left--;
        }
        if (!left) break;
        waited = true;
        const uint64_t tw = g_cmb_timing ? ns_now() : 0;
        g.unlock();
        std::this_thread::sleep_for(std::chrono::microseconds(2));
        g.lock();
        if (g_cmb_timing) t_idle += ns_now() - tw;
    }
    if (waited) ix->commit_waits++;
    if (ix->pub_seq < q) ix->pub_seq = q;
    if (g_cmb_timing) {
        g_cmt.n++;
        g_cmt.apply_ns += tb - ta; g_cmt.lock_ns += tc - tb; g_cmt.collect_ns += td - tc;
        g_cmt.idle_ns += t_idle; g_cmt.ship_ns += t_ship;
    }
    return TM_OK;
}

int tm_read_begin(tm_index *ix, uint64_t *ticket) {
    if (!ix || !ticket) return fail(ix, TM_EINVAL, "tm_read_begin: null argument");
    std::lock_guard<std::mutex> g(ix->ep_mu);
    const uint64_t e = ix->epoch.load(std::memory_order_acquire);
    *ticket = ix->next_ticket++;
    ix->readers.emplace(*ticket, e);
    ix->reader_epochs.insert(e);
    return TM_OK;
}

int tm_read_end(tm_index *ix, uint64_t ticket) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_read_end: null handle");
    std::lock_guard<std::mutex> g(ix->ep_mu);
    auto it = ix->readers.find(ticket);
    if (it == ix->readers.end()) return fail(ix, TM_EINVAL, "tm_read_end: unknown ticket");
    ix->reader_epochs.erase(ix->reader_epochs.find(it->second));
    ix->readers.erase(it);
    return TM_OK;
}

int tm_epoch(tm_index *ix, uint64_t *current, uint64_t *safe) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_epoch: null handle");
    std::lock_guard<std::mutex> g(ix->ep_mu);
    const uint64_t e = ix->epoch.load(std::memory_order_acquire);
    if (current) *current = e;
    if (safe) *safe = ix->reader_epochs.empty() ? e : *ix->reader_epochs.begin();
    return TM_OK;
}

int tm_sync(tm_index *ix, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_sync: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    int dev = 0, r0 = 0;   // `stream` belongs to the current device: its replica (else replica 0, its patch stream)
    HIPCHK(ix, hipGetDevice(&dev));
    hipStream_t s = pick_stream(ix, stream);
    bool found = false;
    for (int r = 0; r < ix->nrep && !found; r++) if (ix->rep[r].device == dev) { r0 = r; found = true; }
    if (!found) s = ix->rep[0].ps;
    return sync_locked(ix, r0, s);
}

int tm_match_batch_dev_ex(tm_index *ix, uint64_t n, const uint8_t *bytes, const uint64_t *offs, uint64_t *hit_offs,
                          uint32_t *out, uint64_t cap, uint8_t *err, uint32_t order, uint32_t *ucnt, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch_dev: null handle");
    if (!hit_offs || (n && (!offs || !bytes || !err))) return fail(ix, TM_EINVAL, "tm_match_batch_dev: null buffer");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch_dev: batch too large");
    if (order > TM_ORDER_UNIQUE) return fail(ix, TM_EINVAL, "tm_match_batch_dev: bad order");
    std::lock_guard<std::mutex> g(ix->mu);
    hipStream_t s = pick_stream(ix, stream);
    int rc, grp = 0;
    Lane *ln;
    if ((rc = dev_group(ix, grp))) return rc;
    if ((rc = collect_patch(ix))) return rc;
    const int r = pick_copy(ix, grp, nullptr, s, true);
    ix->rep[r].last_use = ++ix->tick;
    ix->rep[r].batches++;
    if ((rc = dev_lane(ix, s, r, ln))) return rc;
    if ((rc = sync_locked(ix, ln->r, s))) return rc;
    if ((rc = ensure_ws(ix, n, *ln))) return rc;
    const DevIndex d = dev_view(ix, ln->r);
    tm_index::ProfEv ev;
    if ((rc = prof_begin(ix, ev, s))) return rc;
    uint32_t tag;
    if ((rc = next_tag(ix, *ln, s, tag))) return rc;
    // (asynchronous: a failed look-back reaches the caller as err 4 flags, include/tmatch.h)
    int path = PATH_PHASES;
    HIPCHK(ix, launch_match(d, ln->w, n, bytes, offs, hit_offs, err, out, out ? cap : 0, tag, next_lb(ix),
                            ix->dbg_phases, ix->small_kind, s, ev.w0, ev.w1, &path));
    ix->path_batches[path]++;
    if (order != TM_ORDER_TRAVERSAL && out)
        HIPCHK(ix, launch_sort_segments(ln->w, n, hit_offs, out, cap, order == TM_ORDER_UNIQUE, ucnt, s));
    if ((rc = batch_done(ix, *ln))) return rc;
    return prof_end(ix, ev, s);
}

int tm_match_batch_dev_pairs(tm_index *ix, uint64_t n, const uint8_t *bytes, const uint64_t *offs, uint32_t *pairs,
                             uint32_t *out, uint64_t cap, uint8_t *err, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch_dev_pairs: null handle");
    if (!pairs || (n && (!offs || !bytes || !err))) return fail(ix, TM_EINVAL, "tm_match_batch_dev_pairs: null buffer");
    if (reinterpret_cast<uintptr_t>(pairs) & 7) return fail(ix, TM_EINVAL, "tm_match_batch_dev_pairs: pairs not 8-byte aligned");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch_dev_pairs: batch too large");
    if (!out) cap = 0;
    if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;   // (32-bit positions)
    std::lock_guard<std::mutex> g(ix->mu);
    hipStream_t s = pick_stream(ix, stream);
    int rc, grp = 0;
    Lane *ln;
    if ((rc = dev_group(ix, grp))) return rc;
    if ((rc = collect_patch(ix))) return rc;
    const int r = pick_copy(ix, grp, nullptr, s, true);
    ix->rep[r].last_use = ++ix->tick;
    ix->rep[r].batches++;
    if ((rc = dev_lane(ix, s, r, ln))) return rc;
    if ((rc = sync_locked(ix, ln->r, s))) return rc;
    if ((rc = ensure_ws(ix, n, *ln))) return rc;
    const DevIndex d = dev_view(ix, ln->r);
    tm_index::ProfEv ev;
    if ((rc = prof_begin(ix, ev, s))) return rc;
    HIPCHK(ix, launch_match_pairs(d, ln->w, n, bytes, offs, err, pairs, out, cap, s, ev.w0, ev.w1));
    ix->path_batches[PATH_PHASES]++;
    if ((rc = batch_done(ix, *ln))) return rc;
    return prof_end(ix, ev, s);
}

int tm_match_batch_dev(tm_index *ix, uint64_t n, const uint8_t *bytes, const uint64_t *offs, uint64_t *hit_offs,
                       uint32_t *out, uint64_t cap, uint8_t *err, void *stream) {
    return tm_match_batch_dev_ex(ix, n, bytes, offs, hit_offs, out, cap, err, TM_ORDER_TRAVERSAL, nullptr, stream);
}

int tm_sort_segments(tm_index *ix, uint64_t n, const uint64_t *hit_offs, uint32_t *vals, uint64_t cap, uint32_t order,
                     uint32_t *ucnt, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_sort_segments: null handle");
    if (!hit_offs || (cap && !vals) || order > TM_ORDER_UNIQUE) return fail(ix, TM_EINVAL, "tm_sort_segments: bad argument");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_sort_segments: too many segments");
    if (order == TM_ORDER_TRAVERSAL || !n) return TM_OK;
    std::lock_guard<std::mutex> g(ix->mu);
    hipStream_t s = pick_stream(ix, stream);
    Lane *ln;
    int rc, grp = 0;
    if ((rc = dev_group(ix, grp))) return rc;
    int r = 0;
    while (ix->rep[r].group != grp) r++;
    if ((rc = dev_lane(ix, s, r, ln))) return rc;
    if ((rc = ensure_ws(ix, n, *ln))) return rc;
    HIPCHK(ix, launch_sort_segments(ln->w, n, hit_offs, vals, cap, order == TM_ORDER_UNIQUE, ucnt, s));
    return batch_done(ix, *ln);
}

int tm_stream_release(tm_index *ix, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_stream_release: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    hipStream_t s = pick_stream(ix, stream);
    int dev = 0;
    HIPCHK(ix, hipGetDevice(&dev));
    for (size_t i = 0; i < ix->lanes.size(); i++) {
        Lane &l = *ix->lanes[i];
        if (l.owned || l.s != s || ix->rep[l.r].device != dev) continue;
        if (l.used) HIPCHK(ix, hipEventSynchronize(l.done));
        free_lane(l);
        ix->lanes.erase(ix->lanes.begin() + i);
        break;
    }
    return TM_OK;
}

namespace {

// Batches of up to ZC_TOPICS topics are staged zero-copy: the kernels read the
// topics from, and write offsets / flags / values into, mapped pinned host
// memory over PCIe.  A small batch then costs its kernels plus one host
// synchronisation -- no copy commands and no gaps between them.  Larger
// batches move in one H2D and one D2H transfer.
constexpr uint64_t ZC_TOPICS = 65536;

int pin_mapped(tm_index *ix, hipStream_t s, uint8_t *&host, uint8_t *&dev, uint64_t &cap, uint64_t need) {
    if (need <= cap) return TM_OK;
    HIPCHK(ix, hipStreamSynchronize(s));
    if (host) HIPCHK(ix, hipHostFree(host));
    host = dev = nullptr;
    cap = need + need / 4;
    HIPCHK(ix, hipHostMalloc(&host, cap, hipHostMallocMapped));
    HIPCHK(ix, hipHostGetDevicePointer(reinterpret_cast<void **>(&dev), host, 0));
    return TM_OK;
}

// the TM_ALLOC_VRAM buffer holding [p, p + bytes), or null (caller holds ix->mu)
const tm_index::Pinned *vram_buf(tm_index *ix, const void *p, uint64_t bytes) {
    const uint8_t *q = static_cast<const uint8_t *>(p);
    for (const auto &b : ix->pinned)
        if (b.vram && q >= b.host && bytes <= b.size && q - b.host <= (ptrdiff_t)(b.size - bytes)) return &b;
    return nullptr;
}

// A host topic batch -> what the kernels read: rebased offsets, then the bytes
// (16-aligned: the walk's aligned 16-byte loads), in one buffer of the lane.
// Inputs in TM_ALLOC_VRAM memory are read where they lie, never by the host
// (each host read of it is an uncached PCIe round trip, ~0.6 us):
// bytes there are used in place with the offsets unrebased; u64 offsets there
// too are used in place; u32 offsets there (to32v, the 32-bit API) are widened
// by a kernel into the lane's scratch.  Only `to[0]`/`to[n]` (or to32v[n])
// are read by the host for a VRAM batch.
int stage_in(tm_index *ix, Lane &ln, uint64_t n, const uint8_t *tb, const uint64_t *to, const uint32_t *to32v,
             const uint8_t *&dbytes, const uint64_t *&doffs) {
    int rc;
    const uint64_t end = to32v ? to32v[n] : to[n];
    const uint64_t b0 = to32v ? 0 : to[0];
    const bool vbytes = vram_buf(ix, tb, std::max<uint64_t>(end, 1)) != nullptr;
    const bool voffs = to32v || vram_buf(ix, to, (n + 1) * 8) != nullptr;
    if (vbytes && voffs) {   // both in HBM already: nothing crosses PCIe
        dbytes = tb;
        if (to32v) {
            if ((rc = grow_dev(ix, ln.s, ln.d_o64, ln.d_o64_cap, n + 1))) return rc;
            HIPCHK(ix, launch_offs_widen(to32v, ln.d_o64, n + 1, ln.s));
            doffs = ln.d_o64;
        } else {
            doffs = to;
        }
        return TM_OK;
    }
    if (to32v || voffs) {   // offsets in HBM, bytes in host memory (no caller of the library does this)
        uint64_t *o = nullptr;
        if ((rc = pin_mapped(ix, ln.s, ln.pin_in, ln.pin_in_dev, ln.pin_in_cap, (n + 1) * 8 + end + 32))) return rc;
        o = reinterpret_cast<uint64_t *>(ln.pin_in);
        if (to32v) HIPCHK(ix, launch_offs_widen(to32v, reinterpret_cast<uint64_t *>(ln.pin_in_dev), n + 1, ln.s));
        else HIPCHK(ix, hipMemcpyAsync(o, to, (n + 1) * 8, hipMemcpyDeviceToHost, ln.s));
        const uint64_t boff = ((n + 1) * 8 + 15) & ~15ull;
        if (end) memcpy(ln.pin_in + boff, tb, end);   // bytes [0, end): the offsets stay unrebased
        dbytes = ln.pin_in_dev + boff;
        doffs = reinterpret_cast<const uint64_t *>(ln.pin_in_dev);
        if (n > ZC_TOPICS) {
            if ((rc = grow_dev(ix, ln.s, ln.d_in, ln.d_in_cap, boff + end + 16))) return rc;
            HIPCHK(ix, hipMemcpyAsync(ln.d_in, ln.pin_in, boff + end, hipMemcpyHostToDevice, ln.s));
            dbytes = ln.d_in + boff;
            doffs = reinterpret_cast<const uint64_t *>(ln.d_in);
        }
        return TM_OK;
    }
    const uint64_t nbytes = vbytes ? 0 : end - b0;   // bytes in HBM: only the offsets move
    const uint64_t boff = ((n + 1) * 8 + 15) & ~15ull;
    const uint64_t need = boff + nbytes + 16;
    if ((rc = pin_mapped(ix, ln.s, ln.pin_in, ln.pin_in_dev, ln.pin_in_cap, need))) return rc;
    uint64_t *po = reinterpret_cast<uint64_t *>(ln.pin_in);
    const uint64_t rb = vbytes ? 0 : b0;
    for (uint64_t i = 0; i <= n; i++) po[i] = to[i] - rb;
    if (nbytes) memcpy(ln.pin_in + boff, tb + b0, nbytes);
    const uint8_t *base = ln.pin_in_dev;
    if (n > ZC_TOPICS) {
        if ((rc = grow_dev(ix, ln.s, ln.d_in, ln.d_in_cap, need))) return rc;
        HIPCHK(ix, hipMemcpyAsync(ln.d_in, ln.pin_in, boff + nbytes, hipMemcpyHostToDevice, ln.s));
        base = ln.d_in;
    }
    doffs = reinterpret_cast<const uint64_t *>(base);
    dbytes = vbytes ? tb : base + boff;
    return TM_OK;
}

// where the kernels write `bytes` of per-topic results (read back by fetch_out)
int stage_out(tm_index *ix, Lane &ln, uint64_t n, uint64_t bytes, uint8_t *&dout) {
    int rc;
    if ((rc = pin_mapped(ix, ln.s, ln.pin_out, ln.pin_out_dev, ln.pin_out_cap, bytes + 16))) return rc;
    dout = ln.pin_out_dev;
    if (n > ZC_TOPICS) {
        if ((rc = grow_dev(ix, ln.s, ln.d_res, ln.d_res_cap, bytes + 16))) return rc;
        dout = ln.d_res;
    }
    return TM_OK;
}

int fetch_out(tm_index *ix, Lane &ln, uint64_t n, uint64_t bytes) {
    if (n > ZC_TOPICS && bytes) HIPCHK(ix, hipMemcpyAsync(ln.pin_out, ln.d_res, bytes, hipMemcpyDeviceToHost, ln.s));
    return TM_OK;
}

}  // namespace

// device address of [p, p + bytes) if the range lies in one tm_host_alloc buffer
static uint8_t *pinned_dev(tm_index *ix, const void *p, uint64_t bytes) {
    const uint8_t *q = static_cast<const uint8_t *>(p);
    for (const auto &b : ix->pinned)
        if (q >= b.host && bytes <= b.size && q - b.host <= (ptrdiff_t)(b.size - bytes)) return b.dev + (q - b.host);
    return nullptr;
}

int tm_host_alloc_ex(tm_index *ix, uint64_t bytes, uint32_t flags, void **out) {
    if (!ix || !out) return fail(ix, TM_EINVAL, "tm_host_alloc: null argument");
    *out = nullptr;
    if (flags & ~TM_ALLOC_VRAM) return fail(ix, TM_EINVAL, "tm_host_alloc_ex: unknown flags");
    std::lock_guard<std::mutex> g(ix->mu);
    HIPCHK(ix, hipSetDevice(ix->rep[0].device));
    void *h = nullptr, *d = nullptr;
    if (flags & TM_ALLOC_VRAM) {
        // a replica on another device would read it over the fabric: one device only
        for (int r = 1; r < ix->nrep; r++)
            if (ix->rep[r].device != ix->rep[0].device)
                return fail(ix, TM_EINVAL, "tm_host_alloc_ex: TM_ALLOC_VRAM needs a one-device index");
        // the host writes it through the PCIe BAR: only where the whole of the
        // device's memory is mapped there (large / resizable BAR) -- else a host
        // store could fault the caller; TM_EINVAL, and the caller
        // keeps its inputs in tm_host_alloc memory (the NIF does)
        int large_bar = 0;
        if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, ix->rep[0].device) != hipSuccess || !large_bar)
            return fail(ix, TM_EINVAL, "tm_host_alloc_ex: the device's memory is not mapped for the host (no large BAR)");
        // fine-grained: the host maps it through the BAR (same virtual address)
        if (hipExtMallocWithFlags(&d, bytes ? bytes : 1, hipDeviceMallocFinegrained) != hipSuccess || !d)
            return fail(ix, TM_ENOMEM, "tm_host_alloc_ex: fine-grained device allocation failed");
        hipPointerAttribute_t pa;
        if (hipPointerGetAttributes(&pa, d) != hipSuccess || pa.type != hipMemoryTypeDevice) {
            (void)hipFree(d);
            return fail(ix, TM_EINVAL, "tm_host_alloc_ex: the allocation is not device memory");
        }
        ix->pinned.push_back({static_cast<uint8_t *>(d), static_cast<uint8_t *>(d), bytes, true});
        *out = d;
        return TM_OK;
    }
    // portable: every replica's device reads it in place (one virtual address on ROCm)
    if (hipHostMalloc(&h, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess || !h)
        return fail(ix, TM_ENOMEM, "tm_host_alloc: hipHostMalloc failed");
    HIPCHK(ix, hipHostGetDevicePointer(&d, h, 0));
    ix->pinned.push_back({static_cast<uint8_t *>(h), static_cast<uint8_t *>(d), bytes, false});
    *out = h;
    return TM_OK;
}

int tm_host_alloc(tm_index *ix, uint64_t bytes, void **out) { return tm_host_alloc_ex(ix, bytes, 0, out); }

int tm_host_free(tm_index *ix, void *p) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_host_free: null handle");
    if (!p) return TM_OK;
    std::lock_guard<std::mutex> g(ix->mu);
    for (size_t i = 0; i < ix->pinned.size(); i++) {
        if (ix->pinned[i].host != p) continue;
        int rc = drain_lanes(ix);   // no batch may still read or write it
        if (rc) return rc;
        if (ix->pinned[i].vram) HIPCHK(ix, hipFree(p));
        else HIPCHK(ix, hipHostFree(p));
        ix->pinned.erase(ix->pinned.begin() + i);
        return TM_OK;
    }
    return fail(ix, TM_EINVAL, "tm_host_free: not a tm_host_alloc buffer of this index");
}

// TM_HOST_TIMING=1: per-phase host timings of tm_match_batch on stderr (diagnostics)
static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// After a failed one-launch batch (its look-back wait expired: err 4 flags,
// never a client error -- the reference raises badarg only for a '+'/'#'
// level, emqx_trie_search.erl:374-375): the first failure runs the batch
// again, on the same lane with the current device view; the second returns
// TM_EDEVICE for the whole call.  Retakes the index lock (released for the
// GPU wait).
static int retry_or_fail(tm_index *ix, std::unique_lock<std::mutex> &g, Lane &ln, int tries) {
    if (tries >= 1)
        return fail(ix, TM_EDEVICE, "tm_match_batch: the batch failed on the device twice (look-back wait expired, "
                                    "err 4); not matched");
    ix->retried_batches++;
    g.lock();
    HIPCHK(ix, hipSetDevice(ix->rep[ln.r].device));
    return sync_locked(ix, ln.r, ln.s);
}

// ---- the host-batch combiner (32-bit in-place batches, the NIF's calls)
//
// Concurrent callers' small batches run better as fewer, larger launches: a
// lone 4k batch keeps the GPU ~26 us for fixed costs a 64k batch pays once
// (host to host: 4k 0.040 ms, 64k 0.19 ms), and 8 callers' kernels do not
// overlap beyond ~3 at a time.  A caller queues its batch;
// while fewer than cmb_leaders launches are running it takes the lead: it
// takes the queued batches (in order, up to SMALL_SEGS of them and
// ZC_TOPICS topics), runs them as ONE k_walk_small launch with a segment
// table (each segment its own inputs, outputs and look-back region), and
// marks them done, waking each of their callers (one condition variable per
// request: no herd of every waiting caller per launch).  A lone caller leads
// its own batch at once: its latency is the single-batch path's.
// TM_DEBUG_CMB_GATHER (us, study knob, 0 = off): a new leader first waits up to
// that long while fewer batches are queued or in flight than the recent
// high-water mark (callers between two batches are about to queue theirs), so
// launches carry more batches.  (Round 6 measured, and removed, a landing
// variant: the launch writing its outputs to an HBM arena and one copy kernel
// moving them to the callers' buffers -- slower than the walk's in-place
// writes)
struct SmallReq {
    uint64_t n;
    const uint8_t *db; const uint8_t *dof; uint8_t *dh; uint8_t *de; uint8_t *dv;
    uint64_t cap;
    bool pairs = false;         // (offset, count) pairs out (tm_match_batch32_pairs); a launch carries one kind
    int rc = TM_OK;
    bool done = false;
    std::condition_variable cv;
    std::atomic<int> poke{0};   // done, or it may lead: a spinning waiter stops spinning
};
constexpr int CMB_LEGACY = 1;   // (not a TM_ code) the index no longer allows the one-launch path
constexpr uint64_t CMB_HW_NS = 2000000;   // the high-water mark's memory (2 ms)

static int run_small_group(tm_index *ix, const std::vector<SmallReq *> &grp, uint64_t *t_sync_end) {
    uint64_t total = 0;
    for (auto *r : grp) total += r->n;
    const uint64_t ta = g_cmb_timing ? ns_now() : 0;
    std::unique_lock<std::mutex> g(ix->mu);
    const uint64_t tb = g_cmb_timing ? ns_now() : 0;
    LaneLease lease{ix, g};
    int rc;
    if ((rc = host_lane(ix, g, lease.ln))) return rc;
    Lane &ln = *lease.ln;
    const hipStream_t s = ln.s;
    if ((rc = sync_locked(ix, ln.r, s))) return rc;
    if ((rc = ensure_ws(ix, total + (uint64_t)SMALL_SEGS * SM_TOPICS, ln))) return rc;
    if (!small_path_ok(dev_view(ix, ln.r), total)) return CMB_LEGACY;
    ix->rep[ln.r].batches++;
    SmallSegs sg{};
    sg.count = (uint32_t)grp.size();
    sg.pairs = grp[0]->pairs ? 1u : 0u;
    for (size_t k = 0; k < grp.size(); k++) {
        const SmallReq &r = *grp[k];
        const uint64_t vcap = r.dv ? r.cap : 0;
        sg.s[k] = SmallSeg{r.db ? r.db : r.dof, r.dof, r.dh, r.de, reinterpret_cast<uint32_t *>(r.dv), vcap,
                           (uint32_t)r.n, 0};
    }
    const uint64_t tc = g_cmb_timing ? ns_now() : 0;
    for (int tries = 0;; tries++) {
        const DevIndex d = dev_view(ix, ln.r);
        uint32_t tag;
        if ((rc = next_tag(ix, ln, s, tag))) return rc;
        int path = PATH_SMALL;
        HIPCHK(ix, launch_small_segs(d, ln.w, sg, true, tag, next_lb(ix), ix->small_kind, s, &path));
        ix->path_batches[path]++;
        ix->cmb_launches++;
        ix->cmb_batches += grp.size();
        if ((rc = batch_done(ix, ln))) return rc;
        g.unlock();
        const uint64_t td = g_cmb_timing ? ns_now() : 0;
        HIPCHK(ix, hipStreamSynchronize(s));
        if (g_cmb_timing) {
            const uint64_t te = ns_now();
            g_cmbt.groups++;
            g_cmbt.lock_ns += tb - ta; g_cmbt.setup_ns += tc - tb; g_cmbt.launch_ns += td - tc; g_cmbt.sync_ns += te - td;
            *t_sync_end = te;
        }
        if (!batch_failed(ix, ln)) break;
        if ((rc = retry_or_fail(ix, g, ln, tries))) return rc;
    }
    return TM_OK;
}

// (caller holds cmb_mu) queued + in flight, against the recent high-water mark
static void cmb_note_load(tm_index *ix) {
    const int cur = (int)ix->cmb_q.size() + ix->cmb_inflight;
    const uint64_t t = ns_now();
    if (cur >= ix->cmb_hw || t - ix->cmb_hw_ns > CMB_HW_NS) { ix->cmb_hw = cur; ix->cmb_hw_ns = t; }
}

static int small_combined(tm_index *ix, SmallReq &rq) {
    const uint64_t t_in = g_cmb_timing ? ns_now() : 0;
    struct ReqTime {   // (on every return path)
        uint64_t t;
        ~ReqTime() { if (g_cmb_timing) { g_cmbt.reqs++; g_cmbt.req_ns += ns_now() - t; } }
    } rt{t_in};
    std::unique_lock<std::mutex> lk(ix->cmb_mu);
    ix->cmb_q.push_back(&rq);
    cmb_note_load(ix);
    if (ix->cmb_gathering) ix->cmb_gcv.notify_all();
    while (!rq.done) {
        if (ix->cmb_running < std::max(ix->cmb_leaders.load(), 1) && !ix->cmb_q.empty()) {
            ix->cmb_running++;
            const int gus = ix->cmb_gather_us.load(std::memory_order_relaxed);
            if (gus > 0) {   // the gather window (study knob)
                const auto dl = std::chrono::steady_clock::now() + std::chrono::microseconds(gus);
                ix->cmb_gathering++;
                for (;;) {
                    uint64_t q = 0;
                    for (auto *r : ix->cmb_q) q += r->n;
                    if ((int)ix->cmb_q.size() + ix->cmb_inflight >= ix->cmb_hw || ix->cmb_q.size() >= (size_t)SMALL_SEGS ||
                        q >= ZC_TOPICS)
                        break;
                    if (ix->cmb_gcv.wait_until(lk, dl) == std::cv_status::timeout) break;
                }
                ix->cmb_gathering--;
            }
            std::vector<SmallReq *> grp;
            uint64_t total = 0;
            const bool pairs = ix->cmb_q.front()->pairs;   // a launch carries one output kind: the front's
            for (auto it = ix->cmb_q.begin(); it != ix->cmb_q.end() && grp.size() < (size_t)SMALL_SEGS;) {
                if ((*it)->pairs != pairs || total + (*it)->n > ZC_TOPICS) { ++it; continue; }
                total += (*it)->n;
                grp.push_back(*it);
                it = ix->cmb_q.erase(it);
            }
            ix->cmb_inflight += (int)grp.size();
            if (!ix->cmb_q.empty() && ix->cmb_running < ix->cmb_leaders.load()) ix->cmb_q.front()->cv.notify_one();
            lk.unlock();
            uint64_t t_sync_end = 0;
            const int rc = run_small_group(ix, grp, &t_sync_end);   // (the lane is released on return)
            const uint64_t t_rel = g_cmb_timing ? ns_now() : 0;
            lk.lock();
            if (g_cmb_timing && t_sync_end) {
                g_cmbt.release_ns += t_rel - t_sync_end;
                g_cmbt.done_ns += ns_now() - t_rel;
            }
            for (auto *r : grp) {
                r->rc = rc;
                r->done = true;
                if (r != &rq) { r->poke.store(1, std::memory_order_release); r->cv.notify_one(); }
            }
            ix->cmb_inflight -= (int)grp.size();
            ix->cmb_running--;
            if (!ix->cmb_q.empty()) {   // it may lead now
                ix->cmb_q.front()->poke.store(1, std::memory_order_release);
                ix->cmb_q.front()->cv.notify_one();
            }
            continue;
        }
        const int spin = ix->cmb_spin_us.load(std::memory_order_relaxed);
        if (spin > 0) {   // TM_DEBUG_CMB_SPIN: spin a while before sleeping (no futex wake-up on the reply path)
            rq.poke.store(0, std::memory_order_relaxed);
            lk.unlock();
            const uint64_t dl = ns_now() + (uint64_t)spin * 1000;
            while (!rq.poke.load(std::memory_order_acquire) && ns_now() < dl) __builtin_ia32_pause();
            lk.lock();
            if (rq.done || rq.poke.load(std::memory_order_relaxed)) continue;
        }
        rq.cv.wait(lk);
    }
    return rq.rc;
}

// Host-API batches hold the index lock only to ship pending patches, pick up
// the index's current device view and queue the kernels on the caller's lane;
// they wait for the GPU and copy results out without it, so concurrent callers
// overlap on the device (each lane is its own stream) and deltas keep flowing.
// tm_match_batch_ex, or (to32v) the same over u32 offsets that lie in
// TM_ALLOC_VRAM memory with their bytes (tm_match_batch32_ex's batches the
// one-launch path does not take): widened on the device, never read by the host
static int match_batch_impl(tm_index *ix, uint64_t n, const uint8_t *tb, const uint64_t *to, const uint32_t *to32v,
                            uint64_t *out_hit, uint32_t *out_vals, uint64_t cap, uint8_t *out_err, uint32_t order,
                            uint32_t *out_unique) {
    static const bool timing = getenv("TM_HOST_TIMING") != nullptr;
    double tt[8]; int nt = 0;
    if (timing) tt[nt++] = now_us();
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch: batch too large");
    if (order > TM_ORDER_UNIQUE) return fail(ix, TM_EINVAL, "tm_match_batch: bad order");
    const bool sorted = order != TM_ORDER_TRAVERSAL, unique = order == TM_ORDER_UNIQUE;
    std::unique_lock<std::mutex> g(ix->mu);
    LaneLease lease{ix, g};
    int rc;
    if ((rc = host_lane(ix, g, lease.ln))) return rc;
    Lane &ln = *lease.ln;
    const hipStream_t s = ln.s;
    if ((rc = sync_locked(ix, ln.r, s))) return rc;
    if ((rc = ensure_ws(ix, n, ln))) return rc;
    ix->rep[ln.r].batches++;
    if (timing) tt[nt++] = now_us();
    if (n && n <= ZC_TOPICS && !to32v) {
        // every buffer from tm_host_alloc: the kernels read the topics and
        // write the hit lists in place (no staging copy in, no copy out)
        const uint64_t nbytes = to[n];
        uint8_t *db = nbytes ? pinned_dev(ix, tb, nbytes) : nullptr;
        uint8_t *dof = pinned_dev(ix, to, (n + 1) * 8);
        uint8_t *dh = pinned_dev(ix, out_hit, (n + 1) * 8);
        uint8_t *dv = out_vals ? pinned_dev(ix, out_vals, cap * 4) : nullptr;
        uint8_t *de = out_err ? pinned_dev(ix, out_err, n) : nullptr;
        uint8_t *du = out_unique ? pinned_dev(ix, out_unique, n * 4) : nullptr;
        const bool aligned = ((uintptr_t)tb & 15) == 0;
        if ((db || !nbytes) && aligned && dof && dh && (dv || !out_vals) && (de || !out_err) && (du || !out_unique)) {
            if (!de) {   // flags nobody reads still need a home
                if ((rc = stage_out(ix, ln, n, n, de))) return rc;
            }
            const uint8_t *dbytes = db ? db : dof;   // no bytes: any valid address
            uint64_t *dhit = reinterpret_cast<uint64_t *>(dh);
            uint32_t *vdst = reinterpret_cast<uint32_t *>(dv);
            if (sorted && dv) {   // sorted in HBM, then copied into the caller's buffer
                if ((rc = grow_dev(ix, s, ln.d_vals, ln.d_vals_cap, cap))) return rc;
                vdst = ln.d_vals;
            }
            for (int tries = 0;; tries++) {
                const DevIndex d = dev_view(ix, ln.r);
                uint32_t tag;
                if (int rc = next_tag(ix, ln, s, tag)) return rc;
                int path = PATH_PHASES;
                HIPCHK(ix, launch_match(d, ln.w, n, dbytes, reinterpret_cast<const uint64_t *>(dof), dhit, de, vdst,
                                        dv ? cap : 0, tag, next_lb(ix), ix->dbg_phases, ix->small_kind, s, nullptr,
                                        nullptr, &path));
                ix->path_batches[path]++;
                if (sorted && dv) {
                    HIPCHK(ix, launch_sort_segments(ln.w, n, dhit, vdst, cap, unique, reinterpret_cast<uint32_t *>(du), s));
                    HIPCHK(ix, launch_copy_values(dhit, n, vdst, reinterpret_cast<uint32_t *>(dv), cap, s));
                }
                if ((rc = batch_done(ix, ln))) return rc;
                g.unlock();
                if (timing) tt[nt++] = now_us();
                HIPCHK(ix, hipStreamSynchronize(s));
                if (!batch_failed(ix, ln)) break;
                if ((rc = retry_or_fail(ix, g, ln, tries))) return rc;
                if (timing) nt = 1;
            }
            if (timing) {
                tt[nt++] = now_us();
                fprintf(stderr, "tm_match_batch n=%lu (in place): sync %.1f launch %.1f wait %.1f us\n",
                        (unsigned long)n, tt[1] - tt[0], tt[2] - tt[1], tt[3] - tt[2]);
            }
            return (out_vals && out_hit[n] > cap) ? TM_ECAP : TM_OK;
        }
    }
    const uint8_t *dbytes;
    const uint64_t *doffs;
    if ((rc = stage_in(ix, ln, n, tb, to, to32v, dbytes, doffs))) return rc;
    if (timing) tt[nt++] = now_us();
    // results: hit offsets (n + 1) x u64, then the badarg flags (then the
    // distinct counts, u32, for UNIQUE); the values are written by k_emit
    // straight into mapped pinned memory (sorted orders: sorted in HBM, then
    // copied there), so the batch costs one host synchronisation (a second
    // one only when that buffer must grow)
    const uint64_t uoff = ((n + 1) * 8 + n + 3) & ~3ull;
    const uint64_t rbytes = (sorted && out_unique) ? uoff + 4 * n : (n + 1) * 8 + n;
    uint8_t *dres;
    if ((rc = stage_out(ix, ln, n, rbytes, dres))) return rc;
    uint64_t *dhit = reinterpret_cast<uint64_t *>(dres);
    uint8_t *derr = dres + (n + 1) * 8;
    uint32_t *dunq = (sorted && out_unique) ? reinterpret_cast<uint32_t *>(dres + uoff) : nullptr;
    uint64_t total = 0;
    for (int attempt = 0, tries = 0; attempt < 3; attempt++) {
        if (!ln.pin_vals) {
            ln.pin_vals_cap = std::max<uint64_t>(ln.pin_vals_cap, 1 << 16);
            HIPCHK(ix, hipHostMalloc(&ln.pin_vals, ln.pin_vals_cap * 4, hipHostMallocMapped));
            HIPCHK(ix, hipHostGetDevicePointer(reinterpret_cast<void **>(&ln.pin_vals_dev), ln.pin_vals, 0));
        }
        uint32_t *vdst = ln.pin_vals_dev;
        if (sorted && (rc = grow_dev(ix, s, ln.d_vals, ln.d_vals_cap, ln.pin_vals_cap))) return rc;
        if (sorted) vdst = ln.d_vals;
        const DevIndex d = dev_view(ix, ln.r);
        uint32_t tag;
        if (int rc = next_tag(ix, ln, s, tag)) return rc;
        int path = PATH_PHASES;
        HIPCHK(ix, launch_match(d, ln.w, n, dbytes, doffs, dhit, derr, vdst, ln.pin_vals_cap, tag, next_lb(ix),
                                ix->dbg_phases, ix->small_kind, s, nullptr, nullptr, &path));
        ix->path_batches[path]++;
        if (sorted) {
            HIPCHK(ix, launch_sort_segments(ln.w, n, dhit, vdst, ln.pin_vals_cap, unique, dunq, s));
            HIPCHK(ix, launch_copy_values(dhit, n, vdst, ln.pin_vals_dev, ln.pin_vals_cap, s));
        }
        if ((rc = fetch_out(ix, ln, n, rbytes))) return rc;
        if ((rc = batch_done(ix, ln))) return rc;
        g.unlock();
        if (timing && nt < 5) tt[nt++] = now_us();
        HIPCHK(ix, hipStreamSynchronize(s));
        if (timing && nt < 6) tt[nt++] = now_us();
        if (batch_failed(ix, ln)) {   // the look-back failed: run the batch again, once
            if ((rc = retry_or_fail(ix, g, ln, tries++))) return rc;
            attempt--;
            continue;
        }
        memcpy(&total, ln.pin_out + n * 8, 8);
        if (total <= ln.pin_vals_cap || !out_vals || total <= 0) break;
        if (attempt == 2) return fail(ix, TM_EDEVICE, "tm_match_batch: hit total kept growing past the staging buffer");
        // grow the mapped buffer and run the batch again (rare: sizes are sticky)
        g.lock();
        HIPCHK(ix, hipHostFree(ln.pin_vals));
        ln.pin_vals = nullptr;
        ln.pin_vals_cap = total + total / 4;
        HIPCHK(ix, hipSetDevice(ix->rep[ln.r].device));
        if ((rc = sync_locked(ix, ln.r, s))) return rc;
        if ((rc = ensure_ws(ix, n, ln))) return rc;
    }
    memcpy(out_hit, ln.pin_out, (n + 1) * 8);
    if (out_err && n) memcpy(out_err, ln.pin_out + (n + 1) * 8, n);
    if (dunq && n) memcpy(out_unique, ln.pin_out + uoff, 4 * n);
    const uint64_t keep = std::min(total, out_vals ? cap : 0);
    if (keep) memcpy(out_vals, ln.pin_vals, keep * 4);
    if (timing) {
        tt[nt++] = now_us();
        fprintf(stderr, "tm_match_batch n=%lu: sync %.1f stage %.1f launch %.1f wait %.1f copy-out %.1f us\n",
                (unsigned long)n, tt[1] - tt[0], tt[2] - tt[1], tt[3] - tt[2], tt[4] - tt[3], tt[nt - 1] - tt[4]);
    }
    return (out_vals && total > cap) ? TM_ECAP : TM_OK;
}

int tm_match_batch_ex(tm_index *ix, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t *out_hit,
                      uint32_t *out_vals, uint64_t cap, uint8_t *out_err, uint32_t order, uint32_t *out_unique) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch: null handle");
    if (!to || !out_hit || (n && !tb && to[n] != to[0])) return fail(ix, TM_EINVAL, "tm_match_batch: null buffer");
    return match_batch_impl(ix, n, tb, to, nullptr, out_hit, out_vals, cap, out_err, order, out_unique);
}

int tm_match_batch(tm_index *ix, uint64_t n, const uint8_t *tb, const uint64_t *to, uint64_t *out_hit,
                   uint32_t *out_vals, uint64_t cap, uint8_t *out_err) {
    return tm_match_batch_ex(ix, n, tb, to, out_hit, out_vals, cap, out_err, TM_ORDER_TRAVERSAL, nullptr);
}

// 32-bit offsets (include/tmatch.h).  An in-place batch the one-launch small
// kernel takes runs on 32-bit offsets end to end (k_walk_small<.., uint32_t>):
// half the offset bytes cross PCIe in each direction.  Any other batch is
// widened on the host, matched as tm_match_batch_ex, and narrowed.
int tm_match_batch32_ex(tm_index *ix, uint64_t n, const uint8_t *tb, const uint32_t *to, uint32_t *out_hit,
                        uint32_t *out_vals, uint64_t cap, uint8_t *out_err, uint32_t order, uint32_t *out_unique) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch32: null handle");
    if (!to || !out_hit || (n && !tb && to[n] != to[0])) return fail(ix, TM_EINVAL, "tm_match_batch32: null buffer");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch32: batch too large");
    if (order > TM_ORDER_UNIQUE) return fail(ix, TM_EINVAL, "tm_match_batch32: bad order");
    if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;   // (a 32-bit offset addresses no more)
    if (n && n <= ZC_TOPICS && order == TM_ORDER_TRAVERSAL && ((uintptr_t)tb & 15) == 0) {
        const uint64_t nbytes = to[n];   // (before the lock: in TM_ALLOC_VRAM memory a host read is a PCIe round trip)
        std::unique_lock<std::mutex> g(ix->mu);
        uint8_t *db = nbytes ? pinned_dev(ix, tb, nbytes) : nullptr;
        uint8_t *dof = pinned_dev(ix, to, (n + 1) * 4);
        uint8_t *dh = pinned_dev(ix, out_hit, (n + 1) * 4);
        uint8_t *dv = out_vals ? pinned_dev(ix, out_vals, cap * 4) : nullptr;
        uint8_t *de = out_err ? pinned_dev(ix, out_err, n) : nullptr;
        if ((db || !nbytes) && dof && dh && (dv || !out_vals) && (de || !out_err)) {
            if (ix->cmb_leaders > 0 && de) {   // through the combiner (the flags have a home)
                g.unlock();
                SmallReq rq;
                rq.n = n; rq.db = db; rq.dof = dof; rq.dh = dh; rq.de = de; rq.dv = dv; rq.cap = dv ? cap : 0;
                const int rc = small_combined(ix, rq);
                if (rc != CMB_LEGACY) {
                    if (rc) return rc;
                    return (out_vals && out_hit[n] > cap) ? TM_ECAP : TM_OK;
                }
                g.lock();
            }
            LaneLease lease{ix, g};
            int rc;
            if ((rc = host_lane(ix, g, lease.ln))) return rc;
            Lane &ln = *lease.ln;
            const hipStream_t s = ln.s;
            if ((rc = sync_locked(ix, ln.r, s))) return rc;
            if ((rc = ensure_ws(ix, n, ln))) return rc;
            if (small_path_ok(dev_view(ix, ln.r), n)) {
                ix->rep[ln.r].batches++;
                if (!de && (rc = stage_out(ix, ln, n, n, de))) return rc;   // flags nobody reads still need a home
                for (int tries = 0;; tries++) {
                    const DevIndex d = dev_view(ix, ln.r);
                    uint32_t tag;
                    if ((rc = next_tag(ix, ln, s, tag))) return rc;
                    int path = PATH_SMALL;
                    HIPCHK(ix, launch_match32(d, ln.w, n, db ? db : dof, reinterpret_cast<const uint32_t *>(dof),
                                              reinterpret_cast<uint32_t *>(dh), de, reinterpret_cast<uint32_t *>(dv),
                                              dv ? cap : 0, tag, next_lb(ix), ix->small_kind, s, &path));
                    ix->path_batches[path]++;
                    if ((rc = batch_done(ix, ln))) return rc;
                    g.unlock();
                    HIPCHK(ix, hipStreamSynchronize(s));
                    if (!batch_failed(ix, ln)) break;
                    if ((rc = retry_or_fail(ix, g, ln, tries))) return rc;
                }
                return (out_vals && out_hit[n] > cap) ? TM_ECAP : TM_OK;
            }
        }
    }
    // widened: the 64-bit path, then the offsets narrowed.  Offsets in
    // TM_ALLOC_VRAM memory are widened on the device (the host never reads
    // them: ADVICE r5 -- a deep index, > 65536 topics or a sorted order took
    // this path and read the NIF's device buffers back over the BAR)
    bool voffs;
    {
        std::lock_guard<std::mutex> g(ix->mu);
        voffs = vram_buf(ix, to, (n + 1) * 4) != nullptr;
    }
    std::vector<uint64_t> o64, h64;
    try {
        if (!voffs) o64.assign(to, to + n + 1);
        h64.resize(n + 1);
    } catch (const std::bad_alloc &) {
        return fail(ix, TM_ENOMEM, "tm_match_batch32: out of host memory");
    }
    const int rc = voffs ? match_batch_impl(ix, n, tb, nullptr, to, h64.data(), out_vals, cap, out_err, order, out_unique)
                         : tm_match_batch_ex(ix, n, tb, o64.data(), h64.data(), out_vals, cap, out_err, order, out_unique);
    if (rc != TM_OK && rc != TM_ECAP) return rc;
    if (h64[n] > 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch32: more than 2^32 - 1 values");
    for (uint64_t i = 0; i <= n; i++) out_hit[i] = (uint32_t)h64[i];
    return rc;
}

// (offset, count) pairs (include/tmatch.h): an in-place batch the one-launch
// kernel takes runs through the combiner as a pairs launch -- no look-back,
// so no block waits for another; any other batch takes the CSR path and is
// converted on the host.
int tm_match_batch32_pairs(tm_index *ix, uint64_t n, const uint8_t *tb, const uint32_t *to, uint32_t *out_pairs,
                           uint32_t *out_vals, uint64_t cap, uint8_t *out_err) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch32_pairs: null handle");
    if (!to || !out_pairs || !out_err || (n && !tb && to[n] != to[0]))
        return fail(ix, TM_EINVAL, "tm_match_batch32_pairs: null buffer");
    if (n >= 0x7FFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch32_pairs: batch too large");
    if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;
    if (!n) { out_pairs[0] = 0; return TM_OK; }
    if (n <= ZC_TOPICS && ((uintptr_t)tb & 15) == 0) {
        const uint64_t nbytes = to[n];   // (before the lock: in TM_ALLOC_VRAM memory a host read is a PCIe round trip)
        SmallReq rq;
        {
            std::lock_guard<std::mutex> g(ix->mu);
            rq.db = nbytes ? pinned_dev(ix, tb, nbytes) : nullptr;
            rq.dof = pinned_dev(ix, to, (n + 1) * 4);
            rq.dh = pinned_dev(ix, out_pairs, (2 * n + 1) * 4);
            rq.dv = out_vals ? pinned_dev(ix, out_vals, cap * 4) : nullptr;
            rq.de = pinned_dev(ix, out_err, n);
        }
        if ((rq.db || !nbytes) && rq.dof && rq.dh && (rq.dv || !out_vals) && rq.de) {
            rq.n = n; rq.cap = rq.dv ? cap : 0; rq.pairs = true;
            uint64_t t_end = 0;   // (TM_DEBUG_COMBINE 0: every batch its own launch)
            const int rc = ix->cmb_leaders.load() > 0 ? small_combined(ix, rq)
                                                      : run_small_group(ix, std::vector<SmallReq *>{&rq}, &t_end);
            if (rc != CMB_LEGACY) {
                if (rc) return rc;
                return (out_vals && out_pairs[2 * n] > cap) ? TM_ECAP : TM_OK;
            }
        }
    }
    std::vector<uint32_t> h;
    try {
        h.resize(n + 1);
    } catch (const std::bad_alloc &) {
        return fail(ix, TM_ENOMEM, "tm_match_batch32_pairs: out of host memory");
    }
    const int rc = tm_match_batch32_ex(ix, n, tb, to, h.data(), out_vals, cap, out_err, TM_ORDER_TRAVERSAL, nullptr);
    if (rc != TM_OK && rc != TM_ECAP) return rc;
    for (uint64_t i = 0; i < n; i++) { out_pairs[2 * i] = h[i]; out_pairs[2 * i + 1] = h[i + 1] - h[i]; }
    out_pairs[2 * n] = h[n];
    return rc;
}

int tm_match_batch32_dev(tm_index *ix, uint64_t n, const uint8_t *bytes, const uint32_t *offs, uint32_t *hit_offs,
                         uint32_t *out, uint64_t cap, uint8_t *err, void *stream) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_match_batch32_dev: null handle");
    if (!hit_offs || (n && (!offs || !bytes || !err))) return fail(ix, TM_EINVAL, "tm_match_batch32_dev: null buffer");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_match_batch32_dev: batch too large");
    if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;
    std::lock_guard<std::mutex> g(ix->mu);
    hipStream_t s = pick_stream(ix, stream);
    int rc, grp = 0;
    Lane *ln;
    if ((rc = dev_group(ix, grp))) return rc;
    if ((rc = collect_patch(ix))) return rc;
    const int r = pick_copy(ix, grp, nullptr, s, true);
    ix->rep[r].last_use = ++ix->tick;
    ix->rep[r].batches++;
    if ((rc = dev_lane(ix, s, r, ln))) return rc;
    if ((rc = sync_locked(ix, ln->r, s))) return rc;
    if ((rc = ensure_ws(ix, n, *ln))) return rc;
    const DevIndex d = dev_view(ix, ln->r);
    tm_index::ProfEv ev;
    if ((rc = prof_begin(ix, ev, s))) return rc;
    uint32_t tag;
    if ((rc = next_tag(ix, *ln, s, tag))) return rc;
    if (small_path_ok(d, n)) {
        if (ev.w0) HIPCHK(ix, hipEventRecord(ev.w0, s));
        int path = PATH_SMALL;
        HIPCHK(ix, launch_match32(d, ln->w, n, bytes, offs, hit_offs, err, out, out ? cap : 0, tag, next_lb(ix),
                                  ix->small_kind, s, &path));
        if (ev.w1) HIPCHK(ix, hipEventRecord(ev.w1, s));
        ix->path_batches[path]++;
    } else {
        // widened into the lane's scratch, matched, narrowed into the caller's offsets
        if ((rc = grow_dev(ix, s, ln->d_o64, ln->d_o64_cap, n + 1))) return rc;
        if ((rc = grow_dev(ix, s, ln->d_h64, ln->d_h64_cap, n + 1))) return rc;
        HIPCHK(ix, launch_offs_widen(offs, ln->d_o64, n + 1, s));
        int path = PATH_PHASES;
        HIPCHK(ix, launch_match(d, ln->w, n, bytes, ln->d_o64, ln->d_h64, err, out, out ? cap : 0, tag, next_lb(ix),
                                ix->dbg_phases, ix->small_kind, s, ev.w0, ev.w1, &path));
        ix->path_batches[path]++;
        HIPCHK(ix, launch_offs_narrow(ln->d_h64, hit_offs, n + 1, s));
    }
    if ((rc = batch_done(ix, *ln))) return rc;
    return prof_end(ix, ev, s);
}

int tm_first_batch(tm_index *ix, uint64_t n, const uint8_t *tb, const uint64_t *to, uint32_t *out_value,
                   uint8_t *out_found) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_first_batch: null handle");
    if (!to || !out_value || !out_found || (n && !tb && to[n] != to[0]))
        return fail(ix, TM_EINVAL, "tm_first_batch: null buffer");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_first_batch: batch too large");
    std::unique_lock<std::mutex> g(ix->mu);
    LaneLease lease{ix, g};
    int rc;
    if ((rc = host_lane(ix, g, lease.ln))) return rc;
    Lane &ln = *lease.ln;
    const hipStream_t s = ln.s;
    if ((rc = sync_locked(ix, ln.r, s))) return rc;
    if ((rc = ensure_ws(ix, n, ln))) return rc;
    ix->rep[ln.r].batches++;
    if (n && n <= ZC_TOPICS) {   // tm_host_alloc buffers: in place, as tm_match_batch
        const uint64_t nbytes = to[n];
        uint8_t *db = nbytes ? pinned_dev(ix, tb, nbytes) : nullptr;
        uint8_t *dof = pinned_dev(ix, to, (n + 1) * 8);
        uint8_t *dv = pinned_dev(ix, out_value, n * 4), *df = pinned_dev(ix, out_found, n);
        if ((db || !nbytes) && ((uintptr_t)tb & 15) == 0 && dof && dv && df) {
            HIPCHK(ix, launch_first(dev_view(ix, ln.r), ln.w, n, db ? db : dof, reinterpret_cast<const uint64_t *>(dof),
                                    reinterpret_cast<uint32_t *>(dv), df, s));
            if ((rc = batch_done(ix, ln))) return rc;
            g.unlock();
            HIPCHK(ix, hipStreamSynchronize(s));
            return TM_OK;
        }
    }
    const uint8_t *dbytes;
    const uint64_t *doffs;
    if ((rc = stage_in(ix, ln, n, tb, to, nullptr, dbytes, doffs))) return rc;
    const uint64_t rbytes = n * 5;   // first value u32 per topic, then the found flags
    uint8_t *dres;
    if ((rc = stage_out(ix, ln, n, rbytes, dres))) return rc;
    HIPCHK(ix, launch_first(dev_view(ix, ln.r), ln.w, n, dbytes, doffs, reinterpret_cast<uint32_t *>(dres), dres + n * 4, s));
    if ((rc = fetch_out(ix, ln, n, rbytes))) return rc;
    if ((rc = batch_done(ix, ln))) return rc;
    g.unlock();
    HIPCHK(ix, hipStreamSynchronize(s));
    if (n) {
        memcpy(out_value, ln.pin_out, n * 4);
        memcpy(out_found, ln.pin_out + n * 4, n);
    }
    return TM_OK;
}

int tm_merge_shards(uint32_t world, uint64_t n, const uint64_t *shard_hit, const uint32_t *shard_vals,
                    uint64_t stride, uint64_t *out_hit, uint32_t *out, uint64_t cap, void *stream) {
    if (!world || !shard_hit || !out_hit || (cap && !out) || (n && !shard_vals))
        return fail(nullptr, TM_EINVAL, "tm_merge_shards: bad argument");
    hipError_t e = launch_merge_shards(world, n, shard_hit, shard_vals, stride, out_hit, out, cap,
                                       reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return fail(nullptr, TM_EDEVICE, std::string("tm_merge_shards: ") + hipGetErrorString(e));
    return TM_OK;
}

int tm_profile_enable(tm_index *ix, int enable) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_profile_enable: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    ix->prof = enable != 0;
    return TM_OK;
}

int tm_profile_read(tm_index *ix, double *walk_ms, double *batch_ms, uint64_t *batches, int reset) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_profile_read: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    for (auto &ev : ix->prof_pending) {
        HIPCHK(ix, hipEventSynchronize(ev.b1));
        float w = 0, b = 0;
        if (ev.w0) { HIPCHK(ix, hipEventElapsedTime(&w, ev.w0, ev.w1)); }
        HIPCHK(ix, hipEventElapsedTime(&b, ev.b0, ev.b1));
        ix->prof_walk_ms += w; ix->prof_batch_ms += b; ix->prof_batches++;
        ix->prof_free.push_back(ev);
    }
    ix->prof_pending.clear();
    if (walk_ms) *walk_ms = ix->prof_walk_ms;
    if (batch_ms) *batch_ms = ix->prof_batch_ms;
    if (batches) *batches = ix->prof_batches;
    if (reset) { ix->prof_walk_ms = ix->prof_batch_ms = 0; ix->prof_batches = 0; }
    return TM_OK;
}

int tm_debug_set(tm_index *ix, uint32_t key, uint64_t value) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_debug_set: null handle");
    std::lock_guard<std::mutex> g(ix->mu);
    switch (key) {
    case TM_DEBUG_LB_SPINS: ix->dbg_lb.spins = value > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)value; break;
    case TM_DEBUG_LB_FAIL_BLOCK: ix->dbg_lb.fail_block = value > 0xFFFFFFFFull ? NONE : (uint32_t)value; break;
    case TM_DEBUG_LB_LAUNCHES: ix->dbg_lb_launches = value; break;
    case TM_DEBUG_PHASES: ix->dbg_phases = value != 0; break;
    case TM_DEBUG_COMBINE: ix->cmb_leaders = value > 16 ? 16 : (int)value; break;
    case TM_DEBUG_CMB_GATHER: ix->cmb_gather_us = value > 1000 ? 1000 : (int)value; break;
    case TM_DEBUG_CMB_LAND: if (value) return fail(ix, TM_EINVAL, "tm_debug_set: TM_DEBUG_CMB_LAND was removed"); break;
    case TM_DEBUG_CMB_SPIN: ix->cmb_spin_us = value > 1000 ? 1000 : (int)value; break;
    case TM_DEBUG_SMALL_TICKET: ix->small_ticket = value != 0; break;
    case TM_DEBUG_PATCH_ZC: ix->patch_zc = value != 0; break;
    case TM_DEBUG_SMALL_KERNEL:
        if (value != SMALL_AUTO && value != SMALL_WAVE && value != SMALL_WAVE8)
            return fail(ix, TM_EINVAL, "tm_debug_set: TM_DEBUG_SMALL_KERNEL is 0, 1 or 3 (2, the lane kernel, was removed)");
        ix->small_kind = (int)value;
        break;
    default: return fail(ix, TM_EINVAL, "tm_debug_set: unknown key");
    }
    return TM_OK;
}

int tm_debug_get(tm_index *ix, uint32_t key, uint64_t *value) {
    if (!ix || !value) return fail(ix, TM_EINVAL, "tm_debug_get: null argument");
    switch (key) {
    case TM_DEBUG_FAILED_BATCHES: *value = ix->failed_batches.load(); break;
    case TM_DEBUG_RETRIED_BATCHES: *value = ix->retried_batches.load(); break;
    case TM_DEBUG_PATH_PHASES: *value = ix->path_batches[PATH_PHASES].load(); break;
    case TM_DEBUG_PATH_SMALL: *value = ix->path_batches[PATH_SMALL].load(); break;
    case TM_DEBUG_PATH_LANE: *value = ix->path_batches[PATH_LANE].load(); break;
    case TM_DEBUG_COMBINE: *value = (uint64_t)ix->cmb_leaders.load(); break;
    case TM_DEBUG_CMB_GATHER: *value = (uint64_t)ix->cmb_gather_us.load(); break;
    case TM_DEBUG_CMB_LAND: *value = 0; break;
    case TM_DEBUG_CMB_SPIN: *value = (uint64_t)ix->cmb_spin_us.load(); break;
    case TM_DEBUG_COMMITS: *value = ix->commits.load(); break;
    case TM_DEBUG_SMALL_TICKET: *value = ix->small_ticket; break;
    case TM_DEBUG_PATCH_ZC: *value = ix->patch_zc; break;
    case TM_DEBUG_COMMIT_WAITS: *value = ix->commit_waits.load(); break;
    case TM_DEBUG_COMMIT_FORCED: *value = ix->commit_forced.load(); break;
    case TM_DEBUG_COMBINED_LAUNCHES: *value = ix->cmb_launches.load(); break;
    case TM_DEBUG_COMBINED_BATCHES: *value = ix->cmb_batches.load(); break;
    case TM_DEBUG_WIDE_NODES:
    case TM_DEBUG_DENSE_WIDE: {   // wide nodes / those of them that probe their table without the bitmap
        std::lock_guard<std::mutex> g(ix->img);
        uint64_t v = 0;
        for (uint32_t node : ix->wide) v += key == TM_DEBUG_WIDE_NODES || ix->nodes.h[node].kw[2] == NONE;
        *value = v;
        break;
    }
    default: return fail(ix, TM_EINVAL, "tm_debug_get: unknown key");
    }
    return TM_OK;
}

// ------------------------------------------------------- matches_filter/3

}  // extern "C"

namespace {

void mf_words_of(const uint8_t *p, uint32_t n, std::vector<std::string> &out) {
    out.clear();
    uint32_t s0 = 0;
    for (uint32_t i = 0; i <= n; i++)
        if (i == n || p[i] == '/') { out.emplace_back(reinterpret_cast<const char *>(p) + s0, i - s0); s0 = i + 1; }
}

// rank of a word: '#' 0, '+' 1, a binary word 3 + 2 i if it is words[i], else
// 2 + 2 i (i = the words before it): term order (atoms < binaries, bytes)
uint32_t mf_rank(const std::vector<std::string> &words, const std::string &w, bool wild) {
    if (wild) return w == "#" ? 0 : 1;
    const auto it = std::lower_bound(words.begin(), words.end(), w);
    const uint32_t i = (uint32_t)(it - words.begin());
    return it != words.end() && *it == w ? 3 + 2 * i : 2 + 2 * i;
}

// the words of a key (or query) in bytes + flags form: escaped word lists
// decoded, else split on '/' with bare "+" / "#" the wildcards
void mf_key_words(const uint8_t *p, uint32_t n, uint8_t flags, std::vector<std::pair<std::string, bool>> &out) {
    if (flags & TM_KEY_ESCAPED) { esc_words(p, n, out); return; }
    std::vector<std::string> ws;
    mf_words_of(p, n, ws);
    out.clear();
    for (auto &x : ws) out.emplace_back(x, x == "+" || x == "#");
}

void mf_free_keys(tm_index::MfState &m) {
    for (void *p : {(void *)m.pool, (void *)m.koff, (void *)m.val}) if (p) (void)hipFree(p);
    m.pool = nullptr; m.koff = nullptr; m.val = nullptr; m.K = 0; m.pcap = m.kcap = m.vcap = 0;
}

// the filter of trie node `node` (words joined by '/'), for the snapshot
void mf_path(tm_index *ix, uint32_t node, std::string &out) {
    std::vector<uint32_t> up;
    for (uint32_t x = node; x != ROOT; x = ix->aux[x].parent) up.push_back(x);
    out.clear();
    std::string w;
    for (size_t i = up.size(); i-- > 0;) {
        const NodeAux &a = ix->aux[up[i]];
        if (a.is_plus) w = "+";
        else vocab_bytes(ix, ix->vocab.h[ix->wslot[a.wid]], w);
        if (i + 1 != up.size()) out.push_back('/');
        out += w;
    }
}

// Fuzzy snapshot of the word-list keys (caller holds m.mu, not ix->mu): the
// log starts first, then the trie's nodes are read in slices under the image
// lock (ix->img), each ending after MF_SLICE_US (checked every 64 nodes); replaying the
// log afterwards makes the copy exact (a key untouched since the log started
// sits on a node that cannot move, so a slice sees it; any other key ends as
// its last logged op leaves it).
constexpr double MF_SLICE_US = 100.0;

void mf_snapshot(tm_index *ix) {
    auto &m = ix->mf;
    m.keys.clear();
    {
        std::lock_guard<std::mutex> g(ix->img);
        m.log.clear();
        m.log_on = true;
        m.log_lost = false;
        for (const std::string &k : ix->dead) m.keys.insert(k);
    }
    std::string path, key;
    for (uint64_t cur = 0;;) {
        std::lock_guard<std::mutex> g(ix->img);
        const auto t0 = std::chrono::steady_clock::now();
        uint64_t end = ix->nodes.h.size(), x = cur;
        for (; x < end; x++) {
            if ((x & 63) == 63 &&
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > MF_SLICE_US) {
                end = x;
                break;
            }
            const Node &n = ix->nodes.h[x];
            if (!(n.exact_cnt & RUN_CNT) && !(n.hash_cnt & RUN_CNT)) continue;
            mf_path(ix, (uint32_t)x, path);
            const NodeAux &a = ix->aux[x];
            auto add = [&](uint32_t roff, uint32_t cnt, bool hash) {
                for (uint32_t i = 0; i < cnt; i++) {
                    const uint32_t v = ix->vals.h[roff + i];
                    // (the root has no words; a node whose path is one empty word has path "")
                    std::string f = hash ? (x == ROOT ? std::string("#") : path + "/#") : path;
                    m.keys.insert(dead_key(reinterpret_cast<const uint8_t *>(f.data()), (uint32_t)f.size(), v,
                                           TM_KEY_WORDS));
                }
            };
            add(a.exact_roff, n.exact_cnt & RUN_CNT, false);
            add(a.hash_roff, n.hash_cnt & RUN_CNT, true);
        }
        m.slices++;
        cur = end;
        if (cur >= ix->nodes.h.size()) break;
    }
    m.snapshots++;
    m.have_keys = true;
}

// the device's term-ordered key arrays from m.keys (caller holds m.mu only)
int mf_upload(tm_index *ix) {
    auto &m = ix->mf;
    std::vector<std::pair<std::string, bool>> dw;
    std::vector<std::string> sorted;
    std::unordered_set<std::string> distinct;
    for (const std::string &k : m.keys) {
        if ((uint8_t)k[0] & TM_KEY_EMPTY_LIST) continue;
        mf_key_words(reinterpret_cast<const uint8_t *>(k.data()) + 5, (uint32_t)k.size() - 5, (uint8_t)k[0], dw);
        for (auto &x : dw) if (!x.second) distinct.insert(x.first);
    }
    sorted.assign(distinct.begin(), distinct.end());
    std::sort(sorted.begin(), sorted.end());
    std::vector<uint32_t> pool;
    struct K { uint64_t off; uint32_t len, val; };
    std::vector<K> keys;
    keys.reserve(m.keys.size());
    for (const std::string &k : m.keys) {
        uint32_t v;
        memcpy(&v, k.data() + 1, 4);
        const uint64_t off = pool.size();
        if (!((uint8_t)k[0] & TM_KEY_EMPTY_LIST)) {
            mf_key_words(reinterpret_cast<const uint8_t *>(k.data()) + 5, (uint32_t)k.size() - 5, (uint8_t)k[0], dw);
            for (auto &x : dw) pool.push_back(mf_rank(sorted, x.first, x.second));
        }
        keys.push_back(K{off, (uint32_t)(pool.size() - off), v});
    }
    std::sort(keys.begin(), keys.end(), [&](const K &x, const K &y) {
        const uint32_t m2 = std::min(x.len, y.len);
        for (uint32_t i = 0; i < m2; i++)
            if (pool[x.off + i] != pool[y.off + i]) return pool[x.off + i] < pool[y.off + i];
        if (x.len != y.len) return x.len < y.len;
        return x.val < y.val;
    });
    std::vector<uint32_t> spool;
    spool.reserve(pool.size());
    std::vector<uint64_t> koff(keys.size() + 1, 0);
    std::vector<uint32_t> kval(keys.size());
    for (size_t i = 0; i < keys.size(); i++) {
        koff[i] = spool.size();
        spool.insert(spool.end(), pool.begin() + keys[i].off, pool.begin() + keys[i].off + keys[i].len);
        kval[i] = keys[i].val;
    }
    koff[keys.size()] = spool.size();
    // grow-only device arrays (a free would wait for the device), async copies on the mf stream
    auto grow = [&](auto *&p, uint64_t &cap, uint64_t need, size_t elt) -> int {
        if (need <= cap && p) return TM_OK;
        if (p) { HIPCHK(ix, hipStreamSynchronize(m.s)); HIPCHK(ix, hipFree(p)); }
        p = nullptr;
        cap = need + need / 4 + 1024;
        HIPCHK(ix, hipMalloc(reinterpret_cast<void **>(&p), cap * elt));
        return TM_OK;
    };
    int rc;
    if ((rc = grow(m.pool, m.pcap, spool.size(), 4))) return rc;
    if ((rc = grow(m.koff, m.kcap, koff.size(), 8))) return rc;
    if ((rc = grow(m.val, m.vcap, kval.size(), 4))) return rc;
    if (!spool.empty()) HIPCHK(ix, hipMemcpyAsync(m.pool, spool.data(), spool.size() * 4, hipMemcpyHostToDevice, m.s));
    HIPCHK(ix, hipMemcpyAsync(m.koff, koff.data(), koff.size() * 8, hipMemcpyHostToDevice, m.s));
    if (!kval.empty()) HIPCHK(ix, hipMemcpyAsync(m.val, kval.data(), kval.size() * 4, hipMemcpyHostToDevice, m.s));
    HIPCHK(ix, hipStreamSynchronize(m.s));   // the host vectors die here
    m.K = keys.size();
    m.words.swap(sorted);
    m.dev_stale = false;
    return TM_OK;
}

// bring m.keys up to date: a new snapshot when there is none (or its log was
// dropped), else the logged ops since the last call -- the index lock is
// held only to swap the log out
int mf_refresh(tm_index *ix) {
    auto &m = ix->mf;
    std::vector<std::pair<bool, std::string>> log;
    bool lost;
    {
        std::lock_guard<std::mutex> g(ix->img);
        lost = m.log_lost || !m.log_on;
        if (!lost) log.swap(m.log);
    }
    if (lost || !m.have_keys) {
        mf_snapshot(ix);
        std::lock_guard<std::mutex> g(ix->img);
        log.swap(m.log);
        m.dev_stale = true;
    }
    for (auto &op : log) {
        if (op.first) m.keys.insert(op.second); else m.keys.erase(op.second);
    }
    if (!log.empty()) m.dev_stale = true;
    m.nkeys.store(m.keys.size(), std::memory_order_relaxed);
    return m.dev_stale ? mf_upload(ix) : TM_OK;
}

template <class T>
int mf_grow(tm_index *ix, T *&p, uint64_t &cap, uint64_t need) {
    if (need <= cap && p) return TM_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = std::max<uint64_t>(need + need / 2, 1024);
    HIPCHK(ix, hipMalloc(&p, cap * sizeof(T)));
    return TM_OK;
}

}  // namespace

extern "C" {

int tm_matches_filter(tm_index *ix, uint64_t n, const uint8_t *fb, const uint64_t *fo, uint64_t *out_hit_offsets,
                      uint32_t *out_values, uint64_t cap, uint8_t *out_err) {
    return tm_matches_filter_ex(ix, n, fb, fo, nullptr, out_hit_offsets, out_values, cap, out_err);
}

int tm_matches_filter_ex(tm_index *ix, uint64_t n, const uint8_t *fb, const uint64_t *fo, const uint8_t *ff,
                         uint64_t *out_hit_offsets, uint32_t *out_values, uint64_t cap, uint8_t *out_err) {
    if (!ix) return fail(nullptr, TM_EINVAL, "tm_matches_filter: null handle");
    if (!fo || !out_hit_offsets || !out_err || (n && !fb && fo[n] != fo[0]) || (cap && !out_values))
        return fail(ix, TM_EINVAL, "tm_matches_filter: null buffer");
    if (n >= 0xFFFFFFFFull) return fail(ix, TM_EINVAL, "tm_matches_filter: batch too large");
    auto &m = ix->mf;
    std::lock_guard<std::mutex> g(m.mu);   // control plane: one call at a time; the index lock stays free
    HIPCHK(ix, hipSetDevice(ix->rep[0].device));   // matches_filter's arrays live on replica 0
    if (!m.s) HIPCHK(ix, hipStreamCreateWithFlags(&m.s, hipStreamNonBlocking));
    int rc;
    if ((rc = mf_refresh(ix))) return rc;
    // queries: filter_words/1 (:359-366) -> ranks; base_init on a '$' first word
    std::vector<uint32_t> qoff(n + 1, 0), qr, qbase(n, NONE);
    std::vector<std::pair<std::string, bool>> w;
    for (uint64_t i = 0; i < n; i++) {
        mf_key_words(fb + fo[i], (uint32_t)(fo[i + 1] - fo[i]), ff ? ff[i] : 0, w);
        for (auto &x : w) qr.push_back(mf_rank(m.words, x.first, x.second));
        if (!w[0].second && !w[0].first.empty() && w[0].first[0] == '$') qbase[i] = mf_rank(m.words, w[0].first, false);
        qoff[i + 1] = (uint32_t)qr.size();
    }
    const uint64_t qwords = (n + 1) + qr.size() + n + n;   // offsets, ranks, bases, counts
    if ((rc = mf_grow(ix, m.q, m.qcap, qwords))) return rc;
    if ((rc = mf_grow(ix, m.err, m.ecap, n + 1))) return rc;
    if ((rc = mf_grow(ix, m.hit, m.hcap, n + 1))) return rc;
    uint32_t *d_qoff = m.q, *d_qr = m.q + n + 1, *d_qbase = d_qr + qr.size(), *d_cnt = d_qbase + n;
    HIPCHK(ix, hipMemcpyAsync(d_qoff, qoff.data(), (n + 1) * 4, hipMemcpyHostToDevice, m.s));
    if (!qr.empty()) HIPCHK(ix, hipMemcpyAsync(d_qr, qr.data(), qr.size() * 4, hipMemcpyHostToDevice, m.s));
    if (n) HIPCHK(ix, hipMemcpyAsync(d_qbase, qbase.data(), n * 4, hipMemcpyHostToDevice, m.s));
    HIPCHK(ix, hipMemsetAsync(m.err, 0, n + 1, m.s));
    HIPCHK(ix, launch_matches_filter(n, d_qoff, d_qr, d_qbase, m.pool, m.koff, m.val, m.K, d_cnt, nullptr, nullptr,
                                     0, m.err, m.s));
    std::vector<uint32_t> cnt(n);
    if (n) HIPCHK(ix, hipMemcpyAsync(cnt.data(), d_cnt, n * 4, hipMemcpyDeviceToHost, m.s));
    HIPCHK(ix, hipStreamSynchronize(m.s));
    out_hit_offsets[0] = 0;
    for (uint64_t i = 0; i < n; i++) out_hit_offsets[i + 1] = out_hit_offsets[i] + cnt[i];
    const uint64_t total = out_hit_offsets[n];
    if (total && cap) {
        const uint64_t wcap = std::min(total, cap);
        if ((rc = mf_grow(ix, m.out, m.ocap, wcap))) return rc;
        HIPCHK(ix, hipMemcpyAsync(m.hit, out_hit_offsets, (n + 1) * 8, hipMemcpyHostToDevice, m.s));
        HIPCHK(ix, launch_matches_filter(n, d_qoff, d_qr, d_qbase, m.pool, m.koff, m.val, m.K, d_cnt, m.hit, m.out,
                                         wcap, m.err, m.s));
        HIPCHK(ix, hipMemcpyAsync(out_values, m.out, wcap * 4, hipMemcpyDeviceToHost, m.s));
    }
    if (n) HIPCHK(ix, hipMemcpyAsync(out_err, m.err, n, hipMemcpyDeviceToHost, m.s));
    HIPCHK(ix, hipStreamSynchronize(m.s));
    if (total > cap) return fail(ix, TM_ECAP, "tm_matches_filter: output capacity too small");
    return TM_OK;
}

int tm_stats(tm_index *ix, tm_stats_t *o) {
    if (!ix || !o) return fail(ix, TM_EINVAL, "tm_stats: null argument");
    std::lock_guard<std::mutex> g(ix->img);
    memset(o, 0, sizeof *o);
    o->n_wild_keys = ix->n_wild;
    o->n_exact_keys = ix->n_exact;
    o->n_dead_keys = ix->dead.size();
    o->n_keys = ix->n_wild + ix->n_exact + ix->dead.size();
    o->n_nodes = ix->live_nodes;
    o->n_edges = ix->nlinks;
    o->n_words = ix->vcount;
    o->device_bytes = ix->vocab.dcap * sizeof(VocabEntry)   /* per replica */ + ix->wpool.dcap + ix->nodes.dcap * sizeof(Node) +
                      ix->ctab.dcap * sizeof(CSlot) + ix->vals.dcap * 4 + ix->exact.dcap * sizeof(ExactEntry) + ix->xfp.dcap * 2 +
                      ix->wseq.dcap * 4 + ix->wbits.dcap * 4;
    o->uploads = ix->uploads;
    o->patch_bytes = ix->patch_bytes;
    return TM_OK;
}

}  // extern "C"
