// tm_kernels.hip -- gfx950 kernels of the topic-match pipeline.
//
// One publish topic = one unit of work (the unit of emqx_topic_index:matches/3,
// apps/emqx/src/emqx_trie_search.erl:182-226).  A batch of topics is matched in
// two phases on one HIP stream:
//
//   phase 1  k_walk_fast     one lane per topic: tokenise on '/', look every
//                            level up in the vocab (hash + byte verification),
//                            then walk the trie as an NFA depth first
//                            ('#' terminal, '+' subtree, literal subtree -- the
//                            reference's term order, so hits come out in
//                            traversal order without a sort), then the exact
//                            (binary-key) table.  Hits are recorded as value
//                            ranges; the pending literal branch of every level
//                            and the level word ids live in LDS.
//            k_walk_list     the same for topics deeper than FAST_L (LDS, 32
//                            levels) or MID_L (global scratch), driven by
//                            device-side lists (no host round trip).
//            k_scan_*        exclusive scan of per-topic hit counts -> CSR offsets.
//   phase 2  k_emit          wave-cooperative load-balanced copy of the value
//                            ranges into the CSR (coalesced stores).
//            k_rewalk_list   topics with more than RCAP ranges are walked again
//                            and write their values directly.
//
// Integer/byte work only; the path is HBM-latency bound, so the
// design goal is many independent loads in flight per CU, not MFMA.
#include "tm_dev.h"

// The tail kernels' last-block ticket (k_walk_tail, reset_lists_if_last) and
// k_walk_small's look-back read totals other blocks published with relaxed
// device-scope atomics, ordered only by s_waitcnt(0) before the ticket and
// by agent-scope (sc1) loads in the reader -- no release/acquire fence, which
// writes back and invalidates the whole L2 of the XCD (C3deep tail +68 us,
// DESIGN.md 0 item 6).  That relies on the gfx94x/gfx95x memory system:
// device-scope atomics are performed at the coherence point across the XCDs
// and a completed s_waitcnt means they were.  Built for gfx950 only (ADVICE
// r5): any other target must revisit it, so it does not compile.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "tm_kernels.hip: the tail tickets' ordering is argued for gfx950 only (see above)"
#endif

namespace tmx {

// ----------------------------------------------------------------- helpers

__device__ __forceinline__ uint4 ld4(const void *p) { return *reinterpret_cast<const uint4 *>(p); }
// topic bytes: read once per batch, non-temporal so they do not evict trie
// lines (bench, three streams: +0.5 %, neutral on one stream)
__device__ __forceinline__ uint4 ld4_once(const void *p) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// bit b (0..191) of a table-mode node's Bloom: words kw[2..3], kc[0..3]
__device__ __forceinline__ uint32_t bloom_bit(const uint4 &n2, const uint4 &n3, uint32_t b) {
    const uint32_t j = b >> 5;
    const uint32_t w = j == 0 ? n2.z : j == 1 ? n2.w : j == 2 ? n3.x : j == 3 ? n3.y : j == 4 ? n3.z : n3.w;
    return (w >> (b & 31)) & 1u;
}

// may a table-mode node (line words n1, n2, n3) have a literal child for word
// w?  Wide nodes answer exactly from their bitmap (an L2-resident line) --
// unless the node is dense (its line's bitmap pointer NONE: nearly every word
// of its level is a child, tm_host.cpp wide_dense), where the answer is
// almost always yes and the table is probed at once -- the others from the
// 192-bit Bloom in the line
__device__ __forceinline__ uint32_t child_maybe(const DevIndex &ix, const uint4 &n1, const uint4 &n2, const uint4 &n3,
                                                uint32_t w, uint32_t h) {
    if ((n1.y & NLIT_MASK) >= WIDE_LIT)
        return n2.z == NONE ? 1u : w < ix.wcap ? (ix.wbits[n2.z + (w >> 5)] >> (w & 31)) & 1u : 0u;
    return bloom_bit(n2, n3, child_bit(h));
}

// can a child Q (summarised as Node.psum / CSlot.sum, tm_layout.h) matter to
// a topic of L levels when entered at level lq?  At lq == L, Q must emit or cut
// the walk (NLIT_HDESC); below it Q must emit ('#' terminal) or go on: a
// literal child for word wq, or its '+' child QQ, which in turn must be able to
// matter at lq + 1 (word wq2)
__device__ __forceinline__ bool child_alive(uint32_t lo, uint32_t hi, uint32_t lq, uint32_t L, uint32_t wq,
                                            uint32_t wq2) {
    const uint64_t m = (uint64_t)hi << 32 | lo;
    constexpr uint32_t AT_END = PSUM_HASH | PSUM_EXACT | PSUM_HDESC;
    if (lq == L) return (m & AT_END) != 0;
    if (m & PSUM_HASH) return true;
    if (wq != NONE && ((m >> (PSUM_BQ + psum_bit(child_hash(wq)))) & 1u)) return true;
    if (!(m & PSUM_PLUS)) return false;
    const uint32_t qq = (uint32_t)(m >> PSUM_QQ) & 15u;
    if (lq + 1 == L) return (qq & AT_END) != 0;
    if (qq & (PSUM_HASH | PSUM_PLUS)) return true;
    return wq2 != NONE && ((m >> (PSUM_BQQ + psum_bit(child_hash(wq2)))) & 1u);
}

// Empty asm "uses": pin a loaded value at this point on every path.  Without
// them the compiler sinks loads into the branches that read each field (one
// dependent round trip per field: the exact entry took three, a child slot
// two), and a load left pending on a skipped branch makes it drain vmcnt(0)
// before the next reuse of its registers.
__device__ __forceinline__ void pin(uint32_t &v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(uint2 &v) { pin(v.x); pin(v.y); }
__device__ __forceinline__ void pin(uint4 &v) { pin(v.x); pin(v.y); pin(v.z); pin(v.w); }

// A word being scanned: its length and first 8 bytes.  Words longer than VINL
// bytes (rare) are hashed from their bytes in memory when they end, so the
// per-byte loop carries no 64-bit FNV multiply.
struct WordAcc {
    uint32_t len, b0, b1;       // length, first 8 bytes packed little endian
    uint64_t start;
    __device__ __forceinline__ void reset(uint64_t s) {
        len = 0; b0 = b1 = 0; start = s;
    }
    __device__ __forceinline__ void push(uint32_t c) {
        uint32_t v = c << ((len & 3) * 8);
        if (len < 4) b0 |= v; else if (len < 8) b1 |= v;
        len++;
    }
};

// Where a walk reads its topic's bytes (offsets are the batch's own):
//  - GlobalSrc: the batch in global memory (HBM, or mapped host memory for
//    in-place host batches), or any byte pointer;
//  - StagedSrc: the block's byte span copied into LDS by coalesced loads
//    (k_walk_small's fallback lane walk), read at offset p - b0 from the LDS
//    array itself -- never
//    through a pointer rebased below it.  (The round-4 stage1 study formed
//    `s_stage - B0`: the compiler did that arithmetic on the 32-bit LDS
//    address, which wraps for B0 above the array's LDS offset, then cast it to
//    a flat pointer whose 64-bit add of the topic offset carried into the
//    aperture bits: HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION on every block
//    with B0 > 0x1300, so 1- and 64-topic batches (one block, B0 = 0) passed
//    and the 1,024-topic batch faulted -- DESIGN.md 8.)  When the span does not
//    fit (`staged` false, block-uniform) the lanes read global memory.
struct GlobalSrc {
    const uint8_t *g;
    __device__ __forceinline__ uint4 ld16(uint64_t p) const { return ld4_once(g + p); }
    __device__ __forceinline__ uint32_t byte(uint64_t p) const { return g[p]; }
};
struct StagedSrc {
    const uint8_t *g;
    const uint4 *lds;
    uint64_t b0;
    bool staged;
    __device__ __forceinline__ uint4 ld16(uint64_t p) const {
        return staged ? lds[(uint32_t)(p - b0) >> 4] : ld4_once(g + p);
    }
    __device__ __forceinline__ uint32_t byte(uint64_t p) const {
        return staged ? reinterpret_cast<const uint8_t *>(lds)[(uint32_t)(p - b0)] : g[p];
    }
};

template <class Src>
__device__ bool bytes_eq(const uint8_t *a, const Src &src, uint64_t b, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) if (a[i] != src.byte(b + i)) return false;
    return true;
}

template <class Src>
__device__ __forceinline__ uint64_t word_hash_dev(const WordAcc &w, const Src &src) {
    if (w.len <= VINL) return word_hash_short(w.b0, w.b1, w.len);
    uint64_t h = FNV_OFF;   // FNV-1a, as the host's word_hash (tm_host.cpp)
    for (uint32_t i = 0; i < w.len; i++) h = (h ^ src.byte(w.start + i)) * FNV_PRIME;
    return word_hash_finish(h, w.len);
}

// continue a vocab probe sequence from `slot` (exact: tag, then bytes: the
// word at `start` of src when it is longer than VINL)
template <class Src>
__device__ uint32_t vocab_probe(const DevIndex &ix, uint32_t slot, uint32_t tag, uint32_t len, uint32_t b0,
                                uint32_t b1, const Src &src, uint64_t start) {
    for (;;) {
        const uint4 e = ld4(ix.vocab + slot);   // tag, wid, b0, b1
        if (e.y == NONE) return NONE;
        if (e.x == tag) {
            if (len <= VINL) {
                if (e.z == b0 && e.w == b1) return e.y;
            } else if (e.w == len && bytes_eq(ix.wpool + e.z, src, start, len)) {
                return e.y;
            }
        }
        slot = (slot + 1) & ix.vmask;
    }
}

// the same for a word of <= VINL bytes (tag, then its packed bytes)
__device__ uint32_t vocab_probe_short(const DevIndex &ix, uint32_t slot, uint32_t tag, uint32_t b0, uint32_t b1) {
    for (;;) {
        const uint4 e = ld4(ix.vocab + slot);   // tag, wid, b0, b1
        if (e.y == NONE) return NONE;
        if (e.x == tag && e.z == b0 && e.w == b1) return e.y;
        slot = (slot + 1) & ix.vmask;
    }
}

// vocab: word -> wid, exact by construction (hash tag, then length and bytes)
template <class Src>
__device__ uint32_t vocab_find(const DevIndex &ix, const WordAcc &w, const Src &src) {
    const uint64_t h = word_hash_dev(w, src);
    return vocab_probe(ix, (uint32_t)h & ix.vmask, vocab_tag(h, w.len), w.len, w.b0, w.b1, src, w.start);
}

// literal child in a node's private table (table mode, nlit > KINL), with the
// slot's summary of the child
__device__ __forceinline__ uint32_t ctab_find(const DevIndex &ix, uint32_t off, uint32_t mask, uint32_t wid,
                                              uint32_t h, uint32_t &slo, uint32_t &shi) {
    for (uint32_t s = h & mask;; s = (s + 1) & mask) {
        uint4 e = ld4(ix.ctab + off + s);
        pin(e);
        if (e.x == wid) { slo = e.z; shi = e.w; return e.y; }
        if (e.x == NONE) return NONE;
    }
}

// ------------------------------------------------------- frontier storage

// LDS frontier: wid[level] and the pending literal child of each level,
// laid out [level][thread] so that any mix of levels is bank-conflict free.
//
// Stores deeper than the main walk's also carry what the cut of a '#'-not-last
// key needs (tm_layout.h NLIT_HDESC): which levels of the current path were
// entered through '+' (pm, bit q: the node at depth q + 1 is a '+' child).  The
// main walk's store does not: a topic that meets such a cut is handed to the
// tail lists (DFS_REROUTE), keeping k_walk_fast within its register budget.
//
// LITE (k_walk_small<8>'s fallback lane walk, lite_path_ok indexes): the main
// walk's FAST_L levels, but tokenised like the deeper stores -- every level
// scanned (count, badarg), only the levels a walk can use resolved
// (need_levels) -- which lite_path_ok guarantees fit FAST_L.
template <int ML, bool LITE = false>
struct LdsStore {
    static constexpr uint32_t maxl = ML;
    static constexpr bool deferred = true;   // vocab probes of short words after tokenisation
    static constexpr bool cuts = ML > FAST_L;
    static constexpr bool need = ML > FAST_L || LITE;   // resolve only need_levels(), scan the rest
    uint32_t *wid, *pend;
    uint8_t *len8;                           // [level][thread] word lengths (deferred probes)
    uint32_t stride;
    uint64_t mask;
    uint32_t pm;
    __device__ __forceinline__ void down(uint32_t l, bool via_plus) {   // depth l -> l + 1
        if constexpr (cuts) pm = via_plus ? pm | (1u << l) : pm & ~(1u << l);
    }
    __device__ __forceinline__ void popped(uint32_t l) {   // resumed at depth l (>= 1): a literal child
        if constexpr (cuts) pm &= (1u << (l - 1)) - 1u;
    }
    // the walk hit the cut at the topic's last level: keep the pending literal
    // branches up to the innermost '+' of the path (the seek target), or none
    __device__ __forceinline__ void cut(uint32_t) {
        if constexpr (cuts) mask &= pm ? (1ull << (33u - __clz(pm))) - 1ull : 0ull;
    }
    __device__ __forceinline__ uint32_t get_wid(uint32_t l) const { return wid[l * stride]; }
    __device__ __forceinline__ void set_wid(uint32_t l, uint32_t w) { wid[l * stride] = w; }
    __device__ __forceinline__ void reset() { mask = 0; pm = 0; }
    // deferred vocab probes: a short word's packed bytes + length, parked in
    // the wid / pend slots of its level until the probe resolves it
    __device__ __forceinline__ void put_word(uint32_t l, uint32_t b0, uint32_t b1, uint32_t len) {
        wid[l * stride] = b0; pend[l * stride] = b1; len8[l * stride] = (uint8_t)len;
    }
    __device__ __forceinline__ uint32_t word_b0(uint32_t l) const { return wid[l * stride]; }
    __device__ __forceinline__ uint32_t word_b1(uint32_t l) const { return pend[l * stride]; }
    __device__ __forceinline__ uint32_t word_len(uint32_t l) const { return len8[l * stride]; }
    __device__ __forceinline__ void push(uint32_t l, uint32_t node) {
        pend[l * stride] = node; mask |= 1ull << l;
    }
    __device__ __forceinline__ bool pop(uint32_t &l, uint32_t &node) {
        if (!mask) return false;
        l = 63u - (uint32_t)__clzll(mask);
        mask &= ~(1ull << l);
        node = pend[l * stride];
        return true;
    }
};

// Global-scratch frontier for arbitrarily deep topics (one slot per lane);
// plus_at[q] = 1: the path's node at depth q + 1 is a '+' child (for cut()).
struct GlobalStore {
    static constexpr uint32_t maxl = MAX_LEVELS;
    static constexpr bool deferred = false;
    static constexpr bool cuts = true;
    static constexpr bool need = true;
    uint32_t *wid;
    uint2 *stk;
    uint8_t *plus_at;
    uint32_t top;
    __device__ __forceinline__ uint32_t get_wid(uint32_t l) const { return wid[l]; }
    __device__ __forceinline__ void set_wid(uint32_t l, uint32_t w) { wid[l] = w; }
    __device__ __forceinline__ void reset() { top = 0; }
    __device__ __forceinline__ void down(uint32_t l, bool via_plus) { plus_at[l] = via_plus; }
    __device__ __forceinline__ void popped(uint32_t l) { plus_at[l - 1] = 0; }
    __device__ void cut(uint32_t L) {   // as LdsStore::cut, the path being L levels deep
        int64_t q = (int64_t)L - 1;
        while (q >= 0 && !plus_at[q]) q--;
        while (top && (int64_t)stk[top - 1].x > q + 1) top--;
    }
    __device__ __forceinline__ void push(uint32_t l, uint32_t node) { stk[top++] = make_uint2(l, node); }
    __device__ __forceinline__ bool pop(uint32_t &l, uint32_t &node) {
        if (!top) return false;
        uint2 e = stk[--top]; l = e.x; node = e.y;
        return true;
    }
};

// ---------------------------------------------------------- tokenisation

enum { RC_OK = 0, RC_BADARG = 1, RC_DEEP = 2 };

// levels whose vocab probes are in flight together (6 covers MQTT's usual
// topic depths in one round trip and keeps k_walk_fast within 64 VGPRs, i.e.
// 8 waves per SIMD -- a budget small code changes can tip: check the
// -Rpass-analysis=kernel-resource-usage remark after every change)
constexpr uint32_t VGROUP = 6;

// '/' bytes in [p, end), p 16-byte aligned: four 16-byte loads in flight per
// round trip, bytes compared a word at a time
template <class Src>
__device__ __noinline__ uint32_t count_slashes(const Src src, uint64_t p, uint64_t end) {   // (by value: a reference to a
                                                                                            // temporary put it in scratch)
    uint32_t n = 0;
    for (; p < end; p += 64) {
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; c++) v[c] = p + 16 * c < end ? src.ld16(p + 16 * c) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t w[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
            const uint64_t q = p + 16 * c;
            const int k1 = q >= end ? 0 : end - q < 16 ? (int)(end - q) : 16;   // bytes of the chunk inside [p, end)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t x = w[j] ^ 0x2F2F2F2Fu;   // '/' bytes -> 0
                uint32_t nz = (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;   // bit 7 set: byte != '/'
                const int valid = k1 - 4 * j;
                if (valid < 4) nz |= valid <= 0 ? 0x80808080u : 0x80808080u << (8 * valid);
                n += 4 - __popc(nz);
            }
        }
    }
    return n;
}

// topic_words/1 (emqx_trie_search.erl:369-378): split on '/', a level that is
// exactly '+' or '#' is badarg; level words are resolved to wids.  Also
// computes base_init's '$' flag (:160-163) and the exact-key hash.
//
// Two passes.  The scan (ALU only once the first two 16-byte chunks of the
// topic are in) keeps each word's packed bytes and length in the frontier's
// LDS slots; words longer than VINL bytes are looked up after it.
// Then the vocab probes of up to VGROUP levels are issued together, so a topic's
// words cost one memory round trip instead of one per level, and the lanes of a
// wave no longer serialise on the byte position where each of their words ends.
template <class S, class Src>
__device__ int tokenize(const DevIndex &ix, const Src &src, uint64_t beg, uint64_t end, S &st,
                        uint32_t &L, bool &dollar, uint64_t &xh, bool &all_found) {
    uint64_t longmask = 0;   // levels resolved before the deferred probes
    all_found = true; dollar = false; xh = FNV_OFF;
    const uint64_t p0 = beg & ~15ull;
    // aligned 16-byte loads (the first two issued together): a chunk shares its 16-byte granule with a valid
    // byte, so it never crosses a page the caller does not own
    const uint4 z = make_uint4(0, 0, 0, 0);
    const uint4 c0 = p0 < end ? src.ld16(p0) : z;
    const uint4 c1 = p0 + 16 < end ? src.ld16(p0 + 16) : z;
    if constexpr (S::deferred) {
        // The scan keeps only (first 8 bytes, length) per word and parks them in
        // the level's LDS slots when a '/' ends it; the checks (badarg, depth,
        // '$', long words) run per level afterwards, so the divergent work at a
        // word end is three LDS stores.  A word longer than VINL bytes parks
        // its length and start instead (len8 = 255), resolved below.
        // The main walk's store (FAST_L levels) takes topics that fit it whole;
        // deeper ones go to the tail lists.  The tail's store (MID_L levels)
        // resolves only the levels a walk can use: down to the trie's depth,
        // or all of them when a binary key of L levels exists -- so a 64-level
        // topic against a 6-level trie stays on the LDS path (need_levels).
        constexpr bool NEED = S::need;
        uint32_t lev = 0, len = 0, b0 = 0, b1 = 0;
        uint64_t ws = beg;
        bool bad = false;   // tail store: a level past the stored ones is exactly '+' or '#'
        auto park = [&]() {
            if (lev < S::maxl) {
                if (len <= VINL) st.put_word(lev, b0, b1, len);
                else st.put_word(lev, len, (uint32_t)(ws - beg), 255);
            } else if constexpr (NEED) {
                bad |= len == 1 && ((b0 & 0xFFu) == '+' || (b0 & 0xFFu) == '#');
            }
            lev++;
        };
        uint32_t ci = 0;
        uint64_t p = p0;
        uint4 ra = c0, rb = c1;   // tail store: chunks loaded two ahead (deep topics run hundreds of bytes)
        for (; p < end; p += 16, ci++) {
            if (!NEED && lev > S::maxl) break;   // deeper than the main walk's store
            uint4 v;
            if constexpr (NEED) {
                v = ra; ra = rb;
                rb = p + 32 < end ? src.ld16(p + 32) : z;
            } else {
                v = ci == 0 ? c0 : ci == 1 ? c1 : src.ld16(p);
            }
            const uint32_t k0 = p < beg ? (uint32_t)(beg - p) : 0;
            const uint32_t k1 = end - p < 16 ? (uint32_t)(end - p) : 16;
#pragma unroll
            for (uint32_t k = 0; k < 16; k++) {
                if (k < k0 || k >= k1) continue;
                const uint32_t word = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
                const uint32_t c = (word >> ((k & 3) * 8)) & 0xFFu;
                if (c == '/') {
                    park();
                    len = 0; b0 = 0; b1 = 0; ws = p + k + 1;
                } else {
                    const uint32_t sh = (len & 3) * 8;
                    b0 |= len < 4 ? c << sh : 0u;
                    b1 |= len - 4 < 4 ? c << sh : 0u;
                    len++;
                }
            }
        }
        if (!NEED && p < end) {   // left early: hand the topic over to the tail lists
            // The level count only picks the tail list.  With no binary key
            // deeper than this store and a trie the LDS tail resolves, every
            // count from here on picks the LDS list (need_levels <= depth), so
            // the rest is not scanned: a long topic made its whole wave wait
            const bool any = ix.xlen_max <= S::maxl && ix.depth + 2 <= (uint32_t)MID_L &&
                             end - beg < (uint64_t)MAX_LEVELS;
            L = any ? lev + 1 : lev + 1 + count_slashes(src, p, end);
            return RC_DEEP;
        }
        park();
        if (lev > (NEED ? MAX_LEVELS : S::maxl)) { L = lev; return RC_DEEP; }   // (> MAX_LEVELS: the global walk flags it)
        L = lev;
        // a level exactly '+' or '#' is badarg (:374-375), at any depth: the
        // stored levels here, the rest during the scan (park)
        for (uint32_t l = 0; l < L && l < S::maxl; l++) {
            const uint32_t n = st.word_len(l), c = st.word_b0(l) & 0xFFu;
            bad |= n == 1 && (c == '+' || c == '#');
        }
        if (bad) return RC_BADARG;
        if constexpr (NEED) {
            const uint32_t Lw = need_levels(ix, L);
            if (Lw + (Lw < L ? 2 : 0) > S::maxl) return RC_DEEP;
            L |= Lw << 24;   // Lw rides in L's top byte until the probes are done
        }
        // base_init (:160-163): the first level starts with '$'
        dollar = st.word_len(0) == 255 ? src.byte(beg) == '$' : st.word_len(0) >= 1 && (st.word_b0(0) & 0xFFu) == '$';
        for (uint32_t l = 0; l < (S::need ? L >> 24 : L); l++) {
            if (st.word_len(l) != 255) continue;
            WordAcc w; w.reset(beg + st.word_b1(l)); w.len = st.word_b0(l);
            st.set_wid(l, vocab_find(ix, w, src));
            longmask |= 1ull << l;
        }
    } else {
        WordAcc w; w.reset(beg);
        uint32_t lev = 0;
        auto finish = [&]() -> int {
            if (w.len == 1 && (w.b0 == '+' || w.b0 == '#')) return RC_BADARG;
            if (lev >= S::maxl) return RC_DEEP;
            if (lev == 0 && w.len >= 1 && (w.b0 & 0xFF) == '$') dollar = true;
            st.set_wid(lev, vocab_find(ix, w, src));
            lev++;
            return RC_OK;
        };
        uint32_t ci = 0;
        for (uint64_t p = p0; p < end; p += 16, ci++) {
            const uint4 v = ci == 0 ? c0 : ci == 1 ? c1 : src.ld16(p);
            const uint32_t k0 = p < beg ? (uint32_t)(beg - p) : 0;
            const uint32_t k1 = end - p < 16 ? (uint32_t)(end - p) : 16;
            for (uint32_t k = k0; k < k1; k++) {
                const uint32_t word = k < 4 ? v.x : k < 8 ? v.y : k < 12 ? v.z : v.w;
                const uint32_t c = (word >> ((k & 3) * 8)) & 0xFFu;
                if (c == '/') {
                    int rc = finish();
                    if (rc) return rc;
                    w.reset(p + k + 1);
                } else {
                    w.push(c);
                }
            }
        }
        int rc = finish();
        if (rc) return rc;
        L = lev;
    }
    if constexpr (S::deferred) {
        // Branch-free issue and consumption: every lane issues VGROUP loads
        // (unused levels read slot 0) and consumes all of them, so no load is
        // left pending on a skipped branch -- the compiler would otherwise drain
        // vmcnt(0) before reusing its registers and serialise the probes.
        for (uint32_t base = 0; base < (S::need ? L >> 24 : L); base += VGROUP) {
            uint4 e[VGROUP];
            uint32_t tg[VGROUP];
            bool use[VGROUP];
#pragma unroll
            for (uint32_t k = 0; k < VGROUP; k++) {
                const uint32_t l = base + k;
                use[k] = l < (S::need ? L >> 24 : L) && !((longmask >> l) & 1);
                const uint32_t ls = use[k] ? l : 0;
                const uint32_t len = st.word_len(ls);
                const uint64_t h = word_hash_short(st.word_b0(ls), st.word_b1(ls), len);
                tg[k] = vocab_tag(h, len);
                e[k] = ld4(ix.vocab + (use[k] ? ((uint32_t)h & ix.vmask) : 0u));
            }
#pragma unroll
            for (uint32_t k = 0; k < VGROUP; k++) {
                const uint32_t l = use[k] ? base + k : 0;
                const uint32_t b0 = st.word_b0(l), b1 = st.word_b1(l);
                const bool hit = e[k].x == tg[k] && e[k].z == b0 && e[k].w == b1;
                uint32_t wid = e[k].y == NONE ? NONE : hit ? e[k].y : NONE - 1;
                pin(wid);   // consume e[k] here on every path
                if (use[k]) {
                    if (wid == NONE - 1) {   // rare at load <= 1/2: walk the probe sequence on
                        const uint32_t len = st.word_len(l);
                        const uint64_t h = word_hash_short(b0, b1, len);
                        wid = vocab_probe_short(ix, ((uint32_t)h + 1) & ix.vmask, tg[k], b0, b1);
                    }
                    st.set_wid(l, wid);
                }
            }
        }
    }
    if constexpr (S::deferred && S::need) {
      const uint32_t Lw = L >> 24;
      L &= 0xFFFFFFu;
      if (Lw < L) {
        // No binary key has L levels, and no trie node below level Lw has
        // children: the walk reads levels Lw and Lw + 1 at most (a node's
        // word and its summaries' look-ahead), which never match anything.
        st.set_wid(Lw, NONE);
        st.set_wid(Lw + 1, NONE);
        all_found = false;
        return RC_OK;
      }
    }
    for (uint32_t l = 0; l < L; l++) {
        const uint32_t wid = st.get_wid(l);
        all_found &= wid != NONE;
        xh = seq_hash_step(xh, wid);
    }
    xh = seq_hash_finish(xh, L);
    return RC_OK;
}

// the tail list of a topic of nl levels the main walk could not take: the LDS
// frontier (MID_L levels) if the levels it must resolve fit, else global scratch
__device__ __forceinline__ int tail_list(const DevIndex &ix, uint32_t nl) {
    return nl <= MAX_LEVELS && need_levels(ix, nl) <= MID_L ? L_MID : L_DEEP;
}

// match_topics/4 (emqx_trie_search.erl:381-389): binary keys equal to the topic.
// The probe walks the 2-byte fingerprint array (`f` = the home slot's, loaded
// before the trie walk so its latency hides behind it) and reads a 64-byte
// entry only where the fingerprint matches; the entry is then verified
// exactly (hash, level count, every wid).
template <class S>
__device__ void exact_find(const DevIndex &ix, uint64_t xh, uint32_t L, const S &st, uint32_t slot, uint32_t f,
                           uint32_t &off, uint32_t &cnt) {
    cnt = 0; off = 0;
    const uint32_t fp = exact_fp(xh);
    for (;;) {
        if (f == 0) return;
        if (f == fp) {
            const uint4 *e = reinterpret_cast<const uint4 *>(ix.exact + slot);
            uint4 a = e[0], b = e[1], c = e[2], d = e[3];
            pin(a); pin(b); pin(c); pin(d);
            if (a.x == (uint32_t)xh && a.y == (uint32_t)(xh >> 32) && a.z == L) {
                bool eq = true;
                if (L <= XINL) {
                    const uint32_t iw[XINL] = {b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
#pragma unroll
                    for (uint32_t l = 0; l < XINL; l++)
                        if (l < L) eq &= iw[l] == st.get_wid(l);
                } else {
                    for (uint32_t l = 0; l < L && eq; l++) eq = ix.wseq[b.y + l] == st.get_wid(l);
                }
                if (eq) { off = a.w; cnt = b.x; return; }
            }
        }
        slot = (slot + 1) & ix.xmask;
        f = ix.xfp[slot];
    }
}

// --------------------------------------------------------------- the walk

// Depth-first NFA walk.  At node P on level l (P = the filter prefix matched so
// far) the keys under P in Erlang term order are: [P] (exact terminal, only a
// hit when l == L), [P,'#'] ('#' terminal: 'a/#' also matches 'a'), the '+'
// subtree, then the literal subtree -- so visiting them in that order emits
// hits in exactly the reference's traversal order (search_up, :239-253).
// First-level '$' words skip the root's '+' and '#' (base_init, :160-163).
// A '#'-not-last key below P (NLIT_HDESC) skips P's '+' subtree when the topic
// goes on, and cuts the walk when it ends at P (tm_layout.h).
enum { DFS_DONE = 0, DFS_STOP = 1, DFS_REROUTE = 2 };   // STOP: the emitter asked (match/2 first hit)
template <class S, class EM>
__device__ int dfs(const DevIndex &ix, uint32_t L, bool dollar, S &st, EM &em) {
    uint32_t cur = ROOT, l = 0;
    for (;;) {
        // the whole state is one 64-byte line (tm_layout.h Node)
        const uint4 *np = reinterpret_cast<const uint4 *>(ix.nodes + cur);
        const uint4 n0 = np[0];   // plus, hash_off, hash_cnt, exact_off
        const uint4 n1 = np[1];   // exact_cnt, nlit | NLIT_HDESC, psum_lo, psum_hi
        const uint4 n2 = np[2];   // kw[0..3] (table mode: offset, size-1)
        const uint4 n3 = np[3];   // kc[0..3]
        const bool droot = dollar && l == 0;
        // The inline-child match reads n2/n3 on every path (pinned): a line
        // load left pending on a skipped branch would make the compiler drain
        // vmcnt(0) at the top of the next step, before its loads are issued --
        // serialising them behind the exact-table fingerprint load that is
        // meant to overlap the walk.
        const uint32_t w = l < L ? st.get_wid(l) : NONE;
        uint32_t inl = n2.x == w ? n3.x : n2.y == w ? n3.y : n2.z == w ? n3.z : n2.w == w ? n3.w : NONE;
        pin(inl);
        if (l == L) {
            if (!em(n0.w, n1.x)) return DFS_STOP;
            if (!droot && !em(n0.y, n0.z)) return DFS_STOP;
            if (n1.y & NLIT_HDESC) {   // [P,'#',...] returns lower here (compare/3, :333-340)
                if constexpr (!S::cuts) return DFS_REROUTE;
                st.cut(L);
            }
        } else {
            uint32_t lit = NONE;
            if (w != NONE) {
                if ((n1.y & NLIT_MASK) <= KINL) {
                    lit = inl;
                } else {
                    const uint32_t h = child_hash(w);
                    if (child_maybe(ix, n1, n2, n3, w, h) & 1u) {
                        uint32_t slo, shi;
                        lit = ctab_find(ix, n2.x, n2.y, w, h, slo, shi);
                        if (lit != NONE && !child_alive(slo, shi, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                                        l + 2 < L ? st.get_wid(l + 2) : NONE))
                            lit = NONE;
                    }
                }
            }
            if (!droot && !em(n0.y, n0.z)) return DFS_STOP;
            // [P,'#',...] seeks to P/W past the '+' subtree (:341-348)
            uint32_t plus = droot || (n1.y & NLIT_HDESC) ? NONE : n0.x;
            if (plus != NONE && !child_alive(n1.z, n1.w, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                             l + 2 < L ? st.get_wid(l + 2) : NONE))
                plus = NONE;
            if (plus != NONE) {
                if (lit != NONE) st.push(l + 1, lit);
                st.down(l, true);
                cur = plus; l++;
                continue;
            }
            if (lit != NONE) {
                st.down(l, false);
                cur = lit; l++;
                continue;
            }
        }
        if (!st.pop(l, cur)) return DFS_DONE;
        st.popped(l);
    }
}

// ---------------------------------------------------------------- emitters

struct RangeEmit {          // phase 1: count hits, keep up to RCAP value ranges in registers
    uint2 r[RCAP];
    uint32_t cnt, nr;
    __device__ __forceinline__ bool operator()(uint32_t off, uint32_t n) {   // n: a run's device count
        if (n) {
#pragma unroll
            for (uint32_t i = 0; i < RCAP; i++)
                if (nr == i) r[i] = make_uint2(off, n);
            nr++; cnt += n & RUN_CNT;
        }
        return true;
    }
    // ranges are stored rank-major (rng[i * n + t]): lanes of a wave write and
    // k_emit reads them coalesced
    __device__ __forceinline__ void store(uint2 *rng, uint64_t n, uint64_t t) const {
#pragma unroll
        for (uint32_t i = 0; i < RCAP; i++)
            if (i < nr) __builtin_nontemporal_store((uint64_t)r[i].x | ((uint64_t)r[i].y << 32),
                                                    reinterpret_cast<uint64_t *>(rng) + (uint64_t)i * n + t);
    }
};

struct DirectEmit {         // re-walk: write values straight into the CSR
    const uint32_t *vals;
    uint32_t *out;
    uint64_t pos, cap;
    __device__ __forceinline__ bool operator()(uint32_t off, uint32_t n) {
        const uint32_t c = n & RUN_CNT;
        for (uint32_t i = 0; i < c; i++, pos++)
            if (pos < cap) out[pos] = (n & RUN_INLINE) ? off : vals[off + i];
        return true;
    }
};

struct FirstEmit {          // match/2: stop at the first hit
    const uint32_t *vals;
    uint32_t v;
    bool found;
    __device__ __forceinline__ bool operator()(uint32_t off, uint32_t n) {
        if (n) { v = (n & RUN_INLINE) ? off : vals[off]; found = true; return false; }
        return true;
    }
};

template <class S, class EM, class Src>
__device__ __forceinline__ int match_topic(const DevIndex &ix, const Src &src, uint64_t beg, uint64_t end, S &st,
                                           EM &em, uint32_t *levels = nullptr) {
    uint32_t L = 0; bool dollar, allf; uint64_t xh;
    int rc = tokenize(ix, src, beg, end, st, L, dollar, xh, allf);
    if (levels) *levels = L;   // RC_DEEP: the topic's level count (the tail list's choice)
    if (rc) return rc;
    st.reset();
    const uint32_t xslot = (uint32_t)xh & ix.xmask;
    const uint32_t xf = allf ? ix.xfp[xslot] : 0;
    const int d = dfs(ix, L, dollar, st, em);
    if (d == DFS_STOP) return RC_OK;
    if (d == DFS_REROUTE) {   // a cut the main walk's store cannot make: the tail lists walk it
        if (levels) *levels = L;
        return RC_DEEP;
    }
    if (allf) {
        uint32_t xoff, xcnt;
        exact_find(ix, xh, L, st, xslot, xf, xoff, xcnt);
        em(xoff, xcnt);
    }
    return RC_OK;
}

enum { MODE_COUNT = 0, MODE_FIRST = 1 };

struct Outs {               // per-mode outputs
    uint8_t *err;
    uint32_t *first_val;
    uint8_t *first_found;
};

// Wave-aggregated push (every lane of the wave calls it; k = -1: nothing to
// push): one atomic per list and wave.  Per-lane atomics on one counter
// serialise at the L2 -- a batch with 10 % deep topics spent 1 ms of its walk
// on them.
__device__ __forceinline__ void list_push_wave(const Workspace &ws, uint64_t n, int k, uint32_t t) {
    const uint32_t lane = threadIdx.x & 63;
    for (int j = 0; j < L_COUNT; j++) {
        if (!__ballot(k >= 0)) break;   // (nothing to push: the common case, one ballot)
        const uint64_t m = __ballot(k == j);
        if (!m) continue;
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&ws.list_n[j], (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, (int)leader, 64);
        if (k == j) ws.lists[(uint64_t)j * n + base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = t;
    }
}

__device__ __forceinline__ void list_push(const Workspace &ws, uint64_t n, int k, uint32_t t) {
    uint32_t i = atomicAdd(&ws.list_n[k], 1u);
    ws.lists[(uint64_t)k * n + i] = t;
}

// one topic in phase-1 (count) or first-hit mode; returns RC_DEEP if the
// storage is too shallow (caller routes the topic to a list kernel).  *hits
// receives the topic's hit count (count mode).
template <int MODE, class S>
__device__ int run_topic(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *blob,
                         const uint64_t *offs, uint64_t t, S &st, const Outs &o, uint32_t *hits,
                         int *ovf = nullptr) {
    const uint64_t beg = offs[t], end = offs[t + 1];
    if (MODE == MODE_COUNT) {
        RangeEmit em;
        em.cnt = 0; em.nr = 0;
        uint32_t levels;
        int rc = match_topic(ix, GlobalSrc{blob}, beg, end, st, em, &levels);
        // more levels than the global scratch holds (> 65536: longer than any
        // MQTT topic, emqx_mqtt.hrl:44): flagged err 2, no hits
        const bool toolong = rc == RC_DEEP && S::maxl == MAX_LEVELS;
        if (rc == RC_DEEP && !toolong) { *hits = levels; return rc; }   // the caller lists it by depth
        if (rc != RC_OK) { em.cnt = 0; em.nr = 0; }
        // per-topic outputs, read once by k_emit: non-temporal (bench +1.6 %)
        __builtin_nontemporal_store(em.cnt, ws.cnt + t);
        __builtin_nontemporal_store(em.nr, ws.nr + t);
        em.store(ws.rng, n, t);
        __builtin_nontemporal_store((uint8_t)(rc == RC_BADARG ? 1 : (toolong ? 2 : 0)), o.err + t);
        if (em.nr > RCAP) {   // re-walked by k_rewalk_tail (ovf: the caller pushes it)
            const int k = S::maxl <= MID_L ? L_OVF_MID : L_OVF_DEEP;
            if (ovf) *ovf = k; else list_push(ws, n, k, (uint32_t)t);
        }
        *hits = em.cnt;
        return rc;
    } else {
        FirstEmit em{ix.vals, 0, false};
        uint32_t levels;
        int rc = match_topic(ix, GlobalSrc{blob}, beg, end, st, em, &levels);
        const bool toolong = rc == RC_DEEP && S::maxl == MAX_LEVELS;
        if (rc == RC_DEEP && !toolong) { *hits = levels; return rc; }
        o.first_val[t] = toolong ? 0 : em.v;
        o.first_found[t] = rc == RC_BADARG ? 2 : (toolong ? 3 : (em.found ? 1 : 0));
        *hits = 0;
        return rc;
    }
}

// ------------------------------------------------------------ wave / block scans

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Decoupled look-back of the one-launch kernels, by one whole wave: block vb
// publishes its own total `sum` (LB_AGG), reads its predecessors' words 64 at
// a time (lane k: block hi - k) back to the nearest inclusive prefix, summing
// the totals in between, publishes its own inclusive prefix and returns its
// exclusive one (in every lane).  A predecessor started before vb (dispatch
// order, include/tmatch.h "Forward progress"), so it
// publishes soon; the wait for one word is still bounded: past lb.spins polls
// -- or when a predecessor failed, or vb is the test hook's lb.fail_block --
// the result is LBR_FAIL and vb publishes LB_FAIL, which every later block
// meets and propagates: nothing after a failed block is trusted, the caller
// flags its topics err 4 and raises the workspace's fail word (a
// failed block used to publish a partial prefix its successors took as
// correct).
enum { LBR_OK = 0, LBR_FAIL = 1 };
__device__ __forceinline__ uint64_t look_back(uint64_t *look, uint32_t vb, uint32_t tag, uint64_t sum, const LbCtl &lb,
                                              int &res) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t pre = 0;
    res = vb == lb.fail_block ? LBR_FAIL : LBR_OK;
    if (res == LBR_OK && vb > 0 && lane == 0)
        __hip_atomic_store(&look[(uint64_t)vb * LB_STRIDE], lb_word(tag, LB_AGG, sum), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    for (int64_t hi = (int64_t)vb - 1; hi >= 0 && res == LBR_OK;) {
        const int64_t j = hi - (int64_t)lane;
        uint64_t f = lb_word(tag, LB_INCL, 0);   // before block 0: an inclusive prefix of 0
        if (j >= 0)
            for (;;) {
                f = __hip_atomic_load(&look[(uint64_t)j * LB_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lb_tag(f) == tag || ++spins > lb.spins) break;
                __builtin_amdgcn_s_sleep(LB_SLEEP);
            }
        if (__ballot(lb_tag(f) != tag || lb_state(f) == LB_FAIL)) { res = LBR_FAIL; break; }
        const uint64_t mi = __ballot(lb_state(f) == LB_INCL);
        const uint32_t k = mi ? (uint32_t)__ffsll((long long)mi) - 1 : 63;   // nearest inclusive prefix
        uint64_t v = lane <= k ? f & LB_VAL_MASK : 0;
        for (int d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
        pre += v;
        if (mi) break;
        hi -= 64;
    }
    if (lane == 0)
        __hip_atomic_store(&look[(uint64_t)vb * LB_STRIDE],
                           res == LBR_OK ? lb_word(tag, LB_INCL, pre + sum) : lb_word(tag, LB_FAIL, sum),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v, uint32_t &total) {
    const int lane = threadIdx.x & 63;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    total = __shfl(inc, 63, 64);
    return inc - v;
}

// block-wide exclusive scan of one value per thread (blockDim = 256)
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t &total, uint64_t *s_w) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint64_t inc = wave_incl_scan(v);
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint64_t pre = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) { if (i < wv) pre += s_w[i]; if (i < nw) total += s_w[i]; }
    __syncthreads();
    return pre + inc - v;
}

// a walk's hits into its topic's tile total (phase 1).  (Adding them into
// the superblock total here as well cost the walk 19 us per 1M C3 topics:
// 256 walk blocks' atomics on each superblock word.)
__device__ __forceinline__ void add_tile_total(const Workspace &ws, uint64_t t, uint64_t v) {
    atomicAdd((unsigned long long *)&ws.blk[t / TILE], (unsigned long long)v);
}

// ----------------------------------------------------------------- kernels
//
// Per batch: phase 1 = k_walk_fast, k_walk_tail; phase 2 = k_emit,
// k_rewalk_tail.  Tiles of TILE = 256 topics line up across kernels: the walks
// add each tile's hit total into ws.blk, the last k_walk_tail block sums each
// superblock's (SUP tiles) into ws.sup; a k_emit block sums the superblock
// totals before its own and the tile totals before it inside its superblock
// (one load per lane, no scan kernel and no waiting: every total is final
// when k_emit starts), then scans inside its tile; k_rewalk_tail, the batch's
// last kernel, zeroes both.

// a walk block is a scan tile, or a part of one (tile totals added
// atomically); 64 vs 256 threads: walk 0.2553 vs 0.2631 ms per 1M C3 topics
// (a block waits for its slowest lane)
constexpr int WALK_BLOCK = 64;
static_assert(TILE % WALK_BLOCK == 0, "walk blocks tile the scan tiles");

template <int MODE>
__global__ __launch_bounds__(WALK_BLOCK, 8) void k_walk_fast(DevIndex ix, Workspace ws, uint64_t n,
                                                          const uint8_t *blob, const uint64_t *offs, Outs o) {
    __shared__ uint32_t s_wid[FAST_L * WALK_BLOCK];
    __shared__ uint32_t s_pend[(FAST_L + 1) * WALK_BLOCK];
    __shared__ uint8_t s_len[FAST_L * WALK_BLOCK];
    __shared__ uint64_t s_w[4];
    const uint64_t t = (uint64_t)blockIdx.x * WALK_BLOCK + threadIdx.x;
    uint32_t hits = 0;
    int deep = -1, ovf = -1;   // tail lists this topic goes to
    if (t < n) {
        LdsStore<FAST_L> st{s_wid + threadIdx.x, s_pend + threadIdx.x, s_len + threadIdx.x, WALK_BLOCK, 0};
        int rc = run_topic<MODE>(ix, ws, n, blob, offs, t, st, o, &hits, &ovf);
        if (rc == RC_DEEP) {   // hits = the topic's level count
            deep = tail_list(ix, hits);
            hits = 0;   // counted by k_walk_tail (atomically added to this tile)
        }
    }
    static_assert(WALK_BLOCK % 64 == 0, "whole waves");
    list_push_wave(ws, n, deep, (uint32_t)t);
    list_push_wave(ws, n, ovf, (uint32_t)t);
    if (MODE == MODE_COUNT) {
        uint64_t total;
        block_excl_scan(hits, total, s_w);
        if (threadIdx.x == 0 && total) add_tile_total(ws, (uint64_t)blockIdx.x * WALK_BLOCK, total);
    }
}

// ------------------------------------------------------ wave per topic
//
// Small batches (latency).  One wavefront per topic: the lanes split the topic
// on '/' together (ballot over 64-byte windows), look its levels up in the
// vocab at once (lane l = level l), then walk the trie breadth first -- the
// live '+'/literal frontier of a level is one state per lane, compacted into
// LDS with ballot + prefix count, so every state of a level is one request in
// the same round trip.  Hits carry their traversal rank as a 64-bit path code
// (2 bits per level, MSB first: '#'-terminal 0 < '+' subtree 1 < literal
// subtree 2; at the topic's last level exact terminal 0 < '#'-terminal 1;
// binary key all ones), and are sorted by it before they are written: the same
// (cnt, nr, ranges) a lane walk produces, in the same order.  The "wave" is a
// group of WAVE_W lanes (16: four topics per wavefront); a topic deeper than
// the group, whose frontier outgrows it, or with more hit ranges than lanes
// goes to the lane-walk tail lists instead.
constexpr uint64_t WAVE_TOPICS = 8192;   // batches of up to this many topics take the wave-per-topic walk (latency)
constexpr int WAVE_W = 16;               // lanes per topic in the wave walk
constexpr int WV_BLOCK = 256;   // 4 waves per block
constexpr int WV_WAVES = WV_BLOCK / 64;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A group of W lanes (W = 16, 32 or 64) of a wavefront working on one topic:
// ballots, ranks and broadcasts restricted to the group.
template <int W>
struct Group {
    uint32_t g, gl;   // group within the wave, lane within the group
    __device__ __forceinline__ Group() : g((threadIdx.x & 63) / W), gl((threadIdx.x & 63) % W) {}
    __device__ __forceinline__ uint64_t ballot(bool p) const {
        const uint64_t m = __ballot(p);
        return W == 64 ? m : (m >> (g * W)) & ((1ull << (W & 63)) - 1);
    }
    __device__ __forceinline__ uint32_t rank(uint64_t gm) const {   // set bits of gm below this lane
        return (uint32_t)__popcll(gm & ((1ull << gl) - 1));
    }
    __device__ __forceinline__ uint32_t bcast(uint32_t v, uint32_t src) const {
        return (uint32_t)__shfl((int)v, (int)src, W);
    }
};

// W lanes per topic: W <= 31 levels (one level per lane; 2 code bits per level
// plus the digit at level L fit 64 bits up to 31), at most W frontier states
// and W hit ranges; anything larger goes to the lane walk's lists.
template <int MODE, int W>
__global__ __launch_bounds__(WV_BLOCK) void k_walk_wave(DevIndex ix, Workspace ws, uint64_t n,
                                                        const uint8_t *blob, const uint64_t *offs, Outs o) {
    constexpr uint32_t G = 64 / W;                        // topics per wave
    constexpr uint32_t MAXL = W < 31 ? W : 31;
    __shared__ uint32_t s_slash[WV_WAVES][64];
    __shared__ uint32_t s_node[WV_WAVES][64];
    __shared__ uint64_t s_code[WV_WAVES][64];
    __shared__ uint64_t s_hcode[WV_WAVES][64];
    __shared__ uint32_t s_hoff[WV_WAVES][64], s_hcnt[WV_WAVES][64];
    const Group<W> grp;
    const uint32_t wv = threadIdx.x >> 6, gl = grp.gl, base = grp.g * W;
    const uint64_t t = ((uint64_t)blockIdx.x * WV_WAVES + wv) * G + grp.g;
    if (t >= n) return;                       // the whole group
    uint32_t *sl_ = s_slash[wv] + base, *sn_ = s_node[wv] + base, *hoff = s_hoff[wv] + base, *hcnt = s_hcnt[wv] + base;
    uint64_t *sc_ = s_code[wv] + base, *hcode = s_hcode[wv] + base;
    const uint64_t beg = offs[t], end = offs[t + 1], len = end - beg;

    // ---- topic_words/1: level boundaries by ballot over W-byte windows
    uint32_t nsl = 0;
    for (uint64_t p = 0; p < len; p += W) {
        const bool sl = p + gl < len && blob[beg + p + gl] == '/';
        const uint64_t m = grp.ballot(sl);
        if (sl) {
            const uint32_t k = nsl + grp.rank(m);
            if (k < W) sl_[k] = (uint32_t)(p + gl);
        }
        nsl += (uint32_t)__popcll(m);
    }
    const uint32_t L = nsl + 1;
    wave_sync();
    auto to_lists = [&]() {
        if (gl == 0) {
            list_push(ws, n, tail_list(ix, L), (uint32_t)t);
        }
    };
    if (L > MAXL) { to_lists(); return; }

    // ---- this lane's level: bytes, badarg check, vocab lookup
    const bool mine = gl < L;
    const uint32_t ws0 = !mine || gl == 0 ? 0 : sl_[gl - 1] + 1;
    const uint32_t we0 = !mine ? 0 : gl == L - 1 ? (uint32_t)len : sl_[gl];
    const uint32_t wl = we0 - ws0;
    const uint8_t *wp = blob + beg + ws0;
    WordAcc w; w.reset(beg + ws0);
    if (mine) for (uint32_t i = 0; i < wl; i++) w.push(wp[i]);
    const bool bad = mine && wl == 1 && (w.b0 == '+' || w.b0 == '#');
    const bool badarg = grp.ballot(bad) != 0;
    const bool dollar = grp.bcast(mine && wl >= 1 && (w.b0 & 0xFFu) == '$' ? 1u : 0u, 0) != 0;
    uint32_t wid = mine && !badarg ? vocab_find(ix, w, GlobalSrc{blob}) : NONE;
    const bool allf = grp.ballot(mine && wid == NONE) == 0;
    uint64_t xh = FNV_OFF;
    for (uint32_t l = 0; l < L; l++) xh = seq_hash_step(xh, grp.bcast(wid, l));
    xh = seq_hash_finish(xh, L);
    const uint32_t xslot = (uint32_t)xh & ix.xmask;
    const uint32_t xf = allf && !badarg ? ix.xfp[xslot] : 0;   // in flight during the walk

    // ---- breadth-first walk: one frontier state per lane
    uint32_t nst = badarg ? 0 : 1, nh = 0;
    uint32_t node = ROOT;
    uint64_t code = 0;
    bool ovf = false;
    auto add_hits = [&](bool h, uint64_t c, uint32_t off, uint32_t cnt) {
        const uint64_t m = grp.ballot(h);
        if (h) {
            const uint32_t k = nh + grp.rank(m);
            if (k < W) { hcode[k] = c; hoff[k] = off; hcnt[k] = cnt; }
        }
        nh += (uint32_t)__popcll(m);
    };
    for (uint32_t l = 0; nst; l++) {
        const bool act = gl < nst;
        uint4 n0 = make_uint4(NONE, 0, 0, 0), n1 = make_uint4(0, 0, 0, 0), n2 = n1, n3 = n1;
        if (act) {
            const uint4 *np = reinterpret_cast<const uint4 *>(ix.nodes + node);
            n0 = np[0]; n1 = np[1]; n2 = np[2]; n3 = np[3];
        }
        pin(n0); pin(n1); pin(n2); pin(n3);
        const bool droot = dollar && l == 0;
        const uint32_t sh = 62 - 2 * l;
        if (l == L) {
            // a '#'-not-last key's cut (NLIT_HDESC) drops later hits: the lane walk's lists make it
            if (grp.ballot(act && (n1.y & NLIT_HDESC))) { to_lists(); return; }
            add_hits(act && n1.x, code, n0.w, n1.x);                              // exact terminal: digit 0
            add_hits(act && !droot && n0.z, code | (1ull << sh), n0.y, n0.z);     // '#' terminal: digit 1
            break;
        }
        add_hits(act && !droot && n0.z, code, n0.y, n0.z);                       // '#' terminal: digit 0
        const uint32_t wl_ = grp.bcast(wid, l);
        const uint32_t wnext = l + 1 < L ? grp.bcast(wid, l + 1) : NONE;
        const uint32_t wnext2 = l + 2 < L ? grp.bcast(wid, l + 2) : NONE;
        uint32_t lit = NONE;
        if (act && wl_ != NONE) {
            if ((n1.y & NLIT_MASK) <= KINL) {
                lit = n2.x == wl_ ? n3.x : n2.y == wl_ ? n3.y : n2.z == wl_ ? n3.z : n2.w == wl_ ? n3.w : NONE;
            } else {
                const uint32_t h = child_hash(wl_);
                const uint32_t mb = child_maybe(ix, n1, n2, n3, wl_, h);
                if (mb & 1u) {
                    uint32_t slo, shi;
                    lit = ctab_find(ix, n2.x, n2.y, wl_, h, slo, shi);
                    if (lit != NONE && !child_alive(slo, shi, l + 1, L, wnext, wnext2)) lit = NONE;
                }
            }
        }
        uint32_t plus = act && !droot && !(n1.y & NLIT_HDESC) ? n0.x : NONE;   // seek past '+' (dfs)
        if (plus != NONE && !child_alive(n1.z, n1.w, l + 1, L, wnext, wnext2)) plus = NONE;
        const uint64_t mp = grp.ballot(plus != NONE), ml = grp.ballot(lit != NONE);
        const uint32_t np_ = (uint32_t)__popcll(mp), nn = np_ + (uint32_t)__popcll(ml);
        if (nn > W) { ovf = true; break; }
        wave_sync();   // every lane has read its state before the slots are reused
        if (plus != NONE) { const uint32_t k = grp.rank(mp); sn_[k] = plus; sc_[k] = code | (1ull << sh); }
        if (lit != NONE) { const uint32_t k = np_ + grp.rank(ml); sn_[k] = lit; sc_[k] = code | (2ull << sh); }
        wave_sync();
        nst = nn;
        if (gl < nst) { node = sn_[gl]; code = sc_[gl]; }
    }

    // ---- match_topics/4: the binary key equal to the topic, after every list key
    if (!ovf && allf && !badarg) {
        uint32_t slot = xslot, f = xf, xoff = 0, xcnt = 0;
        const uint32_t fp = exact_fp(xh);
        for (;;) {
            if (f == 0) break;
            if (f == fp) {
                const uint32_t *e = reinterpret_cast<const uint32_t *>(ix.exact + slot);
                const bool keyok = e[0] == (uint32_t)xh && e[1] == (uint32_t)(xh >> 32) && e[2] == L;
                if (keyok) {
                    const uint32_t ew = !mine ? wid : L <= XINL ? e[6 + gl] : ix.wseq[e[5] + gl];
                    if (grp.ballot(mine && ew != wid) == 0) { xoff = e[3]; xcnt = e[4]; break; }
                }
            }
            slot = (slot + 1) & ix.xmask;
            f = ix.xfp[slot];
        }
        add_hits(gl == 0 && xcnt, ~0ull, xoff, xcnt);
    }
    if (ovf || nh > W) { to_lists(); return; }

    // ---- rank the hits by path code (traversal order) and write them out
    wave_sync();
    const bool hv = gl < nh;
    const uint64_t my = hv ? hcode[gl] : 0;
    uint32_t rank = 0, total = 0;
    for (uint32_t j = 0; j < nh; j++) {
        rank += hcode[j] < my;
        total += hcnt[j] & RUN_CNT;
    }
    if (MODE == MODE_COUNT) {
        if (hv && rank < RCAP) ws.rng[(uint64_t)rank * n + t] = make_uint2(hoff[gl], hcnt[gl]);
        if (gl == 0) {
            ws.cnt[t] = total;
            ws.nr[t] = nh;
            o.err[t] = badarg;
            if (total) add_tile_total(ws, t, total);
            if (nh > RCAP) list_push(ws, n, L_OVF_MID, (uint32_t)t);
        }
    } else {
        if (hv && rank == 0) o.first_val[t] = (hcnt[gl] & RUN_INLINE) ? hoff[gl] : ix.vals[hoff[gl]];
        if (gl == 0) {
            if (!nh) o.first_val[t] = 0;
            o.first_found[t] = badarg ? 2 : (nh ? 1 : 0);
        }
    }
}

// ------------------------------------------- small batches in one launch
//
// A batch of <= SMALL_TOPICS topics is latency: its walk, scan and emit as
// separate kernels (k_walk_wave, the tail kernels, k_emit) cost ~4 launches
// of mostly idle grids.  k_walk_small does all of it in one: each group of W
// lanes walks its topic as k_walk_wave does; a topic the group cannot take
// (deeper than the group, a frontier or hit list wider than it, a
// '#'-not-last cut) is walked by the group's first lane with an LDS store of
// MID_L levels (small_path_ok: the index never needs more); the block's 16
// hit counts get their global offset from a single-pass decoupled look-back
// scan over the blocks in dispatch order (a block only ever waits for blocks
// already running); then each group puts its values in
// the block's LDS span, written out as one contiguous run (or, for a block
// whose values do not fit or that holds a lane-walked topic, straight into the
// CSR).  The caller's buffers may be host memory (in-place host batches): the
// block reads its offsets and its whole topic byte span once each, and writes
// its offsets, flags and values as contiguous runs -- a few whole PCIe
// transactions per block instead of several per topic.  No range lists, no
// device-side lists, no other kernel.
struct CountEmit {          // one-launch path: hit count only (the values come from a re-walk)
    uint64_t cnt;
    __device__ __forceinline__ bool operator()(uint32_t, uint32_t n) { cnt += n & RUN_CNT; return true; }
};

// Batches of up to SMALL_TOPICS topics take the one-launch path.  Up to 8192
// topics it replaced the wave walk + tails + emit; up to 64k it also beats the
// lane walk's five kernels, because it writes each block's values while the
// other blocks still walk (C3, host-to-host p50, in place: 16k topics 0.112
// -> 0.075 ms, 32k 0.173 -> 0.111, 64k 0.208 -> 0.189; profiles/r3/sm64k/).
constexpr uint64_t SMALL_TOPICS = 65536;

// the one-launch kernels' fallback store resolves need_levels() (+2 look-ahead
// levels) within MID_L for every topic of this index
bool one_launch_ok(const DevIndex &ix) {
    return ix.depth + 2 <= (uint32_t)MID_L && ix.xlen_max + 2 <= (uint32_t)MID_L;
}

bool small_path_ok(const DevIndex &ix, uint64_t n) { return n && n <= SMALL_TOPICS && one_launch_ok(ix); }

// OT: the offsets' type, in and out -- uint64_t (tm_match_batch*), or uint32_t
// (tm_match_batch32*: half the offset bytes of an in-place host batch cross
// PCIe in each direction)
// sg.count > 0 (count mode): the launch carries several host batches
// (SmallSegs); each block finds its segment and works on it as a launch of
// that batch alone would -- its own block index, look-back region and last block.
// W: lanes per topic -- 16 (four topics per wave), or 8 (eight: twice the
// topics per wave slot for concurrent callers, whose launches together fill
// every slot of the GPU; levels and frontier states per topic <= 8, else the
// lane walk).  A group keeps up to HC hit ranges (C3: 8.4 per topic).
// LITE: the fallback lane walk's store holds FAST_L levels and resolves only
// need_levels() (lite_path_ok indexes: shallow, no
// '#'-not-last key) instead of MID_L: 76 instead of 292 B of LDS per topic.
template <int W>
struct SmallShape {
    static constexpr uint32_t G = 64 / W;                          // topics per wave
    static constexpr uint32_t ST = WV_WAVES * G;                   // topics per block
    static constexpr uint32_t MAXL = W < 31 ? W : 31;              // levels a group takes
    static constexpr uint32_t HC = W < 16 ? 16 : W;                // hit ranges a group keeps
    static constexpr uint32_t TBQ = (W >= 16 ? SM_TB : SM_TB / 2) / 16 + 1;   // 16-B chunks of a topic staged
};
static_assert(SmallShape<16>::ST == SM_TOPICS, "SM_TOPICS: the most blocks a small batch launches per topic");

template <int MODE, class OT, int W, bool LITE>
__global__ __launch_bounds__(WV_BLOCK) void k_walk_small(DevIndex ix, Workspace ws, uint64_t n_, const uint8_t *blob_,
                                                         const OT *offs_, Outs o, OT *hit_offs_,
                                                         uint32_t *out_, uint64_t cap_, uint32_t tag, LbCtl lb,
                                                         SmallSegs sg) {
    uint64_t n = n_, cap = cap_;
    const uint8_t *blob = blob_;
    const OT *offs = offs_;
    OT *hit_offs = hit_offs_;
    uint32_t *out = out_;
    uint32_t vb = blockIdx.x, nblk = gridDim.x, sb0 = 0;   // sb0: the segment's first block
    uint32_t k = 0;   // the segment
    if (MODE == MODE_COUNT && sg.count) {
        while (k + 1 < sg.count && blockIdx.x >= sg.s[k + 1].block0) k++;
        const SmallSeg &S = sg.s[k];
        n = S.n; cap = S.cap; blob = S.blob;
        offs = static_cast<const OT *>(S.offs);
        hit_offs = static_cast<OT *>(S.hit);
        out = S.out; o.err = S.err;
        sb0 = S.block0;
        nblk = (k + 1 < sg.count ? sg.s[k + 1].block0 : gridDim.x) - sb0;
        vb = blockIdx.x - sb0;
    }
    if (MODE == MODE_COUNT && lb.ticket) {
        // start-order ticket (include/tmatch.h "Forward progress"): the block
        // takes the segment's next virtual index, so every block it may wait
        // for in the look-back below has started; the segment's last ticket
        // resets the word for the next launch on this workspace
        __shared__ uint32_t s_tk;
        if (threadIdx.x == 0) {
            const uint32_t tk = atomicAdd(&ws.list_n[SM_TICK + k], 1u);
            if (tk == nblk - 1) atomicExch(&ws.list_n[SM_TICK + k], 0u);
            s_tk = tk;
        }
        __syncthreads();
        vb = s_tk;
    }
    using SH = SmallShape<W>;
    constexpr uint32_t G = SH::G, ST = SH::ST, MAXL = SH::MAXL, HC = SH::HC;
    __shared__ uint32_t s_slash[WV_WAVES][64];
    __shared__ uint32_t s_node[WV_WAVES][64];
    __shared__ uint64_t s_code[WV_WAVES][64];
    // a group's hits (path code, value run) -- by rank once they are ranked
    // (then the code's slot holds the hit's first output position)
    __shared__ uint64_t s_hcode[WV_WAVES][G * HC];
    __shared__ uint32_t s_hoff[WV_WAVES][G * HC], s_hcnt[WV_WAVES][G * HC];
    constexpr uint32_t FBL = LITE ? FAST_L : MID_L;       // levels of the fallback lane walk's store
    using FbStore = LdsStore<FBL, LITE>;
    __shared__ uint32_t s_mwid[ST][FBL], s_mpend[ST][FBL + 1];   // fallback lane-walk stores
    __shared__ uint8_t s_mlen[ST][FBL];
    __shared__ uint64_t s_cnt[ST];
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_fail;
    constexpr uint32_t TBQ = SH::TBQ;                     // 16-B chunks of a topic staged in LDS
    constexpr uint32_t TBQ_ALL = ST * TBQ;
    // topic bytes in LDS: the block's whole byte span in one cooperative round
    // of 16-B loads when it fits (each chunk read once -- consecutive topics
    // share the chunk at their boundary), else one row per topic
    __shared__ uint4 s_tb[TBQ_ALL];
    __shared__ uint64_t s_off[ST + 1];
    __shared__ uint8_t s_err[ST], s_fbk[ST];
    // the block's values staged in LDS and written as one contiguous span
    // (in place batches: a few whole PCIe writes instead of one per group)
    __shared__ uint32_t s_vals[SM_VSTAGE];
    __shared__ uint64_t s_sum;
    // blocks scan in blockIdx order (workgroups are dispatched in that order),
    // or in start order with lb.ticket (include/tmatch.h "Forward progress")
    // the block's ST + 1 topic offsets, read once by one wave (the caller's
    // buffers may be host memory: one coalesced read, not one per group)
    if (threadIdx.x <= ST && (uint64_t)vb * ST + threadIdx.x <= n)
        s_off[threadIdx.x] = offs[(uint64_t)vb * ST + threadIdx.x];
    __syncthreads();
    const Group<W> grp;
    const uint32_t wv = threadIdx.x >> 6, gl = grp.gl, base = grp.g * W;
    const uint32_t gi = wv * G + grp.g;                   // topic slot in the block
    const uint64_t t = (uint64_t)vb * ST + gi;
    const bool live = t < n;
    const uint32_t hbase = grp.g * HC;
    uint32_t *sl_ = s_slash[wv] + base, *sn_ = s_node[wv] + base, *hoff = s_hoff[wv] + hbase, *hcnt = s_hcnt[wv] + hbase;
    uint64_t *sc_ = s_code[wv] + base, *hcode = s_hcode[wv] + hbase;
    const uint64_t beg = live ? s_off[gi] : 0, end = live ? s_off[gi + 1] : 0, len = end - beg;

    // ---- the topic into LDS: one round of 16-B loads by the group's lanes
    // (the caller's buffers may be host memory read over PCIe: every byte
    // read from there would be a round trip).  Aligned chunks share their
    // granule with a valid byte, so they never touch a page the caller does
    // not own.  A topic longer than its row (TBQ chunks) goes to the lane walk.
    const uint64_t a0 = beg & ~15ull;
    const uint32_t nq = live ? (uint32_t)((end - a0 + 15) >> 4) : 0;
    bool fb = nq > TBQ;   // the group's first lane walks this topic (lane walk, global reads)
    const uint32_t nt = (uint64_t)vb * ST + ST <= n ? ST : (uint32_t)(n - (uint64_t)vb * ST);
    const uint64_t B0 = s_off[0] & ~15ull;
    const uint64_t nqb = (s_off[nt] - B0 + 15) >> 4;
    const bool span = nqb <= TBQ_ALL;                     // (block-uniform)
    if (span) {
        for (uint32_t c = threadIdx.x; c < nqb; c += WV_BLOCK) s_tb[c] = ld4_once(blob + B0 + 16ull * c);
        __syncthreads();
    } else {
        if (!fb)
            for (uint32_t c = gl; c < nq; c += W) s_tb[gi * TBQ + c] = ld4_once(blob + a0 + 16ull * c);
        wave_sync();
    }
    const uint8_t *tb = span ? reinterpret_cast<const uint8_t *>(s_tb) + (live ? beg - B0 : 0)   // topic byte i = tb[i]
                             : reinterpret_cast<const uint8_t *>(s_tb + gi * TBQ) + (beg - a0);
    const uint64_t tlen = fb ? 0 : len;

    // ---- the wave walk (k_walk_wave), falling back instead of listing
    uint32_t nsl = 0;
    for (uint64_t p = 0; p < tlen; p += W) {
        const bool sl = p + gl < tlen && tb[p + gl] == '/';
        const uint64_t m = grp.ballot(sl);
        if (sl) {
            const uint32_t k = nsl + grp.rank(m);
            if (k < W) sl_[k] = (uint32_t)(p + gl);
        }
        nsl += (uint32_t)__popcll(m);
    }
    const uint32_t L = nsl + 1;
    wave_sync();
    fb = live && (fb || L > MAXL);
    const bool mine = live && !fb && gl < L;
    const uint32_t ws0 = !mine || gl == 0 ? 0 : sl_[gl - 1] + 1;
    const uint32_t we0 = !mine ? 0 : gl == L - 1 ? (uint32_t)len : sl_[gl];
    const uint32_t wl = we0 - ws0;
    const uint8_t *wp = tb + ws0;
    WordAcc w; w.reset(ws0);
    if (mine) for (uint32_t i = 0; i < wl; i++) w.push(wp[i]);
    const bool bad = mine && wl == 1 && (w.b0 == '+' || w.b0 == '#');
    const bool badarg = grp.ballot(bad) != 0;
    const bool dollar = grp.bcast(mine && wl >= 1 && (w.b0 & 0xFFu) == '$' ? 1u : 0u, 0) != 0;
    uint32_t wid = mine && !badarg ? vocab_find(ix, w, GlobalSrc{tb}) : NONE;   // (long words: bytes from LDS)
    const bool allf = grp.ballot(mine && wid == NONE) == 0;
    uint64_t xh = FNV_OFF;
    for (uint32_t l = 0; l < L && !fb; l++) xh = seq_hash_step(xh, grp.bcast(wid, l));
    xh = seq_hash_finish(xh, L);
    const uint32_t xslot = (uint32_t)xh & ix.xmask;
    const uint32_t xf = live && !fb && allf && !badarg ? ix.xfp[xslot] : 0;   // in flight during the walk

    uint32_t nst = live && !fb && !badarg ? 1 : 0, nh = 0;
    uint32_t node = ROOT;
    uint64_t code = 0;
    auto add_hits = [&](bool h, uint64_t c, uint32_t off, uint32_t cnt) {
        const uint64_t m = grp.ballot(h);
        if (h) {
            const uint32_t k = nh + grp.rank(m);
            if (k < HC) { hcode[k] = c; hoff[k] = off; hcnt[k] = cnt; }
        }
        nh += (uint32_t)__popcll(m);
    };
    for (uint32_t l = 0; nst; l++) {
        const bool act = gl < nst;
        uint4 n0 = make_uint4(NONE, 0, 0, 0), n1 = make_uint4(0, 0, 0, 0), n2 = n1, n3 = n1;
        if (act) {
            const uint4 *np = reinterpret_cast<const uint4 *>(ix.nodes + node);
            n0 = np[0]; n1 = np[1]; n2 = np[2]; n3 = np[3];
        }
        pin(n0); pin(n1); pin(n2); pin(n3);
        const bool droot = dollar && l == 0;
        const uint32_t sh = 62 - 2 * l;
        if (l == L) {
            if (grp.ballot(act && (n1.y & NLIT_HDESC))) { fb = true; break; }   // the cut: the lane walk makes it
            add_hits(act && n1.x, code, n0.w, n1.x);                              // exact terminal: digit 0
            add_hits(act && !droot && n0.z, code | (1ull << sh), n0.y, n0.z);     // '#' terminal: digit 1
            break;
        }
        add_hits(act && !droot && n0.z, code, n0.y, n0.z);                       // '#' terminal: digit 0
        const uint32_t wl_ = grp.bcast(wid, l);
        const uint32_t wnext = l + 1 < L ? grp.bcast(wid, l + 1) : NONE;
        const uint32_t wnext2 = l + 2 < L ? grp.bcast(wid, l + 2) : NONE;
        uint32_t lit = NONE;
        if (act && wl_ != NONE) {
            if ((n1.y & NLIT_MASK) <= KINL) {
                lit = n2.x == wl_ ? n3.x : n2.y == wl_ ? n3.y : n2.z == wl_ ? n3.z : n2.w == wl_ ? n3.w : NONE;
            } else {
                const uint32_t h = child_hash(wl_);
                // a wide node's bitmap line would be one more round trip before
                // the probe: at a small batch's load the probe itself is cheaper
                const uint32_t mb = (n1.y & NLIT_MASK) >= WIDE_LIT ? 1u : child_maybe(ix, n1, n2, n3, wl_, h);
                if (mb & 1u) {
                    uint32_t slo, shi;
                    lit = ctab_find(ix, n2.x, n2.y, wl_, h, slo, shi);
                    if (lit != NONE && !child_alive(slo, shi, l + 1, L, wnext, wnext2)) lit = NONE;
                }
            }
        }
        uint32_t plus = act && !droot && !(n1.y & NLIT_HDESC) ? n0.x : NONE;   // seek past '+' (dfs)
        if (plus != NONE && !child_alive(n1.z, n1.w, l + 1, L, wnext, wnext2)) plus = NONE;
        const uint64_t mp = grp.ballot(plus != NONE), ml = grp.ballot(lit != NONE);
        const uint32_t np_ = (uint32_t)__popcll(mp), nn = np_ + (uint32_t)__popcll(ml);
        if (nn > W) { fb = true; break; }
        wave_sync();   // every lane has read its state before the slots are reused
        if (plus != NONE) { const uint32_t k = grp.rank(mp); sn_[k] = plus; sc_[k] = code | (1ull << sh); }
        if (lit != NONE) { const uint32_t k = np_ + grp.rank(ml); sn_[k] = lit; sc_[k] = code | (2ull << sh); }
        wave_sync();
        nst = nn;
        if (gl < nst) { node = sn_[gl]; code = sc_[gl]; }
    }
    // ---- match_topics/4: the binary key equal to the topic, after every list key
    if (live && !fb && allf && !badarg) {
        uint32_t slot = xslot, f = xf, xoff = 0, xcnt = 0;
        const uint32_t fp = exact_fp(xh);
        for (;;) {
            if (f == 0) break;
            if (f == fp) {
                const uint32_t *e = reinterpret_cast<const uint32_t *>(ix.exact + slot);
                const bool keyok = e[0] == (uint32_t)xh && e[1] == (uint32_t)(xh >> 32) && e[2] == L;
                if (keyok) {
                    const uint32_t ew = !mine ? wid : L <= XINL ? e[6 + gl] : ix.wseq[e[5] + gl];
                    if (grp.ballot(mine && ew != wid) == 0) { xoff = e[3]; xcnt = e[4]; break; }
                }
            }
            slot = (slot + 1) & ix.xmask;
            f = ix.xfp[slot];
        }
        add_hits(gl == 0 && xcnt, ~0ull, xoff, xcnt);
    }
    fb |= live && nh > HC;

    // ---- the hits' total (every lane); their ranks by path code below
    wave_sync();
    uint64_t total = 0;
    if (live && !fb)
        for (uint32_t j = 0; j < nh; j++) total += hcnt[j] & RUN_CNT;

    // ---- topics the group could not take: its first lane walks them (LDS store of FBL levels)
    FbStore st{s_mwid[gi], s_mpend[gi], s_mlen[gi], 1, 0};
    // its bytes from the LDS copy above (the block's span, or the topic's row),
    // not from the caller's buffer: for an in-place batch every byte the walk
    // read from there was a PCIe round trip on the launch's critical path (the
    // block's count waits for it, and every later block for the block's count)
    const StagedSrc fsrc{blob, span ? s_tb : s_tb + gi * TBQ, span ? B0 : a0, span || nq <= TBQ};
    int frc = RC_OK;
    const bool walker = fb && gl == 0;
    if (walker) {
        if (MODE == MODE_COUNT) {
            CountEmit em{0};
            frc = match_topic(ix, fsrc, beg, end, st, em);
            total = frc == RC_OK ? em.cnt : 0;
        } else {
            FirstEmit em{ix.vals, 0, false};
            frc = match_topic(ix, fsrc, beg, end, st, em);
            o.first_val[t] = frc == RC_OK ? em.v : 0;
            o.first_found[t] = frc == RC_BADARG ? 2 : frc == RC_DEEP ? 3 : (em.found ? 1 : 0);
        }
    }
    if (MODE == MODE_FIRST) {
        if (live && !fb) {
            for (uint32_t h = gl; h < nh; h += W) {   // the hit ranked first
                uint32_t rank = 0;
                for (uint32_t j = 0; j < nh; j++) rank += hcode[j] < hcode[h];
                if (!rank) o.first_val[t] = (hcnt[h] & RUN_INLINE) ? hoff[h] : ix.vals[hoff[h]];
            }
            if (gl == 0) {
                if (!nh) o.first_val[t] = 0;
                o.first_found[t] = badarg ? 2 : (nh ? 1 : 0);
            }
        }
        return;
    }

    // ---- the block's offset: exclusive scan of its ST counts + decoupled look-back
    if (gl == 0) {
        s_cnt[gi] = live ? total : 0;
        s_err[gi] = fb ? (frc == RC_BADARG ? 1 : frc == RC_DEEP ? 2 : 0) : badarg;
        s_fbk[gi] = live && fb;
    }
    __syncthreads();
    if (wv == 0 && sg.pairs) {
        // (offset, count) pairs (tm_match_batch32_pairs): the block reserves
        // its values' span with ONE atomic on the segment's counter and never
        // waits for another block -- no look-back, so a finished block frees
        // its slot at once for the other callers' launches; the segment's
        // last block (a ticket taken after its reservation returned) writes
        // the total and resets both words for the next launch
        if (threadIdx.x == 0) {
            uint64_t sum = 0;
            for (uint32_t i = 0; i < ST; i++) sum += s_cnt[i];
            s_base = atomicAdd(&ws.pairs[2 * k], (uint32_t)sum);
            s_sum = sum;
            s_fail = 0;
            if (atomicAdd(&ws.pairs[2 * k + 1], 1u) == nblk - 1) {
                hit_offs[2 * n] = (OT)__hip_atomic_load(&ws.pairs[2 * k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicExch(&ws.pairs[2 * k], 0u);
                atomicExch(&ws.pairs[2 * k + 1], 0u);
            }
        }
    } else if (wv == 0) {
        uint64_t sum = 0;
        for (uint32_t i = 0; i < ST; i++) sum += s_cnt[i];
        // one flag round trip per 64 predecessors (look_back); a failed wait
        // fails this block and every later one: err 4, the fail word raised
        int res;
        const uint64_t pre = look_back(ws.look + (uint64_t)sb0 * LB_STRIDE, vb, tag, sum, lb, res);
        const bool fail = res != LBR_OK;
        if (threadIdx.x == 0) {
            s_fail = fail;
            s_sum = sum;
            s_base = pre;
            if (fail) ws.hint_d[HINT_FAIL] = 1;
            if (vb == nblk - 1 && !fail) hit_offs[n] = (OT)(pre + sum);
        }
    }
    __syncthreads();
    // the block's hit offsets (pairs: first position and count) and flags:
    // lanes 0..ST-1 of wave 0, one coalesced store each
    if (threadIdx.x < ST && (uint64_t)vb * ST + threadIdx.x < n) {
        uint64_t p = s_base;
        for (uint32_t i = 0; i < threadIdx.x; i++) p += s_cnt[i];
        const uint64_t t_ = (uint64_t)vb * ST + threadIdx.x;
        if (sg.pairs) {
            hit_offs[2 * t_] = (OT)p;
            hit_offs[2 * t_ + 1] = (OT)s_cnt[threadIdx.x];
        } else {
            hit_offs[t_] = (OT)p;
        }
        o.err[t_] = s_fail ? 4 : s_err[threadIdx.x];
    }
    if (s_fail) return;   // (block-uniform)
    // stage the block's values in LDS when they fit and no topic of the block
    // took the lane walk (which writes its values itself)
    bool stage = s_sum <= SM_VSTAGE;
    for (uint32_t i = 0; i < ST; i++) stage &= !s_fbk[i];
    const uint64_t b0 = s_base;
    uint64_t pos = b0;
    for (uint32_t i = 0; i < gi; i++) pos += s_cnt[i];
    auto put = [&](uint64_t P, uint32_t v) {
        if (stage) s_vals[P - b0] = v;
        else if (P < cap) out[P] = v;
    };

    // ---- the values
    if (walker && frc == RC_OK) {   // (never with stage)
        DirectEmit em{ix.vals, out, pos, cap};
        match_topic(ix, fsrc, beg, end, st, em);
    }
    if (live && !fb) {
        // each lane ranks its hits (HC / W of them) in registers, then writes
        // them back in rank order: run in hoff / hcnt, first position in hcode
        constexpr uint32_t HPL = HC / W;
        uint32_t rk[HPL], ro[HPL], rc[HPL];
        uint64_t rp[HPL];
#pragma unroll
        for (uint32_t q = 0; q < HPL; q++) {
            const uint32_t h = gl + q * W;
            rk[q] = NONE; ro[q] = rc[q] = 0; rp[q] = 0;
            if (h < nh) {
                const uint64_t my = hcode[h];
                uint32_t rank = 0;
                uint64_t before = 0;   // values of the hits ranked before this one
                for (uint32_t j = 0; j < nh; j++)
                    if (hcode[j] < my) { rank++; before += hcnt[j] & RUN_CNT; }
                rk[q] = rank; ro[q] = hoff[h]; rc[q] = hcnt[h]; rp[q] = pos + before;
            }
        }
        wave_sync();   // every hit read before the slots take them by rank
#pragma unroll
        for (uint32_t q = 0; q < HPL; q++)
            if (rk[q] != NONE) { hoff[rk[q]] = ro[q]; hcnt[rk[q]] = rc[q]; hcode[rk[q]] = rp[q]; }
        const uint32_t *roff = hoff, *rcnt = hcnt;
        const uint64_t *rpos = hcode;
        wave_sync();
        // single-value runs (C3: almost every hit): lane r writes the one ranked r
        for (uint32_t r = gl; r < nh; r += W)
            if (rcnt[r] & RUN_INLINE) put(rpos[r], roff[r]);
        for (uint32_t r = 0; r < nh; r++) {
            const uint32_t ro = roff[r], rc = rcnt[r];
            const uint64_t P = rpos[r];
            if (rc & RUN_INLINE) continue;
            for (uint32_t k = gl; k < (rc & RUN_CNT); k += W) put(P + k, ix.vals[ro + k]);
        }
    }
    if (stage) {   // (block-uniform)
        __syncthreads();
        const uint32_t m = (uint32_t)s_sum;
        for (uint32_t i = threadIdx.x; i < m; i += WV_BLOCK)
            if (b0 + i < cap) out[b0 + i] = s_vals[i];
    }
}

constexpr int MID_BLOCK = 64;
constexpr int MID_GRID = 512;                         // LDS-frontier blocks of the tail kernels (at most)
// k_walk_tail of a large count-mode batch: more LDS-frontier blocks (it takes
// no grid-wide ticket then, so idle blocks cost only their dispatch).  512
// blocks = 2 waves per CU: C3deep (100k topics of 33-64 levels per 1M batch)
// spent 0.57 ms per batch in the tail; 2048: 0.25 ms
constexpr int MID_GRID_BIG = 2048;
constexpr int MID_GRID_MIN = 32;

// LDS-frontier blocks for a tail list: one lane per topic the list held in the
// last count-mode batch on this workspace (scaled to this batch, x2 + 2048
// topics of slack), between MID_GRID_MIN and `most`.  Idle blocks are not
// free when other streams' walks fill the GPU: each waits for a workgroup
// slot, so a 2049-block tail kernel took 110 us per C3 batch with three
// streams (4 us alone); any grid is correct (the lists are walked grid-stride).
static uint32_t tail_blocks(const Workspace &ws, uint64_t n, int list, uint32_t most) {
    if (!ws.hint_h) return most;
    const volatile uint32_t *h = ws.hint_h;
    const uint32_t hn = h[L_COUNT];
    if (!hn) return most;   // no count-mode batch has finished here yet
    const double want = 2.0 * (double)h[list] * (double)n / (double)hn + 2048.0;
    const double b = want / MID_BLOCK;
    return b >= most ? most : (b <= MID_GRID_MIN ? (uint32_t)MID_GRID_MIN : (uint32_t)b);
}

// last block of a grid (atomic ticket) resets the list counters for the next
// batch; hint_n != 0 (the count-mode batch's last kernel): it also leaves the
// list lengths and hint_n in the workspace's mapped hint words (tail_blocks)
// (no fence: a block only READ the list counters, and those loads completed
// before its ticket was taken, so the reset cannot overtake them)
__device__ __forceinline__ void reset_lists_if_last(const Workspace &ws, uint32_t hint_n = 0) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t ticket = atomicAdd(&ws.list_n[L_COUNT], 1u);
        if (ticket == gridDim.x - 1) {
            for (int k = 0; k < L_COUNT; k++) {
                const uint32_t len = atomicExch(&ws.list_n[k], 0u);
                if (hint_n && ws.hint_d) ws.hint_d[k] = len;
            }
            if (hint_n && ws.hint_d) ws.hint_d[L_COUNT] = hint_n;
            atomicExch(&ws.list_n[L_COUNT], 0u);
        }
    }
}

// topics deeper than FAST_L: blocks < MID_GRID take the MID list (LDS frontier,
// <= MID_L levels), the rest take the DEEP list (global scratch, any depth)
template <int MODE>
__global__ __launch_bounds__(MID_BLOCK) void k_walk_tail(DevIndex ix, Workspace ws, uint64_t n,
                                                         const uint8_t *blob, const uint64_t *offs, Outs o,
                                                         uint32_t mid_grid) {
    __shared__ uint32_t s_wid[MID_L * MID_BLOCK];
    __shared__ uint32_t s_pend[(MID_L + 1) * MID_BLOCK];
    __shared__ uint8_t s_len[MID_L * MID_BLOCK];
    uint32_t hits = 0;
    if (blockIdx.x < mid_grid) {
        const uint32_t cnt = ws.list_n[L_MID];
        const uint32_t *lst = ws.lists + (uint64_t)L_MID * n;
        LdsStore<MID_L> st{s_wid + threadIdx.x, s_pend + threadIdx.x, s_len + threadIdx.x, MID_BLOCK, 0};
        for (uint32_t i = blockIdx.x * MID_BLOCK + threadIdx.x; i < cnt; i += mid_grid * MID_BLOCK) {
            run_topic<MODE>(ix, ws, n, blob, offs, lst[i], st, o, &hits);
            if (MODE == MODE_COUNT && hits) add_tile_total(ws, lst[i], hits);
        }
    } else {
        const uint32_t lane = (blockIdx.x - mid_grid) * 64 + threadIdx.x;   // < DEEP_LANES
        const uint32_t cnt = ws.list_n[L_DEEP];
        const uint32_t *lst = ws.lists + (uint64_t)L_DEEP * n;
        GlobalStore st{ws.deep_wid + (uint64_t)lane * MAX_LEVELS, ws.deep_stk + (uint64_t)lane * (MAX_LEVELS + 1),
                       ws.deep_plus + (uint64_t)lane * MAX_LEVELS, 0};
        for (uint32_t i = lane; i < cnt; i += DEEP_LANES) {
            run_topic<MODE>(ix, ws, n, blob, offs, lst[i], st, o, &hits);
            if (MODE == MODE_COUNT && hits) add_tile_total(ws, lst[i], hits);
        }
    }
    if (MODE == MODE_FIRST) reset_lists_if_last(ws);   // count mode: k_rewalk_tail resets
    if (MODE == MODE_COUNT) {
        // the grid's last block: the superblock totals from the (now final)
        // tile totals.  The tile totals are written only by device-scope
        // atomics, which are performed coherently across the XCDs: each block
        // drains its own (s_waitcnt) before its ticket, and the last block
        // reads them with agent-scope (sc1) loads -- no L2 write-back per
        // block (an agent-scope release, __threadfence, in every block cost
        // C3deep's tail 68 us: 159 -> 227 us, profiles/r5/scan/).
        __shared__ uint32_t s_last;
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (threadIdx.x == 0) s_last = atomicAdd(&ws.list_n[L_COUNT + 1], 1u) == gridDim.x - 1;
        __syncthreads();
        if (!s_last) return;
        const uint64_t nb = (n + TILE - 1) / TILE, ns = (nb + SUP - 1) / SUP;
        for (uint64_t sb = threadIdx.x; sb < ns; sb += MID_BLOCK) {   // a lane per superblock
            const uint64_t t0 = sb * SUP, t1 = t0 + SUP < nb ? t0 + SUP : nb;
            uint64_t v = 0;
#pragma unroll 1
            for (uint64_t c = t0; c < t1; c += 8) {   // 8 loads in flight
                uint64_t x[8];
#pragma unroll
                for (int i = 0; i < 8; i++)
                    x[i] = c + i < t1 ? __hip_atomic_load(&ws.blk[c + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#pragma unroll
                for (int i = 0; i < 8; i++) v += x[i];
            }
            ws.sup[sb] = v;
        }
        if (threadIdx.x == 0) atomicExch(&ws.list_n[L_COUNT + 1], 0u);
    }
}

// re-walk of topics with more than RCAP hit ranges: values go straight to the CSR
template <class S>
__device__ void rewalk(const DevIndex &ix, const uint8_t *blob, const uint64_t *offs, uint64_t t,
                       const uint64_t *hit_offs, uint32_t *out, uint64_t cap, S &st) {
    DirectEmit em{ix.vals, out, hit_offs[t], cap};
    match_topic(ix, GlobalSrc{blob}, offs[t], offs[t + 1], st, em);
}

__global__ __launch_bounds__(MID_BLOCK) void k_rewalk_tail(DevIndex ix, Workspace ws, uint64_t n, const uint8_t *blob,
                                                           const uint64_t *offs, const uint64_t *hit_offs,
                                                           uint32_t *out, uint64_t cap, uint32_t mid_grid) {
    __shared__ uint32_t s_wid[MID_L * MID_BLOCK];
    __shared__ uint32_t s_pend[(MID_L + 1) * MID_BLOCK];
    __shared__ uint8_t s_len[MID_L * MID_BLOCK];
    {   // every k_emit block has read the totals: zero them for the next batch
        const uint64_t nb = (n + TILE - 1) / TILE, ns = (nb + SUP - 1) / SUP;
        for (uint64_t i = (uint64_t)blockIdx.x * MID_BLOCK + threadIdx.x; i < nb + ns; i += (uint64_t)gridDim.x * MID_BLOCK)
            if (i < nb) ws.blk[i] = 0; else ws.sup[i - nb] = 0;
    }
    if (blockIdx.x < mid_grid) {
        const uint32_t cnt = ws.list_n[L_OVF_MID];
        const uint32_t *lst = ws.lists + (uint64_t)L_OVF_MID * n;
        LdsStore<MID_L> st{s_wid + threadIdx.x, s_pend + threadIdx.x, s_len + threadIdx.x, MID_BLOCK, 0};
        for (uint32_t i = blockIdx.x * MID_BLOCK + threadIdx.x; i < cnt; i += mid_grid * MID_BLOCK)
            rewalk(ix, blob, offs, lst[i], hit_offs, out, cap, st);
    } else {
        const uint32_t lane = (blockIdx.x - mid_grid) * 64 + threadIdx.x;
        const uint32_t cnt = ws.list_n[L_OVF_DEEP];
        const uint32_t *lst = ws.lists + (uint64_t)L_OVF_DEEP * n;
        GlobalStore st{ws.deep_wid + (uint64_t)lane * MAX_LEVELS, ws.deep_stk + (uint64_t)lane * (MAX_LEVELS + 1),
                       ws.deep_plus + (uint64_t)lane * MAX_LEVELS, 0};
        for (uint32_t i = lane; i < cnt; i += DEEP_LANES)
            rewalk(ix, blob, offs, lst[i], hit_offs, out, cap, st);
    }
    reset_lists_if_last(ws, n < 0xFFFFFFFFull ? (uint32_t)n : 0xFFFFFFFFu);
}

// ------------------------------------------------------------------- emit

constexpr int EMIT_BLOCK = TILE;
constexpr int EMIT_WAVES = EMIT_BLOCK / 64;
constexpr int WR = 64 * RCAP;   // ranges per wave
typedef uint4 __attribute__((aligned(4))) uint4u;   // dword-aligned 16-B load (global_load_dwordx4)
constexpr int EMIT_Q = 1;   // quads per lane per iteration (loads in flight before the stores)
constexpr uint64_t EMIT_RUNS = 16;   // average run length from which a wave copies run by run
constexpr uint8_t RF_INLINE = 1, RF_SKIP = 2;   // s_flg: a one-value run kept inline / an overflowed topic's positions

// One wave writes the values of R ranges flattened in LDS into out[base, endp):
// s_off = the range's value offset (RF_INLINE: the value itself), s_rel = its
// first position relative to base (s_rel[R] = endp - base), s_flg (RF_SKIP: a
// re-walked topic's positions, written by its re-walk).  k_emit's inner copy
// (ranges read back from the walk's range lists).
__device__ __forceinline__ void wave_emit(const DevIndex &ix, const uint32_t *s_off, const uint32_t *s_rel,
                                          const uint8_t *s_flg, uint32_t R, uint64_t base, uint64_t endp,
                                          uint32_t *out, uint64_t cap) {
    const int lane = threadIdx.x & 63;
    if (!R) return;
    const bool vec = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    const uint64_t q1 = (endp + 3) >> 2;
    if (endp - base >= (uint64_t)EMIT_RUNS * R) {
        // Long runs (C2: 250 IDs per filter; average run >= EMIT_RUNS values):
        // copy run by run.  The wave walks its ranges in order; for each, lane
        // l writes the l-th 16-B quad of the run's output with one dword-
        // aligned 16-B load from the run (the vals device copy has a 4-word
        // guard before the first run and >= 16 words after the last, so the
        // load may overhang the run) and one non-temporal store: a few
        // instructions per KiB instead of a range search per quad.  The quads
        // a run shares with its neighbours take dword stores of its own
        // elements.  C2 batch 1.43 -> 1.10 ms (profiles/r2_emit_variants.txt;
        // the variants that wrote every quad once, whole -- a window of <= 4
        // ranges per 1 KiB, extra loads of the next runs, a quad carried
        // between runs in scalar registers -- all measured slower: each extra
        // load or cross-lane step per quad costs more than the partial writes).
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        for (uint32_t i = 0; i < R; i++) {
            const uint32_t ro = s_off[i], rf = s_flg[i];
            const uint64_t P = base + s_rel[i];
            if (rf & RF_SKIP) continue;
            if (rf & RF_INLINE) {
                if (lane == 0 && P < cap) out[P] = ro;
                continue;
            }
            const uint64_t E = base + s_rel[i + 1];
            for (uint64_t Q = (P >> 2) + lane; (Q << 2) < E; Q += 64) {
                const uint64_t p0 = Q << 2;
                const uint4 a = *reinterpret_cast<const uint4u *>(ix.vals + ro + (int64_t)(p0 - P));
                if (vec && p0 >= P && p0 + 4 <= E && p0 + 3 < cap) {
                    const u32x4 x = {a.x, a.y, a.z, a.w};
                    __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(out + p0));
                } else {
                    const uint32_t e[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        if (p0 + k >= P && p0 + k < E && p0 + k < cap) out[p0 + k] = e[k];
                }
            }
        }
        return;
    }
    uint32_t r = 0;   // last range starting at or before the lane's position (positions only grow)
    // one quad: its range found from the lane's previous one (positions only
    // grow; a lane moves 256 positions per quad, so a few steps forward cover
    // long ranges -- C2: 250 values -- and a binary search the rest), then its
    // four values
    auto fetch = [&](uint64_t q, uint32_t (&v)[4], bool (&ok)[4]) {
        const uint64_t p0 = q << 2;
        const uint32_t first = (uint32_t)((p0 > base ? p0 : base) - base);
        uint32_t k = 0;
        while (k < 2 && r + 1 < R && s_rel[r + 1] <= first) { r++; k++; }
        if (r + 1 < R && s_rel[r + 1] <= first) {
            uint32_t lo = r + 1, hi = R - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (s_rel[mid] <= first) lo = mid; else hi = mid - 1;
            }
            r = lo;
        }
        if (q < q1 && p0 >= base && p0 + 3 < endp) {   // whole quad inside one run: one 16-B load
            const uint32_t rs = s_rel[r], re = s_rel[r + 1];
            if (!s_flg[r] && first >= rs && first + 3 < re) {
                const uint4 a = *reinterpret_cast<const uint4u *>(ix.vals + s_off[r] + (first - rs));
                v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
                ok[0] = ok[1] = ok[2] = ok[3] = true;
                return;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t p = p0 + k;
            ok[k] = false; v[k] = 0;
            if (q >= q1 || p < base || p >= endp) continue;
            const uint32_t x = (uint32_t)(p - base);
            while (r + 1 < R && s_rel[r + 1] <= x) r++;
            const uint32_t rs = s_rel[r], rf = s_flg[r];
            if (!(rf & RF_SKIP) && x >= rs && x < s_rel[r + 1]) {
                v[k] = (rf & RF_INLINE) ? s_off[r] : ix.vals[s_off[r] + (x - rs)];
                ok[k] = true;
            }
        }
    };
    auto put = [&](uint64_t q, const uint32_t (&v)[4], const bool (&ok)[4]) {
        const uint64_t p0 = q << 2;
        if (vec && ok[0] && ok[1] && ok[2] && ok[3] && p0 + 3 < cap) {
            // non-temporal: the hit lists are not read back by the GPU, and
            // dirty output lines left in L2 slow the next batch's walk (C2
            // walk 0.150 -> 0.124 ms, C3 batch -1 %)
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 x = {v[0], v[1], v[2], v[3]};
            __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(out + p0));
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (ok[k] && p0 + k < cap) out[p0 + k] = v[k];
        }
    };
    // EMIT_Q quads per iteration, all their value loads issued before any
    // store (the compiler cannot move a vals load above a store to out).  The
    // lanes start at the 128-byte line holding the span's first quad, so every
    // store instruction covers 8 whole lines instead of 9 partial ones
    // (tools/store_bench: 16-B- but not 128-B-aligned 1 KiB stores write at
    // 4.2-4.8 TB/s, aligned ones at 5.2-5.7); lanes before the span store
    // nothing.
    for (uint64_t q = ((base >> 2) & ~7ull) + lane; q < q1; q += 64 * EMIT_Q) {
        uint32_t v[EMIT_Q][4];
        bool ok[EMIT_Q][4];
#pragma unroll
        for (int j = 0; j < EMIT_Q; j++) fetch(q + 64 * j, v[j], ok[j]);
#pragma unroll
        for (int j = 0; j < EMIT_Q; j++) put(q + 64 * j, v[j], ok[j]);
    }
}

// One block = one tile of 256 topics: finishes the scan (tile prefix + local
// exclusive scan -> hit_offs), then each wave flattens its 64 topics' value
// ranges into LDS (sorted by output position) and every lane produces whole
// aligned quads of the wave's CSR span: the quad's range found from the lane's
// previous one (a few steps, else a binary search), four value reads, one
// 16-byte store -- a wave writes 1 KiB per store instruction
// whatever the per-topic hit counts are.  Positions of topics that overflowed
// RCAP ranges are skipped (k_rewalk_tail writes them).
__global__ __launch_bounds__(EMIT_BLOCK) void k_emit(DevIndex ix, Workspace ws, uint64_t n,
                                                     uint64_t *hit_offs, uint32_t *out, uint64_t cap) {
    // 9 B per range: a range's count is the distance to the next one's start
    // (s_rel[R] = the wave's span), so 18 KiB per block: 8 waves per SIMD
    // instead of 6 with an explicit count (C3 batch 0.338 -> 0.327 ms with the
    // range prefetch below, profiles/r3/emit/)
    __shared__ uint32_t s_off[EMIT_WAVES][WR];
    __shared__ uint32_t s_rel[EMIT_WAVES][WR + 1];
    __shared__ uint8_t s_flg[EMIT_WAVES][WR];
    __shared__ uint64_t s_w[4];
    __shared__ uint64_t s_end[EMIT_WAVES];
    __shared__ uint64_t s_pre;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * EMIT_BLOCK + threadIdx.x;
    const bool valid = t < n;
    // per-topic walk outputs are read once: non-temporal loads keep them from
    // evicting the concurrent walk's lines (bench, three streams: +1.3 %)
    const uint32_t c = valid ? __builtin_nontemporal_load(ws.cnt + t) : 0;
    uint32_t nr = valid ? __builtin_nontemporal_load(ws.nr + t) : 0;
    const bool ovf = nr > RCAP;   // written by k_rewalk_tail: one skip range over its positions
    if (ovf) nr = 0;
    // the topic's ranges do not depend on the scan: all its loads are issued
    // here and fly across it (one round trip instead of one per range; loading
    // all RCAP slots whatever nr is measured slower: +55 % range bytes)
    uint64_t gr[RCAP];
#pragma unroll
    for (int i = 0; i < RCAP; i++)
        gr[i] = (uint32_t)i < nr ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(ws.rng) + (uint64_t)i * n + t) : 0;
    // the tile's prefix: the superblocks before this one, then the tiles
    // before this one in its superblock (wave 0; <= 64 of each per lane round)
    if (wv == 0) {
        const uint64_t b = blockIdx.x, sb = b / SUP;
        uint64_t v = 0;
        for (uint64_t i = lane; i < sb; i += 64) v += ws.sup[i];
        if (sb * SUP + lane < b) v += ws.blk[sb * SUP + lane];
        v = wave_incl_scan(v);
        if (lane == 63) s_pre = v;
    }
    uint64_t total;
    const uint64_t ex = block_excl_scan(c, total, s_w);   // (its barrier publishes s_pre)
    const uint64_t my = s_pre + ex;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) hit_offs[n] = s_pre + total;   // the grand total
    // the GPU never reads the offsets (or the err flags) back: non-temporal
    if (valid) __builtin_nontemporal_store(my, hit_offs + t);
    if (lane == 63) s_end[wv] = my + c;
    __syncthreads();
    const uint64_t t0 = t - lane;
    if (t0 >= n) return;   // whole wave leaves; only wave-level sync below
    const uint64_t base = __shfl(my, 0, 64);
    const uint64_t endp = s_end[wv];
    const uint32_t rel = (uint32_t)(my - base);
    uint32_t R;
    const uint32_t r0 = wave_excl_scan32(ovf ? (c ? 1u : 0u) : nr, R);
    if (ovf && c) {
        s_off[wv][r0] = 0;
        s_rel[wv][r0] = rel;
        s_flg[wv][r0] = RF_SKIP;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < RCAP; i++) {
        if ((uint32_t)i >= nr) break;
        const uint2 g = make_uint2((uint32_t)gr[i], (uint32_t)(gr[i] >> 32));
        s_off[wv][r0 + i] = g.x;          // RUN_INLINE: the value itself
        s_rel[wv][r0 + i] = rel + acc;
        s_flg[wv][r0 + i] = (g.y & RUN_INLINE) ? RF_INLINE : 0;
        acc += g.y & RUN_CNT;
    }
    if (lane == 0) s_rel[wv][R] = (uint32_t)(endp - base);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    wave_emit(ix, s_off[wv], s_rel[wv], s_flg[wv], R, base, endp, out, cap);
}

// ------------------------------------------------- one-pass batches as pairs
//
// tm_match_batch_dev_pairs: the hit lists as per-topic (first position, count)
// pairs, so a walk block writes its own values -- no scan, no range lists, no
// k_emit.  A block of 64 topics walks as k_walk_fast does (ranges in
// registers), scans its counts in the wave, reserves its values' span with ONE
// atomic on its region's counter (vres_reserve), writes its topics' pairs, then
// flattens its ranges into the (now dead) walk LDS and writes the span as
// whole aligned quads (wave_emit, k_emit's copy).  Spans are disjoint, in
// completion order, and may leave gaps.  Deep topics (the tail lists) and
// topics with more than RCAP ranges (span reserved here, values re-walked) are
// finished by k_tail_pairs, whose last block writes the total and the extent.
struct WalkLds {
    uint32_t wid[FAST_L * WALK_BLOCK];
    uint32_t pend[(FAST_L + 1) * WALK_BLOCK];
    uint8_t len[FAST_L * WALK_BLOCK];
};
struct SpanLds {
    uint32_t off[WR];
    uint32_t rel[WR + 1];
    uint8_t flg[WR];
};
static_assert(WALK_BLOCK == 64, "k_walk_pairs: one wave per block");

// A span of T values for region g of K (Workspace::vres): [g Rg, (g + 1) Rg)
// while the region has room, else the pool [K Rg, cap); a position past cap
// means the values were dropped (the caller's extent check).  The regions take
// 7/8 of cap; a region's unused tail is a gap in the output.  K: one region per
// 128 walk blocks, at most VRES_K (a batch of < 16k topics has one region and
// fills it in order; a larger one spreads its blocks' atomics over K lines).
__device__ __forceinline__ uint32_t vres_k(uint64_t n) {
    const uint64_t k = (n + WALK_BLOCK - 1) / WALK_BLOCK / 128;
    return k < 1 ? 1u : (k > VRES_K ? (uint32_t)VRES_K : (uint32_t)k);
}
__device__ __forceinline__ uint64_t vres_region(uint64_t cap, uint32_t K) { return (cap - cap / 8) / K; }
__device__ __forceinline__ uint64_t vres_reserve(const Workspace &ws, uint64_t cap, uint32_t K, uint32_t g, uint32_t T) {
    const uint64_t Rg = vres_region(cap, K);
    if (g < K && Rg) {
        const uint64_t old = atomicAdd((unsigned long long *)&ws.vres[g * VRES_STRIDE], (unsigned long long)T);
        if (old + T <= Rg) return g * Rg + old;
        atomicAdd((unsigned long long *)&ws.vres[g * VRES_STRIDE + 1], (unsigned long long)T);
    }
    return K * Rg + atomicAdd((unsigned long long *)&ws.vres[VRES_POOL], (unsigned long long)T);
}

__global__ __launch_bounds__(WALK_BLOCK, 8) void k_walk_pairs(DevIndex ix, Workspace ws, uint64_t n,
                                                           const uint8_t *blob, const uint64_t *offs, uint8_t *err,
                                                           uint32_t *pairs, uint32_t *out, uint64_t cap) {
    __shared__ union { WalkLds w; SpanLds e; } s;
    const uint32_t lane = threadIdx.x;
    const uint64_t t = (uint64_t)blockIdx.x * WALK_BLOCK + lane;
    RangeEmit em;
    em.cnt = 0; em.nr = 0;
    int deep = -1, ovf = -1;
    if (t < n) {
        LdsStore<FAST_L> st{s.w.wid + lane, s.w.pend + lane, s.w.len + lane, WALK_BLOCK, 0};
        uint32_t levels;
        const int rc = match_topic(ix, GlobalSrc{blob}, offs[t], offs[t + 1], st, em, &levels);
        if (rc == RC_DEEP) {   // k_tail_pairs walks it (flag, pair and values)
            deep = tail_list(ix, levels);
            em.cnt = 0; em.nr = 0;
        } else {
            if (rc != RC_OK) { em.cnt = 0; em.nr = 0; }
            __builtin_nontemporal_store((uint8_t)(rc == RC_BADARG ? 1 : 0), err + t);
            if (em.nr > RCAP) ovf = L_OVF_MID;   // span reserved below, values re-walked by k_tail_pairs
        }
    }
    list_push_wave(ws, n, deep, (uint32_t)t);
    list_push_wave(ws, n, ovf, (uint32_t)t);
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(em.cnt, tot);
    uint64_t base = 0;
    if (lane == 0 && tot) {
        const uint32_t K = vres_k(n);
        base = vres_reserve(ws, cap, K, blockIdx.x % K, tot);
    }
    base = ((uint64_t)(uint32_t)__shfl((int)(base >> 32), 0, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)base, 0, 64);
    if (t < n && deep < 0) {
        const uint64_t p = base + ex < cap ? base + ex : cap;   // (past cap: dropped)
        const uint64_t pc = (uint64_t)(uint32_t)p | ((uint64_t)em.cnt << 32);
        __builtin_nontemporal_store(pc, reinterpret_cast<uint64_t *>(pairs) + t);
    }
    if (!tot) return;   // (wave-uniform)
    wave_sync();   // every lane is done with the walk's LDS
    const bool skip = ovf >= 0;
    constexpr uint32_t VST = sizeof(s) / 4;   // values the dead walk LDS holds (1,216)
    if (tot <= VST) {
        // Most spans (C3: ~540 values per wave, nearly all single-value runs
        // kept inline): each lane stages its topic's values in LDS at its own
        // offset, then the wave copies the span out in coalesced non-temporal
        // dwords -- no range search per quad.  An overflowed topic's positions
        // hold stale words until k_tail_pairs re-walks it (stream order).
        uint32_t *sv = reinterpret_cast<uint32_t *>(&s);
        uint32_t p = ex;
#pragma unroll
        for (int i = 0; i < RCAP; i++) {
            if (skip || (uint32_t)i >= em.nr) break;
            const uint2 r = em.r[i];
            if (r.y & RUN_INLINE) { sv[p++] = r.x; continue; }
#pragma unroll 2
            for (uint32_t k = 0; k < (r.y & RUN_CNT); k++) sv[p++] = ix.vals[r.x + k];
        }
        wave_sync();
        for (uint32_t i = lane; i < tot; i += 64)
            if (base + i < cap) __builtin_nontemporal_store(sv[i], out + base + i);
        return;
    }
    // a larger span: its ranges flattened (one skip range for an overflowed
    // topic) and copied as whole aligned quads
    uint32_t R;
    const uint32_t r0 = wave_excl_scan32(skip ? (em.cnt ? 1u : 0u) : em.nr, R);
    if (skip && em.cnt) {
        s.e.off[r0] = 0;
        s.e.rel[r0] = ex;
        s.e.flg[r0] = RF_SKIP;
    }
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < RCAP; i++) {
        if (skip || (uint32_t)i >= em.nr) break;
        s.e.off[r0 + i] = em.r[i].x;   // RUN_INLINE: the value itself
        s.e.rel[r0 + i] = ex + acc;
        s.e.flg[r0 + i] = (em.r[i].y & RUN_INLINE) ? RF_INLINE : 0;
        acc += em.r[i].y & RUN_CNT;
    }
    if (lane == 0) s.e.rel[R] = tot;
    wave_sync();
    wave_emit(ix, s.e.off, s.e.rel, s.e.flg, R, base, base + tot, out, cap);
}

// one tail-list topic of a pairs batch (every lane of the wave calls it; live:
// the lane has a topic): walk, reserve (one atomic per wave), pair, flag; the
// wave's values written as k_walk_pairs writes them (ranges flattened into
// LDS, whole aligned quads); a topic with more than RCAP ranges is re-walked
// into its span afterwards.  sp aliases the MID store's LDS: a wave's walks
// are done before it is written (wave_sync), and read before the re-walk.
template <class S>   // (inlined: a call would pass the kernel's DevIndex and Workspace through scratch)
__device__ __forceinline__ void tail_pair(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *blob,
                          const uint64_t *offs, bool live, uint64_t t, uint8_t *err, uint32_t *pairs, uint32_t *out,
                          uint64_t cap, uint32_t wave_no, S &st, SpanLds &sp) {
    // the walk is k_walk_tail's (run_topic: count, ranges and flag into the
    // workspace at t -- its own register budget, no scratch); the ranges are
    // read back below by the lane that wrote them
    uint32_t c = 0;
    if (live) {
        int ovf = -1;   // (more than RCAP ranges: re-walked below, no list)
        const Outs o{err, nullptr, nullptr};
        const int rc = run_topic<MODE_COUNT>(ix, ws, n, blob, offs, t, st, o, &c, &ovf);
        if (rc == RC_DEEP) c = 0;   // (not on the lists' stores: they hold every level a walk uses)
    }
    uint32_t tot;
    const uint32_t ex = wave_excl_scan32(c, tot);
    const uint32_t lane = threadIdx.x & 63;
    uint64_t base = 0;
    if (lane == 0 && tot) {   // the waves of a list take the regions in turn, as the walk's blocks do
        const uint32_t K = vres_k(n);
        base = vres_reserve(ws, cap, K, wave_no % K, tot);
    }
    base = ((uint64_t)(uint32_t)__shfl((int)(base >> 32), 0, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)base, 0, 64);
    const uint64_t pos = base + ex;
    if (live)
        reinterpret_cast<uint64_t *>(pairs)[t] = (uint64_t)(uint32_t)(pos < cap ? pos : cap) | ((uint64_t)c << 32);
    if (!tot) return;   // (wave-uniform)
    const uint32_t nr = live && c ? ws.nr[t] : 0;
    const bool skip = nr > RCAP;
    wave_sync();   // every lane is done with the store's LDS
    uint32_t R;
    const uint32_t r0 = wave_excl_scan32(skip ? 1u : nr, R);
    if (skip) {
        sp.off[r0] = 0;
        sp.rel[r0] = ex;
        sp.flg[r0] = RF_SKIP;
    }
    uint32_t acc = 0;
    for (uint32_t i = 0; !skip && i < nr; i++) {
        const uint64_t g = reinterpret_cast<const uint64_t *>(ws.rng)[(uint64_t)i * n + t];
        sp.off[r0 + i] = (uint32_t)g;
        sp.rel[r0 + i] = ex + acc;
        sp.flg[r0 + i] = ((uint32_t)(g >> 32) & RUN_INLINE) ? RF_INLINE : 0;
        acc += (uint32_t)(g >> 32) & RUN_CNT;
    }
    if (lane == 0) sp.rel[R] = tot;
    wave_sync();
    wave_emit(ix, sp.off, sp.rel, sp.flg, R, base, base + tot, out, cap);
    wave_sync();   // the span table read before the store's LDS is walked again
    if (skip) {   // (rare)
        DirectEmit de{ix.vals, out, pos, cap};
        match_topic(ix, GlobalSrc{blob}, offs[t], offs[t + 1], st, de);
    }
}

// The second (last) launch of a pairs batch: the MID / DEEP lists (topics the
// walk handed over, walked here from scratch) and the overflow list (span
// reserved by the walk, values re-walked into it); the grid's last block
// writes the total, zeroes the value counter and resets the lists
struct MidLds {
    uint32_t wid[MID_L * MID_BLOCK];
    uint32_t pend[(MID_L + 1) * MID_BLOCK];
    uint8_t len[MID_L * MID_BLOCK];
};
__global__ __launch_bounds__(MID_BLOCK) void k_tail_pairs(DevIndex ix, Workspace ws, uint64_t n, const uint8_t *blob,
                                                          const uint64_t *offs, uint8_t *err, uint32_t *pairs,
                                                          uint32_t *out, uint64_t cap, uint32_t mid_grid) {
    __shared__ union { MidLds w; SpanLds e; } s;
    static_assert(MID_BLOCK == 64, "one wave per tail block");
    if (blockIdx.x < mid_grid) {
        LdsStore<MID_L> st{s.w.wid + threadIdx.x, s.w.pend + threadIdx.x, s.w.len + threadIdx.x, MID_BLOCK, 0};
        const uint32_t cnt = ws.list_n[L_MID];
        const uint32_t *lst = ws.lists + (uint64_t)L_MID * n;
        for (uint32_t i0 = blockIdx.x * MID_BLOCK; i0 < cnt; i0 += mid_grid * MID_BLOCK) {
            const uint32_t i = i0 + threadIdx.x;
            tail_pair(ix, ws, n, blob, offs, i < cnt, i < cnt ? lst[i] : 0, err, pairs, out, cap, i0 / MID_BLOCK, st,
                      s.e);
        }
        const uint32_t co = ws.list_n[L_OVF_MID];
        const uint32_t *lo = ws.lists + (uint64_t)L_OVF_MID * n;
        for (uint32_t i = blockIdx.x * MID_BLOCK + threadIdx.x; i < co; i += mid_grid * MID_BLOCK) {
            const uint64_t t = lo[i];
            DirectEmit de{ix.vals, out, pairs[2 * t], cap};
            match_topic(ix, GlobalSrc{blob}, offs[t], offs[t + 1], st, de);
        }
    } else {
        const uint32_t lane = (blockIdx.x - mid_grid) * 64 + threadIdx.x;   // < DEEP_LANES
        GlobalStore st{ws.deep_wid + (uint64_t)lane * MAX_LEVELS, ws.deep_stk + (uint64_t)lane * (MAX_LEVELS + 1),
                       ws.deep_plus + (uint64_t)lane * MAX_LEVELS, 0};
        const uint32_t cnt = ws.list_n[L_DEEP];
        const uint32_t *lst = ws.lists + (uint64_t)L_DEEP * n;
        for (uint32_t i0 = lane - threadIdx.x; i0 < cnt; i0 += DEEP_LANES) {
            const uint32_t i = i0 + threadIdx.x;
            tail_pair(ix, ws, n, blob, offs, i < cnt, i < cnt ? lst[i] : 0, err, pairs, out, cap, i0 / 64 + 1, st, s.e);
        }
    }
    // the grid's last block: every block's reservations have returned (their
    // atomics drained before its ticket), so the counter is the total
    __shared__ uint32_t s_last;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&ws.list_n[L_COUNT + 1], 1u) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    // the total (every region's successful reservations and the pool's) and
    // the extent (the end of the last value position used; past cap: values
    // were dropped), then the counters zeroed for the next batch
    const uint32_t K = vres_k(n);
    const uint64_t Rg = vres_region(cap, K);
    uint64_t total = 0, extent = 0;
    for (uint32_t k = threadIdx.x; k <= VRES_K; k += MID_BLOCK) {
        const uint64_t f = __hip_atomic_load(&ws.vres[k * VRES_STRIDE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k < VRES_K) {
            const uint64_t x = __hip_atomic_load(&ws.vres[k * VRES_STRIDE + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            total += f - x;
            if (f - x) extent = max(extent, k * Rg + (f - x));
        } else {
            total += f;
            if (f) extent = max(extent, K * Rg + f);
        }
        ws.vres[k * VRES_STRIDE] = 0;
        ws.vres[k * VRES_STRIDE + 1] = 0;
    }
    for (int d = 32; d; d >>= 1) {
        total += (uint64_t)__shfl_xor((long long)total, d, 64);
        extent = max(extent, (uint64_t)__shfl_xor((long long)extent, d, 64));
    }
    if (threadIdx.x) return;
    pairs[2 * n] = total > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)total;
    pairs[2 * n + 1] = extent > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)extent;
    for (int k = 0; k < L_COUNT; k++) {
        const uint32_t len = atomicExch(&ws.list_n[k], 0u);
        if (ws.hint_d) ws.hint_d[k] = len;
    }
    if (ws.hint_d) ws.hint_d[L_COUNT] = n < 0xFFFFFFFFull ? (uint32_t)n : 0xFFFFFFFFu;
    atomicExch(&ws.list_n[L_COUNT + 1], 0u);
}

// The LITE fallback store of k_walk_small<8> (FAST_L levels resolving only
// need_levels()) holds every topic of a shallow index without a
// '#'-not-last key.  (Round 5's k_walk_lane, one lane per topic, ran on the same
// condition; it lost to k_walk_small on every measured path -- 4k 0.077 vs
// 0.040 ms, 8 callers 2.5e8 vs 3.1e8 -- and was removed in round 6.)
bool lite_path_ok(const DevIndex &ix) {
    return !ix.hdesc && ix.depth + 2 <= (uint32_t)FAST_L && ix.xlen_max <= (uint32_t)FAST_L;
}

__global__ void k_patch(const PatchRun *runs, const uint32_t *data, uint64_t n, PatchBases bases) {
    const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const uint32_t g = threadIdx.x & 15;
    if (i >= n) return;
    const PatchRun r = runs[i];
    uint32_t *dst = reinterpret_cast<uint32_t *>(bases.b[r.dst >> 48]) + (r.dst & PATCH_OFF);
    for (uint32_t k = g; k < r.n; k += 16) dst[k] = data[r.src + k];
}

// ------------------------------------------------------ filter-sharded merge

// Filter-sharded mode: `world` shards matched the same n topics
// against disjoint key sets; their CSR hit lists were exchanged (RCCL) into
// shard_hit [world][n+1] and shard_vals [world][stride].  Topic t's merged list
// is shard 0's list, then shard 1's, ... -- the union of disjoint key sets, so
// the same value set as one index holding every key.  Merged offsets are the
// sums of the shards' offsets (a sum of exclusive prefix sums is the prefix sum
// of the summed counts): no scan needed.  One wave per MERGE_TOPICS topics; a
// segment (one shard's list of one topic) is copied by all 64 lanes, so loads
// and stores are coalesced (one thread per segment walked its own range:
// C4's 62 values per topic became 62 M scattered requests, 1.6 ms per batch).
constexpr int MERGE_TOPICS = 16;
constexpr int MERGE_LDS_WORLD = 16;   // shards whose offsets a wave stages in LDS (more: read in place)
__global__ __launch_bounds__(256) void k_merge_shards(uint32_t world, uint64_t n, const uint64_t *shard_hit,
                                                      const uint32_t *shard_vals, uint64_t stride,
                                                      uint64_t *out_hit, uint32_t *out, uint64_t cap) {
    __shared__ uint64_t s_h[4][MERGE_LDS_WORLD][MERGE_TOPICS + 1];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t t0 = w * MERGE_TOPICS;
    if (t0 > n) return;
    const uint64_t t1 = t0 + MERGE_TOPICS < n ? t0 + MERGE_TOPICS : n;
    const bool staged = world <= MERGE_LDS_WORLD;
    // the wave's offsets, every shard at once (one round trip instead of one per topic)
    if (staged) {
        for (uint32_t q = 0; q < world; q++)
            if (lane <= t1 - t0) s_h[wv][q][lane] = shard_hit[(uint64_t)q * (n + 1) + t0 + lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    auto H = [&](uint32_t q, uint64_t t) -> uint64_t {
        return staged ? s_h[wv][q][t - t0] : shard_hit[(uint64_t)q * (n + 1) + t];
    };
    for (uint64_t t = t0; t <= t1; t++) {
        if (t == t1 && t1 != n) break;   // the next wave writes its own first offset
        uint64_t d = 0;
        for (uint32_t q = 0; q < world; q++) d += H(q, t);
        if (lane == 0) out_hit[t] = d;
        if (t == n) break;
        for (uint32_t q = 0; q < world; q++) {
            const uint64_t s0 = H(q, t), len = H(q, t + 1) - s0;
            const uint32_t *src = shard_vals + (uint64_t)q * stride + s0;
            for (uint64_t i = lane; i < len; i += 64)
                if (d + i < cap) out[d + i] = src[i];
            d += len;
        }
    }
}

// ------------------------------------------------------ sorted hit lists
//
// Ascending-u32 output ("hit lists come out sorted (ascending
// u32), plus a mode that emits the reference traversal order"): a post-pass
// over any CSR of hit lists (the emit's, or the merged shards') sorts each
// topic's segment in place; UNIQUE also drops repeated values (the
// [unique] option of matches/3, emqx_trie_search.erl:201-211, when the u32
// is the interned ID): the distinct values first, the rest of the segment
// padded with 0xFFFFFFFF, and the distinct count per topic in ucnt.
//
// Segments of up to SS_SMALL values: one lane each (insertion sort in LDS,
// laid out [k][thread]: conflict free).  Longer ones are listed and sorted by
// one block each (bitonic, LDS up to SS_LDS values; beyond that chunks sorted
// in LDS and merged with global-memory steps).  The bitonic network is the
// all-ascending ("flip") form, so a segment of any length c sorts as if
// padded to a power of two with +inf: comparators touching index >= c are
// no-ops and never run.
constexpr int SS_SMALL = 32;
constexpr int SS_BLOCK = 256;
constexpr int SS_LDS = 8192;
constexpr int SS_GRID_BIG = 512;
enum { SS_CNT = L_COUNT + 2, SS_TICKET = L_COUNT + 3 };   // Workspace::list_n slots

__device__ __forceinline__ void cas_up(uint32_t *v, uint64_t i, uint64_t j) {
    const uint32_t a = v[i], b = v[j];
    if (a > b) { v[i] = b; v[j] = a; }
}

// comparator k of a step whose partner bit is b: index i has bit b clear
__device__ __forceinline__ uint64_t cmp_index(uint64_t k, uint32_t b) {
    return ((k >> b) << (b + 1)) | (k & ((1ull << b) - 1));
}

// bitonic steps of sizes [size0, size1] (flip + half-cleaners down to stride
// smin) over v[0, c), by the block; v is LDS or global
template <bool LDS>
__device__ void bitonic_steps(uint32_t *v, uint64_t c, uint64_t P, uint64_t size0, uint64_t size1, uint64_t smin) {
    for (uint64_t size = size0; size <= size1; size <<= 1) {
        const uint32_t bf = 63 - __clzll(size >> 1);
        for (uint64_t k = threadIdx.x; k < P / 2; k += blockDim.x) {   // flip: i <-> i ^ (size - 1)
            const uint64_t i = cmp_index(k, bf), j = i ^ (size - 1);
            if (j < c) cas_up(v, i, j);
        }
        if (!LDS) __threadfence_block();
        __syncthreads();
        for (uint64_t st = size >> 2; st >= smin && st > 0; st >>= 1) {   // half-cleaners: i <-> i + st
            const uint32_t b = 63 - __clzll(st);
            for (uint64_t k = threadIdx.x; k < P / 2; k += blockDim.x) {
                const uint64_t i = cmp_index(k, b), j = i + st;
                if (j < c) cas_up(v, i, j);
            }
            if (!LDS) __threadfence_block();
            __syncthreads();
        }
    }
}

// the remaining half-cleaner strides < SS_LDS of a merge step, chunk by chunk in LDS
__device__ void bitonic_tail_lds(uint32_t *g, uint64_t c, uint32_t *s, uint64_t st0) {
    for (uint64_t base = 0; base < c; base += SS_LDS) {
        const uint64_t len = c - base < (uint64_t)SS_LDS ? c - base : SS_LDS;
        for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) s[k] = g[base + k];
        __syncthreads();
        for (uint64_t st = st0; st > 0; st >>= 1) {
            const uint32_t b = 63 - __clzll(st);
            for (uint64_t k = threadIdx.x; k < SS_LDS / 2; k += blockDim.x) {
                const uint64_t i = cmp_index(k, b), j = i + st;
                if (j < len) cas_up(s, i, j);
            }
            __syncthreads();
        }
        for (uint64_t k = threadIdx.x; k < len; k += blockDim.x) g[base + k] = s[k];
        __syncthreads();
    }
}

__global__ __launch_bounds__(SS_BLOCK) void k_segsort_small(uint64_t n, const uint64_t *hit, uint32_t *out, uint64_t cap,
                                                            int unique, uint32_t *ucnt, Workspace ws) {
    __shared__ uint32_t s[SS_SMALL * SS_BLOCK];
    const uint64_t t = (uint64_t)blockIdx.x * SS_BLOCK + threadIdx.x;
    if (t >= n) return;
    const uint64_t o = hit[t], e = hit[t + 1], c = e - o;
    if (e > cap) {   // not (wholly) written: the caller gets TM_ECAP and retries
        if (ucnt) ucnt[t] = 0;
        return;
    }
    if (c > SS_SMALL) {
        const uint32_t i = atomicAdd(&ws.list_n[SS_CNT], 1u);
        ws.lists[(uint64_t)L_COUNT * n + i] = (uint32_t)t;
        return;
    }
    uint32_t *v = s + threadIdx.x;
    for (uint32_t k = 0; k < c; k++) v[k * SS_BLOCK] = out[o + k];
    for (uint32_t i = 1; i < c; i++) {
        const uint32_t x = v[i * SS_BLOCK];
        uint32_t j = i;
        while (j > 0 && v[(j - 1) * SS_BLOCK] > x) { v[j * SS_BLOCK] = v[(j - 1) * SS_BLOCK]; j--; }
        v[j * SS_BLOCK] = x;
    }
    uint32_t u = 0;
    for (uint32_t k = 0; k < c; k++) {
        const uint32_t x = v[k * SS_BLOCK];
        if (!unique || k == 0 || x != v[(k - 1) * SS_BLOCK]) out[o + u++] = x;
    }
    for (uint32_t k = u; k < c; k++) out[o + k] = NONE;
    if (ucnt) ucnt[t] = u;
}

__global__ __launch_bounds__(SS_BLOCK) void k_segsort_big(uint64_t n, const uint64_t *hit, uint32_t *out, int unique,
                                                          uint32_t *ucnt, Workspace ws) {
    __shared__ uint32_t s[SS_LDS];
    __shared__ uint64_t s_w[4];
    const uint32_t cnt = ws.list_n[SS_CNT];
    const uint32_t *lst = ws.lists + (uint64_t)L_COUNT * n;
    for (uint32_t li = blockIdx.x; li < cnt; li += gridDim.x) {
        const uint64_t t = lst[li];
        const uint64_t o = hit[t], c = hit[t + 1] - o;
        uint64_t P = 1;
        while (P < c) P <<= 1;
        uint32_t *g = out + o;
        if (c <= SS_LDS) {
            for (uint64_t k = threadIdx.x; k < c; k += SS_BLOCK) s[k] = g[k];
            __syncthreads();
            bitonic_steps<true>(s, c, P, 2, P, 1);
            for (uint64_t k = threadIdx.x; k < c; k += SS_BLOCK) g[k] = s[k];
            __syncthreads();
        } else {
            for (uint64_t base = 0; base < c; base += SS_LDS) {   // every SS_LDS chunk sorted in LDS
                const uint64_t len = c - base < (uint64_t)SS_LDS ? c - base : SS_LDS;
                for (uint64_t k = threadIdx.x; k < len; k += SS_BLOCK) s[k] = g[base + k];
                __syncthreads();
                bitonic_steps<true>(s, len, SS_LDS, 2, SS_LDS, 1);
                for (uint64_t k = threadIdx.x; k < len; k += SS_BLOCK) g[base + k] = s[k];
                __syncthreads();
            }
            for (uint64_t size = 2 * SS_LDS; size <= P; size <<= 1) {   // merge levels: strides >= SS_LDS in global
                bitonic_steps<false>(g, c, P, size, size, SS_LDS);
                bitonic_tail_lds(g, c, s, SS_LDS / 2);
            }
        }
        if (unique) {   // distinct values first (block scan of "differs from its left neighbour"), then padding
            uint64_t carry = 0;
            for (uint64_t b0 = 0; b0 < c; b0 += SS_BLOCK) {
                const uint64_t k = b0 + threadIdx.x;
                const uint32_t x = k < c ? g[k] : 0;
                const bool f = k < c && (k == 0 || g[k - 1] != x);
                uint64_t tot;
                const uint64_t pos = carry + block_excl_scan(f ? 1 : 0, tot, s_w);
                __syncthreads();   // every read of this window before any write into it
                if (f) g[pos] = x;
                carry += tot;
                __threadfence_block();
                __syncthreads();
            }
            for (uint64_t k = carry + threadIdx.x; k < c; k += SS_BLOCK) g[k] = NONE;
            if (ucnt && threadIdx.x == 0) ucnt[t] = (uint32_t)carry;
        } else if (ucnt && threadIdx.x == 0) {
            ucnt[t] = (uint32_t)c;
        }
        __syncthreads();
    }
    // the last block resets the list for the next batch
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t ticket = atomicAdd(&ws.list_n[SS_TICKET], 1u);
        if (ticket == gridDim.x - 1) {
            atomicExch(&ws.list_n[SS_CNT], 0u);
            atomicExch(&ws.list_n[SS_TICKET], 0u);
        }
    }
}

// copy a CSR's values (total = hit[n], at most cap) to dst (e.g. mapped host memory)
__global__ __launch_bounds__(256) void k_copy_values(const uint64_t *hit, uint64_t n, const uint32_t *src, uint32_t *dst,
                                                     uint64_t cap) {
    const uint64_t total = hit[n] < cap ? hit[n] : cap;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256)
        dst[i] = src[i];
}

// ------------------------------------------------------------ launchers

static inline uint32_t blocks_for(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

constexpr uint32_t WV_TOPICS_PER_BLOCK = WV_WAVES * (64 / WAVE_W);

hipError_t launch_match_phase1(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                               const uint64_t *offs, uint64_t *hit_offs, uint8_t *err, hipStream_t s,
                               hipEvent_t ev_walk0, hipEvent_t ev_walk1) {
    hipError_t e;
    Outs o{err, nullptr, nullptr};
    // tile and superblock totals are zero between batches (k_rewalk_tail
    // leaves them so): the walks add their topics' hits into them
    const bool wave = n && n <= WAVE_TOPICS;
    if (n) {
        if (ev_walk0 && (e = hipEventRecord(ev_walk0, s)) != hipSuccess) return e;
        if (wave)
            hipLaunchKernelGGL((k_walk_wave<MODE_COUNT, WAVE_W>), dim3(blocks_for(n, WV_TOPICS_PER_BLOCK)),
                               dim3(WV_BLOCK), 0, s, ix, ws, n, bytes, offs, o);
        else
            hipLaunchKernelGGL(k_walk_fast<MODE_COUNT>, dim3(blocks_for(n, WALK_BLOCK)), dim3(WALK_BLOCK), 0, s, ix, ws,
                               n, bytes, offs, o);
        if (ev_walk1 && (e = hipEventRecord(ev_walk1, s)) != hipSuccess) return e;
        const uint32_t mg = tail_blocks(ws, n, L_MID, wave ? MID_GRID : MID_GRID_BIG);
        hipLaunchKernelGGL(k_walk_tail<MODE_COUNT>, dim3(mg + DEEP_LANES / 64), dim3(MID_BLOCK), 0, s, ix, ws, n,
                           bytes, offs, o, mg);
    }
    return hipGetLastError();
}

hipError_t launch_match_phase2(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                               const uint64_t *offs, uint64_t *hit_offs, uint32_t *out, uint64_t cap,
                               hipStream_t s) {
    // (an empty batch: one k_emit block writes hit_offs[0] = 0)
    hipLaunchKernelGGL(k_emit, dim3(n ? blocks_for(n, TILE) : 1), dim3(EMIT_BLOCK), 0, s, ix, ws, n, hit_offs, out, cap);
    if (!n) return hipGetLastError();
    const uint32_t mg = tail_blocks(ws, n, L_OVF_MID, MID_GRID);
    hipLaunchKernelGGL(k_rewalk_tail, dim3(mg + DEEP_LANES / 64), dim3(MID_BLOCK), 0, s, ix, ws, n, bytes, offs,
                       hit_offs, out, cap, mg);
    return hipGetLastError();
}

// a pairs batch (tm_match_batch_dev_pairs): the walk writing its own values,
// then the tail (deep and overflowed topics, the total): two launches
hipError_t launch_match_pairs(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                              const uint64_t *offs, uint8_t *err, uint32_t *pairs, uint32_t *out, uint64_t cap,
                              hipStream_t s, hipEvent_t ev_walk0, hipEvent_t ev_walk1) {
    hipError_t e;
    if (!n) return hipMemsetAsync(pairs, 0, 2 * sizeof(uint32_t), s);
    if (ev_walk0 && (e = hipEventRecord(ev_walk0, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_walk_pairs, dim3(blocks_for(n, WALK_BLOCK)), dim3(WALK_BLOCK), 0, s, ix, ws, n, bytes, offs, err,
                       pairs, out, cap);
    if (ev_walk1 && (e = hipEventRecord(ev_walk1, s)) != hipSuccess) return e;
    const uint32_t mg = tail_blocks(ws, n, L_MID, MID_GRID_BIG);
    hipLaunchKernelGGL(k_tail_pairs, dim3(mg + DEEP_LANES / 64), dim3(MID_BLOCK), 0, s, ix, ws, n, bytes, offs, err,
                       pairs, out, cap, mg);
    return hipGetLastError();
}

// The one-launch kernel of a small batch (small_kind): k_walk_small with 16
// or 8 lanes per topic.  The default (SMALL_AUTO): 8 lanes per topic for a
// launch of >= SMALL_W8_MIN topics or of several host batches (the
// combiner's) -- throughput, twice the topics per wave slot -- and 16 for a
// lone smaller batch (latency: a topic's levels tokenised in half the ballot
// rounds).  8 lanes per topic run only on a lite_path_ok index (the LITE
// fallback store); elsewhere 16.
constexpr uint64_t SMALL_W8_MIN = 8192;
static int small_w(const DevIndex &ix, int kind, uint64_t n, uint32_t segs) {
    const bool w8 = kind == SMALL_WAVE8 || (kind == SMALL_AUTO && (n >= SMALL_W8_MIN || segs > 1));
    return w8 && lite_path_ok(ix) ? 8 : 16;
}
static uint32_t small_topics_per_block(int w) { return w == 8 ? SmallShape<8>::ST : SmallShape<16>::ST; }

template <class OT>
static void launch_small_kernel(int w, uint32_t blocks, const DevIndex &ix, const Workspace &ws, uint64_t n,
                                const uint8_t *bytes, const OT *offs, uint8_t *err, OT *hit_offs, uint32_t *out,
                                uint64_t cap, uint32_t tag, LbCtl lb, const SmallSegs &sg, hipStream_t s) {
    Outs o{err, nullptr, nullptr};
    if (w == 8)
        hipLaunchKernelGGL((k_walk_small<MODE_COUNT, OT, 8, true>), dim3(blocks), dim3(WV_BLOCK), 0, s, ix, ws, n,
                           bytes, offs, o, hit_offs, out, cap, tag, lb, sg);
    else
        hipLaunchKernelGGL((k_walk_small<MODE_COUNT, OT, 16, false>), dim3(blocks), dim3(WV_BLOCK), 0, s, ix, ws, n,
                           bytes, offs, o, hit_offs, out, cap, tag, lb, sg);
}

hipError_t launch_match(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                        const uint64_t *offs, uint64_t *hit_offs, uint8_t *err, uint32_t *out, uint64_t cap,
                        uint32_t tag, LbCtl lb, bool phases, int small_kind, hipStream_t s, hipEvent_t ev_walk0,
                        hipEvent_t ev_walk1, int *path) {
    if (n && !phases && small_path_ok(ix, n)) {
        const int w = small_w(ix, small_kind, n, 1);
        if (path) *path = PATH_SMALL;
        hipError_t e;
        if (ev_walk0 && (e = hipEventRecord(ev_walk0, s)) != hipSuccess) return e;
        launch_small_kernel<uint64_t>(w, blocks_for(n, small_topics_per_block(w)), ix, ws, n, bytes, offs, err,
                                      hit_offs, out, cap, tag & LB_TAG_MASK, lb, SmallSegs{}, s);
        if (ev_walk1 && (e = hipEventRecord(ev_walk1, s)) != hipSuccess) return e;
        return hipGetLastError();
    }
    if (path) *path = PATH_PHASES;
    hipError_t e = launch_match_phase1(ix, ws, n, bytes, offs, hit_offs, err, s, ev_walk0, ev_walk1);
    if (e != hipSuccess) return e;
    return launch_match_phase2(ix, ws, n, bytes, offs, hit_offs, out, cap, s);
}

hipError_t launch_match32(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                          const uint32_t *offs, uint32_t *hit_offs, uint8_t *err, uint32_t *out, uint64_t cap,
                          uint32_t tag, LbCtl lb, int small_kind, hipStream_t s, int *path) {
    if (!small_path_ok(ix, n)) return hipErrorInvalidValue;   // (the caller converts instead)
    const int w = small_w(ix, small_kind, n, 1);
    if (path) *path = PATH_SMALL;
    launch_small_kernel<uint32_t>(w, blocks_for(n, small_topics_per_block(w)), ix, ws, n, bytes, offs, err, hit_offs,
                                  out, cap, tag & LB_TAG_MASK, lb, SmallSegs{}, s);
    return hipGetLastError();
}

// the combiner's launch: sg's segments (block0 filled here) in one grid
hipError_t launch_small_segs(const DevIndex &ix, const Workspace &ws, const SmallSegs &sg0, bool u32, uint32_t tag,
                             LbCtl lb, int small_kind, hipStream_t s, int *path) {
    SmallSegs sg = sg0;
    uint64_t total = 0;
    for (uint32_t q = 0; q < sg.count; q++) total += sg.s[q].n;
    const int w = small_w(ix, small_kind, total, sg.count);
    const uint32_t per = small_topics_per_block(w);
    uint32_t blocks = 0;
    for (uint32_t q = 0; q < sg.count; q++) {
        if (!sg.s[q].n) return hipErrorInvalidValue;
        sg.s[q].block0 = blocks;
        blocks += blocks_for(sg.s[q].n, per);
    }
    if (!sg.count || sg.count > (uint32_t)SMALL_SEGS) return hipErrorInvalidValue;
    if (path) *path = PATH_SMALL;
    const SmallSeg &F = sg.s[0];
    const uint32_t tg = tag & LB_TAG_MASK;
    if (u32)
        launch_small_kernel<uint32_t>(w, blocks, ix, ws, F.n, F.blob, static_cast<const uint32_t *>(F.offs), F.err,
                                      static_cast<uint32_t *>(F.hit), F.out, F.cap, tg, lb, sg, s);
    else
        launch_small_kernel<uint64_t>(w, blocks, ix, ws, F.n, F.blob, static_cast<const uint64_t *>(F.offs), F.err,
                                      static_cast<uint64_t *>(F.hit), F.out, F.cap, tg, lb, sg, s);
    return hipGetLastError();
}

// 32-bit offsets <-> the 64-bit ones every other kernel takes (tm_match_batch32_dev
// on a batch the one-launch small kernel does not take)
__global__ __launch_bounds__(256) void k_offs_widen(const uint32_t *in, uint64_t *out, uint64_t m) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}
__global__ __launch_bounds__(256) void k_offs_narrow(const uint64_t *in, uint32_t *out, uint64_t m) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256)
        out[i] = in[i] > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)in[i];
}

hipError_t launch_offs_widen(const uint32_t *in, uint64_t *out, uint64_t m, hipStream_t s) {
    const uint32_t g = blocks_for(m, 256) < 4096 ? blocks_for(m, 256) : 4096;
    hipLaunchKernelGGL(k_offs_widen, dim3(g), dim3(256), 0, s, in, out, m);
    return hipGetLastError();
}
hipError_t launch_offs_narrow(const uint64_t *in, uint32_t *out, uint64_t m, hipStream_t s) {
    const uint32_t g = blocks_for(m, 256) < 4096 ? blocks_for(m, 256) : 4096;
    hipLaunchKernelGGL(k_offs_narrow, dim3(g), dim3(256), 0, s, in, out, m);
    return hipGetLastError();
}

hipError_t launch_first(const DevIndex &ix, const Workspace &ws, uint64_t n, const uint8_t *bytes,
                        const uint64_t *offs, uint32_t *out_value, uint8_t *out_found, hipStream_t s) {
    if (!n) return hipSuccess;
    Outs o{nullptr, out_value, out_found};
    if (small_path_ok(ix, n)) {
        hipLaunchKernelGGL((k_walk_small<MODE_FIRST, uint64_t, 16, false>), dim3(blocks_for(n, SM_TOPICS)), dim3(WV_BLOCK), 0, s,
                           ix, ws, n, bytes, offs, o, nullptr, nullptr, (uint64_t)0, 0u, LbCtl{LB_SPINS, NONE},
                           SmallSegs{});
        return hipGetLastError();
    }
    if (n <= WAVE_TOPICS)
        hipLaunchKernelGGL((k_walk_wave<MODE_FIRST, WAVE_W>), dim3(blocks_for(n, WV_TOPICS_PER_BLOCK)),
                           dim3(WV_BLOCK), 0, s, ix, ws, n, bytes, offs, o);
    else
        hipLaunchKernelGGL(k_walk_fast<MODE_FIRST>, dim3(blocks_for(n, WALK_BLOCK)), dim3(WALK_BLOCK), 0, s,
                           ix, ws, n, bytes, offs, o);
    hipLaunchKernelGGL(k_walk_tail<MODE_FIRST>, dim3(MID_GRID + DEEP_LANES / 64), dim3(MID_BLOCK), 0, s, ix, ws, n, bytes, offs, o,
                       (uint32_t)MID_GRID);
    return hipGetLastError();
}

hipError_t launch_merge_shards(uint32_t world, uint64_t n, const uint64_t *shard_hit, const uint32_t *shard_vals,
                               uint64_t stride, uint64_t *out_hit, uint32_t *out, uint64_t cap, hipStream_t s) {
    const uint64_t threads = (n / MERGE_TOPICS + 1) * 64;   // one wave per MERGE_TOPICS topics (+ the final offset)
    hipLaunchKernelGGL(k_merge_shards, dim3(blocks_for(threads, 256)), dim3(256), 0, s, world, n, shard_hit,
                       shard_vals, stride, out_hit, out, cap);
    return hipGetLastError();
}

hipError_t launch_sort_segments(const Workspace &ws, uint64_t n, const uint64_t *hit_offs, uint32_t *out, uint64_t cap,
                                int unique, uint32_t *ucnt, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_segsort_small, dim3(blocks_for(n, SS_BLOCK)), dim3(SS_BLOCK), 0, s, n, hit_offs, out, cap, unique,
                       ucnt, ws);
    hipLaunchKernelGGL(k_segsort_big, dim3(SS_GRID_BIG), dim3(SS_BLOCK), 0, s, n, hit_offs, out, unique, ucnt, ws);
    return hipGetLastError();
}

hipError_t launch_copy_values(const uint64_t *hit_offs, uint64_t n, const uint32_t *src, uint32_t *dst, uint64_t cap,
                              hipStream_t s) {
    if (!cap) return hipSuccess;
    const uint64_t blocks = cap / 256 + 1 < 2048 ? cap / 256 + 1 : 2048;
    hipLaunchKernelGGL(k_copy_values, dim3((uint32_t)blocks), dim3(256), 0, s, hit_offs, n, src, dst, cap);
    return hipGetLastError();
}

// ------------------------------------------------------- matches_filter/3
//
// emqx_topic_index:matches_filter/3 -> emqx_trie_search:search/3 with
// [topic_filter] (:186-189): the ordered walk over the key set with the filter
// clauses of compare/3 (:291-300).  Its result depends on where that walk stops
// (a query '+' passes a stored word without leaving a seek point, so one
// stored key above the query ends the whole search), so it runs on the keys in
// Erlang term order, not on the trie: the word-list keys as sequences of word
// ranks ('#' = 0, '+' = 1, binary words 3 + 2 i in byte order; a query word
// the index lacks ranks 2 + 2 i, between its neighbours), sorted by (ranks,
// value), with the reference's seeks as binary searches.  Binary keys sort
// after every list and compare `lower` (:260-261): the walk ends at the last
// list key.  One thread per query; pass 1 counts, pass 2 writes.
struct MfSeek { uint64_t ks; uint32_t pos, w; bool fin; };   // key ks's first pos ranks, then w if fin

__device__ __forceinline__ int mf_cmp(const uint32_t *pool, const uint64_t *koff, uint64_t k, const MfSeek &sk) {
    const uint64_t a0 = koff[k], kl = koff[k + 1] - a0;
    const uint64_t b0 = sk.ks == ~0ull ? 0 : koff[sk.ks];
    const uint64_t sl = sk.pos + (sk.fin ? 1 : 0);
    const uint64_t m = kl < sl ? kl : sl;
    for (uint64_t i = 0; i < m; i++) {
        const uint32_t a = pool[a0 + i], b = i < sk.pos ? pool[b0 + i] : sk.w;
        if (a != b) return a < b ? -1 : 1;
    }
    return kl < sl ? -1 : kl == sl ? 0 : 1;
}

__device__ __forceinline__ uint64_t mf_lower_bound(const uint32_t *pool, const uint64_t *koff, uint64_t K,
                                                   const MfSeek &sk) {
    uint64_t lo = 0, hi = K;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (mf_cmp(pool, koff, mid, sk) < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

constexpr int64_t MF_FULL = -1, MF_PREFIX = -2, MF_LOWER = -3;

// compare/3 with a filter as the query (tm_oracle.c compare_filter restates
// the clauses; ranks as above)
__device__ __forceinline__ int64_t mf_compare(const uint32_t *pool, const uint64_t *koff, uint64_t k,
                                              const uint32_t *q, uint32_t nq) {
    const uint64_t a0 = koff[k];
    const uint32_t kl = (uint32_t)(koff[k + 1] - a0);
    int64_t lastplus = -1;
    for (uint32_t i = 0;; i++) {
        if (i == kl) return i == nq ? MF_FULL : MF_PREFIX;          // :262-281
        const uint32_t f = pool[a0 + i];
        if (f == 0 && i == kl - 1) return MF_FULL;                  // stored '#' last, :282-290
        if (i < nq && q[i] == 0 && i == nq - 1) return MF_FULL;     // query '#' last, :292-293
        if (i == nq) break;                                         // :333-340
        if (q[i] == 1) continue;                                    // query '+', :294-300
        if (f == 1) { lastplus = i; continue; }                     // stored '+', :302-320
        if (f == q[i]) continue;                                    // :321-324
        if (f > q[i]) break;                                        // :325-332
        return (int64_t)i;                                          // seek, :341-348
    }
    return lastplus >= 0 ? lastplus : MF_LOWER;
}

__global__ __launch_bounds__(64) void k_matches_filter(uint64_t n, const uint32_t *qoff, const uint32_t *qr,
                                                       const uint32_t *qbase, const uint32_t *pool,
                                                       const uint64_t *koff, const uint32_t *kval, uint64_t K,
                                                       uint32_t *cnt, const uint64_t *hit, uint32_t *out,
                                                       uint64_t cap, uint8_t *err) {
    const uint64_t t = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (t >= n) return;
    const uint32_t *q = qr + qoff[t];
    const uint32_t nq = qoff[t + 1] - qoff[t];
    // base_init (:160-163): a query whose first word starts with '$' starts at base([W0])
    MfSeek sk{~0ull, 0, qbase[t], qbase[t] != NONE};
    uint64_t cur = mf_lower_bound(pool, koff, K, sk);
    uint64_t o = hit ? hit[t] : 0, c = 0;
    const uint64_t limit = 2 * K + 64;   // every step moves forward; a bound every thread reaches regardless
    for (uint64_t steps = 0; cur < K; steps++) {
        if (steps > limit) { err[t] = 1; break; }
        const int64_t r = mf_compare(pool, koff, cur, q, nq);
        if (r == MF_FULL) {
            if (hit && o < cap) out[o] = kval[cur];
            o++; c++; cur++;
        } else if (r == MF_PREFIX) {
            cur++;
        } else if (r == MF_LOWER) {
            break;
        } else {
            const MfSeek s2{cur, (uint32_t)r, q[r], true};
            const uint64_t nx = mf_lower_bound(pool, koff, K, s2);
            cur = nx > cur ? nx : cur + 1;   // a seek target is above the current key (:341-348)
        }
    }
    if (!hit) cnt[t] = (uint32_t)c;
}

hipError_t launch_matches_filter(uint64_t n, const uint32_t *qoff, const uint32_t *qr, const uint32_t *qbase,
                                 const uint32_t *pool, const uint64_t *koff, const uint32_t *kval, uint64_t K,
                                 uint32_t *cnt, const uint64_t *hit, uint32_t *out, uint64_t cap, uint8_t *err,
                                 hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_matches_filter, dim3(blocks_for(n, 64)), dim3(64), 0, s, n, qoff, qr, qbase, pool, koff,
                       kval, K, cnt, hit, out, cap, err);
    return hipGetLastError();
}

hipError_t launch_patch(const PatchRun *d_runs, const uint32_t *d_data, uint64_t n, PatchBases bases, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_patch, dim3(blocks_for(n * 16, 256)), dim3(256), 0, s, d_runs, d_data, n, bases);
    return hipGetLastError();
}

}  // namespace tmx
