// tm_layout.h -- HBM layout of the compiled topic index, shared by the host
// compiler (tm_host.cpp) and the gfx950 kernels (tm_kernels.hip).
//
// The reference keeps every index entry as an ETS ordered_set key
// {Words | Binary, {ID}} (apps/emqx/src/emqx_trie_search.erl:107-128) and walks
// it with ets:next/2.  Here the same key set is compiled into four
// open-addressing tables + two pools, all flat arrays of 4-byte words so the
// host can patch them in place and mirror the patches to HBM:
//
//   vocab  : word bytes  -> word id (wid)       16 B/entry, verified by bytes
//   ctab   : private child tables (wid -> child) of nodes with more than 4
//            literal children                    8 B/slot
//   nodes  : per trie node: '+' child, '#'-terminal and exact-terminal value
//            ranges, up to 4 inline literal children  64 B/node (one line)
//   exact  : wid sequence -> value range         64 B/entry   (binary keys)
//   xfp    : 16-bit fingerprint per exact slot   2 B/slot: the walk probes
//            this compact array first and reads a 64-byte entry only on a
//            fingerprint match (most topics have no binary key)
//   vals   : u32 values (caller IDs), one sorted run per terminal
//   wpool  : bytes of words longer than 8 B; wseq: wid runs of exact keys
//            longer than XINL levels
//
// A word-list key (wildcard filter, or make_key(Words, ID)) is a path in the
// trie ending in a terminal: exact terminal of node P for filter P, '#'
// terminal of node P for filter P/#.  A binary key without wildcards lives in
// the exact table (emqx_trie_search.erl:121-125 keeps it as a binary too).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define TM_HD __host__ __device__ __forceinline__
#else
#define TM_HD inline
#endif

namespace tmx {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t ROOT = 0;
constexpr uint32_t VINL = 8;    // inline word bytes in a vocab entry
constexpr uint32_t XINL = 10;   // inline wids in an exact entry

struct alignas(16) VocabEntry {   // 16 B
    uint32_t tag;                  // hash bits 32..55 | min(len, 255); 0 with wid NONE = empty
    uint32_t wid;                  // NONE = empty slot
    uint32_t b0, b1;               // len <= 8: the bytes, little endian, zero padded
                                   // len  > 8: b0 = offset of the word in wpool, b1 = len
};

struct alignas(16) CSlot {          // 16 B: one literal child in a node's private table
    uint32_t wid;                  // NONE = empty slot
    uint32_t child;
    uint32_t sum_lo, sum_hi;       // summary of the child (PSUM_* bits + Bloom, as Node.psum):
                                   // the probe that finds a child also says if visiting it can matter
};

constexpr uint32_t KINL = 4;     // literal children kept inside the node's line

// A table-mode node with at least WIDE_LIT literal children (its 192-bit Bloom
// would be saturated: every probe passes it) keeps an exact bitmap over the
// whole wid space instead, in the `wbits` pool (kw[2] = its word offset; NONE
// for a dense wide node, whose children are most of its level's words: the
// walk then probes its child table without asking the bitmap first).
// The few such nodes are the widest of the upper trie -- C3: the level-1
// nodes and the (w0,+) / (+,+) level-2 nodes -- so their bitmaps stay in L2
// and a probe for a word the node has no child for costs an L2 hit instead of
// a memory-side request into a multi-megabyte child table.
constexpr uint32_t WIDE_LIT = 256;

// One 64-byte line per trie state: everything a walk step needs -- the '+'
// child, both terminals and, for nodes with <= KINL literal children (almost
// every node below the top levels), the literal children themselves.  A node
// with more children keeps them in a private open-addressing table of CSlots
// (contiguous, so the hot top of the trie packs densely in L2), and six of the
// line's spare words hold a 192-bit Bloom of its child wids, so the walk skips
// most probes for a word the node has no child for.
//
// `psum` summarises the '+' child Q (when there is one): whether Q has a '#'
// terminal, an exact terminal, a '+' child, and a 61-bit Bloom of Q's literal
// child wids.  From it the walk decides, without reading Q's line, that Q can
// neither emit nor lead anywhere for this topic -- a dead-end '+' visit (2.8
// of the 12.3 node visits per C3 topic before this summary existed).
struct alignas(64) Node {          // 64 B
    uint32_t plus;                 // '+' child or NONE
    uint32_t hash_off, hash_cnt;   // values of filter <path>/#
    uint32_t exact_off, exact_cnt; // values of filter <path> (word-list form)
    uint32_t nlit;                 // literal children (NLIT_MASK; > KINL: table mode) | NLIT_HDESC
    uint32_t psum_lo, psum_hi;     // summary of the '+' child (PSUM_*)
    uint32_t kw[KINL];             // inline: child wids (NONE = free); table mode: kw[0] = table
                                   // offset (CSlots), kw[1] = table size - 1, kw[2..3] Bloom bits 0-63
    uint32_t kc[KINL];             // inline: child node ids; table mode: Bloom bits 64-191
};

// NLIT_HDESC: some stored key continues past this node P with a '#' that is
// not its last word (P/#/X..., a filter emqx_topic:validate/2 would reject but
// an index that does not validate -- the rule engine's FROM topics,
// emqx_rule_engine.erl:534-540 -- may hold).  Such a key never matches, but it
// moves the reference's ordered walk: compare/3 has no clause for a non-final
// '#' (emqx_trie_search.erl:282-290 vs :341-348), so at that key it
//   - seeks to P/W when the topic has a word W at that level: the walk skips
//     P's '+' subtree ('#' < '+' < binaries in term order);
//   - returns `lower` when the topic ends at P: the wildcard phase ends, or,
//     under the innermost '+' of P's path at position q, it seeks to the
//     literal branch P[0..q)/W_q (the '+' frame turns lower into a seek,
//     :302-320).
constexpr uint32_t NLIT_HDESC = 0x80000000u;
constexpr uint32_t NLIT_MASK = 0x7FFFFFFFu;

// Summary of a child Q (Node.psum for the '+' child, CSlot.sum for a literal
// child), two levels deep so a '+' chain that dies one level down is skipped too:
//   bits 0-3  Q has a '#' terminal / an exact terminal / a '+' child (QQ) /
//             NLIT_HDESC (a visit at the topic's last level cuts the walk)
//   bits 4-7  the same for QQ (0 if Q has no '+' child)
//   bits 8-35  28-bit Bloom of Q's literal child wids  (all ones past 28 children)
//   bits 36-63 28-bit Bloom of QQ's literal child wids
constexpr uint32_t PSUM_HASH = 1u, PSUM_EXACT = 2u, PSUM_PLUS = 4u, PSUM_HDESC = 8u;   // psum_lo bits (<< 4: QQ's)
constexpr uint32_t PSUM_QQ = 4, PSUM_BQ = 8, PSUM_BQQ = 36, PSUM_BLOOM = 28;

struct alignas(16) ExactEntry {    // 64 B
    uint32_t h_lo, h_hi;           // hash of the wid sequence
    uint32_t nlev;                 // NONE = empty slot
    uint32_t val_off, val_cnt;
    uint32_t seq_off;              // nlev > XINL: wids in wseq[seq_off ..)
    uint32_t wids[XINL];
};

// Value runs as the device sees them (Node hash_/exact_ fields, ExactEntry
// val_*): (offset into vals, count), except that a run of exactly ONE value is
// stored inline -- off = the value itself, cnt = 1 | RUN_INLINE -- so emitting
// the (common) single-subscriber filter reads no `vals` line.
constexpr uint32_t RUN_INLINE = 0x80000000u;
constexpr uint32_t RUN_CNT = 0x7FFFFFFFu;

static_assert(sizeof(VocabEntry) == 16, "vocab entry");
static_assert(sizeof(CSlot) == 16, "child slot");
static_assert(sizeof(Node) == 64, "node");
static_assert(sizeof(ExactEntry) == 64, "exact entry");

// ---- hashing (identical on host and device) -------------------------------

TM_HD uint64_t mix64(uint64_t x) {          // splitmix64 finaliser
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

constexpr uint64_t FNV_OFF = 0xcbf29ce484222325ull;
constexpr uint64_t FNV_PRIME = 0x100000001b3ull;

// Word hash.  A word of <= VINL bytes is hashed from its packed little-endian
// bytes (b0 = bytes 0..3, b1 = bytes 4..7, zero padded) and its length, so the
// walk kernel can defer its vocab probe to after tokenisation with nothing but
// (b0, b1, len) kept per level; a longer word is FNV-1a over its bytes.
TM_HD uint64_t word_hash_short(uint32_t b0, uint32_t b1, uint32_t len) {
    return mix64((((uint64_t)b1 << 32) | b0) + 0x9e3779b97f4a7c15ull * (len + 1));
}
TM_HD uint64_t word_hash_finish(uint64_t fnv, uint32_t len) { return mix64(fnv ^ ((uint64_t)len << 56)); }

TM_HD uint32_t vocab_tag(uint64_t h, uint32_t len) {
    return ((uint32_t)(h >> 32) & 0xFFFFFF00u) | (len < 255 ? len : 255);
}

// child table hash: low bits pick the slot, the high 16 bits the Bloom bits
TM_HD uint32_t child_hash(uint32_t wid) { return (uint32_t)mix64((uint64_t)wid * 0x9e3779b97f4a7c15ull + 1); }
TM_HD uint32_t child_bit(uint32_t h) { return ((h >> 16) * 192u) >> 16; }      // 0..191, table-mode Bloom
TM_HD uint32_t psum_bit(uint32_t h) { return ((h >> 16) * PSUM_BLOOM) >> 16; }   // 0..27, + PSUM_BQ / PSUM_BQQ
// Bloom word j (bits 32j .. 32j+31) of a table-mode node line
TM_HD uint32_t &bloom_word(Node &n, uint32_t j) { return j < 2 ? n.kw[2 + j] : n.kc[j - 2]; }

// exact-table fingerprint of a wid-sequence hash (never 0: 0 marks an empty slot)
TM_HD uint16_t exact_fp(uint64_t h) { return (uint16_t)((h >> 48) | 1u); }

TM_HD uint64_t seq_hash_step(uint64_t h, uint32_t wid) { return (h ^ wid) * FNV_PRIME; }
TM_HD uint64_t seq_hash_finish(uint64_t h, uint32_t nlev) { return mix64(h + 0x9e3779b97f4a7c15ull * (nlev + 1)); }

}  // namespace tmx
