// tm_layout.h -- HBM layout of the compiled topic index, shared by the host
// compiler (tm_host.cpp) and the gfx950 kernels (tm_kernels.hip).
//
// The reference keeps every index entry as an ETS ordered_set key
// {Words | Binary, {ID}} (apps/emqx/src/emqx_trie_search.erl:107-128) and walks
// it with ets:next/2.  Here the same key set is compiled into four
// open-addressing tables + two pools, all flat arrays of 4-byte words so the
// host can patch them in place and mirror the patches to HBM:
//
//   vocab  : word bytes  -> word id (wid)       32 B/entry, verified by bytes
//   edges  : (node, wid) -> child node           16 B/entry   (literal levels)
//   nodes  : per trie node: '+' child, '#'-terminal and exact-terminal value
//            ranges                              32 B/node
//   exact  : wid sequence -> value range         64 B/entry   (binary keys)
//   vals   : u32 values (caller IDs), one sorted run per terminal
//   wpool  : bytes of words longer than 16 B; wseq: wid runs of exact keys
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
constexpr uint32_t VINL = 16;   // inline word bytes in a vocab entry
constexpr uint32_t XINL = 10;   // inline wids in an exact entry

struct alignas(16) VocabEntry {   // 32 B
    uint32_t h_lo, h_hi;           // 64-bit word hash
    uint32_t wid;                  // NONE = empty slot
    uint32_t len;                  // word length in bytes
    uint32_t b[4];                 // len <= 16: the bytes, little endian, zero padded
                                   // len  > 16: b[0] = offset of the word in wpool
};

struct alignas(16) Edge {          // 16 B
    uint32_t parent;               // NONE = empty slot
    uint32_t wid;
    uint32_t child;
    uint32_t pad;
};

struct alignas(16) Node {          // 32 B
    uint32_t plus;                 // '+' child or NONE
    uint32_t hash_off, hash_cnt;   // values of filter <path>/#
    uint32_t exact_off, exact_cnt; // values of filter <path> (word-list form)
    uint32_t pad[3];
};

struct alignas(16) ExactEntry {    // 64 B
    uint32_t h_lo, h_hi;           // hash of the wid sequence
    uint32_t nlev;                 // NONE = empty slot
    uint32_t val_off, val_cnt;
    uint32_t seq_off;              // nlev > XINL: wids in wseq[seq_off ..)
    uint32_t wids[XINL];
};

static_assert(sizeof(VocabEntry) == 32, "vocab entry");
static_assert(sizeof(Edge) == 16, "edge");
static_assert(sizeof(Node) == 32, "node");
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

TM_HD uint64_t word_hash_finish(uint64_t fnv, uint32_t len) { return mix64(fnv ^ ((uint64_t)len << 56)); }

TM_HD uint32_t edge_slot(uint32_t parent, uint32_t wid, uint32_t mask) {
    return (uint32_t)mix64(((uint64_t)parent << 32) | wid) & mask;
}

TM_HD uint64_t seq_hash_step(uint64_t h, uint32_t wid) { return (h ^ wid) * FNV_PRIME; }
TM_HD uint64_t seq_hash_finish(uint64_t h, uint32_t nlev) { return mix64(h + 0x9e3779b97f4a7c15ull * (nlev + 1)); }

}  // namespace tmx
