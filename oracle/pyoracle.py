"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
checker / timed CPU reference.  The product (emqx_amd/) never imports this.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "liboracle.so"
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            import subprocess
            subprocess.run(["make", "-s", "liboracle.so"], cwd=LIB.parent, check=True)
        lib = C.CDLL(str(LIB))
        vp, u32, i64, u64 = C.c_void_p, C.c_uint32, C.c_int64, C.c_uint64
        lib.orc_new.restype = vp
        lib.orc_free.argtypes = [vp]
        lib.orc_insert.argtypes = [vp, C.c_char_p, u32, u32, C.c_int]
        lib.orc_delete.argtypes = [vp, C.c_char_p, u32, u32, C.c_int]
        lib.orc_apply.argtypes = [vp, i64, vp, vp, vp, vp, vp]
        lib.orc_size.argtypes = [vp]
        lib.orc_size.restype = i64
        lib.orc_prepare.argtypes = [vp]
        lib.orc_matches.argtypes = [vp, C.c_char_p, u32, vp, i64]
        lib.orc_matches.restype = i64
        lib.orc_matches_filter.argtypes = [vp, C.c_char_p, u32, vp, i64]
        lib.orc_matches_filter.restype = i64
        lib.orc_first.argtypes = [vp, C.c_char_p, u32, vp]
        lib.orc_first.restype = C.c_int
        lib.orc_match_batch.argtypes = [vp, vp, vp, i64, vp, vp, vp, vp, C.c_int]
        lib.orc_match_batch.restype = i64
        lib.orc_frontier_batch.argtypes = [vp, vp, vp, i64, vp, vp, C.c_int]
        lib.orc_spec_match.argtypes = [C.c_char_p, u32, C.c_char_p, u32, C.c_int]
        lib.orc_spec_match.restype = C.c_int
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    """The reference's ordered-set seek walker (emqx_trie_search) on the CPU."""

    def __init__(self):
        self._l = load()
        self._h = self._l.orc_new()

    def __del__(self):
        try:
            self._l.orc_free(self._h)
        except Exception:
            pass

    def insert(self, f: bytes, v: int, flags: int = 0):
        self._l.orc_insert(self._h, f, len(f), v, flags)

    def delete(self, f: bytes, v: int, flags: int = 0):
        self._l.orc_delete(self._h, f, len(f), v, flags)

    def apply(self, ops, blob, offs, vals, flags=None):
        ops = np.ascontiguousarray(ops, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        vals = np.ascontiguousarray(vals, np.uint32)
        blob = np.ascontiguousarray(blob, np.uint8)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint8)
        self._l.orc_apply(self._h, len(ops), _p(ops), _p(blob), _p(offs), _p(vals), _p(fl))

    def size(self) -> int:
        return self._l.orc_size(self._h)

    def prepare(self):
        self._l.orc_prepare(self._h)

    def matches(self, topic: bytes):
        """traversal-order values, or None for badarg"""
        cap = 64
        while True:
            out = np.empty(cap, np.uint32)
            r = self._l.orc_matches(self._h, topic, len(topic), _p(out), cap)
            if r < 0:
                return None
            if r <= cap:
                return out[:r].tolist()
            cap = int(r)

    def matches_filter(self, flt: bytes):
        """matches_filter/3 values in traversal order (the query split by filter_words/1)"""
        cap = 64
        while True:
            out = np.empty(cap, np.uint32)
            r = self._l.orc_matches_filter(self._h, flt, len(flt), _p(out), cap)
            if r <= cap:
                return out[:r].tolist()
            cap = int(r)

    def first(self, topic: bytes):
        """(found, value); found = -1 badarg, -2 more than 65536 levels, 0 false, 1 hit"""
        v = np.zeros(1, np.uint32)
        r = self._l.orc_first(self._h, topic, len(topic), _p(v))
        return r, int(v[0])

    def match_batch(self, blob, offs, nthreads: int = 8, with_values: bool = True):
        """-> (counts i64[n] (-1 badarg, -2 more than 65536 levels), hashes u64[n], hit_offs u64[n+1] | None, values | None)"""
        n = len(offs) - 1
        blob = np.ascontiguousarray(blob, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        counts = np.zeros(max(n, 1), np.int64)
        hashes = np.zeros(max(n, 1), np.uint64)
        self._l.orc_match_batch(self._h, _p(blob), _p(offs), n, _p(counts), _p(hashes), None, None, nthreads)
        if not with_values:
            return counts[:n], hashes[:n], None, None
        hit = np.zeros(n + 1, np.int64)
        hit[1:] = np.cumsum(np.maximum(counts[:n], 0))
        vals = np.empty(max(int(hit[n]), 1), np.uint32)
        self._l.orc_match_batch(self._h, _p(blob), _p(offs), n, None, None, _p(hit), _p(vals), nthreads)
        return counts[:n], hashes[:n], hit.astype(np.uint64), vals[: int(hit[n])]


def frontier(o: "Oracle", blob, offs, nthreads: int = 8):
    """-> (levels u32[n], sum_{l<L} |F_l| i64[n]) per topic (-1 = badarg)."""
    n = len(offs) - 1
    lv = np.zeros(max(n, 1), np.uint32)
    st = np.zeros(max(n, 1), np.int64)
    blob = np.ascontiguousarray(blob, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    o._l.orc_frontier_batch(o._h, _p(blob), _p(offs), n, _p(lv), _p(st), nthreads)
    return lv[:n], st[:n]


def spec_match(topic: bytes, flt: bytes, words_form: bool = False) -> bool:
    """emqx_topic:match/2 restated (brute-force oracle)."""
    return bool(load().orc_spec_match(topic, len(topic), flt, len(flt), int(words_form)))


# ------------------------------------------------------------ matches_filter
#
# The reference's ordered matches_filter/3 walk restated in Python over a
# sorted key list (emqx_trie_search.erl:186-253 with the filter clauses of
# compare/3, :260-348): a second, independent restatement next to
# tm_oracle.c's orc_matches_filter, for tests/test_matches_filter_cpu.py.  The
# product runs this walk on the device only (tm_matches_filter_ex).

from emqx_amd.trie_search import HASH, PLUS, term_key  # noqa: E402

FULL, PREFIX, LOWER = "match_full", "match_prefix", "lower"


def compare_filter(f, w):
    """compare/3 (emqx_trie_search.erl:260-348) with a FILTER query `w`: the
    filter clauses (:291-300) come before the stored-'+' clause, so a query '+'
    passes any stored word over without turning a later 'lower' into a seek.
    -> FULL / PREFIX / LOWER / seek position (int)."""
    if not isinstance(f, tuple):
        return LOWER                                         # :260-261 binary key
    lastplus = -1
    i = 0
    while True:
        if i == len(f):
            return FULL if i == len(w) else PREFIX           # :262-281
        if f[i] == HASH and i == len(f) - 1:
            return FULL                                      # :282-290
        if i < len(w) and w[i] == HASH and i == len(w) - 1:
            return FULL                                      # :292-293
        if i == len(w):
            break                                            # :333-340 lower
        if w[i] == PLUS:
            i += 1                                           # :294-300
            continue
        if f[i] == PLUS:
            lastplus = i                                     # :302-320
            i += 1
            continue
        a, b = term_key(f[i]), term_key(w[i])
        if a == b:
            i += 1                                           # :321-324
            continue
        if a > b:
            break                                            # :325-332 lower
        return i                                             # :341-348 seek
    return lastplus if lastplus >= 0 else LOWER


def _base_order(prefix):
    """order key of base(Prefix) = {Prefix, {}}: before every {Prefix, {ID}}"""
    return ((8, tuple(term_key(x) for x in prefix)), (-1,))


def search_filter(keys, order, words):
    """matches_filter's ordered search (emqx_trie_search.erl:186-253, no
    match_topics phase) over `keys` sorted in term order (`order[i]` =
    key_order(keys[i])).  -> matching keys in traversal order."""
    import bisect
    base = (words[0],) if words and isinstance(words[0], bytes) and words[0][:1] == b"$" else ()   # :160-163
    cur = bisect.bisect_right(order, _base_order(base))
    out = []
    while cur < len(keys):
        k = keys[cur]
        r = compare_filter(k[0], words)
        if r == FULL:
            out.append(k)
            cur = bisect.bisect_right(order, order[cur])
        elif r == PREFIX:
            cur = bisect.bisect_right(order, order[cur])
        elif r == LOWER:
            break
        else:
            cur = bisect.bisect_right(order, _base_order(tuple(k[0][:r]) + (words[r],)))   # seek/3 :255-258
    return out
