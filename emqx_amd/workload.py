"""Synthetic workloads of BASELINE.json's configs (ctypes over libtmwork.so).

Bench / test infrastructure: generates filter, topic and delta sets as
(blob, offsets, values, flags) numpy arrays.  See emqx_amd/csrc/workload.cpp
for the exact shapes; seeds are 0x454D5158 + config index.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .build import LIB_WORK

SEED_BASE = 0x454D5158


class _Set(C.Structure):
    _fields_ = [("bytes", C.POINTER(C.c_uint8)), ("offs", C.POINTER(C.c_uint64)),
                ("vals", C.POINTER(C.c_uint32)), ("flags", C.POINTER(C.c_uint8)),
                ("n", C.c_uint64), ("nbytes", C.c_uint64)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        if not LIB_WORK.exists():
            from .build import build_work
            build_work()
        lib = C.CDLL(str(LIB_WORK))
        P = C.POINTER(_Set)
        lib.tmw_filters.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, P]
        lib.tmw_topics.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, P]
        lib.tmw_deltas.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, P]
        lib.tmw_free.argtypes = [P]
        for f in (lib.tmw_filters, lib.tmw_topics, lib.tmw_deltas):
            f.restype = C.c_int
        _lib = lib
    return _lib


class ItemSet:
    """blob (u8, 16 B of zero padding), offs (u64[n+1]), vals (u32[n]), flags (u8[n])."""

    def __init__(self, blob, offs, vals, flags):
        self.blob, self.offs, self.vals, self.flags = blob, offs, vals, flags

    def __len__(self):
        return len(self.offs) - 1

    def item(self, i) -> bytes:
        return self.blob[int(self.offs[i]):int(self.offs[i + 1])].tobytes()

    def items(self):
        return [self.item(i) for i in range(len(self))]

    def slice(self, lo, hi) -> "ItemSet":
        b0, b1 = int(self.offs[lo]), int(self.offs[hi])
        blob = np.concatenate([self.blob[b0:b1], np.zeros(16, np.uint8)])
        return ItemSet(blob, self.offs[lo:hi + 1] - np.uint64(b0), self.vals[lo:hi].copy(), self.flags[lo:hi].copy())


def take(s: ItemSet, idx) -> ItemSet:
    """The items s[idx] (idx: ascending int array) as a new packed set."""
    idx = np.asarray(idx, dtype=np.int64)
    starts = s.offs[idx].astype(np.int64)
    lens = (s.offs[idx + 1] - s.offs[idx]).astype(np.int64)
    offs = np.zeros(len(idx) + 1, np.uint64)
    np.cumsum(lens, out=offs[1:].view(np.int64))
    total = int(offs[-1])
    pos = np.repeat(starts - offs[:-1].astype(np.int64), lens) + np.arange(total, dtype=np.int64)
    blob = np.concatenate([s.blob[pos], np.zeros(16, np.uint8)])
    return ItemSet(blob, offs, s.vals[idx].copy(), s.flags[idx].copy())


def concat(sets) -> ItemSet:
    """The items of several packed sets, in order, as one set."""
    sets = list(sets)
    if not sets:
        return ItemSet(np.zeros(16, np.uint8), np.zeros(1, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
    blobs, offs, base = [], [np.zeros(1, np.uint64)], 0
    for x in sets:
        nb = int(x.offs[-1])
        blobs.append(x.blob[:nb])
        offs.append(x.offs[1:] + np.uint64(base))
        base += nb
    blobs.append(np.zeros(16, np.uint8))
    return ItemSet(np.concatenate(blobs), np.concatenate(offs), np.concatenate([x.vals for x in sets]),
                   np.concatenate([x.flags for x in sets]))


def _take(s: _Set) -> ItemSet:
    n, nb = s.n, s.nbytes
    blob = np.ctypeslib.as_array(s.bytes, shape=(nb + 16,)).copy()
    offs = np.ctypeslib.as_array(s.offs, shape=(n + 1,)).copy()
    vals = np.ctypeslib.as_array(s.vals, shape=(max(n, 1),))[:n].copy()
    flags = np.ctypeslib.as_array(s.flags, shape=(max(n, 1),))[:n].copy()
    _load().tmw_free(C.byref(s))
    return ItemSet(blob, offs, vals, flags)


def config_seed(cfg: int) -> int:
    return SEED_BASE + {1: 0, 2: 1, 20: 1, 3: 2, 30: 2, 4: 3, 5: 4}[cfg]


def filters(cfg: int, n: int, seed: int | None = None, shard: int = 0, nshards: int = 1) -> ItemSet:
    """cfg 1, 2, 20 (C2 with non-matching globals) or 3 (also the C3deep/C4/C5 base)."""
    s = _Set()
    gen_cfg = 3 if cfg in (4, 5, 30) else cfg
    rc = _load().tmw_filters(gen_cfg, config_seed(cfg) if seed is None else seed, n, shard, nshards, C.byref(s))
    if rc:
        raise ValueError("tmw_filters failed")
    return _take(s)


def topics(cfg: int, n_filters: int, n: int, first: int = 0, seed: int | None = None) -> ItemSet:
    s = _Set()
    gen_cfg = 3 if cfg in (4, 5) else (2 if cfg == 20 else cfg)
    rc = _load().tmw_topics(gen_cfg, config_seed(cfg) if seed is None else seed, n_filters, first, n, C.byref(s))
    if rc:
        raise ValueError("tmw_topics failed")
    return _take(s)


def deltas(n_filters: int, first: int, n: int, seed: int | None = None) -> ItemSet:
    """C5 churn: flags = 1 subscribe / 0 unsubscribe; vals = key value."""
    s = _Set()
    rc = _load().tmw_deltas(config_seed(5) if seed is None else seed, n_filters, first, n, C.byref(s))
    if rc:
        raise ValueError("tmw_deltas failed")
    return _take(s)
