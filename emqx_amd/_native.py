"""ctypes binding of ``libtmatch.so`` (the C ABI in ``include/tmatch.h``).

This is the only way the Python host layer reaches the match path.  There is
no fallback: if the library is missing or no GPU is visible, calls raise
:class:`NativeUnavailable` (the product path never routes through a CPU
implementation).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from .build import LIB_TMATCH

TM_OK, TM_EINVAL, TM_ENOMEM, TM_EDEVICE, TM_ECAP = 0, -1, -2, -3, -4
TM_OP_DELETE, TM_OP_INSERT = 0, 1
TM_KEY_BINARY, TM_KEY_WORDS, TM_KEY_EMPTY_LIST, TM_KEY_ESCAPED = 0, 1, 2, 4
TM_ORDER_TRAVERSAL, TM_ORDER_SORTED, TM_ORDER_UNIQUE = 0, 1, 2

# every symbol include/tmatch.h declares (tests check the export table)
EXPORTS = ("tm_create", "tm_destroy", "tm_apply_deltas", "tm_sync", "tm_match_batch",
           "tm_match_batch_dev", "tm_first_batch", "tm_stats", "tm_profile_enable", "tm_profile_read",
           "tm_last_error", "tm_abi_version", "tm_merge_shards", "tm_host_alloc", "tm_host_free",
           "tm_stream_release", "tm_match_batch_ex", "tm_match_batch_dev_ex", "tm_sort_segments",
           "tm_matches_filter", "tm_apply_deltas_ex", "tm_read_begin", "tm_read_end", "tm_epoch",
           "tm_create_replicas", "tm_replica_stats", "tm_debug_set", "tm_debug_get", "tm_match_batch32_ex",
           "tm_match_batch32_dev", "tm_matches_filter_ex", "tm_host_alloc_ex", "tm_commit",
           "tm_match_batch32_pairs", "tm_match_batch_dev_pairs")
TM_ALLOC_VRAM = 1
TM_DEBUG_LB_SPINS, TM_DEBUG_LB_FAIL_BLOCK, TM_DEBUG_LB_LAUNCHES, TM_DEBUG_PHASES = 1, 2, 3, 4
TM_DEBUG_FAILED_BATCHES, TM_DEBUG_RETRIED_BATCHES = 5, 6
TM_DEBUG_PATH_PHASES, TM_DEBUG_PATH_SMALL, TM_DEBUG_PATH_LANE = 7, 8, 9
TM_DEBUG_SMALL_KERNEL = 10
SMALL_AUTO, SMALL_WAVE, SMALL_WAVE8 = 0, 1, 3   # (2: round 5's lane kernel, removed)
TM_DEBUG_COMBINE, TM_DEBUG_COMBINED_LAUNCHES, TM_DEBUG_COMBINED_BATCHES = 12, 13, 14
TM_DEBUG_WIDE_NODES, TM_DEBUG_DENSE_WIDE = 15, 16
TM_DEBUG_CMB_GATHER, TM_DEBUG_CMB_LAND = 17, 18
TM_DEBUG_COMMITS, TM_DEBUG_COMMIT_WAITS, TM_DEBUG_COMMIT_FORCED = 19, 20, 21
TM_DEBUG_SMALL_TICKET = 22
TM_DEBUG_CMB_SPIN = 23
TM_DEBUG_PATCH_ZC = 24


class NativeUnavailable(RuntimeError):
    pass


class TmError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"tmatch error {code}: {msg}")
        self.code = code


class DeviceError(TmError):
    """TM_EDEVICE: the GPU failed the call (e.g. a batch whose look-back wait
    expired twice, include/tmatch.h err flag 4).  Never a client error: the
    reference raises badarg only for a '+'/'#' topic level
    (emqx_trie_search.erl:374-375)."""


class tm_options(C.Structure):
    _fields_ = [("device", C.c_int32), ("copies", C.c_uint32), ("hint_keys", C.c_uint64)]


class tm_stats_t(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_keys", "n_wild_keys", "n_exact_keys", "n_dead_keys",
                                          "n_nodes", "n_edges", "n_words", "device_bytes",
                                          "uploads", "patch_bytes")]


_lib = None


def load_library(path: Path | None = None):
    """Load libtmatch.so (does not touch the GPU)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    import os
    # TM_LIB: an experimental build of the same library (emqx_amd.build.build_variant)
    p = Path(path) if path else Path(os.environ.get("TM_LIB", LIB_TMATCH))
    if not p.exists():
        raise NativeUnavailable(f"{p} is not built (run emqx_amd.build.build_all())")
    lib = C.CDLL(str(p))
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    sig = {
        "tm_create": (i32, [C.POINTER(tm_options), C.POINTER(vp)]),
        "tm_destroy": (i32, [vp]),
        "tm_apply_deltas": (i32, [vp, u64, vp, vp, vp, vp, vp]),
        "tm_sync": (i32, [vp, vp]),
        "tm_match_batch": (i32, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "tm_match_batch_dev": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, vp]),
        "tm_first_batch": (i32, [vp, u64, vp, vp, vp, vp]),
        "tm_matches_filter": (i32, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "tm_matches_filter_ex": (i32, [vp, u64, vp, vp, vp, vp, vp, u64, vp]),
        "tm_stats": (i32, [vp, C.POINTER(tm_stats_t)]),
        "tm_profile_enable": (i32, [vp, i32]),
        "tm_profile_read": (i32, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(u64), i32]),
        "tm_last_error": (C.c_char_p, [vp]),
        "tm_abi_version": (u32, []),
        "tm_merge_shards": (i32, [u32, u64, vp, vp, u64, vp, vp, u64, vp]),
        "tm_host_alloc": (i32, [vp, u64, C.POINTER(vp)]),
        "tm_host_free": (i32, [vp, vp]),
        "tm_host_alloc_ex": (i32, [vp, u64, u32, C.POINTER(vp)]),
        "tm_stream_release": (i32, [vp, vp]),
        "tm_match_batch_ex": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, u32, vp]),
        "tm_match_batch_dev_ex": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, u32, vp, vp]),
        "tm_match_batch_dev_pairs": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, vp]),
        "tm_sort_segments": (i32, [vp, u64, vp, vp, u64, u32, vp, vp]),
        "tm_apply_deltas_ex": (i32, [vp, u64, vp, vp, vp, vp, vp, C.POINTER(u64)]),
        "tm_commit": (i32, [vp, u64, vp, vp, vp, vp, vp, C.POINTER(u64)]),
        "tm_read_begin": (i32, [vp, C.POINTER(u64)]),
        "tm_read_end": (i32, [vp, u64]),
        "tm_epoch": (i32, [vp, C.POINTER(u64), C.POINTER(u64)]),
        "tm_create_replicas": (i32, [C.POINTER(tm_options), C.POINTER(C.c_int32), u32, C.POINTER(vp)]),
        "tm_replica_stats": (i32, [vp, u32, C.POINTER(u64), C.POINTER(C.c_int32)]),
        "tm_match_batch32_ex": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, u32, vp]),
        "tm_match_batch32_dev": (i32, [vp, u64, vp, vp, vp, vp, u64, vp, vp]),
        "tm_match_batch32_pairs": (i32, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "tm_debug_set": (i32, [vp, u32, u64]),
        "tm_debug_get": (i32, [vp, u32, C.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        try:
            f = getattr(lib, name)
        except AttributeError:
            if p == LIB_TMATCH:
                raise
            continue   # (an older TM_LIB study build: newer entry points absent)
        f.restype, f.argtypes = res, args
    if path is None:
        _lib = lib
    return lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _gpu_present() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def merge_shards(world: int, n: int, d_shard_hit: int, d_shard_vals: int, stride: int, d_out_hit: int,
                 d_out_vals: int, cap: int, stream: int | None = None):
    """tm_merge_shards on device pointers (filter-sharded mode)."""
    if not _gpu_present():
        raise NativeUnavailable("no HIP device visible: the shard merge runs on the GPU only")
    lib = load_library()
    rc = lib.tm_merge_shards(world, n, d_shard_hit, d_shard_vals, stride, d_out_hit, d_out_vals, cap, stream)
    if rc != TM_OK:
        raise TmError(rc, lib.tm_last_error(None).decode())


def pack_strings(items) -> tuple[np.ndarray, np.ndarray]:
    """bytes-likes -> (uint8 blob, uint64 offsets[n+1])."""
    items = [bytes(x) for x in items]
    offs = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        offs[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    blob = np.frombuffer(b"".join(items) + b"\0" * 16, dtype=np.uint8)
    return blob, offs


class Index:
    """Owning handle of one device-resident topic index (tm_index*)."""

    def __init__(self, device: int = -1, hint_keys: int = 0, devices=None, copies: int = 1):
        """devices: a list of HIP devices -> one host image with a replica on
        each (tm_create_replicas); otherwise one device.  copies: copies of the
        tables per device (tm_options.copies: deltas never wait for batches in
        flight on another copy)."""
        if not _gpu_present():
            raise NativeUnavailable("no HIP device visible: the topic index runs on the GPU only")
        self._lib = load_library()
        opts = tm_options(device, copies, hint_keys)
        h = C.c_void_p()
        if devices is not None:
            devs = (C.c_int32 * len(devices))(*devices)
            rc = self._lib.tm_create_replicas(C.byref(opts), devs, len(devices), C.byref(h))
        else:
            rc = self._lib.tm_create(C.byref(opts), C.byref(h))
        if rc != TM_OK:
            raise TmError(rc, self._lib.tm_last_error(None).decode())
        self._h = h

    def _check(self, rc):
        if rc != TM_OK:
            cls = DeviceError if rc == TM_EDEVICE else TmError
            raise cls(rc, self._lib.tm_last_error(self._h).decode())

    def close(self):
        if getattr(self, "_h", None):
            self._pinned = []   # tm_destroy frees the tm_host_alloc buffers
            self._lib.tm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- deltas
    def apply(self, ops: np.ndarray, blob: np.ndarray, offs: np.ndarray, values: np.ndarray,
              flags: np.ndarray | None = None, commit: bool = False):
        """tm_apply_deltas_ex, or (commit) tm_commit: published on a table copy no
        batch is reading, so no batch waits for the patch.  -> the delta epoch."""
        ops = np.ascontiguousarray(ops, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        values = np.ascontiguousarray(values, dtype=np.uint32)
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        if flags is not None:
            flags = np.ascontiguousarray(flags, dtype=np.uint8)
        e = C.c_uint64()
        fn = self._lib.tm_commit if commit else self._lib.tm_apply_deltas_ex
        self._check(fn(self._h, len(ops), _ptr(ops), _ptr(blob), _ptr(offs), _ptr(values), _ptr(flags), C.byref(e)))
        return e.value

    # ---- reader epochs (include/tmatch.h "Reader epochs")
    def read_begin(self) -> int:
        t = C.c_uint64()
        self._check(self._lib.tm_read_begin(self._h, C.byref(t)))
        return t.value

    def read_end(self, ticket: int):
        self._check(self._lib.tm_read_end(self._h, ticket))

    def epoch(self) -> tuple[int, int]:
        """-> (current epoch, safe epoch: the oldest running reader's, or current)."""
        cur, safe = C.c_uint64(), C.c_uint64()
        self._check(self._lib.tm_epoch(self._h, C.byref(cur), C.byref(safe)))
        return cur.value, safe.value

    def sync(self, stream: int | None = None):
        self._check(self._lib.tm_sync(self._h, stream))

    # ---- pinned host buffers (tm_host_alloc)
    def host_array(self, n: int, dtype, vram: bool = False) -> np.ndarray:
        """A numpy array in pinned host memory mapped into the device.  Batches
        whose buffers (topics 16-byte aligned, offsets, outputs) all come from
        here run in place, without staging copies (include/tmatch.h).  Valid
        until host_free() or close().  vram: device memory mapped into the host
        (TM_ALLOC_VRAM) for a batch's inputs -- write it, never read it back
        (each host read is an uncached PCIe round trip)."""
        dtype = np.dtype(dtype)
        nbytes = max(int(n), 1) * dtype.itemsize
        p = C.c_void_p()
        self._check(self._lib.tm_host_alloc_ex(self._h, nbytes, TM_ALLOC_VRAM if vram else 0, C.byref(p)))
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        a = np.frombuffer(buf, dtype=dtype, count=max(int(n), 1))
        if not hasattr(self, "_pinned"):
            self._pinned = []
        self._pinned.append(p.value)
        return a

    def host_free(self, a: np.ndarray):
        addr = a.__array_interface__["data"][0]
        self._check(self._lib.tm_host_free(self._h, C.c_void_p(addr)))
        self._pinned.remove(addr)

    # ---- matching (host buffers)
    def match_batch(self, blob: np.ndarray, offs: np.ndarray, cap: int | None = None, out=None,
                    order: int = TM_ORDER_TRAVERSAL, unique_counts: np.ndarray | None = None):
        """-> (hit_offsets u64[n+1], values u32[total], err u8[n]), each topic's
        values in `order` (traversal by default; TM_ORDER_SORTED ascending;
        TM_ORDER_UNIQUE ascending distinct values first, padded with
        0xFFFFFFFF, the distinct count per topic in `unique_counts`).

        `out` = (hit u64[>= n+1], values u32[cap], err u8[>= n]): caller-owned
        buffers reused across batches (what a NIF keeps per scheduler); the
        results are views into them.  Without it fresh arrays are allocated."""
        n = len(offs) - 1
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        if unique_counts is not None and (len(unique_counts) < n or unique_counts.dtype != np.uint32):
            raise ValueError("match_batch: unique_counts too small or not uint32")
        uc = _ptr(unique_counts)
        if out is not None:
            hit, vals, err = out
            if len(hit) < n + 1 or len(err) < n or hit.dtype != np.uint64 or vals.dtype != np.uint32 \
                    or err.dtype != np.uint8:
                raise ValueError("match_batch: out buffers too small or of the wrong dtype")
            rc = self._lib.tm_match_batch_ex(self._h, n, _ptr(blob), _ptr(offs), _ptr(hit), _ptr(vals), len(vals),
                                             _ptr(err), order, uc)
            self._check(rc)
            return hit[: n + 1], vals[: int(hit[n])], err[:n]
        hit = np.zeros(n + 1, dtype=np.uint64)
        err = np.zeros(max(n, 1), dtype=np.uint8)
        if cap is None:
            cap = max(4 * n, 1024)
        while True:
            out = np.empty(max(cap, 1), dtype=np.uint32)
            rc = self._lib.tm_match_batch_ex(self._h, n, _ptr(blob), _ptr(offs), _ptr(hit), _ptr(out), cap, _ptr(err),
                                             order, uc)
            if rc == TM_ECAP:
                cap = int(hit[n])
                continue
            self._check(rc)
            return hit, out[: int(hit[n])], err[:n]

    def match_batch32(self, blob: np.ndarray, offs: np.ndarray, out, order: int = TM_ORDER_TRAVERSAL,
                      unique_counts: np.ndarray | None = None):
        """tm_match_batch32_ex: u32 topic offsets in, u32 hit offsets out.
        out = (hit u32[>= n+1], values u32[cap], err u8[>= n]); in place when
        every buffer comes from host_array() (a NIF's pooled buffers).  Raises
        TmError(TM_ECAP) when the values do not fit (hit offsets valid)."""
        n = len(offs) - 1
        hit, vals, err = out
        if offs.dtype != np.uint32 or hit.dtype != np.uint32 or len(hit) < n + 1 or len(err) < n:
            raise ValueError("match_batch32: u32 offsets and large enough outputs expected")
        self._check(self._lib.tm_match_batch32_ex(self._h, n, _ptr(blob), _ptr(offs), _ptr(hit), _ptr(vals), len(vals),
                                                  _ptr(err), order, _ptr(unique_counts)))
        return hit[: n + 1], vals[: int(hit[n])], err[:n]

    def match_batch32_pairs(self, blob: np.ndarray, offs: np.ndarray, out):
        """tm_match_batch32_pairs: u32 topic offsets in; out = (pairs u32[>= 2n+1],
        values u32[cap], err u8[>= n]) -> (pairs[:2n+1], values, err[:n]);
        topic i's values are values[pairs[2i] : pairs[2i] + pairs[2i+1]]
        (disjoint spans, not in topic order).  In place, through the combiner,
        when every buffer comes from host_array()."""
        n = len(offs) - 1
        pairs, vals, err = out
        if offs.dtype != np.uint32 or pairs.dtype != np.uint32 or len(pairs) < 2 * n + 1 or len(err) < n:
            raise ValueError("match_batch32_pairs: u32 offsets and large enough outputs expected")
        self._check(self._lib.tm_match_batch32_pairs(self._h, n, _ptr(blob), _ptr(offs), _ptr(pairs), _ptr(vals),
                                                     len(vals), _ptr(err)))
        return pairs[: 2 * n + 1], vals, err[:n]

    def match_batch32_dev(self, n: int, d_blob: int, d_offs: int, d_hit: int, d_out: int, cap: int, d_err: int,
                          stream: int | None = None):
        self._check(self._lib.tm_match_batch32_dev(self._h, n, d_blob, d_offs, d_hit, d_out, cap, d_err, stream))

    def first_batch(self, blob: np.ndarray, offs: np.ndarray):
        """-> (value u32[n], found u8[n]: 1 hit, 0 none, 2 badarg, 3 > 65536 levels)."""
        n = len(offs) - 1
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        val = np.zeros(max(n, 1), dtype=np.uint32)
        found = np.zeros(max(n, 1), dtype=np.uint8)
        self._check(self._lib.tm_first_batch(self._h, n, _ptr(blob), _ptr(offs), _ptr(val), _ptr(found)))
        return val[:n], found[:n]

    def matches_filter_batch(self, blob: np.ndarray, offs: np.ndarray, flags: np.ndarray | None = None):
        """matches_filter/3 for n subscription filters on the device (tm_matches_filter_ex;
        flags: TM_KEY_ESCAPED per filter given as an escaped word list, or None):
        -> (hit_offsets u64[n+1], values u32 in traversal order, err u8[n])."""
        n = len(offs) - 1
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        if flags is not None:
            flags = np.ascontiguousarray(flags, dtype=np.uint8)
        hit = np.zeros(n + 1, dtype=np.uint64)
        err = np.zeros(max(n, 1), dtype=np.uint8)
        cap = 1024
        while True:
            out = np.zeros(max(cap, 1), dtype=np.uint32)
            rc = self._lib.tm_matches_filter_ex(self._h, n, _ptr(blob), _ptr(offs), _ptr(flags), _ptr(hit), _ptr(out),
                                                cap, _ptr(err))
            if rc == TM_ECAP and int(hit[n]) > cap:
                cap = int(hit[n])
                continue
            self._check(rc)
            return hit, out[: int(hit[n])], err[:n]

    # ---- matching (device buffers, e.g. torch tensors' data_ptr())
    def match_batch_dev(self, n: int, d_blob: int, d_offs: int, d_hit: int, d_out: int, cap: int, d_err: int,
                        stream: int | None = None, order: int = TM_ORDER_TRAVERSAL, d_unique: int | None = None):
        self._check(self._lib.tm_match_batch_dev_ex(self._h, n, d_blob, d_offs, d_hit, d_out, cap, d_err, order,
                                                    d_unique, stream))

    def match_batch_dev_pairs(self, n: int, d_blob: int, d_offs: int, d_pairs: int, d_out: int, cap: int, d_err: int,
                              stream: int | None = None):
        """tm_match_batch_dev_pairs: per-topic (first position, count) u32 pairs, d_pairs[2 n] = total."""
        self._check(self._lib.tm_match_batch_dev_pairs(self._h, n, d_blob, d_offs, d_pairs, d_out, cap, d_err, stream))

    def sort_segments(self, n: int, d_hit: int, d_vals: int, cap: int, order: int = TM_ORDER_SORTED,
                      d_unique: int | None = None, stream: int | None = None):
        """tm_sort_segments: sort each of n CSR segments on the device in place."""
        self._check(self._lib.tm_sort_segments(self._h, n, d_hit, d_vals, cap, order, d_unique, stream))

    def release_stream(self, stream: int | None):
        """Drop the batch scratch the library keeps for `stream`."""
        self._check(self._lib.tm_stream_release(self._h, stream))

    def profile(self, enable: bool = True):
        self._check(self._lib.tm_profile_enable(self._h, int(enable)))

    def profile_read(self, reset: bool = True):
        """-> (walk kernel ms, whole batch ms, batches) accumulated on the device."""
        w, b, n = C.c_double(), C.c_double(), C.c_uint64()
        self._check(self._lib.tm_profile_read(self._h, C.byref(w), C.byref(b), C.byref(n), int(reset)))
        return w.value, b.value, n.value

    def replica_stats(self, r: int) -> tuple[int, int]:
        """-> (host-API batches replica r served, its device)."""
        b, d = C.c_uint64(), C.c_int32()
        self._check(self._lib.tm_replica_stats(self._h, r, C.byref(b), C.byref(d)))
        return b.value, d.value

    def debug_set(self, key: int, value: int):
        """tm_debug_set (test hooks, include/tmatch.h)."""
        self._check(self._lib.tm_debug_set(self._h, key, value))

    def debug_get(self, key: int) -> int:
        v = C.c_uint64()
        self._check(self._lib.tm_debug_get(self._h, key, C.byref(v)))
        return v.value

    def stats(self) -> dict:
        s = tm_stats_t()
        self._check(self._lib.tm_stats(self._h, C.byref(s)))
        return {k: getattr(s, k) for k, _ in tm_stats_t._fields_}
