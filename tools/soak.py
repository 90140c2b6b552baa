#!/usr/bin/env python3
"""Concurrent-caller soak (study tool, not product code): one C3 index, then
`--callers` native threads of 4k-topic batches with one more thread applying
256-delta batches every millisecond, for `--seconds` per call placement
(tmb_callers_ex modes: 4 = u32 offsets, host buffers, CSR; 5 = inputs in
TM_ALLOC_VRAM, CSR; 6 = inputs in VRAM, pairs -- the NIF's call), one JSON line
each, with the look-back failures and reruns the library counted meanwhile
(k_walk_small's start-order ticket is the default since round 6: none should
fail).  usage: soak.py [--seconds 60] [--callers 16] [--modes 4,5,6]"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--seconds", type=float, default=60.0)
    p.add_argument("--callers", type=int, default=16)
    p.add_argument("--modes", default="4,5,6")
    p.add_argument("--churn", type=int, default=256, help="deltas per millisecond from one more thread")
    p.add_argument("--copies", type=int, default=2)
    a = p.parse_args()
    import torch
    assert torch.cuda.is_available()
    from bench import host_bench_lib
    from emqx_amd import _native, workload as wl
    fs = wl.filters(3, a.filters)
    ix = _native.Index(device=0, hint_keys=len(fs), copies=a.copies)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    hb = host_bench_lib()
    lb = 4096
    ts = wl.topics(3, a.filters, a.callers * lb)
    hh, _, _ = ix.match_batch(ts.blob, ts.offs)
    cap = int(np.diff(hh.astype(np.int64)).reshape(a.callers, lb).sum(axis=1).max()) + 65536
    keys = (_native.TM_DEBUG_FAILED_BATCHES, _native.TM_DEBUG_RETRIED_BATCHES)
    for mode in [int(x) for x in a.modes.split(",")]:
        f0 = [ix.debug_get(k) for k in keys]
        out = (ctypes.c_double * 6)()
        t = time.time()
        rc = hb.tmb_callers_ex(ix._h, a.callers, lb, _native._ptr(ts.blob), _native._ptr(ts.offs), cap, a.seconds,
                               a.churn, mode, out)
        assert rc == 0, rc
        f1 = [ix.debug_get(k) for k in keys]
        print(json.dumps({"mode": mode, "callers": a.callers, "seconds": round(time.time() - t, 1),
                          "small_ticket": ix.debug_get(_native.TM_DEBUG_SMALL_TICKET), "copies": a.copies,
                          "batches": int(out[0]), "topics": int(out[0]) * lb, "topics_per_s": round(out[1], 1),
                          "p50_ms": round(out[2], 4), "p99_ms": round(out[3], 4), "deltas_per_s": round(out[4], 1),
                          "failed_batches": f1[0] - f0[0], "retried_batches": f1[1] - f0[1]}), flush=True)


if __name__ == "__main__":
    main()
