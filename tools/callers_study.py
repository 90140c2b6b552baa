#!/usr/bin/env python3
"""Native caller threads (emqx_amd/csrc/hostbench.cpp tmb_callers) against a
C3 index: aggregate topics/s and p50/p99 per batch for 1..16 threads, with and
without a delta-churn thread, and single-caller latency per batch size.
usage: callers_study.py [--filters N] [--batch 4096] [--seconds 1.0]"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--seconds", type=float, default=1.0)
    p.add_argument("--threads", default="1,2,4,8,16")
    a = p.parse_args()
    import torch
    assert torch.cuda.is_available()
    from bench import host_bench_lib
    from emqx_amd import _native, workload as wl
    fs = wl.filters(3, a.filters)
    ix = _native.Index(device=0, hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    hb = host_bench_lib()
    nmax = max(int(x) for x in a.threads.split(","))
    ts = wl.topics(3, a.filters, nmax * a.batch)
    for lb in (1, 64, 1024, 4096, 16384, 65536):
        sub = ts.slice(0, lb)
        hh, _, _ = ix.match_batch(sub.blob, sub.offs)
        out = (ctypes.c_double * 3)()
        assert hb.tmb_single(ix._h, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096, 200,
                             out) == 0
        print(json.dumps({"single": lb, "p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4)}), flush=True)
    for churn in (0, 256):
        for nth in (int(x) for x in a.threads.split(",")):
            sub = ts.slice(0, nth * a.batch)
            hh, _, _ = ix.match_batch(sub.blob, sub.offs)
            cap = int(np.diff(hh.astype(np.int64)).reshape(nth, a.batch).sum(axis=1).max()) + 65536
            out = (ctypes.c_double * 6)()
            assert hb.tmb_callers(ix._h, nth, a.batch, _native._ptr(sub.blob), _native._ptr(sub.offs), cap,
                                  a.seconds, churn, out) == 0
            print(json.dumps({"threads": nth, "churn_ops_per_ms": churn, "batches": int(out[0]),
                              "topics_per_s": round(out[1], 1), "p50_ms": round(out[2], 4),
                              "p99_ms": round(out[3], 4), "deltas_per_s": round(out[4], 1)}), flush=True)


if __name__ == "__main__":
    main()
