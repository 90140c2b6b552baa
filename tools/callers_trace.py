#!/usr/bin/env python3
"""Kernel-trace driver for concurrent callers: a C3 index, then `--threads`
native caller threads (tmb_callers, no churn) for a short while, so a
rocprofv3 kernel trace shows whether their kernels overlap on the device.
usage: callers_trace.py [--threads 4] [--seconds 0.3] [--filters N]"""
import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--threads", type=int, default=4)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--seconds", type=float, default=0.3)
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
    ts = wl.topics(3, a.filters, a.threads * a.batch)
    hh, _, _ = ix.match_batch(ts.blob, ts.offs)
    cap = int(hh[-1]) + 65536
    out = (ctypes.c_double * 6)()
    assert hb.tmb_callers(ix._h, a.threads, a.batch, _native._ptr(ts.blob), _native._ptr(ts.offs), cap, a.seconds, 0,
                          out) == 0
    print(f"threads {a.threads}: {out[1]:.3e} topics/s p50 {out[2]:.3f} ms p99 {out[3]:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
