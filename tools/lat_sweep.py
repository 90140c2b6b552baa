#!/usr/bin/env python3
"""Single-caller host-to-host latency sweep (study tool): tmb_single (buffers
from tm_host_alloc, batch run in place) at several batch sizes on a C3 index;
TM_LIB selects a study build.  usage: lat_sweep.py [--sizes 4096,8192,...]"""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--sizes", default="4096,8192,16384,32768,65536")
    p.add_argument("--iters", type=int, default=100)
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
    sizes = [int(x) for x in a.sizes.split(",")]
    ts = wl.topics(3, a.filters, max(sizes))
    for n in sizes:
        sub = ts.slice(0, n)
        hh, _, _ = ix.match_batch(sub.blob, sub.offs)
        out = (ctypes.c_double * 3)()
        assert hb.tmb_single(ix._h, n, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096, a.iters,
                             out) == 0
        print(json.dumps({"lib": os.path.basename(os.environ.get("TM_LIB", "libtmatch.so")), "topics": n,
                          "p50_ms": out[0], "p99_ms": out[1], "mean_ms": out[2]}), flush=True)


if __name__ == "__main__":
    main()
