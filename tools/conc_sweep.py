#!/usr/bin/env python3
"""Concurrent-caller sweep (study tool, not product code): one C3 index, then
tmb_callers (native caller threads, tm_host_alloc buffers, in place) for each
(threads, churn) pair, one JSON line each.  Run it once per HIP setting under
study (e.g. GPU_MAX_HW_QUEUES), since HIP reads those at initialisation.
usage: conc_sweep.py [--dev 0|1] [--filters N] [--batch 4096] [--threads 1,4,8,16] [--churn 0,256] [--seconds 1]"""
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
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--threads", default="1,4,8,16")
    p.add_argument("--churn", default="0,256")
    p.add_argument("--seconds", type=float, default=1.0)
    p.add_argument("--copies", type=int, default=1, help="tm_options.copies of the index")
    p.add_argument("--dev", type=int, default=0, help="1: batches in HBM through the device API (no PCIe leg)")
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
    thr = [int(x) for x in a.threads.split(",")]
    ts = wl.topics(3, a.filters, max(thr) * a.batch)
    hh, _, _ = ix.match_batch(ts.blob, ts.offs)
    cap = int(hh[-1]) + 65536
    for churn in [int(x) for x in a.churn.split(",")]:
        for t in thr:
            out = (ctypes.c_double * 6)()
            rc = hb.tmb_callers_ex(ix._h, t, a.batch, _native._ptr(ts.blob), _native._ptr(ts.offs), cap, a.seconds,
                                   churn, a.dev, out)
            assert rc == 0, rc
            print(json.dumps({"hwq": os.environ.get("GPU_MAX_HW_QUEUES", "default"), "dev": a.dev, "copies": a.copies, "threads": t, "churn": churn,
                              "batches": out[0], "topics_per_s": out[1], "p50_ms": out[2], "p99_ms": out[3],
                              "deltas_per_s": out[4]}), flush=True)


if __name__ == "__main__":
    main()
