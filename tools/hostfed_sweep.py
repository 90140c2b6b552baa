#!/usr/bin/env python3
"""Host-fed pipeline sweep (study tool): tmb_pipeline (pinned host topics ->
H2D -> match -> D2H of offsets and values) over 1M-topic C3 batches for several
stream counts and batch sizes, next to the PCIe copy ceiling (tmb_pcie).
usage: hostfed_sweep.py [--streams 2,3,4,6] [--batches 1000000,262144]"""
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
    p.add_argument("--streams", default="2,3,4,6")
    p.add_argument("--batches", default="1000000,262144")
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
    pc = (ctypes.c_double * 4)()
    assert hb.tmb_pcie(0, 256 << 20, 16, 4, pc) == 0
    print(json.dumps({"pcie_GBps": {"h2d_alone": pc[0], "d2h_alone": pc[1], "both_each": pc[2]}}), flush=True)
    R = 4
    for B in [int(x) for x in a.batches.split(",")]:
        allt = wl.topics(3, a.filters, R * B)
        for ns in [int(x) for x in a.streams.split(",")]:
            out = (ctypes.c_double * 5)()
            iters = max(24, 24 * 1_000_000 // B)
            assert hb.tmb_pipeline(ix._h, 0, _native._ptr(allt.blob), _native._ptr(allt.offs), B, R, ns, iters, out) == 0
            per = max(out[2] / (pc[2] * 1e9), out[3] / (pc[3] * 1e9))
            print(json.dumps({"batch": B, "streams": ns, "topics_per_s": out[0], "ms_per_batch": out[1],
                              "h2d_MB": out[2] / 1e6, "d2h_MB": out[3] / 1e6, "pcie_bound_topics_per_s": B / per,
                              "frac": out[0] * per / B}), flush=True)


if __name__ == "__main__":
    main()
