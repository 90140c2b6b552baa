#!/usr/bin/env python3
"""Where a 4k-topic one-launch batch spends its time: runs the stamped study
build (tools/mk_stamps.py; TM_LIB=emqx_amd/variants/libtmatch_stamps.so) on a
C3 index and prints, per phase of k_walk_small, the median / p90 / max over
waves of the time since the wave's start, and the spread of wave starts and
ends over the grid (10 ns ticks).  usage: stamps_study.py [--filters N] [--batch 4096]"""
import argparse
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
PH = ["entry", "staged", "words", "walk", "exact", "fallback", "lookback", "emitted"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--batch", type=int, default=4096)
    a = p.parse_args()
    assert "stamps" in os.environ.get("TM_LIB", "")
    import torch
    assert torch.cuda.is_available()
    from emqx_amd import _native, workload as wl
    lib = _native.load_library()
    fs = wl.filters(3, a.filters)
    ix = _native.Index(device=0, hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    ts = wl.topics(3, a.filters, a.batch)
    for _ in range(20):
        ix.match_batch(ts.blob, ts.offs)
    nw = (a.batch + 15) // 16 * 4
    st = np.zeros(nw * 8, np.uint64)
    lib.tm_study_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    assert lib.tm_study_stamps(st.ctypes.data, st.size) == 0
    st = st.reshape(nw, 8).astype(np.int64)
    t0 = st[:, 0]
    print(f"batch {a.batch}: {nw} waves; start spread p50 {np.median(t0 - t0.min()) * 10:.0f} ns "
          f"max {(t0.max() - t0.min()) * 10:.0f} ns; last stamp {(st.max() - t0.min()) * 10:.0f} ns after first start")
    for k in range(1, 8):
        d = st[:, k] - t0
        ok = st[:, k] > 0
        d = d[ok]
        if not len(d):
            continue
        print(f"  {PH[k]:9s} n={len(d):5d} median {np.median(d) * 10:8.0f} ns  p90 {np.percentile(d, 90) * 10:8.0f}"
              f"  max {d.max() * 10:8.0f}")
    inc = np.diff(st, axis=1)
    for k in range(1, 8):
        print(f"  step {PH[k - 1]}->{PH[k]}: median {np.median(inc[:, k - 1]) * 10:8.0f} ns  "
              f"p90 {np.percentile(inc[:, k - 1], 90) * 10:8.0f}  max {inc[:, k - 1].max() * 10:8.0f}")


if __name__ == "__main__":
    main()
