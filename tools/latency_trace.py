#!/usr/bin/env python3
"""Small-batch latency driver: build a config's index, then run --reps
host-API batches of --batch topics (topics in host memory, hit lists back in
host memory) so a kernel + memory-copy trace shows where a batch's time goes."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c3")
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--reps", type=int, default=50)
    a = p.parse_args()
    from bench import CONFIGS
    from emqx_amd import _native, workload as wl
    gen, nf, _ = CONFIGS[a.config]
    fs = wl.filters(gen, nf)
    ix = _native.Index(device=0)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    ts = wl.topics(gen, nf, a.batch)
    def report(tag, xs):
        xs = np.array(xs[5:])
        print(f"{a.config} batch={a.batch} {tag}: p50 {np.percentile(xs, 50):.3f} ms p99 {np.percentile(xs, 99):.3f} ms "
              f"min {xs.min():.3f} ms", flush=True)

    xs = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        ix.match_batch(ts.blob, ts.offs)
        xs.append((time.perf_counter() - t1) * 1e3)
    report("match_batch (fresh outputs)", xs)
    # the C ABI call alone, caller-owned output buffers reused across batches
    from emqx_amd._native import _ptr
    n = len(ts)
    blob = np.ascontiguousarray(ts.blob, np.uint8)
    offs = np.ascontiguousarray(ts.offs, np.uint64)
    hit = np.zeros(n + 1, np.uint64)
    err = np.zeros(n, np.uint8)
    cap = 64 * n
    out = np.zeros(cap, np.uint32)
    args = (ix._h, n, _ptr(blob), _ptr(offs), _ptr(hit), _ptr(out), cap, _ptr(err))
    xs = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        ix._lib.tm_match_batch(*args)
        xs.append((time.perf_counter() - t1) * 1e3)
    report("tm_match_batch (reused outputs)", xs)
    # every buffer from tm_host_alloc: the batch runs in place
    nb = int(offs[-1] - offs[0])
    pb, po = ix.host_array(nb + 16, np.uint8), ix.host_array(n + 1, np.uint64)
    pb[:nb] = blob[int(offs[0]):int(offs[-1])]
    po[:] = offs - offs[0]
    ph, pv, pe = ix.host_array(n + 1, np.uint64), ix.host_array(cap, np.uint32), ix.host_array(n, np.uint8)
    args = (ix._h, n, _ptr(pb), _ptr(po), _ptr(ph), _ptr(pv), cap, _ptr(pe))
    xs = []
    for _ in range(a.reps):
        t1 = time.perf_counter()
        ix._lib.tm_match_batch(*args)
        xs.append((time.perf_counter() - t1) * 1e3)
    report("tm_match_batch (tm_host_alloc buffers, in place)", xs)


if __name__ == "__main__":
    main()
