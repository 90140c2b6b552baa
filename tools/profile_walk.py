#!/usr/bin/env python3
"""Minimal profiling driver: build a config's index, then run --batches
device-resident match batches (no oracle, no CPU work) so rocprofv3 passes
(kernel trace or PMC counters) see only the match kernels."""
import argparse
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c3")
    p.add_argument("--filters", type=int, default=None)
    p.add_argument("--batch", type=int, default=1_000_000)
    p.add_argument("--batches", type=int, default=8)
    p.add_argument("--rotate", type=int, default=4, help="distinct batches the launches cycle over (as bench.py)")
    p.add_argument("--order", default="stream", choices=["stream", "sorted", "bucket", "work"],
                   help="topic order in the batch: generator stream, byte-sorted, bucketed "
                        "by the hash of the first two levels (locality study), or by predicted work "
                        "(level count, then hit count from a first device pass: divergence study)")
    p.add_argument("--window", type=int, default=0,
                   help="with --order sorted/bucket: order only inside consecutive windows of this many topics "
                        "(the upper bound of a block-local grouping: its gain without its cost)")
    p.add_argument("--outputs", default="csr", choices=["csr", "pairs"],
                   help="tm_match_batch_dev (CSR) or tm_match_batch_dev_pairs ((first position, count) pairs)")
    p.add_argument("--filter-order", default="stream", choices=["stream", "sorted"],
                   help="insertion order of the filters (node ids follow it): generator stream or "
                        "byte-sorted, i.e. trie nodes numbered depth first (layout study)")
    p.add_argument("--streams", type=int, default=1,
                   help="streams the launches rotate over (3: bench.py's overlapped steps; wall/batch is then the "
                        "step time)")
    p.add_argument("--small-kernel", default="auto", choices=["auto", "wave", "wave8"],
                   help="batches <= 65536 topics: the library's default, k_walk_small with 16 or 8 lanes per topic")
    p.add_argument("--phases", action="store_true", help="every batch on the two-phase path (TM_DEBUG_PHASES)")
    p.add_argument("--noise", default="none", choices=["none", "launch", "host", "native", "events"],
                   help="during the timed launches, a thread that launches one-element kernels on a stream of its "
                        "own as fast as it can (launch; native: a C++ thread enqueueing 4-byte fills, libtmbench; events: event records, no kernel), "
                        "or spins on the host only (host): does another stream's "
                        "launch rate slow the walk (kernel-boundary cache maintenance)?")
    a = p.parse_args()
    import torch
    from bench import CONFIGS
    from emqx_amd import _native, workload as wl
    gen, nf0, _ = CONFIGS[a.config]
    nf = a.filters or nf0
    fs = wl.filters(gen, nf)
    if a.filter_order == "sorted":
        items = fs.items()
        order = sorted(range(len(items)), key=items.__getitem__)
        blob, offs = _native.pack_strings([items[i] for i in order])
        fs = wl.ItemSet(blob, offs, fs.vals[np.array(order)], fs.flags[np.array(order)])
        del items, order
    ix = _native.Index(device=0)
    if a.small_kernel != "auto":
        ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, {"wave": _native.SMALL_WAVE, "wave8": _native.SMALL_WAVE8}[a.small_kernel])
    if a.phases:
        ix.debug_set(_native.TM_DEBUG_PHASES, 1)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    print(f"wide nodes {ix.debug_get(_native.TM_DEBUG_WIDE_NODES)}, dense {ix.debug_get(_native.TM_DEBUG_DENSE_WIDE)}",
          flush=True)
    dev = torch.device("cuda:0")
    R = max(1, a.rotate)
    d_in = []
    for k in range(R):
        ts = wl.topics(gen, nf, a.batch, first=k * a.batch)
        if a.order != "stream":
            items = ts.items()
            W = a.window if a.window > 0 else len(items)
            if a.order == "sorted":
                items = [t for lo in range(0, len(items), W) for t in sorted(items[lo:lo + W])]
            elif a.order == "work":   # lanes of a wave get topics of similar work
                hh, _, _ = ix.match_batch(ts.blob, ts.offs)
                hits = np.diff(hh.astype(np.int64))
                key = [(t.count(b"/"), int(h)) for t, h in zip(items, hits)]
                items = [items[i] for i in sorted(range(len(items)), key=key.__getitem__)]
            else:
                items = [t for lo in range(0, len(items), W)
                         for t in sorted(items[lo:lo + W], key=lambda t: hash(b"/".join(t.split(b"/")[:2])) & 0xFFFF)]
            blob, offs = _native.pack_strings(items)
            ts = wl.ItemSet(blob, offs, np.zeros(len(items), np.uint32), np.zeros(len(items), np.uint8))
        d_in.append((torch.from_numpy(ts.blob).to(dev), torch.from_numpy(ts.offs.view(np.int64)).to(dev)))
    d_hit = torch.zeros(a.batch + 1, dtype=torch.int64, device=dev)
    d_err = torch.zeros(a.batch, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    S = max(1, a.streams)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(S - 1)]
    tot = 0
    pairs = a.outputs == "pairs"

    def run(d_blob, d_offs, h_, o_, cap, e_, sid):
        if pairs:   # (h_ holds the 2 n + 1 u32 pairs)
            ix.match_batch_dev_pairs(a.batch, d_blob.data_ptr(), d_offs.data_ptr(), h_.data_ptr(), o_, cap,
                                     e_.data_ptr(), sid)
        else:
            ix.match_batch_dev(a.batch, d_blob.data_ptr(), d_offs.data_ptr(), h_.data_ptr(), o_, cap, e_.data_ptr(),
                               sid)

    slack = 0
    for d_blob, d_offs in d_in:
        run(d_blob, d_offs, d_hit, 0, 0, d_err, s)
        torch.cuda.synchronize()
        tot = max(tot, int(d_hit[-1]) & (0xFFFFFFFF if pairs else ~0))
        if pairs:   # spans may leave gaps (tmatch.h): + 4096 x the most hits of one topic
            slack = max(slack, 4096 * int(d_hit[:a.batch].view(torch.int32).view(a.batch, 2)[:, 1].max().item()))
    tot += slack
    outs = [(torch.zeros(a.batch + 1, dtype=torch.int64, device=dev), torch.zeros(a.batch, dtype=torch.uint8, device=dev),
             torch.zeros(max(tot, 1), dtype=torch.int32, device=dev)) for _ in range(S)]

    def launch(k):
        d_blob, d_offs = d_in[k % R]
        h_, e_, o_ = outs[k % S]
        run(d_blob, d_offs, h_, o_.data_ptr(), tot, e_, streams[k % S].cuda_stream)

    for k in range(S):   # every stream's workspace exists before the timed launches
        launch(k)
    torch.cuda.synchronize()
    launch(0)   # unprofiled: the profiled launches are enqueued behind a busy stream
    import threading
    stop, nlaunch = threading.Event(), [0]

    def noise():
        ns = torch.cuda.Stream()
        x = torch.zeros(1, device=dev)
        with torch.cuda.stream(ns):
            while not stop.is_set():
                if a.noise == "launch":
                    x.add_(1)
                nlaunch[0] += 1

    th = threading.Thread(target=noise) if a.noise in ("launch", "host") else None
    hb = None
    if a.noise in ("native", "events"):
        import ctypes
        from bench import host_bench_lib
        hb = host_bench_lib()
        assert hb.tmb_noise_start(0, 1 if a.noise == "events" else 0) == 0
    ix.profile(True)
    t = time.perf_counter()
    if th:
        th.start()
    for k in range(a.batches):
        launch(k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    if th:
        stop.set()
        th.join()
        print(f"noise={a.noise}: {nlaunch[0] / el:.0f} loop iterations/s on the other thread", flush=True)
    if hb is not None:
        rate = ctypes.c_double()
        assert hb.tmb_noise_stop(ctypes.byref(rate)) == 0
        print(f"noise={a.noise}: {rate.value:.0f} operations/s on the other stream", flush=True)
    w, b, n = ix.profile_read()
    st = ix.stats()
    paths = [ix.debug_get(k) for k in (_native.TM_DEBUG_PATH_PHASES, _native.TM_DEBUG_PATH_SMALL,
                                       _native.TM_DEBUG_PATH_LANE)]
    assert not any(bool(e_.any().item()) for _, e_, _ in outs), "err flags set"
    print(f"{a.config}/{a.outputs}/{a.order}{'/w' + str(a.window) if a.window else ''}/filters-{a.filter_order} streams={S} paths(phases,small,lane)={paths} filters={len(fs)} batch={a.batch} rotate={R} hits<={tot} "
          f"wall/batch={el / a.batches * 1e3:.3f}ms walk={w / n:.4f}ms batch_dev={b / n:.4f}ms "
          f"rate={a.batch * a.batches / el / 1e9:.3f}G/s device_MiB={st['device_bytes'] / 2**20:.0f}", flush=True)


if __name__ == "__main__":
    main()
