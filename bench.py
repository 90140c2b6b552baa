#!/usr/bin/env python3
"""bench.py -- topic matches/sec at 10M filters on 1..N MI355X (BASELINE.json).

One step = one batch of publish topics matched against the device-resident
index (tokenise + trie walk + exact lookup + CSR emission of every matched
value), inputs already resident in HBM.  Default workload: config C3 (10M
mixed-wildcard filters incl. $share dests, $SYS filters and root globals),
1M-topic batches per GPU.  Multi-GPU = topic-sharded weak scaling: every rank
holds a replica of the index and matches its own batch; there is no
data-path collective.

Other modes (not the headline line):
  --config c4   filter-sharded (100M filters split over the ranks, each rank
                matches the SAME batch against its shard, the hit lists are
                allgathered over RCCL and merged on the device): strong scaling
  --config c5   churn: every step first applies --deltas subscribe/unsubscribe
                ops (one router-syncer batch) to the replicated index, then
                matches the batch; reports deltas/s beside topics/s
  --config c1 / c2 / c2nm   the other BASELINE.json configs, topic-sharded

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
       torchrun ... bench.py --gpus N  (one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

CONFIGS = {
    # name: (generator cfg, default filters, description)
    "c1": (1, 10_000, "emqx_topic_index 10k filters (70% exact, 20% '+', 10% '#'), topics depth 4-6"),
    "c2": (2, 1_000_000, "1M 'fleet/{id}/sensor/+' + 1k global '#' rules"),
    "c2nm": (20, 1_000_000, "1M 'fleet/{id}/sensor/+' + 1k non-matching 'rules/{k}/#' globals"),
    "c3": (3, 10_000_000, "10M mixed-wildcard filters incl. $share groups and '$SYS' exclusion"),
    "c4": (4, 100_000_000, "100M mixed filters filter-sharded over the ranks, RCCL allgatherv of hit lists"),
    "c5": (5, 10_000_000, "churn: 10M mixed filters, subscribe/unsubscribe deltas interleaved with match batches"),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
RANDOM_REQ_CEILING = 5.5e10   # measured random 64-B request rate beyond L2 (profiles/r1_gather.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--filters", type=int, default=None)
    p.add_argument("--batch", type=int, default=1_000_000, help="topics per GPU per step")
    p.add_argument("--deltas", type=int, default=100,
                   help="c5: deltas applied per step (100 x ~2.5k steps/s = 2.5x the configured 100k deltas/s)")
    p.add_argument("--streams", type=int, default=3,
                   help="HIP streams the steps rotate over (batch k+1's walk overlaps batch k's scan/emit)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--latency-batches", type=int, default=20)
    p.add_argument("--frontier-sample", type=int, default=20_000)
    return p.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    from emqx_amd import _native, shard, workload as wl

    gen_cfg, default_f, desc = CONFIGS[a.config]
    filter_sharded = a.config == "c4"
    nf = a.filters or default_f
    B = a.batch

    t = time.time()
    fs = wl.filters(gen_cfg, nf, shard=rank, nshards=world) if filter_sharded else wl.filters(gen_cfg, nf)
    t_gen = time.time() - t
    log(f"[rank {rank}] generated {len(fs)} filters in {t_gen:.1f}s")

    t = time.time()
    ix = _native.Index(device=local, hint_keys=len(fs))
    chunk = 2_000_000
    for lo in range(0, len(fs), chunk):
        part = fs.slice(lo, min(lo + chunk, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    t_compile = time.time() - t
    stream = torch.cuda.current_stream().cuda_stream
    t = time.time()
    ix.sync(stream)
    torch.cuda.synchronize()
    t_upload = time.time() - t
    st = ix.stats()
    log(f"[rank {rank}] index: {st['n_keys']} keys, {st['n_nodes']} nodes, {st['n_edges']} edges, "
        f"{st['n_words']} words, {st['device_bytes'] / 2**20:.0f} MiB HBM; compile {t_compile:.1f}s upload {t_upload:.2f}s")

    # topic-sharded: rank r matches topics [r B, (r+1) B); filter-sharded: all ranks the same batch
    first = 0 if filter_sharded else rank * B
    ts = wl.topics(gen_cfg, nf, B, first=first)
    d_blob = torch.from_numpy(ts.blob).to(dev)
    d_offs = torch.from_numpy(ts.offs.view(np.int64)).to(dev)
    # one output set per stream: consecutive steps rotate over the streams, so
    # step k+1's walk overlaps step k's scan / emit (the library keeps one
    # workspace per stream and orders index patches across streams)
    nstreams = 1 if filter_sharded else max(1, a.streams)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    outs = [{"hit": torch.zeros(B + 1, dtype=torch.int64, device=dev),
             "err": torch.zeros(B, dtype=torch.uint8, device=dev),
             "out": torch.zeros(1, dtype=torch.int32, device=dev)} for _ in range(nstreams)]
    d_hit, d_err = outs[0]["hit"], outs[0]["err"]

    # c5: the delta stream, generated up front (host buffers, as the syncer hands them over)
    dchunks = []
    if a.config == "c5":
        nd = a.deltas * (a.steps + a.warmup + 1)
        dl = wl.deltas(nf, 0, nd)
        dchunks = [dl.slice(k * a.deltas, (k + 1) * a.deltas) for k in range(a.steps + a.warmup + 1)]
    dpos = [0]
    kstep = [0]

    def step(cap):
        k = kstep[0] % nstreams
        kstep[0] += 1
        o = outs[k]
        sid = streams[k].cuda_stream
        if dchunks:
            d = dchunks[dpos[0]]
            dpos[0] += 1
            ix.apply(d.flags, d.blob, d.offs, d.vals)
        ix.match_batch_dev(B, d_blob.data_ptr(), d_offs.data_ptr(), o["hit"].data_ptr(), o["out"].data_ptr(), cap,
                           o["err"].data_ptr(), sid)
        if filter_sharded:
            if world == 1:   # one shard: the merge alone (the exchange is the identity)
                return shard.merge(o["hit"].view(1, B + 1), o["out"].view(1, -1), o["out"].numel(), sid)
            return shard.allgatherv_hits(o["hit"], o["out"], stream=sid)
        return None

    # sizing pass (no values written), then the output buffers
    ix.match_batch_dev(B, d_blob.data_ptr(), d_offs.data_ptr(), d_hit.data_ptr(), outs[0]["out"].data_ptr(), 0,
                       d_err.data_ptr(), stream)
    torch.cuda.synchronize()
    total_hits = int(d_hit[-1].item())
    slack = a.deltas * (a.steps + a.warmup) * 64 if dchunks else 0   # churn may add hits
    cap = total_hits + slack
    for o in outs:
        o["out"] = torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)
    for _ in range(a.warmup):
        step(cap)
    torch.cuda.synchronize()
    assert not any(bool(o["err"].any().item()) for o in outs)

    ix.profile(True)
    ix.profile_read(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    merged = None
    for _ in range(a.steps):
        merged = step(cap)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    walk_ms, batch_ms, nb = ix.profile_read(reset=True)
    # the same kernel alone: a few batches on one stream, one after another
    # (with several streams a launch's duration includes the GPU time it
    # shares with the other streams' kernels)
    for _ in range(5):
        ix.match_batch_dev(B, d_blob.data_ptr(), d_offs.data_ptr(), outs[0]["hit"].data_ptr(),
                           outs[0]["out"].data_ptr(), cap, outs[0]["err"].data_ptr(), stream)
        torch.cuda.synchronize()
    iso_walk_ms, _, iso_nb = ix.profile_read(reset=True)
    ix.profile(False)
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el_max = float(el_t.item())
    last = outs[(kstep[0] - 1) % nstreams]
    d_hit, d_out = last["hit"], last["out"]
    last_hits = int(d_hit[-1].item())
    assert last_hits <= cap
    merged_total = int(merged[0][-1].item()) if merged is not None else None

    # whole-job topics/s: topic-sharded = every rank's own batch; filter-sharded = the one shared batch
    topics_per_step = B if filter_sharded else world * B
    value = topics_per_step * a.steps / el_max
    ms_per_step = el_max / a.steps * 1e3
    walk_avg_ms = walk_ms / max(nb, 1)
    batch_avg_ms = batch_ms / max(nb, 1)

    # p50/p99 batch latency: host topics in, hit lists back in host memory
    # (every rank).  "pinned": the caller's buffers come from tm_host_alloc
    # (what a NIF keeps per scheduler), so the kernels read the topics and
    # write the hit lists in place; "pageable": ordinary caller buffers,
    # staged through the library's pinned buffers (one copy in, one out).
    lat = {}
    if not filter_sharded:
        for lb in sorted({min(4096, B), min(65536, B)}):
            sub = ts.slice(0, lb)
            _, v0, _ = ix.match_batch(sub.blob, sub.offs)          # sizes the value buffer
            nb = int(sub.offs[-1] - sub.offs[0])
            pb = ix.host_array(nb + 16, np.uint8)
            po = ix.host_array(lb + 1, np.uint64)
            pb[:nb] = sub.blob[int(sub.offs[0]):int(sub.offs[-1])]
            po[:] = sub.offs - sub.offs[0]
            kinds = {"pinned": (pb, po, (ix.host_array(lb + 1, np.uint64), ix.host_array(len(v0) + 1024, np.uint32),
                                         ix.host_array(lb, np.uint8))),
                     "pageable": (sub.blob, sub.offs, (np.zeros(lb + 1, np.uint64),
                                                       np.zeros(len(v0) + 1024, np.uint32), np.zeros(lb, np.uint8)))}
            for kind, (tb, to, bufs) in kinds.items():
                xs = []
                for k in range(a.latency_batches + 2):
                    t1 = time.perf_counter()
                    ix.match_batch(tb, to, out=bufs)
                    xs.append((time.perf_counter() - t1) * 1e3)
                xs = np.array(xs[2:])
                lat[f"{kind}/{lb}"] = {"p50_ms": float(np.percentile(xs, 50)), "p99_ms": float(np.percentile(xs, 99))}
    if world > 1 and lat:
        # the slowest rank's percentiles (max over ranks)
        keys = sorted(lat)
        v = torch.tensor([lat[k][q] for k in keys for q in ("p50_ms", "p99_ms")], dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        v = v.tolist()
        lat = {k: {"p50_ms": v[2 * i], "p99_ms": v[2 * i + 1]} for i, k in enumerate(keys)}
    lat_pinned = {k.split("/")[1]: {q: round(x, 3) for q, x in d.items()} for k, d in lat.items()
                  if k.startswith("pinned/")}
    lat_pageable = {k.split("/")[1]: {q: round(x, 3) for q, x in d.items()} for k, d in lat.items()
                    if k.startswith("pageable/")}

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    sys.path.insert(0, str(ROOT / "oracle"))
    from pyoracle import Oracle, frontier

    res_extra = {}
    mism = None
    ns = min(a.frontier_sample, B)
    achieved = walk_bytes = None
    cpu = None
    if not a.no_parity:
        # ---- oracle over this rank's key set (after the churn, for c5): roofline
        # bytes, parity sample, CPU baseline
        t = time.time()
        o = Oracle()
        o.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
        for k in range(dpos[0]):
            d = dchunks[k]
            o.apply(d.flags, d.blob, d.offs, d.vals)
        o.prepare()
        log(f"oracle built in {time.time() - t:.1f}s")
        # the last step's output of this rank (its own shard's lists for c4)
        host_hit = d_hit.cpu().numpy().view(np.uint64)
        host_out = d_out.cpu().numpy().view(np.uint32)
        rng = np.random.default_rng(0x454D5158)
        idx = np.sort(rng.choice(B, ns, replace=False))
        sblob, soffs = _native.pack_strings([ts.item(int(i)) for i in idx])
        levels, states = frontier(o, sblob, soffs, nthreads=a.cpu_threads)
        cnt, _, ohit, ovals = o.match_batch(sblob, soffs, nthreads=a.cpu_threads)
        mism = 0
        for j, i in enumerate(idx):
            g = host_out[int(host_hit[i]):int(host_hit[i + 1])]
            e = ovals[int(ohit[j]):int(ohit[j + 1])]
            mism += int(not np.array_equal(g, e))
        # algorithmic bytes per walk launch (SURVEY.md 8d per topic, minus the
        # 4 H the emit kernel writes):  8 L + 32 sum|F_l| + 4
        L_total = int(np.count_nonzero(ts.blob[: int(ts.offs[-1])] == ord("/"))) + B
        F_total = float(states.sum()) * B / ns
        walk_bytes = 8 * L_total + 32 * F_total + 4 * B
        achieved = walk_bytes / (walk_avg_ms * 1e-3) / 1e9
        iso_ms = iso_walk_ms / max(iso_nb, 1)
        res_extra["walk_isolated"] = {"kernel_avg_ms": round(iso_ms, 4),
                                      "achieved_GBps": round(walk_bytes / (iso_ms * 1e-3) / 1e9, 1),
                                      "frac": round(walk_bytes / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "note": "k_walk_fast alone: 5 batches on one stream after the timed region"}
        res_extra["full_path_GBps"] = round((walk_bytes + 4 * last_hits) / (batch_avg_ms * 1e-3) / 1e9, 1)
        # the walk's algorithmic bytes over the wall time of a step: with steps
        # overlapping on several streams a launch's own duration overstates its
        # share of the GPU, so this is the effective rate beside roofline.achieved
        res_extra["walk_effective_GBps"] = round(walk_bytes / (ms_per_step * 1e-3) / 1e9, 1)

        # ---- CPU baseline: the oracle (restated reference walk) on host threads
        if not a.no_cpu and world == 1 and a.config in ("c1", "c2", "c2nm", "c3"):
            n1 = min(20_000, B)
            probe = ts.slice(0, n1)
            t1 = time.perf_counter()
            o.match_batch(probe.blob, probe.offs, nthreads=a.cpu_threads, with_values=False)
            r1 = n1 / (time.perf_counter() - t1)
            # a bounded sample of about cpu_seconds of CPU work: whole passes over
            # the batch when it is shorter than that, else its first n2 topics
            want = int(max(n1, r1 * a.cpu_seconds))
            passes, n2 = (max(1, round(want / B)), B) if want >= B else (1, want)
            samp = ts.slice(0, n2)
            t1 = time.perf_counter()
            for _ in range(passes):
                o.match_batch(samp.blob, samp.offs, nthreads=a.cpu_threads, with_values=False)
            el_cpu = time.perf_counter() - t1
            what = f"{passes} passes over the {B}-topic batch" if passes > 1 else f"first {n2} topics of the batch"
            cpu = {"value": round(passes * n2 / el_cpu, 1), "unit": "topic matches/s", "cores": a.cpu_threads,
                   "kind": "port",
                   "sample": f"{what} vs all {len(fs)} keys; oracle/tm_oracle.c seek walker (emqx_trie_search "
                             f"restated) over a sorted key array, {a.cpu_threads} pthreads, {el_cpu:.1f}s"}

    traffic = None
    mem_req = None
    pmc = ROOT / "profiles" / f"pmc_{a.config}.json"
    if pmc.exists():
        try:
            pj = json.loads(pmc.read_text())
            if pj.get("filters") == len(fs) and pj.get("batch") == B:
                traffic = pj.get("walk_hbm_bytes_per_launch")
                mem_req = pj.get("walk_mem_requests_per_launch")
        except Exception:
            traffic = None
    # practical roofline of a pointer-chasing walk: the measured memory-side
    # random-request rate (tools/gather_bench.hip, profiles/r1_gather.md)
    req_ceiling = None
    if mem_req and walk_avg_ms:
        rate = mem_req / (walk_avg_ms * 1e-3)
        req_ceiling = {"requests_per_launch": mem_req, "requests_per_s": round(rate, 1),
                       "ceiling_per_s": RANDOM_REQ_CEILING, "frac": round(rate / RANDOM_REQ_CEILING, 4),
                       "source": "profiles/r1_gather.md (64-B random requests beyond L2, 256 MiB-2 GiB tables)"}

    metric = {"c3": "topic matches/sec at 10M filters"}.get(a.config, f"topic matches/sec ({a.config})")
    par = (f"filter-sharded x{world} (RCCL allgatherv of hit lists)" if filter_sharded
           else f"topic-sharded x{world} (trie replicated)")
    res = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "topic matches/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if filter_sharded else "weak",
        "vs_baseline": None,
        "dtype": "u8/u32",
        "data": "synthetic (emqx_amd/csrc/workload.cpp, seed 0x454D5158+cfg)",
        "config": {"workload": f"{a.config}: {desc}", "filters": nf if filter_sharded else len(fs),
                   "topics_per_gpu_step": B, "global_batch": topics_per_step, "parallelism": par,
                   "streams": nstreams},
        "roofline": {"bound": "hbm", "achieved": None if achieved is None else round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "k_walk_fast", "kernel_avg_ms": round(walk_avg_ms, 4),
                     "algorithmic_bytes_per_launch": None if walk_bytes is None else int(walk_bytes),
                     "random_request_roofline": req_ceiling},
        "cpu_baseline": cpu,
        "matched_ids_per_s": round(last_hits * (1 if filter_sharded else world) * a.steps / el_max, 1),
        "hits_per_topic": round((merged_total if merged_total is not None else last_hits) / B, 3),
        "batch_device_ms": round(batch_avg_ms, 4),
        "batch_latency_host_ms": lat_pinned,
        "batch_latency_host_pageable_ms": lat_pageable,
        "parity_sample": None if mism is None else {"topics": ns, "mismatches": mism,
                                                    "against": "oracle over this rank's keys"},
        "build": {"generate_s": round(t_gen, 1), "compile_s": round(t_compile, 1), "upload_s": round(t_upload, 2),
                  "device_MiB": round(st["device_bytes"] / 2**20, 1), "nodes": st["n_nodes"],
                  "edges": st["n_edges"], "words": st["n_words"], "keys_this_rank": st["n_keys"]},
    }
    res.update(res_extra)
    if dchunks:
        res["deltas_per_step"] = a.deltas
        res["deltas_per_s"] = round(a.deltas * a.steps / el_max, 1)
    if filter_sharded:
        res["merged_hits_per_step"] = merged_total
    if cpu:
        res["speedup_vs_cpu"] = round(value / cpu["value"], 1)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
