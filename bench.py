#!/usr/bin/env python3
"""bench.py -- topic matches/sec at 10M filters on 1..N MI355X (BASELINE.json).

One step = one batch of publish topics matched against the device-resident
index (tokenise + trie walk + exact lookup + CSR emission of every matched
value), inputs already resident in HBM.  Default workload: config C3 (10M
mixed-wildcard filters incl. $share dests, $SYS filters and root globals),
1M-topic batches per GPU.  The timed steps rotate over --rotate distinct
1M-topic batches (default 4, 4M different topics), so no step re-matches the
batch the step before it left in the 256 MB Infinity Cache.  Multi-GPU =
topic-sharded weak scaling: every rank holds a replica of the index and
matches its own batches; there is no data-path collective.

Other modes (not the headline line):
  --config c4   filter-sharded (100M filters split over the ranks, each rank
                matches the SAME batch against its shard; every rank receives
                its own slice of the batch from every shard -- all_to_all of
                u32 counts and padded values over RCCL -- and merges it on the
                device): strong scaling
  --config c4l0 the same 100M filters sharded by their first topic level
                (filters whose first level is '+' or '#' on every rank); a
                publish is matched on the ONE rank owning its first level (the
                host routes it there), whose lists are complete and in
                traversal order: no merge, no data-path collective; weak
                scaling (each rank matches its own batches)
  --config c5   churn: every step first applies --deltas subscribe/unsubscribe
                ops (one router-syncer batch) to the replicated index, then
                matches the batch; reports deltas/s beside topics/s
  --config c1 / c2 / c2nm / c3deep   the other BASELINE.json configs (and C3
                with 10 % of the topics 33-64 levels deep), topic-sharded

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
       torchrun ... bench.py --gpus N  (one rank per GPU)
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import math
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
    "c3deep": (30, 10_000_000, "C3 filters; 10% of the topics 33-64 levels deep"),
    "c4": (4, 100_000_000, "100M mixed filters filter-sharded over the ranks, RCCL all_to_all of hit-list slices"),
    "c4l0": (4, 100_000_000, "100M mixed filters sharded by the first topic level ('+'/'#'-rooted filters on "
                             "every rank), publishes routed to the rank owning their first level"),
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
    p.add_argument("--rotate", type=int, default=4, help="distinct topic batches the steps rotate over")
    p.add_argument("--deltas", type=int, default=100,
                   help="c5: deltas applied per application (100 x ~2.5k steps/s = 2.5x the configured 100k deltas/s)")
    p.add_argument("--delta-every", type=int, default=1,
                   help="c5: steps between delta applications (e.g. --deltas 1000 --delta-every 10: the same rate in "
                        "the router syncer's batch size, emqx_router_syncer.erl's <= 1000 ops per run_batch)")
    p.add_argument("--streams", type=int, default=None,
                   help="HIP streams the steps rotate over (batch k+1's walk overlaps batch k's scan/emit); "
                        "default 3; for c5 one per table copy up to 2 (with one copy a churn step's patch waits "
                        "for every batch in flight, so its steps cannot overlap and a second stream only adds "
                        "cross-stream waits: 0.41 vs 0.54-0.64 ms per step measured in round 2)")
    p.add_argument("--split", type=int, default=1,
                   help="sub-batches per step: each step's batch goes to the streams as this many contiguous "
                        "sub-batches (each its own CSR, as that many concurrent NIF batches), so the timed "
                        "region ends one sub-batch's latency after the last launch instead of one whole "
                        "overlapped batch's")
    p.add_argument("--copies", type=int, default=None,
                   help="copies of the tables on the GPU (tm_options.copies): a batch after a delta runs on a "
                        "copy no batch is reading.  Default 1, and 2 for c5 on two streams: each step's patch "
                        "goes to the copy the step before did not read, so consecutive churn steps overlap "
                        "(round 5: 3.30e9 vs 2.89e9 with one copy on one stream; 2 copies on 3 streams 1.65e9, "
                        "3 on 3 2.44e9, profiles/r5/c5/; with stream-aware copies 3 on 3 2.80-2.87e9, 2 on 2 "
                        "3.32-3.36e9, profiles/r5/c5_stream_copies/)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    p.add_argument("--cpu-threads", type=int, default=None,
                   help="CPU baseline threads (default: the CPUs this process may use)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--latency-batches", type=int, default=20)
    p.add_argument("--pool-streams", action="store_true",
                   help="run the steps on streams from torch's pool only (default: the current stream and pool ones)")
    p.add_argument("--combine-leaders", type=int, default=None,
                   help="concurrent combined launches of the callers' legs (TM_DEBUG_COMBINE; default: the library's)")
    p.add_argument("--concurrency", type=int, default=8,
                   help="native caller threads of the concurrent-caller leg (and twice as many; 0 = skip)")
    p.add_argument("--frontier-sample", type=int, default=20_000)
    p.add_argument("--route-writers", type=int, default=16,
                   help="route-write leg: writer threads issuing one-key subscribe/unsubscribe writes through a "
                        "group-committing mirror thread (tm_commit) while --concurrency matcher threads run NIF-shaped "
                        "batches, on a second index of the same filters with --writes-copies table copies (0 = skip)")
    p.add_argument("--writes-copies", type=int, default=3)
    p.add_argument("--cmb-spin", type=int, default=0,
                   help="microseconds a caller waiting in the combiner spins before it sleeps (TM_DEBUG_CMB_SPIN)")
    p.add_argument("--small-ticket", type=int, default=1,
                   help="k_walk_small's blocks take a start-order ticket (TM_DEBUG_SMALL_TICKET; 1 = the library's "
                        "default, 0 = dispatch order)")
    p.add_argument("--replicas", type=int, default=0,
                   help="replica-topology leg: one process, one tm_create_replicas index (one host image) over N "
                        "device entries, native feeder threads submitting in-place host batches while a syncer thread "
                        "applies deltas (the NIF's deployment, INTEGRATION.md 5); with fewer GPUs than N the entries "
                        "repeat the local device -- a rehearsal, not scaling")
    p.add_argument("--outputs", default=None, choices=["csr", "pairs"],
                   help="hit lists as a CSR (tm_match_batch_dev: walk, tails, scan + emit) or as per-topic "
                        "(first position, count) pairs (tm_match_batch_dev_pairs: the walk writes its own values); "
                        "default pairs, CSR for the filter-sharded configs and --split (their merge and sub-batches "
                        "take CSRs)")
    p.add_argument("--small-kernel", default="auto", choices=["auto", "wave", "wave8"],
                   help="the one-launch kernel of batches <= 65536 topics (latency and concurrent-caller legs): "
                        "the library's default, k_walk_small with 16 or 8 lanes per topic (TM_DEBUG_SMALL_KERNEL)")
    return p.parse_args()


def host_cpus():
    """CPUs this process may use: its affinity set, capped by a cgroup CPU
    quota if one is set (the GPU box gives a process a share of the machine),
    and the CPU model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, math.floor(quota)))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"cpu_model": model, "affinity_cpus": aff, "cgroup_cpu_quota": quota}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TM_BENCH_DIST_BACKEND=gloo rehearses the N > 1 path with several ranks on
    # one GPU (the timing collectives then run on host tensors); the driver's
    # multi-GPU runs use the default, RCCL.
    backend = os.environ.get("TM_BENCH_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")
    cdev = dev if backend == "nccl" else torch.device("cpu")   # where the timing collectives' tensors live

    from emqx_amd import _native, shard, workload as wl
    from emqx_amd.build import source_hash

    gen_cfg, default_f, desc = CONFIGS[a.config]
    filter_sharded = a.config == "c4"
    level0 = a.config == "c4l0"
    nf = a.filters or default_f
    B = a.batch
    R = max(1, a.rotate)

    t = time.time()
    l0map = None
    if level0:
        # every rank draws the same owner map from the same samples (filters, and
        # a publish sample: words spread by publish load under a filter cap),
        # then keeps its own words' filters and the '+'/'#'-rooted ones, chunk by chunk
        K = max(1, nf // 10_000_000)
        l0map = shard.Level0Map.from_items(world, wl.filters(gen_cfg, nf, shard=0, nshards=K),
                                           topics=wl.topics(gen_cfg, nf, 200_000, first=1 << 40))
        parts = []
        for k in range(K):
            fk = wl.filters(gen_cfg, nf, shard=k, nshards=K)
            parts.append(wl.take(fk, l0map.filter_rows(fk, rank)))
            del fk
        fs = wl.concat(parts)
        del parts
    elif filter_sharded:
        fs = wl.filters(gen_cfg, nf, shard=rank, nshards=world)
    else:
        fs = wl.filters(gen_cfg, nf)
    t_gen = time.time() - t
    log(f"[rank {rank}] generated {len(fs)} filters in {t_gen:.1f}s")

    t = time.time()
    copies = a.copies if a.copies is not None else (2 if a.config == "c5" else 1)
    ix = _native.Index(device=local, hint_keys=len(fs), copies=copies)
    if a.small_kernel != "auto":
        ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, {"wave": _native.SMALL_WAVE, "wave8": _native.SMALL_WAVE8}[a.small_kernel])
    ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, a.small_ticket)
    if a.cmb_spin:
        ix.debug_set(_native.TM_DEBUG_CMB_SPIN, a.cmb_spin)
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

    # R distinct batches per rank.  Topic-sharded: rank r owns topics
    # [(r R + k) B, (r R + k + 1) B) of the stream; filter-sharded: every rank
    # matches the same R batches against its shard.
    base = 0 if filter_sharded else rank * R
    if level0:
        # c4l0: the host routes each publish to the rank owning its first
        # level; rank r's batches are the topics of the stream it owns
        pool, have, pos, CH = [], 0, 0, max(B, 1_000_000)
        while have < R * B:
            cand = wl.topics(gen_cfg, nf, CH, first=pos)
            pool.append(wl.take(cand, l0map.topic_rows(cand, rank)))
            have += len(pool[-1])
            pos += CH
        allt = wl.concat(pool)
        tsets = [allt.slice(k * B, (k + 1) * B) for k in range(R)]
        del pool, allt
    else:
        tsets = [wl.topics(gen_cfg, nf, B, first=(base + k) * B) for k in range(R)]
    d_in = [(torch.from_numpy(ts.blob).to(dev), torch.from_numpy(ts.offs.view(np.int64)).to(dev)) for ts in tsets]
    # one output set per stream: consecutive steps rotate over the streams, so
    # step k+1's walk overlaps step k's scan / emit (the library keeps one
    # workspace per stream and orders index patches across streams)
    nstreams = 1 if filter_sharded else max(1, a.streams if a.streams is not None else
                                            (copies if a.config == "c5" and copies <= 2 else 3))
    if a.pool_streams:   # every step on a stream of torch's pool, none on the default stream
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
    else:
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]
    split = 1 if (filter_sharded or a.config == "c5") else max(1, min(a.split, nstreams))
    sub = -(-B // split)
    parts = [(j * sub, min(sub, B - j * sub)) for j in range(split)]   # (first topic, topics) of each sub-batch
    outs = [{"hit": torch.zeros(B + 1, dtype=torch.int64, device=dev),
             "err": torch.zeros(B, dtype=torch.uint8, device=dev),
             "out": torch.zeros(1, dtype=torch.int32, device=dev)} for _ in range(nstreams)]

    # c5: the delta stream, generated up front (host buffers, as the syncer hands them over)
    dchunks = []
    every = max(1, a.delta_every)
    if a.config == "c5":
        napp = (a.steps + a.warmup + 1) // every + 1
        dl = wl.deltas(nf, 0, a.deltas * napp)
        dchunks = [dl.slice(k * a.deltas, (k + 1) * a.deltas) for k in range(napp)]
    dpos = [0]
    kstep = [0]
    apply_s = [0.0]   # c5: host time inside tm_apply_deltas (the syncer's side of a churn step)
    xch = shard.Exchange(B, dev) if filter_sharded and world > 1 else None

    if a.outputs is None:
        a.outputs = "csr" if (filter_sharded or level0 or a.split > 1) else "pairs"
    pairs_out = a.outputs == "pairs"
    assert not (pairs_out and (filter_sharded or level0 or a.split > 1)), "--outputs pairs: topic-sharded, no split"

    def match(n, d_blob, d_offs, o, cap, sid, pairs=None):
        if pairs_out if pairs is None else pairs:   # (the "hit" buffer holds the 2 n + 1 u32 pairs)
            ix.match_batch_dev_pairs(n, d_blob.data_ptr(), d_offs.data_ptr(), o["hit"].data_ptr(), o["out"].data_ptr(),
                                     cap, o["err"].data_ptr(), sid)
        else:
            ix.match_batch_dev(n, d_blob.data_ptr(), d_offs.data_ptr(), o["hit"].data_ptr(), o["out"].data_ptr(), cap,
                               o["err"].data_ptr(), sid)

    def total_of(o, n, pairs=None):
        v = int(o["hit"][n].item())
        return v & 0xFFFFFFFF if (pairs_out if pairs is None else pairs) else v

    def step(cap, oset=None):
        k = kstep[0]
        kstep[0] += 1
        o = (oset or outs)[k % nstreams]
        d_blob, d_offs = d_in[k % R]
        if split > 1:   # sub-batch j on stream j, into its own CSR
            for j, (lo, n) in enumerate(parts):
                o = outs[j]
                ix.match_batch_dev(n, d_blob.data_ptr(), d_offs.data_ptr() + 8 * lo, o["hit"].data_ptr(),
                                   o["out"].data_ptr(), cap, o["err"].data_ptr(), streams[j].cuda_stream)
            return None
        sid = streams[k % nstreams].cuda_stream
        if dchunks and k % every == 0:
            d = dchunks[dpos[0]]
            dpos[0] += 1
            ta = time.perf_counter()
            ix.apply(d.flags, d.blob, d.offs, d.vals)
            apply_s[0] += time.perf_counter() - ta
        match(B, d_blob, d_offs, o, cap, sid)
        if filter_sharded:
            if world == 1:   # one shard: the merge alone (the exchange is the identity)
                return shard.merge_local(o["hit"], o["out"], sid)
            return xch.run(o["hit"], o["out"], stream=sid)
        return None

    # sizing pass (no values written) over every batch, then the output buffers
    total_hits = 0
    batch_hits = []
    pairs_slack = [0]
    for d_blob, d_offs in d_in:
        match(B, d_blob, d_offs, outs[0], 0, stream)
        torch.cuda.synchronize()
        batch_hits.append(total_of(outs[0], B))
        # pairs spans may leave gaps: + 4096 x the most hits of one topic (tmatch.h)
        if pairs_out:
            mx = outs[0]["hit"][:B].view(torch.int32).view(B, 2)[:, 1].max()
        elif not (filter_sharded or split > 1):
            mx = (outs[0]["hit"][1:B + 1] - outs[0]["hit"][:B]).max()
        else:
            mx = torch.zeros((), dtype=torch.int64)
        pairs_slack[0] = max(pairs_slack[0], 4096 * int(mx.item()))
        total_hits = max(total_hits, batch_hits[-1])
        if split > 1:   # each sub-batch's CSR is offset from 0: its own capacity is its own hits
            hv = outs[0]["hit"]
            total_hits = max(total_hits, max(int(hv[lo + n].item()) - int(hv[lo].item()) for lo, n in parts))
        if xch is not None:
            xch.size_from(outs[0]["hit"])   # per-peer exchange capacity: setup, not the data path
    slack = a.deltas * (a.steps + a.warmup) * 64 if dchunks else 0   # churn may add hits
    cap = total_hits + slack + (pairs_slack[0] if pairs_out else 0)
    cap_pairs = total_hits + slack + pairs_slack[0]
    for o in outs:
        o["out"] = torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)
    for _ in range(a.warmup):
        step(cap)
    torch.cuda.synchronize()
    assert not any(bool(o["err"].any().item()) for o in outs)

    # (no HIP timing events inside the timed region: the library's profiling
    # events recorded around every walk cost the three-stream step 5-7 %,
    # DESIGN.md 5 -- the per-kernel figures come from the profiled repeat and
    # the isolated pass below)
    ix.profile(False)
    apply_s[0] = 0.0
    # the host loop stands in for the NIF's C caller: keep Python's cyclic
    # collector out of the timed region (a full collection stalled the GPU
    # ~7 ms at a time in c5 traces, where each step waits for its deltas) --
    # collected before the barrier, so the ranks leave it together
    gc.collect()
    gc.freeze()
    gc.disable()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t0_wall = time.time()
    merged = None
    for _ in range(a.steps):
        merged = step(cap)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    log(f"[rank {rank}] timed region {t0_wall:.6f} .. {t0_wall + el:.6f} (wall clock)")
    gc.enable()
    if world > 1:
        dist.barrier()
    # the profiled repeat: the same steps again with the library's events
    # around each walk (the overlapped per-kernel figures), untimed
    prof_steps = 0 if (filter_sharded or split > 1 or dchunks) else a.steps
    kstep0 = kstep[0]
    pouts = [{"hit": torch.zeros(B + 1, dtype=torch.int64, device=dev),
              "err": torch.zeros(B, dtype=torch.uint8, device=dev),
              "out": torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)} for _ in range(nstreams)] \
        if prof_steps else None   # (the timed steps' outputs stay intact for the parity sample)
    ix.profile(True)
    ix.profile_read(reset=True)
    tp = time.perf_counter()
    for _ in range(prof_steps):
        step(cap, pouts)
    torch.cuda.synchronize()
    el_prof = time.perf_counter() - tp
    walk_ms, batch_ms, nb = ix.profile_read(reset=True)
    ix.profile(False)
    kstep[0] = kstep0
    del pouts
    if xch is not None:   # the on-device high-water mark: did any timed batch overflow the capacity?
        assert xch.check(), "filter-sharded exchange capacity overflowed during the timed steps"
    last_k = kstep[0] - 1
    last_batch = last_k % R
    # the last timed step's CSR(s): (first topic, topics, output set) per sub-batch
    last_parts = ([(lo, n, outs[j]) for j, (lo, n) in enumerate(parts)] if split > 1
                  else [(0, B, outs[last_k % nstreams])])
    last_hits = 0
    for lo, n, o in last_parts:
        h = total_of(o, n)
        assert h <= cap
        if pairs_out:   # the extent: no value dropped
            assert (int(o["hit"][n].item()) >> 32) <= cap
        last_hits += h
    merged_total = int(merged[0][-1].item()) if merged is not None else None
    merged_topics = merged[0].numel() - 1 if merged is not None else None
    # The walk kernel alone: two passes over the R batches, back to back on
    # one stream (so no other kernel runs beside a walk), waited for once at
    # the end.  An event recorded on an idle stream is stamped before the
    # host has enqueued the kernel behind it, so one unprofiled batch goes
    # first and every profiled launch is enqueued while the stream is busy:
    # the events then bracket the kernel alone, as rocprof does.  This is the
    # duration roofline.kernel_avg_ms reports; rocprof sees these launches as
    # the last 2 R full-grid k_walk_fast launches of the run
    # (tools/prof_report.py splits them out).
    iso_passes = 2
    spare = {"hit": torch.zeros(B + 1, dtype=torch.int64, device=dev),
             "err": torch.zeros(B, dtype=torch.uint8, device=dev),
             "out": torch.zeros(max(cap, 1), dtype=torch.int32, device=dev)}   # the timed steps' outputs stay intact

    def iso_launch(d_blob, d_offs):
        match(B, d_blob, d_offs, spare, cap, stream)

    ix.profile(False)
    torch.cuda.synchronize()
    iso_launch(*d_in[0])
    ix.profile(True)
    paths0 = [ix.debug_get(k) for k in (_native.TM_DEBUG_PATH_PHASES, _native.TM_DEBUG_PATH_SMALL,
                                        _native.TM_DEBUG_PATH_LANE)]
    for _ in range(iso_passes):
        for d_blob, d_offs in d_in:
            iso_launch(d_blob, d_offs)
    torch.cuda.synchronize()
    iso_walk_ms, iso_batch_ms, iso_nb = ix.profile_read(reset=True)
    ix.profile(False)
    # the kernel the events bracketed: k_walk_fast (the walk of the two-phase
    # path), or for a batch of <= 65536 topics the one-launch k_walk_small /
    # (walk, look-back scan and emit in one kernel)
    paths1 = [ix.debug_get(k) for k in (_native.TM_DEBUG_PATH_PHASES, _native.TM_DEBUG_PATH_SMALL,
                                        _native.TM_DEBUG_PATH_LANE)]
    path = max(range(3), key=lambda i: paths1[i] - paths0[i])
    kernel = "k_walk_pairs" if pairs_out else ("k_walk_fast", "k_walk_small", "k_walk_small")[path]
    one_launch = path != 0 or pairs_out   # (the kernel writes the values too)
    el_t = torch.tensor([el], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el_max = float(el_t.item())

    # The other output form over the same batches, streams and step count
    # (rank 0 of a one-GPU topic-sharded run): the CSR next to the pairs
    # headline, or the pairs next to a CSR one
    alt = None
    if world == 1 and not (filter_sharded or level0 or split > 1 or dchunks):
        alt_pairs = not pairs_out
        aouts = [{"hit": torch.zeros(B + 1, dtype=torch.int64, device=dev),
                  "err": torch.zeros(B, dtype=torch.uint8, device=dev),
                  "out": torch.zeros(max(cap_pairs, 1), dtype=torch.int32, device=dev)} for _ in range(nstreams)]

        def alt_step(k):
            match(B, *d_in[k % R], aouts[k % nstreams], cap_pairs, streams[k % nstreams].cuda_stream, pairs=alt_pairs)

        for k in range(a.warmup):
            alt_step(k)
        torch.cuda.synchronize()
        gc.collect()
        gc.disable()
        t1 = time.perf_counter()
        for k in range(a.steps):
            alt_step(a.warmup + k)
        torch.cuda.synchronize()
        el_alt = time.perf_counter() - t1
        gc.enable()
        assert all(total_of(o, B, pairs=alt_pairs) <= cap_pairs for o in aouts)
        if alt_pairs:   # the extent (nothing dropped)
            assert all((int(o["hit"][B].item()) >> 32) <= cap_pairs for o in aouts)
        alt = {"outputs": "pairs" if alt_pairs else "csr", "value": round(B * a.steps / el_alt, 1),
               "ms_per_step": round(el_alt / a.steps * 1e3, 4),
               "api": "tm_match_batch_dev_pairs" if alt_pairs else "tm_match_batch_dev",
               "note": "same batches, streams, warm-up and step count, timed after the headline region"}
        del aouts

    # whole-job topics/s: topic-sharded = every rank's own batch; filter-sharded = the one shared batch
    topics_per_step = B if filter_sharded else world * B
    value = topics_per_step * a.steps / el_max
    ms_per_step = el_max / a.steps * 1e3
    walk_avg_ms = walk_ms / max(nb, 1)
    batch_avg_ms = batch_ms / max(nb, 1)
    iso_ms = iso_walk_ms / max(iso_nb, 1)
    iso_batch = iso_batch_ms / max(iso_nb, 1)

    # Host-side legs, driven by native threads (emqx_amd/csrc/hostbench.cpp:
    # what the NIF's dirty schedulers do, without Python's GIL in the loop):
    #  - p50/p99 of host-to-host batches of n topics (tm_host_alloc buffers:
    #    the kernels read the topics and write the hit lists in place),
    #  - concurrent callers: 8 and 16 threads of 4k-topic batches while one
    #    thread applies subscribe/unsubscribe deltas,
    #  - host-fed pipeline: 1M-topic batches from pinned host memory, H2D +
    #    match + D2H overlapped on 3 streams (LookupRps's host-side unit,
    #    emqx_broker_bench.erl:68-76), next to the PCIe bytes it moves.
    ts = tsets[0]
    lat_native, conc, hostfed = {}, None, None
    if not filter_sharded and a.latency_batches > 0:
        hb = host_bench_lib()
        for lb in sorted({1, 64, 1024, min(4096, B), min(65536, B)}):
            sub = ts.slice(0, lb)
            hh, _, _ = ix.match_batch(sub.blob, sub.offs)
            out = (ctypes.c_double * 3)()
            rc = hb.tmb_single(ix._h, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096,
                               a.latency_batches * 5, out)
            assert rc == 0, rc
            lat_native[str(lb)] = {"p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4), "mean_ms": round(out[2], 4)}
        # the NIF's entry point (u32 offsets) with the inputs in TM_ALLOC_VRAM
        # memory the caller writes before every batch (the copy is timed)
        lb = min(4096, B)
        sub = ts.slice(0, lb)
        hh, _, _ = ix.match_batch(sub.blob, sub.offs)
        out = (ctypes.c_double * 3)()
        rc = hb.tmb_single_ex(ix._h, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096,
                              a.latency_batches * 5, 5, out)
        assert rc == 0, rc
        lat_native[f"{lb}_u32_vram_inputs"] = {"p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4),
                                               "mean_ms": round(out[2], 4)}
        out = (ctypes.c_double * 3)()   # the same through tm_match_batch32_pairs (the NIF's call)
        rc = hb.tmb_single_ex(ix._h, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096,
                              a.latency_batches * 5, 6, out)
        assert rc == 0, rc
        lat_native[f"{lb}_u32_vram_inputs_pairs"] = {"p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4),
                                                     "mean_ms": round(out[2], 4)}
        # the CSR call with k_walk_small's blocks in dispatch order instead of
        # the start-order ticket (TM_DEBUG_SMALL_TICKET, default 1: forward
        # progress of the look-back by construction, include/tmatch.h) -- what
        # the guarantee costs
        ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, 1 - a.small_ticket)
        out = (ctypes.c_double * 3)()
        rc = hb.tmb_single_ex(ix._h, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh[-1]) + 4096,
                              a.latency_batches * 5, 5, out)
        ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, a.small_ticket)
        assert rc == 0, rc
        lat_native[f"{lb}_u32_vram_inputs_" + ("dispatch_order" if a.small_ticket else "ticket")] = {
            "p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4), "mean_ms": round(out[2], 4)}
        if a.concurrency > 0:
            conc = []
            if a.combine_leaders is not None:
                ix.debug_set(_native.TM_DEBUG_COMBINE, a.combine_leaders)
            # (threads, deltas per ms from one more thread, mode): without churn, then with; mode 4: the
            # u32-offset API the NIF calls (tm_match_batch32_ex), 0: the u64 one
            # mode 5: mode 4 with the inputs in TM_ALLOC_VRAM memory, written by each caller before
            # every batch (as a NIF packs its micro-batch): no PCIe read on the kernel's path
            # mode 6: mode 5 through tm_match_batch32_pairs -- per-topic (offset, count) pairs, no
            # cross-block look-back: what the NIF binds (c_src/tmatch_nif_core.c tmn_match)
            for nth, churn, mode in ((a.concurrency, 0, 0), (a.concurrency, 0, 4), (a.concurrency, 256, 4),
                                     (2 * a.concurrency, 256, 4), (a.concurrency, 0, 5), (a.concurrency, 256, 5),
                                     (2 * a.concurrency, 256, 5), (a.concurrency, 0, 6), (a.concurrency, 256, 6),
                                     (2 * a.concurrency, 0, 6), (2 * a.concurrency, 256, 6)):
                lb = min(4096, B)
                sub = ts.slice(0, nth * lb)
                hh, _, _ = ix.match_batch(sub.blob, sub.offs)
                cap = int(np.diff(hh.astype(np.int64)).reshape(nth, lb).sum(axis=1).max()) + 65536
                out = (ctypes.c_double * 6)()
                fr0 = [ix.debug_get(k) for k in (_native.TM_DEBUG_FAILED_BATCHES, _native.TM_DEBUG_RETRIED_BATCHES)]
                rc = hb.tmb_callers_ex(ix._h, nth, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), cap, 1.0, churn,
                                       mode, out)
                assert rc == 0, rc
                fr1 = [ix.debug_get(k) for k in (_native.TM_DEBUG_FAILED_BATCHES, _native.TM_DEBUG_RETRIED_BATCHES)]
                conc.append({"threads": nth, "topics_per_batch": lb, "batches": int(out[0]),
                             "topics_per_s": round(out[1], 1), "p50_ms": round(out[2], 4), "p99_ms": round(out[3], 4),
                             "deltas_per_s": round(out[4], 1), "offsets": "u32" if mode >= 4 else "u64",
                             # one-launch batches whose look-back wait expired (err 4; each is run
                             # again once, a second failure is TM_EDEVICE): forward progress under
                             # concurrent launches, measured
                             "failed_batches": fr1[0] - fr0[0], "retried_batches": fr1[1] - fr0[1],
                             "inputs": "vram (written per batch)" if mode in (5, 6) else "host",
                             "outputs": "pairs" if mode == 6 else "csr",
                             "combine_leaders": ix.debug_get(_native.TM_DEBUG_COMBINE) if mode >= 4 else None,
                             "callers": "native threads, tm_host_alloc buffers each (in place)"})
        if B >= 65536:
            allt = wl.concat(tsets)
            out = (ctypes.c_double * 5)()
            iters = 48
            # mode bit 1: every H2D on one upload stream, every D2H on one download
            # stream, joined to the batches' compute streams by events -- both PCIe
            # directions then run at once (1.06e9 vs 8.1e8 topics/s with each batch's
            # copies on its own stream, profiles/r4/pipe/)
            rc = hb.tmb_pipeline_ex(ix._h, local, _native._ptr(allt.blob), _native._ptr(allt.offs), B, R, 3, iters, 2,
                                    out)
            assert rc == 0, rc
            out32 = (ctypes.c_double * 5)()   # the same with u32 offsets both ways (tm_match_batch32_dev)
            rc = hb.tmb_pipeline_ex(ix._h, local, _native._ptr(allt.blob), _native._ptr(allt.offs), B, R, 3, iters, 3,
                                    out32)
            assert rc == 0, rc
            h2d, d2h = out[2], out[3]
            hostfed = {"topics_per_s": round(out[0], 1), "ms_per_batch": round(out[1], 4), "batch": B,
                       "streams": 3, "h2d_MB_per_batch": round(h2d / 1e6, 2), "d2h_MB_per_batch": round(d2h / 1e6, 2),
                       "pcie_GBps": {"h2d": round(h2d / (out[1] * 1e-3) / 1e9, 1),
                                     "d2h": round(d2h / (out[1] * 1e-3) / 1e9, 1)},
                       "note": "topics in pinned host memory -> H2D -> match -> D2H of offsets and values into pinned "
                               "host memory; 3 compute streams, H2D on one upload stream and D2H on one download "
                               "stream (event-joined); value bytes per batch from a sizing pass"}
            # the PCIe bound this implies: plain pinned copies of 256 MiB, both directions at once
            pc = (ctypes.c_double * 4)()
            assert hb.tmb_pcie(local, 256 << 20, 16, 4, pc) == 0
            # the bound: full duplex at each direction's one-way peak (the simultaneous
            # two-stream copy rate, both_each, varies 28-44 GB/s between runs)
            per = max(h2d / (pc[0] * 1e9), d2h / (pc[1] * 1e9)) if pc[0] > 0 and pc[1] > 0 else 0.0
            hostfed["pcie_ceiling_GBps"] = {"h2d_alone": round(pc[0], 1), "d2h_alone": round(pc[1], 1),
                                            "both_each": round(pc[2], 1)}
            if per > 0:
                hostfed["pcie_bound_topics_per_s"] = round(B / per, 1)
                hostfed["frac_of_pcie_bound"] = round(out[0] / (B / per), 3)
            per32 = max(out32[2] / (pc[0] * 1e9), out32[3] / (pc[1] * 1e9)) if pc[0] > 0 and pc[1] > 0 else 0.0
            hostfed["u32_offsets"] = {"topics_per_s": round(out32[0], 1), "ms_per_batch": round(out32[1], 4),
                                      "h2d_MB_per_batch": round(out32[2] / 1e6, 2),
                                      "d2h_MB_per_batch": round(out32[3] / 1e6, 2),
                                      "pcie_bound_topics_per_s": round(B / per32, 1) if per32 else None,
                                      "frac_of_pcie_bound": round(out32[0] / (B / per32), 3) if per32 else None,
                                      "note": "tm_match_batch32_dev: u32 topic and hit offsets over PCIe"}
    if world > 1 and lat_native:
        # the slowest rank's percentiles (max over ranks); the caller and
        # host-fed legs are rank 0's (each rank drives its own GPU alike)
        keys = sorted(lat_native)
        v = torch.tensor([lat_native[k][q] for k in keys for q in ("p50_ms", "p99_ms")], dtype=torch.float64,
                         device=cdev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        v = v.tolist()
        lat_native = {k: {"p50_ms": v[2 * i], "p99_ms": v[2 * i + 1], "mean_ms": lat_native[k]["mean_ms"]}
                      for i, k in enumerate(keys)}
    lat_pinned = lat_native
    replicas = replica_leg(a, fs, ix, ts, local) if a.replicas > 0 and rank == 0 else None
    writes = (route_write_leg(a, fs, ts, local) if a.route_writers > 0 and a.concurrency > 0 and rank == 0
              and not filter_sharded and not level0 and a.config in ("c3", "c1") else None)

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    sys.path.insert(0, str(ROOT / "oracle"))
    from pyoracle import Oracle, frontier

    cpu_threads, cpu_info = host_cpus()
    if a.cpu_threads:
        cpu_threads = a.cpu_threads
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
        # the last timed step's output of this rank (its own shard's lists for c4)
        host_parts = [(lo, n, o["hit"][: n + 1].cpu().numpy().view(np.uint64), o["out"].cpu().numpy().view(np.uint32))
                      for lo, n, o in last_parts]
        if pairs_out:   # (first position, count) per topic -> the same slicing as a CSR's [start, end)
            host_parts = [(lo, n, hh.view(np.uint32)[: 2 * n].reshape(n, 2).astype(np.uint64), ho)
                          for lo, n, hh, ho in host_parts]
        rng = np.random.default_rng(0x454D5158)
        idx = np.sort(rng.choice(B, ns, replace=False))
        lts = tsets[last_batch]
        sblob, soffs = _native.pack_strings([lts.item(int(i)) for i in idx])
        cnt, _, ohit, ovals = o.match_batch(sblob, soffs, nthreads=cpu_threads)
        mism = 0
        for j, i in enumerate(idx):
            lo, _, host_hit, host_out = next(p for p in host_parts if p[0] <= i < p[0] + p[1])
            if pairs_out:
                p0, c0 = int(host_hit[i - lo][0]), int(host_hit[i - lo][1])
                g = host_out[p0:p0 + c0]
            else:
                g = host_out[int(host_hit[i - lo]):int(host_hit[i - lo + 1])]
            e = ovals[int(ohit[j]):int(ohit[j + 1])]
            mism += int(not np.array_equal(g, e))
        # algorithmic bytes per launch of the timed kernel (SURVEY.md 8d per
        # topic):  8 L + 32 sum|F_l| + 4 H + 4 for a one-launch batch (the
        # kernel writes the values too), minus the 4 H for k_walk_fast (the
        # emit kernel writes them); averaged over the R batches (L and H
        # exact, sum|F_l| from an ns / R sample of each)
        per = max(1, ns // R)
        wb = []
        for k, tk in enumerate(tsets):
            kidx = np.sort(rng.choice(B, per, replace=False))
            fb, fo = _native.pack_strings([tk.item(int(i)) for i in kidx])
            _, states = frontier(o, fb, fo, nthreads=cpu_threads)
            L_total = int(np.count_nonzero(tk.blob[: int(tk.offs[-1])] == ord("/"))) + B
            F_total = float(states.sum()) * B / per
            wb.append(8 * L_total + 32 * F_total + 4 * B + (4 * batch_hits[k] if one_launch else 0))
        walk_bytes = float(np.mean(wb))
        achieved = walk_bytes / (iso_ms * 1e-3) / 1e9
        res_extra["full_path_GBps"] = round((walk_bytes + (0 if one_launch else 4 * last_hits)) /
                                            (iso_batch * 1e-3) / 1e9, 1)

        # ---- CPU baseline: the oracle (restated reference walk) on the host's CPUs
        if not a.no_cpu and world == 1 and a.config in ("c1", "c2", "c2nm", "c3", "c3deep"):
            n1 = min(20_000, B)
            probe = ts.slice(0, n1)
            t1 = time.perf_counter()
            o.match_batch(probe.blob, probe.offs, nthreads=cpu_threads, with_values=False)
            r1 = n1 / (time.perf_counter() - t1)
            # a bounded sample of about cpu_seconds of CPU work: whole passes over
            # the batch when it is shorter than that, else its first n2 topics
            want = int(max(n1, r1 * a.cpu_seconds))
            passes, n2 = (max(1, round(want / B)), B) if want >= B else (1, want)
            samp = ts.slice(0, n2)
            t1 = time.perf_counter()
            for _ in range(passes):
                o.match_batch(samp.blob, samp.offs, nthreads=cpu_threads, with_values=False)
            el_cpu = time.perf_counter() - t1
            what = f"{passes} passes over the {B}-topic batch" if passes > 1 else f"first {n2} topics of the batch"
            cpu = {"value": round(passes * n2 / el_cpu, 1), "unit": "topic matches/s", "cores": cpu_threads,
                   "kind": "port", **cpu_info,
                   "sample": f"{what} vs all {len(fs)} keys; oracle/tm_oracle.c seek walker (emqx_trie_search "
                             f"restated) over a sorted key array, {cpu_threads} pthreads (one per CPU this "
                             f"process may use), {el_cpu:.1f}s"}

    # memory-side traffic of the walk: PMC counters cannot be read inside this
    # process, so they come from profiles/pmc_<config>.json -- used only if it
    # was measured on the kernels this tree builds (source hash) and the same
    # workload shape
    traffic = mem_req = None
    traffic_note = "no profiles/pmc_{}.json".format(a.config)
    pmc = ROOT / "profiles" / f"pmc_{a.config}.json"
    if pmc.exists():
        try:
            pj = json.loads(pmc.read_text())
            same = (pj.get("filters") == len(fs) and pj.get("batch") == B and pj.get("rotate") == R
                    and kernel in (pj.get("walk_kernel") or ""))
            fresh = pj.get("source_hash") == source_hash()
            if same and fresh:
                traffic = pj.get("walk_hbm_bytes_per_launch")
                mem_req = pj.get("walk_mem_requests_per_launch")
                traffic_note = f"{pj.get('source')} (kernel sources {pj['source_hash']}, this tree)"
            else:
                traffic_note = ("refused: " + ("stale (measured on other kernel sources)" if not fresh
                                              else "different workload shape or kernel") + f" -- {pj.get('source')}")
        except (ValueError, KeyError, OSError) as e:
            traffic_note = f"unreadable: {e!r}"
    # practical roofline of a pointer-chasing walk: the measured memory-side
    # random-request rate (tools/gather_bench.hip, profiles/r1_gather.md)
    req_ceiling = None
    if mem_req and iso_ms:
        rate = mem_req / (iso_ms * 1e-3)
        req_ceiling = {"requests_per_launch": mem_req, "requests_per_s": round(rate, 1),
                       "ceiling_per_s": RANDOM_REQ_CEILING, "frac": round(rate / RANDOM_REQ_CEILING, 4),
                       "source": "profiles/r1_gather.md (64-B random requests beyond L2, 256 MiB-2 GiB tables)"}

    metric = {"c3": "topic matches/sec at 10M filters"}.get(a.config, f"topic matches/sec ({a.config})")
    par = (f"filter-sharded x{world} (RCCL all_to_all of per-slice counts and hit lists, device merge)" if filter_sharded
           else f"level-0 sharded x{world} (first-level words partitioned, '+'/'#' roots replicated; "
                f"topics routed by first level; no data-path collective)" if level0
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
        "config": {"workload": f"{a.config}: {desc}", "filters": nf if (filter_sharded or level0) else len(fs),
                   "topics_per_gpu_step": B, "global_batch": topics_per_step, "parallelism": par,
                   "streams": nstreams, "sub_batches_per_step": split, "distinct_batches": R,
                   "table_copies": copies, "outputs": a.outputs},
        "roofline": {"bound": "hbm", "achieved": None if achieved is None else round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_note,
                     "kernel": kernel, "kernel_avg_ms": round(iso_ms, 4),
                     "kernel_launches": int(iso_nb),
                     "kernel_timing": (f"HIP events on the launch stream around {kernel}, {iso_passes} passes over "
                                       f"the {R} batches back to back on one stream after the timed region"),
                     "kernel_work": ("the walk writing every value into its block's reserved span, pairs out "
                                     "(8 L + 32 sum|F| + 4 H + 4 B per topic)" if pairs_out else
                                     "the whole batch: walk, look-back scan and CSR emission (8 L + 32 sum|F| + "
                                     "4 H + 4 B per topic)" if one_launch else
                                     "the walk (8 L + 32 sum|F| + 4 B per topic; the values are k_emit's)"),
                     "algorithmic_bytes_per_launch": None if walk_bytes is None else int(walk_bytes),
                     "random_request_roofline": req_ceiling,
                     "effective": {"kernel_avg_ms_overlapped": round(walk_avg_ms, 4) if nb else None,
                                   "profiled_repeat_ms_per_step": round(el_prof / prof_steps * 1e3, 4) if prof_steps
                                   else None,
                                   "walk_GBps_per_step": None if walk_bytes is None
                                   else round(walk_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                                   "note": f"the walks of a profiled repeat of the timed steps (overlapping the other "
                                           f"{nstreams - 1} streams' kernels; HIP timing events around each walk, "
                                           f"which the timed region does not carry); "
                                           f"GBps_per_step = algorithmic bytes / ms_per_step"}},
        # a step can be shorter than one walk alone: with three streams the
        # next batch's walk fills the GPU while one batch's walk drains (its
        # last waves leave CUs idle), so the check bounds the step by the
        # isolated walk over the streams instead
        "checks": {"walk_isolated_le_ms_per_step": bool(iso_ms <= ms_per_step),
                   "step_ge_isolated_walk_over_streams": bool(ms_per_step >= iso_ms / nstreams)},
        "other_outputs": alt,
        "cpu_baseline": cpu,
        "matched_ids_per_s": round(last_hits * (1 if filter_sharded else world) * a.steps / el_max, 1),
        "hits_per_topic": round(merged_total / max(merged_topics, 1) if merged_total is not None else last_hits / B, 3),
        "batch_device_ms": round(batch_avg_ms, 4) if nb else None,
        "batch_device_isolated_ms": round(iso_batch, 4),
        "batch_latency_host_ms": lat_pinned,
        "concurrent_callers": conc,
        "host_fed": hostfed,
        "parity_sample": None if mism is None else {"topics": ns, "mismatches": mism,
                                                    "against": "oracle over this rank's keys" + (
                                                        " (every filter that can match a topic this rank owns: "
                                                        "the unsharded answer, order included)" if level0 else "")},
        "build": {"generate_s": round(t_gen, 1), "compile_s": round(t_compile, 1), "upload_s": round(t_upload, 2),
                  "device_MiB": round(st["device_bytes"] / 2**20, 1),
                  "device_MiB_all_copies": round(copies * st["device_bytes"] / 2**20, 1), "nodes": st["n_nodes"],
                  "edges": st["n_edges"], "words": st["n_words"], "keys_this_rank": st["n_keys"],
                  "kernel_source_hash": source_hash()},
    }
    res.update(res_extra)
    if replicas is not None:
        res["replicas"] = replicas
    if writes is not None:
        res["route_writes"] = writes
    if dchunks:
        res["deltas_per_step"] = a.deltas / every
        res["delta_batch"] = {"deltas": a.deltas, "every_steps": every}
        res["deltas_per_s"] = round(a.deltas / every * a.steps / el_max, 1)
        res["delta_apply_host_ms_per_step"] = round(apply_s[0] / a.steps * 1e3, 4)
    if filter_sharded:
        res["merged_hits_this_rank_slice"] = merged_total
        res["merged_topics_this_rank_slice"] = merged_topics
        if xch is not None:
            res["exchange"] = {"per_peer_capacity": xch.per_peer, "slice": xch.s,
                               "collectives": "all_to_all_single of u32 counts + padded u32 values (RCCL)"}
    if cpu:
        res["speedup_vs_cpu"] = round(value / cpu["value"], 1)
    if not res["checks"]["step_ge_isolated_walk_over_streams"]:
        log(f"WARNING: ms_per_step {ms_per_step:.4f} ms < isolated walk {iso_ms:.4f} ms / {nstreams} streams")
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def replica_leg(a, fs, ix, ts, local):
    """One EMQX node's deployment (emqx_router.erl:133-162:
    one replicated route table per node): ONE host image compiled once, N
    device replicas (tm_create_replicas), host-API batches spread over them by
    the library, one syncer thread's tm_apply_deltas reaching every replica.
    Feeder threads submit in-place 64k-topic batches (tm_host_alloc buffers,
    u32 offsets: what the NIF's dirty schedulers do), with and without churn;
    per-replica batch counts from tm_replica_stats.  Its parity: the replica
    index's lists on a sample equal the primary index's (which the oracle
    sample checks) element for element."""
    import torch
    from emqx_amd import _native
    ngpu = torch.cuda.device_count()
    devices = [d % ngpu for d in range(a.replicas)] if ngpu >= a.replicas else [local] * a.replicas
    t = time.time()
    rx = _native.Index(devices=devices, hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        rx.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    t_build = time.time() - t
    sub = ts.slice(0, min(len(ts), 20_000))
    h0, v0, e0 = ix.match_batch(sub.blob, sub.offs)
    h1, v1, e1 = rx.match_batch(sub.blob, sub.offs)
    exact = bool(np.array_equal(h0, h1) and np.array_equal(v0, v1) and np.array_equal(e0, e1))
    hb = host_bench_lib()
    legs = []
    lb = min(65536, len(ts) // max(1, 2 * a.replicas))
    for nth, churn in ((2 * a.replicas, 0), (2 * a.replicas, 256)):
        s2 = ts.slice(0, nth * lb)
        hh, _, _ = rx.match_batch(s2.blob, s2.offs)
        cap = int(np.diff(hh.astype(np.int64)).reshape(nth, lb).sum(axis=1).max()) + 65536
        before = [rx.replica_stats(r)[0] for r in range(a.replicas)]
        fr0 = [rx.debug_get(k) for k in (_native.TM_DEBUG_FAILED_BATCHES, _native.TM_DEBUG_RETRIED_BATCHES)]
        out = (ctypes.c_double * 6)()
        rc = hb.tmb_callers_ex(rx._h, nth, lb, _native._ptr(s2.blob), _native._ptr(s2.offs), cap, 2.0, churn, 4, out)
        assert rc == 0, rc
        fr1 = [rx.debug_get(k) for k in (_native.TM_DEBUG_FAILED_BATCHES, _native.TM_DEBUG_RETRIED_BATCHES)]
        per = [rx.replica_stats(r)[0] - before[r] for r in range(a.replicas)]
        legs.append({"feeder_threads": nth, "topics_per_batch": lb, "topics_per_s": round(out[1], 1),
                     "p50_ms": round(out[2], 4), "p99_ms": round(out[3], 4), "deltas_per_s": round(out[4], 1),
                     "batches_per_replica": per, "failed_batches": fr1[0] - fr0[0],
                     "retried_batches": fr1[1] - fr0[1]})
    st = rx.stats()
    rx.close()
    return {"replicas": a.replicas, "devices": devices,
            "rehearsal": len(set(devices)) < a.replicas,
            "note": ("replicas sharing a GPU: the control flow and balance of the one-process deployment, not "
                     "scaling" if len(set(devices)) < a.replicas else "one replica per GPU"),
            "build_s": round(t_build, 1), "device_MiB_per_replica": round(st["device_bytes"] / 2**20, 1),
            "parity_sample": {"topics": len(sub), "equal_to_primary_index": exact},
            "legs": legs}


def route_write_leg(a, fs, ts, local):
    """Route writes under publish load (the reference's
    broker pool runs do_add_route in up to schedulers x 2 workers,
    emqx_broker_sup.erl:36, emqx_broker.erl:778-808): `--route-writers`
    threads each subscribe and unsubscribe one key at a time and wait for the
    mirror to hold it (the read-your-writes hook); ONE mirror thread takes every
    queued request into ONE tm_commit (src/emqx_router_gpu.erl's group commit),
    published on a table copy no publish batch is reading; meanwhile
    --concurrency matcher threads run 4k-topic batches the NIF's way (u32
    offsets, inputs in TM_ALLOC_VRAM memory, the combiner).  After each
    subscribe the writer publishes its own topic and must see its route
    (ryw_misses counts the failures).  The same with tm_apply_deltas as the
    commit (every publish batch after a write first waits for the batches
    reading the copy it patches) for comparison.  On a second index of the
    same filters with --writes-copies copies of the tables."""
    from emqx_amd import _native
    t = time.time()
    wx = _native.Index(device=local, hint_keys=len(fs), copies=a.writes_copies)
    wx.debug_set(_native.TM_DEBUG_SMALL_TICKET, a.small_ticket)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        wx.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    t_build = time.time() - t
    hb = host_bench_lib()
    lb, nm = 4096, a.concurrency
    sub = ts.slice(0, nm * lb)
    hh, _, _ = wx.match_batch(sub.blob, sub.offs)
    cap = int(np.diff(hh.astype(np.int64)).reshape(nm, lb).sum(axis=1).max()) + 65536
    legs = []
    for commit in (1, 0):
        keys = (_native.TM_DEBUG_COMMITS, _native.TM_DEBUG_COMMIT_WAITS, _native.TM_DEBUG_COMMIT_FORCED,
                _native.TM_DEBUG_FAILED_BATCHES)
        c0 = [wx.debug_get(k) for k in keys]
        out = (ctypes.c_double * 10)()
        rc = hb.tmb_writers(wx._h, a.route_writers, nm, lb, _native._ptr(sub.blob), _native._ptr(sub.offs), cap, 2.0,
                            1, commit, out)
        assert rc == 0, rc
        c1 = [wx.debug_get(k) for k in keys]
        legs.append({"commit": "tm_commit" if commit else "tm_apply_deltas",
                     "writes_per_s": round(out[0], 1), "write_p50_ms": round(out[1], 4),
                     "write_p99_ms": round(out[2], 4), "group_commits_per_s": round(out[3], 1),
                     "matcher_topics_per_s": round(out[4], 1), "matcher_p50_ms": round(out[5], 4),
                     "matcher_p99_ms": round(out[6], 4), "ryw_checks": int(out[7]), "ryw_misses": int(out[8]),
                     "commits_waiting_for_a_copy": c1[1] - c0[1], "commits_forced": c1[2] - c0[2],
                     "failed_batches": c1[3] - c0[3]})
    wx.close()
    return {"writers": a.route_writers, "matchers": nm, "topics_per_batch": lb, "table_copies": a.writes_copies,
            "build_s": round(t_build, 1), "legs": legs,
            "keys": "writer w: 'bench/writer/<w>/<k>' (binary key) and '<that>/+' (word list) alternately, "
                    "subscribed then unsubscribed"}


def host_bench_lib():
    """libtmbench.so (emqx_amd/csrc/hostbench.cpp): native caller threads and
    the host-fed pipeline over the same libtmatch this process loaded."""
    from emqx_amd.build import LIB_BENCH
    lib = ctypes.CDLL(str(LIB_BENCH))
    vp, u64, dp = ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_double)
    lib.tmb_single.argtypes = [vp, u64, vp, vp, u64, ctypes.c_int, dp]
    lib.tmb_single_ex.argtypes = [vp, u64, vp, vp, u64, ctypes.c_int, ctypes.c_int, dp]
    lib.tmb_callers.argtypes = [vp, ctypes.c_int, u64, vp, vp, u64, ctypes.c_double, ctypes.c_int, dp]
    lib.tmb_callers_ex.argtypes = [vp, ctypes.c_int, u64, vp, vp, u64, ctypes.c_double, ctypes.c_int, ctypes.c_int, dp]
    lib.tmb_writers.argtypes = [vp, ctypes.c_int, ctypes.c_int, u64, vp, vp, u64, ctypes.c_double, ctypes.c_int,
                                ctypes.c_int, dp]
    lib.tmb_pipeline.argtypes = [vp, ctypes.c_int, vp, vp, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp]
    lib.tmb_pipeline_ex.argtypes = [vp, ctypes.c_int, vp, vp, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, dp]
    lib.tmb_pcie.argtypes = [ctypes.c_int, u64, ctypes.c_int, ctypes.c_int, dp]
    lib.tmb_noise_start.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.tmb_noise_stop.argtypes = [dp]
    lib.tmb_bind.argtypes = [vp]
    from emqx_amd import _native
    assert lib.tmb_bind(ctypes.c_void_p(_native.load_library()._handle)) == 0   # the libtmatch this process uses
    return lib


if __name__ == "__main__":
    main()
