#!/usr/bin/env python3
"""(Round 6 close: the library's TM_DEBUG_CMB_LAND variant was removed after this sweep measured it slower;
land=1 passes now fail with TM_EINVAL -- run them on the commit that had it, a5371f1.)
Combiner sweep (study, round 6; not product code): native caller threads of
4k-topic C3 batches through tm_match_batch32_ex (the NIF's call; mode 5 =
inputs in TM_ALLOC_VRAM memory, mode 4 = pinned host memory) over combiner
leaders x gather window (TM_DEBUG_CMB_GATHER, us) x landing from HBM
(TM_DEBUG_CMB_LAND), with and without 256-delta churn batches every ms; then
the route-writer leg (tmb_writers: one-key writes group-committed by a mirror
thread while matcher threads run).  One JSON line per point.

Lists take "," or "+" (tools/gpu.sh splits its step arguments on commas);
--combos is "leaders/gather/land[/spin_us]" items.
"""
import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def L(x):
    return [v for v in x.replace("+", ",").split(",") if v]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--threads", default="8,16")
    p.add_argument("--modes", default="5")
    p.add_argument("--churn", default="0,256")
    p.add_argument("--combos", default="4/0/0,4/0/1,2/0/0,2/0/1,1/0/0,1/0/1,4/20/0,2/20/0,1/20/0,2/20/1,1/20/1")
    p.add_argument("--seconds", type=float, default=1.0)
    p.add_argument("--copies", type=int, default=1)
    p.add_argument("--repeat", type=int, default=1)
    p.add_argument("--writers", default="16", help="writer threads of the route-writer leg (0: skip)")
    p.add_argument("--writer-combos", default="4/0/0")
    p.add_argument("--writer-commit", default="1,0", help="1: the mirror ships with tm_commit, 0: tm_apply_deltas")
    p.add_argument("--tickets", default="0", help="TM_DEBUG_SMALL_TICKET values (k_walk_small start-order tickets)")
    p.add_argument("--writer-check", default="1", help="1: each writer publishes its own topic after a subscribe")
    p.add_argument("--patch-zc", default="1", help="TM_DEBUG_PATCH_ZC values")
    p.add_argument("--writer-matchers", default="8")
    p.add_argument("--latency", default="", help="lone-batch sizes for a host-to-host latency leg per ticket value")
    p.add_argument("--latency-modes", default="5", help="tmb_single_ex modes of the latency leg (5: CSR, 6: pairs)")
    p.add_argument("--writer-seconds", type=float, default=2.0)
    a = p.parse_args()
    from bench import CONFIGS, host_bench_lib
    from emqx_amd import _native, workload as wl
    gen, _, _ = CONFIGS["c3"]
    t = time.time()
    fs = wl.filters(gen, a.filters)
    ix = _native.Index(device=0, hint_keys=len(fs), copies=a.copies)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    print(f"# index {len(fs)} keys in {time.time() - t:.1f}s, copies {a.copies}", flush=True)
    hb = host_bench_lib()
    lb = 4096
    thr = [int(x) for x in L(a.threads)]
    ts = wl.topics(gen, a.filters, max(thr) * lb)
    hh, _, _ = ix.match_batch(ts.blob, ts.offs)
    cap = int(np.diff(hh.astype(np.int64)).reshape(max(thr), lb).sum(axis=1).max()) + 65536

    spin = [0]

    def setk(combo):
        f = [int(x) for x in combo.split("/")] + [0]
        lead, gat, land, spin[0] = f[0], f[1], f[2], f[3]
        ix.debug_set(_native.TM_DEBUG_COMBINE, lead)
        try:   # (an older library without these keys: only 0 is meaningful)
            ix.debug_set(_native.TM_DEBUG_CMB_GATHER, gat)
            ix.debug_set(_native.TM_DEBUG_CMB_LAND, land)
            ix.debug_set(_native.TM_DEBUG_CMB_SPIN, spin[0])
        except _native.TmError:
            assert gat == 0 and land == 0 and spin[0] == 0
        return lead, gat, land

    def set_ticket(tk):
        try:
            ix.debug_set(_native.TM_DEBUG_SMALL_TICKET, tk)
        except _native.TmError:
            assert tk == 0

    for n, lm in [(x, m) for x in map(int, L(a.latency)) for m in map(int, L(a.latency_modes))]:
        for rep in range(a.repeat):
            for tk in map(int, L(a.tickets)):
                set_ticket(tk)
                sub = ts.slice(0, n)
                hh2, _, _ = ix.match_batch(sub.blob, sub.offs)
                out = (ctypes.c_double * 3)()
                rc = hb.tmb_single_ex(ix._h, n, _native._ptr(sub.blob), _native._ptr(sub.offs), int(hh2[-1]) + 4096,
                                      400, lm, out)
                assert rc == 0, rc
                print(json.dumps({"leg": "latency", "rep": rep, "topics": n, "ticket": tk, "mode": lm,
                                  "p50_ms": round(out[0], 4), "p99_ms": round(out[1], 4),
                                  "mean_ms": round(out[2], 4)}), flush=True)
    for rep in range(a.repeat):
        for churn in map(int, L(a.churn)):
            for nth in thr:
                for mode in map(int, L(a.modes)):
                    for combo, tk in [(c, t) for c in L(a.combos) for t in map(int, L(a.tickets))]:
                        lead, gat, land = setk(combo)
                        set_ticket(tk)
                        l0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES)
                        b0 = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES)
                        f0 = ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES)
                        out = (ctypes.c_double * 6)()
                        rc = hb.tmb_callers_ex(ix._h, nth, lb, _native._ptr(ts.blob), _native._ptr(ts.offs), cap,
                                               a.seconds, churn, mode, out)
                        assert rc == 0, rc
                        launches = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) - l0
                        batches = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES) - b0
                        print(json.dumps({"rep": rep, "threads": nth, "mode": mode, "leaders": lead, "ticket": tk,
                                          "spin_us": spin[0],
                                          "gather_us": gat,
                                          "land": land, "churn": churn, "topics_per_s": round(out[1]),
                                          "p50_ms": round(out[2], 4), "p99_ms": round(out[3], 4),
                                          "deltas_per_s": round(out[4]),
                                          "batches_per_launch": round(batches / launches, 2) if launches else None,
                                          "failed": ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) - f0}), flush=True)
    for nw in map(int, L(a.writers)):
        if nw <= 0:
            continue
        for combo, cm, ck, zc, nmt in [(c, m, k, z, t) for c in L(a.writer_combos) for m in map(int, L(a.writer_commit))
                                      for k in map(int, L(a.writer_check)) for z in map(int, L(a.patch_zc))
                                      for t in map(int, L(a.writer_matchers))]:
            lead, gat, land = setk(combo)
            set_ticket(0)
            try:
                ix.debug_set(_native.TM_DEBUG_PATCH_ZC, zc)
            except _native.TmError:
                assert zc == 1
            out = (ctypes.c_double * 10)()
            c0 = [ix.debug_get(k) for k in (_native.TM_DEBUG_COMMITS, _native.TM_DEBUG_COMMIT_WAITS,
                                            _native.TM_DEBUG_COMMIT_FORCED)] if cm else [0, 0, 0]
            rc = hb.tmb_writers(ix._h, nw, nmt, lb, _native._ptr(ts.blob), _native._ptr(ts.offs), cap,
                                a.writer_seconds, ck, cm, out)
            assert rc == 0, rc
            c1 = [ix.debug_get(k) for k in (_native.TM_DEBUG_COMMITS, _native.TM_DEBUG_COMMIT_WAITS,
                                            _native.TM_DEBUG_COMMIT_FORCED)] if cm else [0, 0, 0]
            print(json.dumps({"leg": "writers", "commit": cm, "copies": a.copies, "check": ck, "patch_zc": zc,
                              "commits": c1[0] - c0[0], "commit_waits": c1[1] - c0[1], "commit_forced": c1[2] - c0[2],
                              "writers": nw, "matchers": nmt, "leaders": lead, "gather_us": gat,
                              "land": land, "writes_per_s": round(out[0]), "write_p50_ms": round(out[1], 4),
                              "write_p99_ms": round(out[2], 4), "commits_per_s": round(out[3]),
                              "topics_per_s": round(out[4]), "match_p50_ms": round(out[5], 4),
                              "match_p99_ms": round(out[6], 4), "ryw_checks": int(out[7]),
                              "ryw_misses": int(out[8])}), flush=True)


if __name__ == "__main__":
    main()
