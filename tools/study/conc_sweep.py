#!/usr/bin/env python3
"""Concurrent-caller sweep (study): native caller threads of 4k-topic C3
batches (emqx_amd/csrc/hostbench.cpp tmb_callers_ex) over combiner leaders,
small-batch kernel and buffer placement, one second per point.

Modes (tmb_callers_ex): 4 = in place, u32 offsets (the NIF's call, through the
combiner); 0 = in place, u64 offsets (no combiner); 1 = inputs and outputs in
HBM (tm_match_batch_dev, each caller its own stream: no PCIe leg).

Lists take "," or "+" (tools/gpu.sh splits its step arguments on commas).
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--threads", default="8,16")
    p.add_argument("--modes", default="4,1")
    p.add_argument("--leaders", default="1,2,4")
    p.add_argument("--kinds", default="auto,wave,wave8")
    p.add_argument("--churn", type=int, default=0)
    p.add_argument("--seconds", type=float, default=1.0)
    p.add_argument("--copies", type=int, default=1, help="tm_options.copies of the index")
    p.add_argument("--repeat", type=int, default=1, help="passes over the whole sweep (interleaved A/B)")
    a = p.parse_args()
    from bench import CONFIGS, host_bench_lib
    from emqx_amd import _native, workload as wl
    gen, _, _ = CONFIGS["c3"]
    fs = wl.filters(gen, a.filters)
    ix = _native.Index(device=0, copies=a.copies)
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    hb = host_bench_lib()
    kinds = {"auto": _native.SMALL_AUTO, "wave": _native.SMALL_WAVE, "wave8": _native.SMALL_WAVE8,
             "lane": _native.SMALL_LANE}
    lb = 4096
    lead0 = ix.debug_get(_native.TM_DEBUG_COMBINE)
    for rep in range(a.repeat):
        for nth in map(int, a.threads.replace("+", ",").split(",")):
            ts = wl.topics(gen, a.filters, nth * lb)
            hh, _, _ = ix.match_batch(ts.blob, ts.offs)
            cap = int(np.diff(hh.astype(np.int64)).reshape(nth, lb).sum(axis=1).max()) + 65536
            for mode in map(int, a.modes.replace("+", ",").split(",")):
                for kind in a.kinds.replace("+", ",").split(","):
                    ix.debug_set(_native.TM_DEBUG_SMALL_KERNEL, kinds[kind])
                    for lead in (map(int, a.leaders.replace("+", ",").split(",")) if mode in (4, 5) else [0]):
                        if mode in (4, 5):
                            ix.debug_set(_native.TM_DEBUG_COMBINE, lead)
                        l0 = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES)
                        b0 = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES)
                        f0 = ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES)
                        out = (ctypes.c_double * 6)()
                        rc = hb.tmb_callers_ex(ix._h, nth, lb, _native._ptr(ts.blob), _native._ptr(ts.offs), cap,
                                               a.seconds, a.churn, mode, out)
                        assert rc == 0, rc
                        launches = ix.debug_get(_native.TM_DEBUG_COMBINED_LAUNCHES) - l0
                        batches = ix.debug_get(_native.TM_DEBUG_COMBINED_BATCHES) - b0
                        print(json.dumps({"rep": rep, "threads": nth, "mode": mode, "kind": kind, "leaders": lead, "copies": a.copies, "churn": a.churn,
                                          "topics_per_s": round(out[1]), "p50_ms": round(out[2], 4),
                                          "p99_ms": round(out[3], 4), "deltas_per_s": round(out[4]),
                                          "batches_per_launch": round(batches / launches, 2) if launches else None,
                                          "failed": ix.debug_get(_native.TM_DEBUG_FAILED_BATCHES) - f0}), flush=True)
    ix.debug_set(_native.TM_DEBUG_COMBINE, lead0)


if __name__ == "__main__":
    main()
