#!/usr/bin/env python3
"""Study build (TM_STUDY): per-topic DFS node visits and child-table probes,
packed into the err byte by the instrumented k_walk_fast (TM_LIB=...study.so)."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    from bench import CONFIGS
    from emqx_amd import _native, workload as wl
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    gen, nf, _ = CONFIGS[cfg]
    fs = wl.filters(gen, nf)
    ix = _native.Index(device=0)
    for lo in range(0, len(fs), 2_000_000):
        p = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(p), np.uint8), p.blob, p.offs, p.vals)
    st = ix.stats()
    print(f"{cfg}: nodes {st['n_nodes']} edges {st['n_edges']}", flush=True)
    ts = wl.topics(gen, nf, 200_000)
    hit, vals, err = ix.match_batch(ts.blob, ts.offs)
    import os
    if os.environ.get("TM_STUDY_DEAD"):
        dp, dl = (err & 15).astype(np.int64), (err >> 4).astype(np.int64)
        print(f"{cfg}: dead-end visits (emit nothing, lead nowhere) reached via '+' mean {dp.mean():.2f}, "
              f"via a literal edge or a pop mean {dl.mean():.2f} (each capped at 15)", flush=True)
        return
    if os.environ.get("TM_STUDY_MISS"):
        a, b = (err & 15).astype(np.int64), (err >> 4).astype(np.int64)
        what = (("absent at levels 0-1", "absent at level 2") if os.environ["TM_STUDY_MISS"] == "1"
                else ("absent at levels >= 3", "found but dead (any level)"))
        print(f"{cfg}: child-table probes {what[0]} mean {a.mean():.2f}, {what[1]} mean {b.mean():.2f} "
              f"(each capped at 15)", flush=True)
        return
    if os.environ.get("TM_STUDY_LEAF2"):
        imm, pop = (err & 15).astype(np.int64), (err >> 4).astype(np.int64)
        print(f"{cfg}: visits of single-value leaves reached directly ('+' or the only literal child) mean "
              f"{imm.mean():.2f}, off the pending-branch stack mean {pop.mean():.2f} (each capped at 15)", flush=True)
        return
    if os.environ.get("TM_STUDY_LEAF"):
        ct, other = (err & 15).astype(np.int64), (err >> 4).astype(np.int64)
        print(f"{cfg}: visits at the topic's last level (emit only) reached through a child table mean "
              f"{ct.mean():.2f}, through '+' or an inline child mean {other.mean():.2f} (each capped at 15)", flush=True)
        return
    if os.environ.get("TM_STUDY_HITS"):
        hits_, miss_ = (err & 15).astype(np.int64), (err >> 4).astype(np.int64)
        print(f"{cfg}: child-table probes that found the child mean {hits_.mean():.2f}, "
              f"that missed mean {miss_.mean():.2f} (each capped at 15)", flush=True)
        return
    steps = (err & 31).astype(np.int64)
    probes = (err >> 5).astype(np.int64)
    w = steps.reshape(-1, 64)
    print(f"{cfg}: steps mean {steps.mean():.2f} p50 {np.median(steps)} p99 {np.percentile(steps, 99)} "
          f"wave-max mean {w.max(1).mean():.2f}; ctab probes mean {probes.mean():.2f} "
          f"wave-max mean {probes.reshape(-1, 64).max(1).mean():.2f}", flush=True)


if __name__ == "__main__":
    main()
