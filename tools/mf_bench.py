#!/usr/bin/env python3
"""matches_filter/3 on the device at C3 scale (10M filters): the first call
builds the term-ordered key array (host sort + upload), later calls only run
the walk.  Queries are subscription filters drawn from the filter set (valid
MQTT filters), checked against the C oracle on a sample.
usage: mf_bench.py [filters] [queries]"""
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main(nf=10_000_000, nq=10_000):
    nf, nq = int(nf), int(nq)
    from emqx_amd import _native, workload as wl
    fs = wl.filters(3, nf)
    ix = _native.Index(device=0, hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        p = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(p), np.uint8), p.blob, p.offs, p.vals)
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(len(fs), nq, replace=False))
    qs = [fs.item(int(i)) for i in idx]
    blob, offs = _native.pack_strings(qs)
    t = time.perf_counter()
    hit, vals, err = ix.matches_filter_batch(blob[:int(offs[1]) + 16], offs[:2])
    t_build = time.perf_counter() - t
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        hit, vals, err = ix.matches_filter_batch(blob, offs)
        ts.append(time.perf_counter() - t)
    from pyoracle import Oracle
    o = Oracle()
    o.apply(np.ones(len(fs), np.uint8), fs.blob, fs.offs, fs.vals)
    o.prepare()
    sample = list(range(0, nq, max(1, nq // 300)))
    mism = sum(int(vals[hit[i]:hit[i + 1]].tolist() != o.matches_filter(qs[i])) for i in sample)
    print(json.dumps({"filters": len(fs), "queries": nq, "first_call_s (builds the key array)": round(t_build, 2),
                      "batch_s": round(min(ts), 4), "queries_per_s": round(nq / min(ts), 1),
                      "keys_returned": int(hit[-1]), "err": int(err.sum()),
                      "oracle_sample": {"queries": len(sample), "mismatches": mism}}))


if __name__ == "__main__":
    main(*sys.argv[1:])
