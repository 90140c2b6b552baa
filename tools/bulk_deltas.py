#!/usr/bin/env python3
"""Bulk delta paths of the index (VERDICT r1 "bulk and
cold-start paths are unmeasured"):

  boot      a C3 index of --filters keys loaded the way attach/2 loads an
            existing ETS table (src/emqx_topic_index_gpu.erl): batches of
            --boot-batch keys, each ONE tm_apply_deltas call, then the first
            sync (whole tables uploaded);
  cleanup   node down (emqx_router.erl:535-578, emqx_router_helper.erl:147-162):
            every key of one of 10 nodes (value % 10 == 0, 1M keys at 10M)
            deleted as ONE tm_apply_deltas call, then the sync that ships the
            patch and the first 1M-topic match batch after it;
  rejoin    the node's keys inserted again as one call, sync, match.

After cleanup the incremental index is compared with one rebuilt from the
surviving keys on a 1M-topic batch (same CSR expected).  One JSON line."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--filters", type=int, default=10_000_000)
    p.add_argument("--boot-batch", type=int, default=1_000_000)
    p.add_argument("--topics", type=int, default=1_000_000)
    a = p.parse_args()
    import torch
    from emqx_amd import _native, workload as wl

    fs = wl.filters(3, a.filters)
    ts = wl.topics(3, a.filters, a.topics)
    out = {"filters": len(fs), "boot_batch": a.boot_batch}

    def timed(f):
        t = time.perf_counter()
        r = f()
        torch.cuda.synchronize()
        return r, time.perf_counter() - t

    ix = _native.Index(device=0)
    t0 = time.perf_counter()
    calls = 0
    for lo in range(0, len(fs), a.boot_batch):
        part = fs.slice(lo, min(lo + a.boot_batch, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
        calls += 1
    boot_apply = time.perf_counter() - t0
    _, boot_sync = timed(lambda: ix.sync())
    _, first_match = timed(lambda: ix.match_batch(ts.blob, ts.offs))
    st = ix.stats()
    out["boot"] = {"apply_s": round(boot_apply, 3), "calls": calls, "keys_per_s": round(len(fs) / boot_apply),
                   "first_sync_s": round(boot_sync, 3), "first_match_batch_s": round(first_match, 3),
                   "device_MiB": round(st["device_bytes"] / 2**20, 1), "nodes": st["n_nodes"], "words": st["n_words"]}

    gone = np.nonzero(fs.vals % 10 == 0)[0]
    dead = wl.ItemSet(*_native.pack_strings([fs.item(int(i)) for i in gone]), fs.vals[gone], fs.flags[gone])
    _, c_apply = timed(lambda: ix.apply(np.zeros(len(dead), np.uint8), dead.blob, dead.offs, dead.vals))
    up0 = ix.stats()["patch_bytes"]
    _, c_sync = timed(lambda: ix.sync())
    st = ix.stats()
    (hit, vals, err), c_match = timed(lambda: ix.match_batch(ts.blob, ts.offs))
    out["cleanup"] = {"deletes": len(dead), "apply_s": round(c_apply, 3), "deletes_per_s": round(len(dead) / c_apply),
                      "sync_s": round(c_sync, 3), "patch_MiB": round((st["patch_bytes"] - up0) / 2**20, 1),
                      "first_match_batch_s": round(c_match, 3), "keys_left": st["n_keys"]}

    keep = np.nonzero(fs.vals % 10 != 0)[0]
    rest = wl.ItemSet(*_native.pack_strings([fs.item(int(i)) for i in keep]), fs.vals[keep], fs.flags[keep])
    ref = _native.Index(device=0)
    ref.apply(np.ones(len(rest), np.uint8), rest.blob, rest.offs, rest.vals)
    rhit, rvals, rerr = ref.match_batch(ts.blob, ts.offs)
    out["cleanup"]["equals_rebuilt_index"] = bool(np.array_equal(hit, rhit) and np.array_equal(vals, rvals)
                                                  and np.array_equal(err, rerr))
    ref.close()

    _, r_apply = timed(lambda: ix.apply(np.ones(len(dead), np.uint8), dead.blob, dead.offs, dead.vals))
    _, r_sync = timed(lambda: ix.sync())
    (hit2, vals2, _), r_match = timed(lambda: ix.match_batch(ts.blob, ts.offs))
    out["rejoin"] = {"inserts": len(dead), "apply_s": round(r_apply, 3), "inserts_per_s": round(len(dead) / r_apply),
                     "sync_s": round(r_sync, 3), "first_match_batch_s": round(r_match, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
