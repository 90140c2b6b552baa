#!/usr/bin/env python3
"""Read-your-writes soak of the Python Router (study tool, not product code):
the GPU test test_router_concurrent_writers_read_their_writes run for
`--seconds` instead of 25 writes per thread -- `--writers` threads each
subscribe a filter of their own, publish a topic it matches right after the
subscribe returned (the route must be there), and unsubscribe every third one
(the route must be gone), while `--publishers` threads match a C3-shaped batch
stream.  One JSON line per 10 s and a summary line; misses are counted, not
raised.  usage: router_soak.py [--seconds 90] [--writers 12] [--publishers 2] [--old-order]"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=90.0)
    p.add_argument("--writers", type=int, default=12)
    p.add_argument("--publishers", type=int, default=2)
    p.add_argument("--old-order", action="store_true",
                   help="the pre-fix mirror_sync (insert_key each key, then a separate commit flush)")
    a = p.parse_args()
    import torch
    assert torch.cuda.is_available()
    from emqx_amd import router as rt, workload as wl
    if a.old_order:
        def old_sync(self, keys, commit=False):
            with self._tables:
                present = [k in self._filters for k in keys]
            for k, here in zip(keys, present):
                self._mirror.insert_key(k, []) if here else self._mirror.delete_key(k)
            if keys:
                self._mirror.flush(commit=commit)
                self.mirror_calls += 1
        rt.Router.mirror_sync = old_sync
    r = rt.Router(node="n1")
    base = wl.filters(3, 20_000)
    r.do_batch({(base.item(i), "n9"): ("add", 0, None) for i in range(len(base))})
    ts = wl.topics(3, 20_000, 2_000)
    pubs = [ts.item(i) for i in range(len(ts))]
    stop = threading.Event()
    cnt = {"writes": 0, "missing": 0, "stale": 0, "raised": 0, "pub_batches": 0}
    lock = threading.Lock()
    first = []

    def writer(w):
        i = 0
        while not stop.is_set():
            flt = f"wr/{w}/{i}/+".encode()
            topic = f"wr/{w}/{i}/x".encode()
            dest = "n1" if i % 2 else (b"grp", "n2")
            try:
                r.add_route(flt, dest)
                miss = rt.Route(flt, dest) not in r.match_routes(topic)
                stale = False
                n = 1
                if i % 3 == 0:
                    r.delete_route(flt, dest)
                    stale = rt.Route(flt, dest) in r.match_routes(topic)
                    n = 2
                with lock:
                    cnt["writes"] += n
                    cnt["missing"] += miss
                    cnt["stale"] += stale
                    if (miss or stale) and len(first) < 5:
                        first.append((w, i, "missing" if miss else "stale"))
            except Exception as e:   # noqa: BLE001 -- counted and reported
                with lock:
                    cnt["raised"] += 1
                    if len(first) < 5:
                        first.append((w, i, repr(e)))
            i += 1

    def publisher():
        while not stop.is_set():
            r.match_routes_batch(pubs[:500])
            with lock:
                cnt["pub_batches"] += 1

    th = [threading.Thread(target=publisher) for _ in range(a.publishers)]
    th += [threading.Thread(target=writer, args=(w,)) for w in range(a.writers)]
    t0 = time.time()
    for t in th:
        t.start()
    try:
        while time.time() - t0 < a.seconds:
            time.sleep(min(10.0, max(0.0, a.seconds - (time.time() - t0))))
            with lock:
                print(json.dumps({"t_s": round(time.time() - t0, 1), **cnt}), flush=True)
    finally:
        stop.set()
        for t in th:
            t.join()
    dt = time.time() - t0
    print(json.dumps({"summary": True, "old_order": a.old_order, "seconds": round(dt, 1), "writers": a.writers,
                      "publishers": a.publishers,
                      **cnt, "writes_per_s": round(cnt["writes"] / dt, 1), "mirror_commits": r.mirror_commits,
                      "mirror_synced_requests": r.mirror_synced_requests, "first_failures": first}), flush=True)
    # (the old order is run to show the misses: they are its expected outcome)
    return 1 if not a.old_order and (cnt["missing"] or cnt["stale"] or cnt["raised"]) else 0


if __name__ == "__main__":
    sys.exit(main())
