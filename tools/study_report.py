#!/usr/bin/env python3
"""Summarise tools/gpu_study.sh output: per variant, the walk kernel's
memory-side bytes and requests, L1->L2 requests and L2 hit rate per topic
(the last `batches` launches of the full grid).
usage: study_report.py <study_dir> [batch] [batches]"""
import csv
import os
import sys
from collections import defaultdict


def main(d, batch=1_000_000, batches=8):
    batch, batches = int(batch), int(batches)
    grid = (batch + 255) // 256 * 256
    print(open(os.path.join(d, "timing.txt")).read())
    for v in sorted(os.listdir(d)):
        p = os.path.join(d, v)
        if not os.path.isdir(p):
            continue
        vals = defaultdict(dict)
        for sub in sorted(os.listdir(p)):
            f = os.path.join(p, sub, "run_counter_collection.csv")
            if not os.path.isfile(f):
                continue
            for r in csv.DictReader(open(f)):
                if "k_walk_fast" in r["Kernel_Name"] and batch <= int(r["Grid_Size"]) <= grid:
                    vals[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
        c = {k: sum(sorted(x.items())[-batches:][i][1] for i in range(min(batches, len(x)))) / min(batches, len(x))
             for k, x in vals.items() if x}
        fs = c.get("FETCH_SIZE", 0) * 1024
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        print(f"{v}: FETCH {fs / batch:.0f} B/topic = {fs / 64 / batch:.2f} mem-side req/topic; "
              f"L1->L2 {c.get('TCP_TCC_READ_REQ_sum', 0) / batch:.2f}/topic; "
              f"L2 hit {hit / max(hit + miss, 1) * 100:.1f}%")


if __name__ == "__main__":
    main(*sys.argv[1:])
