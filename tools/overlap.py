#!/usr/bin/env python3
"""Kernel overlap in a rocprofv3 kernel trace: how many kernels run at once
(time-weighted), per kernel name.  usage: overlap.py <run_kernel_trace.csv> [name substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2] if len(sys.argv) > 2 else ""
ev = []
for r in rows:
    if sub not in r["Kernel_Name"]:
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ev += [(s, 1), (e, -1)]
ev.sort()
cur, last, acc, busy = 0, None, 0, 0
for t, d in ev:
    if last is not None and cur > 0:
        acc += cur * (t - last)
        busy += t - last
    cur += d
    last = t
n = len(ev) // 2
print(f"{n} kernels; busy {busy / 1e6:.2f} ms; mean concurrency while busy {acc / max(busy, 1):.2f}; "
      f"kernel time sum {acc / 1e6:.2f} ms")
