#!/usr/bin/env python3
"""Per-kernel duration stats from a rocprofv3 kernel-trace csv, over the last
`--window` seconds of the trace (default: all).  usage: kstats.py CSV [--window S]"""
import argparse
import collections
import csv

p = argparse.ArgumentParser()
p.add_argument("csv")
p.add_argument("--window", type=float, default=0.0)
a = p.parse_args()
rows = list(csv.DictReader(open(a.csv)))
t_end = max(int(r["End_Timestamp"]) for r in rows)
if a.window:
    rows = [r for r in rows if int(r["Start_Timestamp"]) > t_end - a.window * 1e9]
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k:40s} n={len(v):6d} mean={sum(v) / len(v):8.1f}us p50={v[len(v) // 2]:8.1f} max={v[-1]:8.1f}")
