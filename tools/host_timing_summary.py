#!/usr/bin/env python3
"""Summarise TM_HOST_TIMING=1 stderr lines of in-place host batches
("tm_match_batch n=... (in place): sync A launch B wait C us"): median / p90
of each phase.  usage: host_timing_summary.py <stderr file>"""
import re
import sys

import numpy as np

rx = re.compile(r"\(in place\): sync ([\d.]+) launch ([\d.]+) wait ([\d.]+) us")
v = np.array([[float(x) for x in m.groups()] for m in map(rx.search, open(sys.argv[1])) if m])
if not len(v):
    sys.exit("no in-place timing lines")
for k, name in enumerate(["lock+lane+sync+ws", "launch", "wait"]):
    print(f"{name:18s} n={len(v)} median {np.median(v[:, k]):7.1f} us  p90 {np.percentile(v[:, k], 90):7.1f}  "
          f"p99 {np.percentile(v[:, k], 99):7.1f}")
