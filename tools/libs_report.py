#!/usr/bin/env python3
"""Summarise tools/gpu_libs_prof.sh output for one kernel: per library build,
the kernel trace's average duration and every counter's average per launch
(the last `last` launches).
usage: libs_report.py <libs_dir> <kernel substring> [last]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, kern, last=8):
    last = int(last)
    for lib in sorted(x for x in os.listdir(d) if os.path.isdir(os.path.join(d, x))):
        rows = defaultdict(dict)
        durs = []
        for f in glob.glob(os.path.join(d, lib, "*", "run_kernel_trace.csv")):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for f in glob.glob(os.path.join(d, lib, "*", "run_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if kern in r["Kernel_Name"]:
                    rows[r["Counter_Name"]][int(r["Dispatch_Id"])] = float(r["Counter_Value"])
        print(f"== {lib}")
        if durs:
            t = durs[-last:]
            print(f"  duration_us {sum(t) / len(t) / 1e3:.1f} (n={len(t)})")
        for k in sorted(rows):
            x = [v for _, v in sorted(rows[k].items())][-last:]
            print(f"  {k} {sum(x) / len(x):.4g}")


if __name__ == "__main__":
    main(*sys.argv[1:])
