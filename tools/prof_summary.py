#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per kernel and grid size
(markdown), so the profile's averages can be compared with bench.py's."""
import csv
import sys
from collections import defaultdict


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        agg[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    lines = ["| kernel | grid (threads) | calls | avg us | min us | max us |", "|---|---|---|---|---|---|"]
    for (name, grid), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"| {name} | {grid} | {len(d)} | {sum(d) / len(d) / 1e3:.2f} | {min(d) / 1e3:.2f} | {max(d) / 1e3:.2f} |")
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
