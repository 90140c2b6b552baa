#!/usr/bin/env python3
"""Turn one tools/gpu.sh `prof` output directory (gpurun_out/<tag>/prof) into the committed evidence
under profiles/:

  profiles/<round>_<tag>.md            kernel-trace summary per kernel and grid
                                       (bench command + profiling driver) and
                                       the PMC counters of the full-grid match
                                       kernels with the derived figures
  profiles/<round>_<tag>_*_stats.csv   rocprofv3 --stats summaries, verbatim
  profiles/pmc_<config>.json           walk-kernel HBM bytes per launch, read by
                                       bench.py for roofline.traffic

HBM bytes: FETCH_SIZE and WRITE_SIZE are reported by rocprofv3 in KiB.
FETCH_SIZE = TCC_EA0_RDREQ x 64 B (MI355X_MICROARCH.md, HBM section); the
walk's reads are 16-B-per-lane loads of scattered 64-B lines, not the wide
streaming reads the guide's x2 correction was calibrated on.  Calibrated with
tools/gather_bench.hip on a known request count (profiles/r1_gather.md): for
scattered 16-B and 64-B reads FETCH_SIZE counts exactly 64 B per memory-side
request, so the value is taken as is (no x2).
It also counts Infinity-Cache (MALL) hits, so it is an upper bound on HBM.

The bench run's kernel trace is split by phase: its last 2 x rotate
full-grid launches of the main kernel (k_walk_small for a one-launch batch,
else k_walk_fast) are the isolated pass bench.py times for
roofline.kernel_avg_ms (one stream, back to back), the launches before them
ran overlapped on three streams.  pmc_<config>.json is stamped with the
kernel-source hash (emqx_amd.build.source_hash) and the workload shape;
bench.py refuses it for any other tree or shape.

usage: prof_report.py <prof_dir> <round> <tag> <config> <filters> <batch> [rotate] [batches]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n


def _open(path):
    if os.path.isfile(path):
        return open(path)
    import gzip
    return gzip.open(path + ".gz", "rt")


def trace_table(path):
    rows = list(csv.DictReader(_open(path)))
    agg = defaultdict(list)
    for r in rows:
        grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        agg[(short(r["Kernel_Name"]), grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = ["| kernel | grid (threads) | calls | avg us | min us | max us |", "|---|---|---|---|---|---|"]
    for (name, grid), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if "tmx::" not in name:
            continue
        out.append(f"| {name} | {grid} | {len(d)} | {sum(d) / len(d) / 1e3:.2f} | {min(d) / 1e3:.2f} | {max(d) / 1e3:.2f} |")
    return out, agg


def pmc_values(prof, grid, last):
    """mean counter value per launch over the LAST `last` launches of each
    kernel at this grid (the profiling driver's timed launches; its sizing
    launches, which write no values, come first)"""
    vals = defaultdict(lambda: defaultdict(dict))
    for d in sorted(os.listdir(prof)):
        p = os.path.join(prof, d, "run_counter_collection.csv")
        if not (d.startswith("pmc") and os.path.isfile(p)):
            continue
        for r in csv.DictReader(open(p)):
            if not (grid - 255 <= int(r["Grid_Size"]) <= grid) or "tmx::" not in r["Kernel_Name"]:
                continue
            k, c, disp = short(r["Kernel_Name"]), r["Counter_Name"], int(r["Dispatch_Id"])
            vals[k][c][disp] = vals[k][c].get(disp, 0.0) + float(r["Counter_Value"])
    out = {}
    for k, cs in vals.items():
        out[k] = {}
        for c, per in cs.items():
            v = [per[d] for d in sorted(per)[-last:]]
            out[k][c] = sum(v) / len(v)
    return out


# the timed kernel: a pairs batch's walk, a one-launch batch, else the two-phase walk
MAIN_KERNELS = ("k_walk_pairs", "k_walk_small", "k_walk_fast")


def main_kernel(names):
    for k in MAIN_KERNELS:
        hit = [n for n in names if k in n]
        if hit:
            return hit[0]
    return None


def split_phases(path, grid, n_iso):
    """full-grid launches of the main kernel (k_walk_small, else k_walk_fast) of
    the bench run in time order -> (timed region + warmup, isolated pass)
    durations in ns"""
    rows = list(csv.DictReader(_open(path)))
    k = main_kernel({r["Kernel_Name"] for r in rows})
    rows = [r for r in rows if k and k in r["Kernel_Name"]
            and grid - 255 <= int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0) <= grid]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    return d[:-n_iso], d[-n_iso:]


def main(prof, rnd, tag, config, filters, batch, rotate=4, batches=8):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from emqx_amd.build import source_hash
    filters, batch, rotate, batches = int(filters), int(batch), int(rotate), int(batches)
    grid = (batch + 255) // 256 * 256   # full-batch launches have grids in [grid - 255, grid]
    lines = [f"# Profile {rnd}/{tag}: config {config}, {filters} filters, {batch}-topic batches", ""]
    bench_json = os.path.join(prof, "bench.json")
    if os.path.isfile(bench_json) and os.path.getsize(bench_json):
        # the stamp names THIS tree's sources: refuse a profile of other sources
        import json
        profiled = json.loads(open(bench_json).read().strip().splitlines()[-1])["build"]["kernel_source_hash"]
        if profiled != source_hash():
            sys.exit(f"refused: {prof} profiled kernel sources {profiled}, this tree is {source_hash()}")
        lines += ["## bench.py line (run under rocprofv3 --kernel-trace --stats)", "", "```",
                  open(bench_json).read().strip(), "```", ""]
    durations = {}
    for sub, title in (("bench", "bench.py with its defaults (includes the 4k/64k latency batches and the isolated walk batches)"),
                       ("trace", "tools/profile_walk.py (full batches only)")):
        p = os.path.join(prof, sub, "run_kernel_trace.csv")
        if not (os.path.isfile(p) or os.path.isfile(p + ".gz")):
            continue
        tab, agg = trace_table(p)
        lines += [f"## Kernel trace: {title}", ""] + tab + [""]
        if sub == "bench":
            timed, iso = split_phases(p, grid, 2 * rotate)
            if iso:
                lines += [f"{main_kernel(agg and {n for n, _ in agg})} (grid {grid}) by phase of the bench run: "
                          f"the last {len(iso)} launches "
                          f"(bench.py's isolated pass, one stream, back to back) avg {sum(iso) / len(iso) / 1e3:.2f} us "
                          f"(min {min(iso) / 1e3:.2f}, max {max(iso) / 1e3:.2f}); the {len(timed)} before them "
                          f"(sizing, warmup, timed steps on three streams) avg {sum(timed) / max(len(timed), 1) / 1e3:.2f} us.",
                          ""]
        if sub == "trace":   # the driver the PMC passes ran: kernels alone on one stream
            for (name, g), d in agg.items():
                if grid - 255 <= g <= grid:   # full batches (walk blocks of 64, emit tiles of 256)
                    durations.setdefault(name, []).extend(d)
        st = os.path.join(prof, sub, "run_kernel_stats.csv")
        if os.path.isfile(st):
            shutil.copy(st, os.path.join("profiles", f"{rnd}_{tag}_{sub}_kernel_stats.csv"))
    pm = pmc_values(prof, grid, batches)
    mk = main_kernel(list(pm))
    walk = [mk] if mk else []
    res = {"config": config, "filters": filters, "batch": batch, "rotate": rotate, "grid": grid,
           "source_hash": source_hash()}
    if pm:
        lines += [f"## PMC counters per launch (grid {grid}, mean over launches; one rocprofv3 --pmc pass per group)", ""]
        names = sorted({c for k in pm for c in pm[k]})
        lines.append("| counter | " + " | ".join(sorted(pm)) + " |")
        lines.append("|---|" + "---|" * len(pm))
        for c in names:
            lines.append(f"| {c} | " + " | ".join(f"{pm[k].get(c, float('nan')):.6g}" for k in sorted(pm)) + " |")
        lines.append("")
        lines += ["## Derived", ""]
        for k in sorted(pm):
            c = pm[k]
            d = durations.get(k)
            dur = sum(d) / len(d) * 1e-9 if d else None
            fb = c.get("FETCH_SIZE", 0) * 1024
            wb = c.get("WRITE_SIZE", 0) * 1024
            hit = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
            lines.append(f"* **{k}**: avg {dur * 1e6:.1f} us; " if dur else f"* **{k}**: ")
            lines[-1] += (f"memory-side reads {fb / 1e6:.1f} MB ({fb / batch:.0f} B/topic), writes {wb / 1e6:.1f} MB "
                          f"({wb / batch:.0f} B/topic)")
            if dur:
                lines[-1] += f", {(fb + wb) / dur / 1e9:.0f} GB/s"
            if hit[0] is not None and hit[1] is not None and hit[0] + hit[1] > 0:
                lines[-1] += f"; L2 hit {hit[0] / (hit[0] + hit[1]) * 100:.1f}%"
            if c.get("TCP_TCC_READ_REQ_sum"):
                lines[-1] += (f"; L1->L2 read requests {c['TCP_TCC_READ_REQ_sum'] / batch:.1f}/topic, "
                              f"mean L2 latency {c.get('TCP_TCC_READ_REQ_LATENCY_sum', 0) / c['TCP_TCC_READ_REQ_sum']:.0f} cycles")
            if c.get("SQ_WAVE_CYCLES"):
                lines[-1] += (f"; waves parked on waitcnt {c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES'] * 100:.0f}% "
                              f"of wave-cycles, VMEM reads {c.get('SQ_INSTS_VMEM_RD', 0) / c.get('SQ_WAVES', 1):.0f}/wave")
            if dur and c.get("GRBM_GUI_ACTIVE"):
                # the PMC passes run the kernel slower than the trace run, so
                # GRBM cycles over the trace duration is not the clock
                lines[-1] += f"; {c['GRBM_GUI_ACTIVE'] / 8 / 1e6:.2f} M GPU-busy cycles per XCD in the PMC pass"
        lines.append("")
        if walk:
            c = pm[walk[0]]
            res["walk_kernel"] = walk[0]
            res["walk_fetch_bytes_per_launch"] = int(c.get("FETCH_SIZE", 0) * 1024)
            res["walk_write_bytes_per_launch"] = int(c.get("WRITE_SIZE", 0) * 1024)
            res["walk_hbm_bytes_per_launch"] = res["walk_fetch_bytes_per_launch"] + res["walk_write_bytes_per_launch"]
            res["walk_mem_requests_per_launch"] = round(res["walk_fetch_bytes_per_launch"] / 64)
            res["note"] = ("FETCH_SIZE (memory-side 64-B read requests, MALL hits included; calibrated at 64 B "
                           "per scattered request, profiles/r1_gather.md) + WRITE_SIZE")
            res["source"] = f"profiles/{rnd}_{tag}.md"
            json.dump(res, open(os.path.join("profiles", f"pmc_{config}.json"), "w"), indent=1)
    open(os.path.join("profiles", f"{rnd}_{tag}.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
