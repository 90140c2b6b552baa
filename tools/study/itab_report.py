"""Summarise a tools/gpu_r4_itab.sh run: per build, the bench line's isolated
walk / batch and parity sample, and the walk kernel's PMC counters per topic
(FETCH_SIZE KiB x 1024 / 64 = memory-side requests, profiles/r1_gather.md).
usage: itab_report.py gpurun_out/itab_<tag> [batch=1000000] [launches=8]"""
import csv, json, os, sys
from collections import defaultdict

d = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
last = int(sys.argv[3]) if len(sys.argv) > 3 else 8
names = sorted({f.split(".")[0] for f in os.listdir(d) if f.endswith(".json")})
print("| build | value | iso walk ms | iso batch ms | parity | mem req/topic | L2 hit | EA rdreq/topic |")
print("|---|---|---|---|---|---|---|---|")
for n in names:
    try:
        b = json.loads(open(os.path.join(d, n + ".json")).read().strip().splitlines()[-1])
    except Exception as e:
        print(f"| {n} | bench failed ({e}) |"); continue
    c = defaultdict(lambda: defaultdict(float))
    for i in (1, 2):
        p = os.path.join(d, f"{n}_p{i}", "run_counter_collection.csv")
        if not os.path.isfile(p):
            for root, _, fs in os.walk(os.path.join(d, f"{n}_p{i}")):
                for f in fs:
                    if f.endswith("counter_collection.csv"): p = os.path.join(root, f)
        if not os.path.isfile(p): continue
        for r in csv.DictReader(open(p)):
            if "k_walk_fast" in r["Kernel_Name"] and int(r["Grid_Size"]) >= batch - 63:
                c[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    m = {k: sum(sorted(v.items())[-last:][j][1] for j in range(min(last, len(v)))) / min(last, len(v)) for k, v in c.items() if v}
    req = m.get("FETCH_SIZE", 0) * 1024 / 64 / batch
    hit = m.get("TCC_HIT_sum", 0) / max(1, m.get("TCC_HIT_sum", 0) + m.get("TCC_MISS_sum", 0))
    ea = m.get("TCC_EA0_RDREQ_sum", 0) / batch
    rl = b["roofline"]
    print(f"| {n} | {b['value']:.3e} | {rl['kernel_avg_ms']:.4f} | {b['batch_device_isolated_ms']:.4f} | "
          f"{b['parity_sample']['mismatches']} / {b['parity_sample']['topics']} | {req:.2f} | {hit:.3f} | {ea:.2f} |")
