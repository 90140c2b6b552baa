#!/usr/bin/env python3
"""VGPRs / scratch per kernel of tm_kernels.hip (hipcc resource-usage remarks):
k_walk_fast must stay within 64 VGPRs and no scratch (8 waves per SIMD).
usage: kernel_regs.py [-Dextra ...]"""
import re
import subprocess
import sys
from pathlib import Path

src = Path(sys.argv.pop(1)) if len(sys.argv) > 1 and sys.argv[1].endswith(".hip") else Path(__file__).resolve().parent.parent / "emqx_amd" / "csrc" / "tm_kernels.hip"
r = subprocess.run(["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", "-o", "/dev/null", str(src),
                    "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:], capture_output=True, text=True)
name, rows = None, {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = re.sub(r"^_ZN3tmx\d+", "", m.group(1)).split("EEEv")[0].split("ENS_")[0]
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and name:
        rows.setdefault(name, {})[m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    print(f"{k:32s} VGPRs {v.get('VGPRs')}  scratch {v.get('ScratchSize')}  occupancy {v.get('Occupancy')}")
w = [v for k, v in rows.items() if k.startswith("k_walk_fast")]
sys.exit(0 if w and all(v.get("VGPRs", 99) <= 64 and v.get("ScratchSize", 1) == 0 for v in w) else 1)
