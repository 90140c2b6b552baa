#!/usr/bin/env python3
"""Host-fed pipeline sweep (bench.py's host_fed leg): 1M-topic C3 batches from
pinned host memory -> H2D -> match -> D2H, for several stream counts and both
offset widths, next to the PCIe copy ceilings.  One JSON line per setting."""
import ctypes, json, os, sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch  # noqa: F401  (device init as bench.py)
    from bench import CONFIGS, host_bench_lib
    from emqx_amd import _native, workload as wl
    gen, nf, _ = CONFIGS["c3"]
    fs = wl.filters(gen, nf)
    ix = _native.Index(device=0, hint_keys=len(fs))
    for lo in range(0, len(fs), 2_000_000):
        part = fs.slice(lo, min(lo + 2_000_000, len(fs)))
        ix.apply(np.ones(len(part), np.uint8), part.blob, part.offs, part.vals)
    B, R = 1_000_000, 4
    allt = wl.concat([wl.topics(gen, nf, B, first=k * B) for k in range(R)])
    hb = host_bench_lib()
    pc = (ctypes.c_double * 4)()
    assert hb.tmb_pcie(0, 256 << 20, 16, 4, pc) == 0
    print(json.dumps({"pcie_GBps": {"h2d": pc[0], "d2h": pc[1], "both_h2d": pc[2], "both_d2h": pc[3]}}), flush=True)
    # interleaved repeats (the PCIe rates drift between and within runs)
    modes = [int(x) for x in os.environ.get("PIPE_MODES", "1,3").split(",")]
    for rep in range(int(os.environ.get("PIPE_REPS", "1"))):
        for u32 in modes:
            for ns in [int(x) for x in (sys.argv[1:] or ["3"])]:
                out = (ctypes.c_double * 5)()
                rc = hb.tmb_pipeline_ex(ix._h, 0, _native._ptr(allt.blob), _native._ptr(allt.offs), B, R, ns, 48, u32,
                                        out)
                assert rc == 0, rc
                per = max(out[2] / (pc[0] * 1e9), out[3] / (pc[1] * 1e9))
                print(json.dumps({"rep": rep, "u32": u32 & 1, "copy_streams": bool(u32 & 2), "streams": ns,
                                  "topics_per_s": out[0], "ms_per_batch": out[1], "h2d_MB": out[2] / 1e6,
                                  "d2h_MB": out[3] / 1e6, "frac_of_pcie_bound": out[0] / (B / per)}), flush=True)


if __name__ == "__main__":
    main()
