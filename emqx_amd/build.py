"""Build recipe for the native parts (in-tree, gfx950 only).

- ``emqx_amd/libtmatch.so``  product: host index compiler + HIP kernels + C ABI
  (``include/tmatch.h``), compiled by hipcc for ``--offload-arch=gfx950``.
- ``emqx_amd/libtmwork.so``  synthetic workload generator (bench / tests).
- ``emqx_amd/libtmbench.so`` native host-side bench drivers (caller threads,
  host-fed pipeline) over libtmatch (bench.py only).
- ``oracle/liboracle.so``    CPU oracle (tests / smoke / bench cpu_baseline only).
"""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"

LIB_TMATCH = PKG / "libtmatch.so"
LIB_WORK = PKG / "libtmwork.so"
LIB_BENCH = PKG / "libtmbench.so"
LIB_ORACLE = ROOT / "oracle" / "liboracle.so"

ARCH = os.environ.get("TM_OFFLOAD_ARCH", "gfx950")


KERNEL_SOURCES = ("tm_kernels.hip", "tm_host.cpp", "tm_layout.h", "tm_dev.h")


def source_hash() -> str:
    """Hash of the sources the match kernels are built from.  Measurements
    that cannot be taken inside bench.py itself (rocprofv3 PMC counters,
    profiles/pmc_<config>.json) are stamped with it, and bench.py refuses a
    stamp that does not match the tree it runs."""
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        h.update(name.encode())
        h.update((CSRC / name).read_bytes())
    return h.hexdigest()[:16]


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")


def build_tmatch(force: bool = False) -> Path:
    srcs = [CSRC / "tm_host.cpp", CSRC / "tm_kernels.hip"]
    deps = srcs + [CSRC / "tm_layout.h", CSRC / "tm_dev.h", ROOT / "include" / "tmatch.h"]
    if force or _stale(LIB_TMATCH, deps):
        tmp = LIB_TMATCH.with_suffix(".so.tmp")
        _run(["hipcc", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
              "-Wall", "-Wno-unused-function", "-o", str(tmp)] + [str(s) for s in srcs])
        os.replace(tmp, LIB_TMATCH)
    return LIB_TMATCH


def build_variant(name: str, kernel_src: str | None = None, force: bool = False,
                  host_src: str | None = None) -> Path:
    """An experimental build of libtmatch (perf studies: tools/gpu.sh export:TM_LIB=...
    loads it through TM_LIB).  `kernel_src` replaces tm_kernels.hip with a
    study copy (e.g. under emqx_amd/study/, not tracked), so experiments never
    put switches into the product source; `host_src` likewise tm_host.cpp.
    Not the product library."""
    out = PKG / "variants" / f"libtmatch_{name}.so"
    out.parent.mkdir(exist_ok=True)
    kern = Path(kernel_src) if kernel_src else CSRC / "tm_kernels.hip"
    srcs = [Path(host_src) if host_src else CSRC / "tm_host.cpp", kern]
    deps = srcs + [CSRC / "tm_layout.h", CSRC / "tm_dev.h", ROOT / "include" / "tmatch.h"]
    if force or _stale(out, deps):
        _run(["hipcc", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-Wall",
              "-Wno-unused-function", f"-I{CSRC}", "-o", str(out)] + [str(s) for s in srcs])
    return out


def build_work(force: bool = False) -> Path:
    src = CSRC / "workload.cpp"
    if force or _stale(LIB_WORK, [src]):
        tmp = LIB_WORK.with_suffix(".so.tmp")
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", str(tmp), str(src)])
        os.replace(tmp, LIB_WORK)
    return LIB_WORK


def build_bench(force: bool = False) -> Path:
    src = CSRC / "hostbench.cpp"
    if force or _stale(LIB_BENCH, [src, ROOT / "include" / "tmatch.h"]):
        tmp = LIB_BENCH.with_suffix(".so.tmp")
        _run(["hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", str(tmp), str(src), "-ldl"])
        os.replace(tmp, LIB_BENCH)
    return LIB_BENCH


def build_oracle(force: bool = False) -> Path:
    src = ROOT / "oracle" / "tm_oracle.c"
    if force or _stale(LIB_ORACLE, [src]):
        _run(["make", "-B" if force else "-s", "liboracle.so"], cwd=ROOT / "oracle")
    return LIB_ORACLE


def build_all(force: bool = False) -> None:
    build_tmatch(force)
    build_work(force)
    build_bench(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force=True)
    print("built", LIB_TMATCH, LIB_WORK, LIB_ORACLE)
