"""Study build (not product): the walk's per-topic outputs (range lists,
counts) stored at agent scope (global_store sc1: written through the XCD's
L2) instead of non-temporal -- does the 5.7 us gap between k_walk_fast's end
and k_walk_tail's start (profiles/r5_fin trace: the end-of-kernel release
writing back the L2's dirty lines) shrink, and what does the walk pay?
Build: python tools/study/mk_wt.py -> emqx_amd/variants/libtmatch_wt.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
k = (CS / "tm_kernels.hip").read_text()
subs = [
    ("""            if (i < nr) __builtin_nontemporal_store((uint64_t)r[i].x | ((uint64_t)r[i].y << 32),
                                                    reinterpret_cast<uint64_t *>(rng) + (uint64_t)i * n + t);""",
     """            if (i < nr) __hip_atomic_store(reinterpret_cast<uint64_t *>(rng) + (uint64_t)i * n + t,
                                           (uint64_t)r[i].x | ((uint64_t)r[i].y << 32), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);"""),
    ("""        __builtin_nontemporal_store(em.cnt, ws.cnt + t);
        __builtin_nontemporal_store(em.nr, ws.nr + t);""",
     """        __hip_atomic_store(ws.cnt + t, em.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ws.nr + t, em.nr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);"""),
]
for a, b in subs:
    assert k.count(a) == 1, a[:60]
    k = k.replace(a, b)
(ST / "wt.hip").write_text(k)
from emqx_amd import build
print(build.build_variant("wt", str(ST / "wt.hip"), force=True))
