"""Study build (not product): k_walk_small asked for 6 waves per SIMD
(__launch_bounds__(256, 6): <= 80 VGPRs, the compiler spills 12-20 B per lane
to scratch) instead of the 5 its 82-83 VGPRs allow -- does the sixth wave pay
for the spill on concurrent small batches?  
Build: python tools/study/mk_occ6.py -> emqx_amd/variants/libtmatch_occ6.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
k = (CS / "tm_kernels.hip").read_text()
old = "__global__ __launch_bounds__(WV_BLOCK) void k_walk_small("
assert old in k
k = k.replace(old, "__global__ __launch_bounds__(WV_BLOCK, 6) void k_walk_small(")
(ST / "occ6.hip").write_text(k)
from emqx_amd import build
print(build.build_variant("occ6", str(ST / "occ6.hip"), force=True))
