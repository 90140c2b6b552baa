"""Study build (not product): k_emit with EMIT_Q = 2 or 3 quads per lane per
iteration (value loads of several quads in flight before the stores; a C3
wave's span is ~135 quads, 2.1 per lane, so Q = 1 serialises ~2 round trips).
Build: python tools/study/mk_emitq.py -> emqx_amd/variants/libtmatch_emitq{2,3}.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
from emqx_amd import build
k0 = (CS / "tm_kernels.hip").read_text()
old = "constexpr int EMIT_Q = 1;"
assert k0.count(old) == 1
for q in (2, 3):
    (ST / f"emitq{q}.hip").write_text(k0.replace(old, f"constexpr int EMIT_Q = {q};"))
    print(build.build_variant(f"emitq{q}", str(ST / f"emitq{q}.hip"), force=True))
