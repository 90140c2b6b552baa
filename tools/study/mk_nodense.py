"""Study build (not product): the product sources with no wide node ever
dense (tm_host.cpp wide_dense: DENSE_NUM huge), i.e. every wide node's visit
asks its bitmap first, as rounds 2-4 did -- the A side of the dense-wide-node
measurement.
Build: python tools/study/mk_nodense.py -> emqx_amd/variants/libtmatch_nodense.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
h = (CS / "tm_host.cpp").read_text()
old = "constexpr uint64_t DENSE_NUM = 3, DENSE_DEN = 5;"
assert old in h
h = h.replace(old, "constexpr uint64_t DENSE_NUM = 1ull << 40, DENSE_DEN = 1;")
(ST / "nodense_host.cpp").write_text(h.replace('#include "../../include/tmatch.h"', f'#include "{ROOT}/include/tmatch.h"'))
from emqx_amd import build
print(build.build_variant("nodense", host_src=str(ST / "nodense_host.cpp"), force=True))
