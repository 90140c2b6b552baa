#!/usr/bin/env python3
"""Study build: k_walk_small with wall-clock stamps (s_memrealtime, 100 MHz)
at its phase boundaries, one row of 8 per wave, readable with
tm_study_stamps().  Writes emqx_amd/study/stamps.hip from the product kernel
file and builds emqx_amd/variants/libtmatch_stamps.so.  Not product code."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
src = (ROOT / "emqx_amd/csrc/tm_kernels.hip").read_text()
a = src.index("__global__ __launch_bounds__(WV_BLOCK) void k_walk_small")
b = src.index("constexpr int MID_BLOCK")
body = src[a:b]


def st(k):
    return f"if ((threadIdx.x & 63) == 0) g_st[((uint64_t)vb * WV_WAVES + wv) * 8 + {k}] = wall_clock64();\n    "


def after(s, anchor, ins):
    assert s.count(anchor) == 1, anchor
    return s.replace(anchor, anchor + ins)


def before(s, anchor, ins):
    assert s.count(anchor) == 1, anchor
    return s.replace(anchor, ins + anchor)


body = after(body, "base = grp.g * W;\n    ", st(0))
body = after(body, "const uint64_t tlen = fb ? 0 : len;\n\n    ", st(1))
body = before(body, "uint32_t nst = live && !fb && !badarg ? 1 : 0, nh = 0;", st(2))
body = before(body, "// ---- match_topics/4: the binary key", st(3))
body = before(body, "fb |= live && nh > W;", st(4))
body = before(body, "if (MODE == MODE_FIRST) {\n        if (live && !fb) {", st(5))
body = before(body, "if (!live) return;\n    uint64_t pos = s_base;", st(6))
body = body.rstrip()
assert body.endswith("}")
body = body[:-1] + "    " + st(7).rstrip() + "\n}\n\n"
out = src[:a] + body + src[b:]
out = before(out, "template <int MODE>\n__global__ __launch_bounds__(WV_BLOCK) void k_walk_small",
             "__device__ uint64_t g_st[4096 * WV_WAVES * 8];\n")
out += '''
extern "C" int tm_study_stamps(uint64_t *out, uint64_t n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(tmx::g_st), 8 * n);
}
'''
dst = ROOT / "emqx_amd/study/stamps.hip"
dst.write_text(out)
from emqx_amd import build  # noqa: E402
print(build.build_variant("stamps", str(dst)))
