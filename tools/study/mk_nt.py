"""Study build (not product): the walk's vocab probes (nt_v), and its exact-key
fingerprint and entry loads (nt_x), as non-temporal loads -- lines a topic
touches once, marked evict-first so they do not push trie lines out of L2.
Build: python tools/study/mk_nt.py -> emqx_amd/variants/libtmatch_nt_v.so, _nt_x.so, _nt_vx.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
k0 = (CS / "tm_kernels.hip").read_text()
helper = '''__device__ __forceinline__ uint32_t ld_once_u16(const uint16_t *p) { return __builtin_nontemporal_load(p); }
'''
def v(k):
    a = "e[k] = ld4(ix.vocab + (use[k] ? ((uint32_t)h & ix.vmask) : 0u));"
    assert a in k
    return k.replace(a, "e[k] = ld4_once(ix.vocab + (use[k] ? ((uint32_t)h & ix.vmask) : 0u));")
def x(k):
    a = "    const uint32_t xf = allf ? ix.xfp[xslot] : 0;"
    assert a in k
    k = k.replace(a, "    const uint32_t xf = allf ? (uint32_t)__builtin_nontemporal_load(ix.xfp + xslot) : 0;")
    a = '''            const uint4 *e = reinterpret_cast<const uint4 *>(ix.exact + slot);
            uint4 a = e[0], b = e[1], c = e[2], d = e[3];'''
    assert a in k
    k = k.replace(a, '''            const uint4 *e = reinterpret_cast<const uint4 *>(ix.exact + slot);
            uint4 a = ld4_once(e), b = ld4_once(e + 1), c = ld4_once(e + 2), d = ld4_once(e + 3);''')
    return k
from emqx_amd import build
for name, f in (("nt_v", v), ("nt_x", x), ("nt_vx", lambda s: x(v(s)))):
    p = ST / f"{name}.hip"
    p.write_text(f(k0))
    print(build.build_variant(name, str(p), force=True))
