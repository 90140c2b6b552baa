"""Study build (not product): at a table-mode node whose '+' child will be
visited next, touch the '+' child's line (one dword load, result unused) in
the same round trip as the literal child's table probe, so the next step's
line loads hit L2 -- a shorter dependent chain with no extra memory-side
request (the line is read next anyway).  Tests the chain-length hypothesis
without round 3's extra requests (cinfo).
Build: python tools/study/mk_touch.py -> emqx_amd/variants/libtmatch_touch.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)
k = (CS / "tm_kernels.hip").read_text()
old = '''            uint32_t lit = NONE;
            if (w != NONE) {
                if ((n1.y & NLIT_MASK) <= KINL) {
                    lit = inl;
                } else {
                    const uint32_t h = child_hash(w);
                    if (child_maybe(ix, n1, n2, n3, w, h) & 1u) {
                        uint32_t slo, shi;
                        lit = ctab_find(ix, n2.x, n2.y, w, h, slo, shi);
                        if (lit != NONE && !child_alive(slo, shi, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                                        l + 2 < L ? st.get_wid(l + 2) : NONE))
                            lit = NONE;
                    }
                }
            }
            if (!droot && !em(n0.y, n0.z)) return DFS_STOP;
            // [P,'#',...] seeks to P/W past the '+' subtree (:341-348)
            uint32_t plus = droot || (n1.y & NLIT_HDESC) ? NONE : n0.x;
            if (plus != NONE && !child_alive(n1.z, n1.w, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                             l + 2 < L ? st.get_wid(l + 2) : NONE))
                plus = NONE;'''
assert old in k
new = '''            // [P,'#',...] seeks to P/W past the '+' subtree (:341-348)
            uint32_t plus = droot || (n1.y & NLIT_HDESC) ? NONE : n0.x;
            if (plus != NONE && !child_alive(n1.z, n1.w, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                             l + 2 < L ? st.get_wid(l + 2) : NONE))
                plus = NONE;
            uint32_t lit = NONE;
            if (w != NONE) {
                if ((n1.y & NLIT_MASK) <= KINL) {
                    lit = inl;
                } else {
                    const uint32_t h = child_hash(w);
                    if (child_maybe(ix, n1, n2, n3, w, h) & 1u) {
                        uint32_t slo, shi;
                        // study: the '+' child's line, read next, in this round trip
                        const uint32_t tch = plus != NONE ? reinterpret_cast<const uint32_t *>(ix.nodes + plus)[0] : 0u;
                        lit = ctab_find(ix, n2.x, n2.y, w, h, slo, shi);
                        asm volatile("" :: "v"(tch));
                        if (lit != NONE && !child_alive(slo, shi, l + 1, L, l + 1 < L ? st.get_wid(l + 1) : NONE,
                                                        l + 2 < L ? st.get_wid(l + 2) : NONE))
                            lit = NONE;
                    }
                }
            }
            if (!droot && !em(n0.y, n0.z)) return DFS_STOP;'''
k = k.replace(old, new, 1)
# control: the same reordering without the touch
kc = k.replace('''                        const uint32_t tch = plus != NONE ? reinterpret_cast<const uint32_t *>(ix.nodes + plus)[0] : 0u;
''', '').replace('''                        asm volatile("" :: "v"(tch));
''', '')
(ST / "touch.hip").write_text(k)
(ST / "touch0.hip").write_text(kc)
from emqx_amd import build
print(build.build_variant("touch", str(ST / "touch.hip"), force=True))
print(build.build_variant("touch0", str(ST / "touch0.hip"), force=True))
