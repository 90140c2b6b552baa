"""Study build (not product): level-D table-mode nodes' literal children stored
as whole node lines inside the parent's child table.

Writes emqx_amd/study/itab_host.cpp (tm_host.cpp + a device-image rewrite at
upload: the host keeps its normal layout, the device copy of `nodes` gets each
depth-D table-mode node's children relocated into a table of 64-B lines, slot
for slot with its ctab, the child's incoming wid in psum_hi) and
emqx_amd/study/itab.hip (tm_kernels.hip whose child probe reads those lines and
synthesises the slot summary from the child's line).  Deltas after the first
upload are NOT supported: measurement only (profile_walk / bench parity sample).
Build: python tools/study/mk_itab.py  ->  emqx_amd/variants/libtmatch_itab.so
Env: TM_STUDY_ITAB=<depths, e.g. "2" or "1,2">  (unset: the normal image)."""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
ST.mkdir(exist_ok=True)

h = (CS / "tm_host.cpp").read_text()
anchor = "template <class T>\nint upload_full(tm_index *ix, Mirror<T> &m) {"
assert anchor in h
fn = r'''
// ---- study: ITAB device image (tools/study/mk_itab.py)
constexpr uint32_t ST_ITAB = 0x40000000u, ST_ITABC = 0x20000000u;
static std::vector<Node> itab_image(tm_index *ix, uint64_t &moved, uint64_t &tabs) {
    const std::vector<Node> &N = ix->nodes.h;
    const std::vector<CSlot> &C = ix->ctab.h;
    std::vector<Node> out(N);
    std::vector<uint8_t> dep(N.size(), 255);
    std::vector<uint32_t> q{ROOT};
    dep[ROOT] = 0;
    for (size_t i = 0; i < q.size(); i++) {
        const uint32_t u = q[i];
        const Node &n = N[u];
        auto visit = [&](uint32_t c) {
            if (c != NONE && c < N.size() && dep[c] == 255) { dep[c] = dep[u] < 254 ? dep[u] + 1 : 254; q.push_back(c); }
        };
        visit(n.plus);
        const uint32_t nl = n.nlit & NLIT_MASK;
        if (nl <= KINL) {
            for (uint32_t k = 0; k < KINL; k++) if (n.kw[k] != NONE) visit(n.kc[k]);
        } else {
            for (uint32_t s = 0; s <= n.kw[1]; s++) if (C[n.kw[0] + s].wid != NONE) visit(C[n.kw[0] + s].child);
        }
    }
    bool want[256] = {};
    const char *e = getenv("TM_STUDY_ITAB");
    for (const char *p = e; p && *p;) { want[atoi(p) & 255] = true; while (*p && *p != ',') p++; if (*p) p++; }
    Node empty;
    memset(&empty, 0, sizeof empty);
    empty.plus = NONE; empty.psum_hi = NONE; empty.nlit = ST_ITABC;
    for (uint32_t k = 0; k < KINL; k++) { empty.kw[k] = NONE; empty.kc[k] = NONE; }
    moved = tabs = 0;
    for (uint32_t u : q) {
        const Node &n = N[u];
        const uint32_t nl = n.nlit & NLIT_MASK;
        if (!want[dep[u]] || nl <= KINL) continue;
        const uint64_t base = out.size(), size = (uint64_t)n.kw[1] + 1;
        out.resize(base + size, empty);
        for (uint64_t s = 0; s < size; s++) {
            const CSlot &sl = C[n.kw[0] + s];
            if (sl.wid == NONE) continue;
            Node c = N[sl.child];
            c.nlit |= ST_ITABC;
            c.psum_hi = sl.wid;
            out[base + s] = c;
            moved++;
        }
        out[u].kw[0] = (uint32_t)base;
        out[u].nlit |= ST_ITAB;
        tabs++;
    }
    return out;
}

'''
h = h.replace(anchor, fn + anchor)
old = "            if (m.bytes()) HIPCHK(ix, hipMemcpy(m.d[r], m.h.data(), m.bytes(), hipMemcpyHostToDevice));"
assert old in h
new = '''            if constexpr (std::is_same<T, Node>::value) {
                if (getenv("TM_STUDY_ITAB")) {
                    uint64_t moved, tabs;
                    std::vector<Node> img = itab_image(ix, moved, tabs);
                    if (m.d[r]) HIPCHK(ix, hipFree(m.d[r]));
                    HIPCHK(ix, hipMalloc(&m.d[r], (img.size() + DEV_GUARD) * sizeof(Node)));
                    HIPCHK(ix, hipMemcpy(m.d[r], img.data(), img.size() * sizeof(Node), hipMemcpyHostToDevice));
                    fprintf(stderr, "study itab: %lu tables, %lu children moved, %zu -> %zu lines\\n",
                            (unsigned long)tabs, (unsigned long)moved, m.h.size(), img.size());
                    continue;
                }
            }
''' + old
h = h.replace(old, new)
if "#include <type_traits>" not in h:
    h = "#include <type_traits>\n" + h
(ST / "itab_host.cpp").write_text(h)

k = (CS / "tm_kernels.hip").read_text()
k = k.replace("NLIT_MASK", "ST_NMASK")
old_ct = k[k.index("__device__ __forceinline__ uint32_t ctab_find("):k.index("// ------------------------------------------------------- frontier storage")]
new_ct = r'''__device__ __forceinline__ uint32_t ctab_find(const DevIndex &ix, uint32_t off, uint32_t mask, uint32_t wid,
                                              uint32_t h, uint32_t &slo, uint32_t &shi) {
    for (uint32_t s = h & mask;; s = (s + 1) & mask) {
        uint4 e = ld4(ix.ctab + off + s);
        pin(e);
        if (e.x == wid) { slo = e.z; shi = e.w; return e.y; }
        if (e.x == NONE) return NONE;
    }
}
// study: the children of an ST_ITAB node are node lines at nodes[off + slot],
// keyed by psum_hi; the slot summary is built from the child's line
__device__ __forceinline__ uint32_t itab_find(const DevIndex &ix, uint32_t off, uint32_t mask, uint32_t wid,
                                              uint32_t h, uint32_t &slo, uint32_t &shi) {
    for (uint32_t s = h & mask;; s = (s + 1) & mask) {
        const uint4 *np = reinterpret_cast<const uint4 *>(ix.nodes + off + s);
        uint4 a = np[0], b = np[1];
        pin(a); pin(b);
        if (b.w == wid) {
            uint64_t m = (a.z ? PSUM_HASH : 0u) | (b.x ? PSUM_EXACT : 0u) | (a.x != NONE ? PSUM_PLUS : 0u) |
                         ((b.y & NLIT_HDESC) ? PSUM_HDESC : 0u);
            m |= (uint64_t)(b.z & 15u) << PSUM_QQ;                  // QQ's flags: Q's own psum
            const uint64_t bq = (1ull << PSUM_BLOOM) - 1;   // (Q's children: the walk visits Q's line anyway)
            m |= bq << PSUM_BQ;
            // QQ's Bloom: Q's psum bits 8-35, whose top 4 (psum_hi) hold the key here
            m |= (((uint64_t)(b.z >> 8) & 0xFFFFFFull) | (0xFull << 24)) << PSUM_BQQ;
            slo = (uint32_t)m; shi = (uint32_t)(m >> 32);
            return off + s;
        }
        if (b.w == NONE) return NONE;
    }
}
__device__ __forceinline__ uint32_t child_find(const DevIndex &ix, const uint4 &n1, uint32_t off, uint32_t mask,
                                               uint32_t wid, uint32_t h, uint32_t &slo, uint32_t &shi) {
    return (n1.y & ST_ITAB) ? itab_find(ix, off, mask, wid, h, slo, shi) : ctab_find(ix, off, mask, wid, h, slo, shi);
}
// a line's '+' summary: an ITAB child's psum_hi is its key (its top Bloom bits unknown: all set)
__device__ __forceinline__ uint32_t psum_hi_of(const uint4 &n1) { return (n1.y & ST_ITABC) ? 0xFFFFFFFFu : n1.w; }

'''
k = k.replace(old_ct, new_ct)
hdr = "// ----------------------------------------------------------------- helpers"
k = k.replace(hdr, "constexpr uint32_t ST_ITAB = 0x40000000u, ST_ITABC = 0x20000000u, ST_NMASK = 0x1FFFFFFFu;\n" + hdr, 1)
n_ct = k.count("lit = ctab_find(ix, n2.x, n2.y,")
k = k.replace("lit = ctab_find(ix, n2.x, n2.y,", "lit = child_find(ix, n1, n2.x, n2.y,")
n_ps = k.count("child_alive(n1.z, n1.w,")
k = k.replace("child_alive(n1.z, n1.w,", "child_alive(n1.z, psum_hi_of(n1),")
print("probe sites", n_ct, "psum sites", n_ps)
assert n_ct == 3 and n_ps >= 3
NOSUM = "nosum" in sys.argv[1:]
if NOSUM:   # no summary from the child's line: every found child is visited
    a = k.index("            uint64_t m = (a.z ? PSUM_HASH")
    b = k.index("            slo = (uint32_t)m; shi = (uint32_t)(m >> 32);")
    k = k[:a] + "            const uint64_t m = ~0ull;\n" + k[b:]
name = "itab_ns" if NOSUM else "itab"
(ST / f"{name}.hip").write_text(k)

from emqx_amd import build
print(build.build_variant(name, str(ST / f"{name}.hip"), force=True, host_src=str(ST / "itab_host.cpp")))
