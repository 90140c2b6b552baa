"""Study build (not product): batches <= 65536 topics on the lane walk
(k_walk_one, one lane per topic) with each block's topic bytes staged in LDS
by one round of coalesced 16-B loads (in-place host batches: one PCIe burst per
block instead of a round trip per lane), look-back without parking, one launch
-- against k_walk_small's wave walk.
Build: python tools/study/mk_stage1.py -> emqx_amd/variants/libtmatch_stage1.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
k = (CS / "tm_kernels.hip").read_text()
old = '''    const uint32_t vb = blockIdx.x;
    const uint64_t t = (uint64_t)vb * WALK_BLOCK + lane;
    const bool live = t < n;

    // ---- 1. the walk (k_walk_fast's)'''
assert old in k
new = '''    const uint32_t vb = blockIdx.x;
    const uint64_t t = (uint64_t)vb * WALK_BLOCK + lane;
    const bool live = t < n;
    // study: the block's topic bytes in LDS (small batches)
    constexpr uint32_t STG_Q = 256;
    __shared__ uint4 s_stage[STG_Q];
    const uint8_t *blob_w = blob;
    if (n <= 65536) {
        const uint64_t tb_ = live ? offs[t] : 0, te_ = live ? offs[t + 1] : 0;
        const uint64_t rem = n - (uint64_t)vb * WALK_BLOCK;
        const uint32_t last = rem > 64 ? 63u : (uint32_t)rem - 1;
        const uint64_t B0 = __shfl(tb_, 0, 64) & ~15ull;
        const uint64_t E = __shfl(te_, (int)last, 64);
        const uint64_t nq = (E - B0 + 15) >> 4;
        if (nq <= STG_Q) {
            for (uint32_t c = lane; c < nq; c += WALK_BLOCK) s_stage[c] = ld4_once(blob + B0 + 16ull * c);
            __syncthreads();
            blob_w = reinterpret_cast<const uint8_t *>(s_stage) - B0;
        }
    }

    // ---- 1. the walk (k_walk_fast's)'''
k = k.replace(old, new, 1)
seg = k[k.index("__global__ __launch_bounds__(WALK_BLOCK, 8) void k_walk_one"):k.index("// The blocks of a k_walk_one launch that parked") if "// The blocks of a k_walk_one launch that parked" in k else k.index("// After k_walk_one every look word is final")]
seg2 = seg.replace("rc = match_topic(ix, blob, offs[t], offs[t + 1], st, em);", "rc = match_topic(ix, blob_w, offs[t], offs[t + 1], st, em);")
seg2 = seg2.replace("const int frc = match_topic(ix, blob, offs[t], offs[t + 1], st, ce);", "const int frc = match_topic(ix, blob_w, offs[t], offs[t + 1], st, ce);")
seg2 = seg2.replace("one_emit(ix, S, blob, offs, t, live, rew, nrr, rg, base, rel, total, A.hit_offs, A.out, A.cap);",
                    "if (lane == 0 && vb == gridDim.x - 1) A.hit_offs[n] = base + total;   // (study: no k_one_scan)\n    one_emit(ix, S, blob_w, offs, t, live, rew, nrr, rg, base, rel, total, A.hit_offs, A.out, A.cap);")
assert seg2.count("blob_w") >= 4, seg2.count("blob_w")
k = k.replace(seg, seg2, 1)
# routing: small batches -> k_walk_one alone (no parking: defer = spins bound), no scan/finish
old = '''        if (n <= SMALL_TOPICS)
            hipLaunchKernelGGL((k_walk_small<MODE_COUNT, uint64_t>), dim3(blocks_for(n, SM_TOPICS)), dim3(WV_BLOCK), 0,
                               s, ix, ws, n, bytes, offs, o, hit_offs, out, cap, tag & LB_TAG_MASK, lb, SmallSegs{});'''
assert old in k
new = '''        if (n <= SMALL_TOPICS && one_pass_ok(ix)) {   // study: the staged lane walk, one launch
            if (path) *path = PATH_ONE;
            LbCtl lb1 = lb;
            lb1.defer = lb.spins;
            const OneArgs a1{n, bytes, offs, ws.look, err, hit_offs, out, cap, ws.cnt, ws.nr, ws.rng,
                             tag & LB_TAG_MASK, lb1};
            hipLaunchKernelGGL(k_walk_one, dim3(blocks_for(n, WALK_BLOCK)), dim3(WALK_BLOCK), 0, s, ix, a1);
        } else if (n <= SMALL_TOPICS)
            hipLaunchKernelGGL((k_walk_small<MODE_COUNT, uint64_t>), dim3(blocks_for(n, SM_TOPICS)), dim3(WV_BLOCK), 0,
                               s, ix, ws, n, bytes, offs, o, hit_offs, out, cap, tag & LB_TAG_MASK, lb, SmallSegs{});'''
k = k.replace(old, new, 1)
(ST / "stage1.hip").write_text(k)
from emqx_amd import build
print(build.build_variant("stage1", str(ST / "stage1.hip"), force=True))
