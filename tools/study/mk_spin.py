"""Study build (not product): an in-place small batch (k_walk_small, count
mode) signals its own completion -- every block, after a system-scope fence,
counts itself done on a device word; the last one writes the launch tag into
a mapped host word -- and the host spins on that word instead of
hipStreamSynchronize (bounded; the stream sync stays the fallback).  Saves the
end-of-kernel fence + completion signal + runtime wake-up on the host-to-host
path the NIF takes.
Build: python tools/study/mk_spin.py -> emqx_amd/variants/libtmatch_spin.so"""
import pathlib, sys
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
CS = ROOT / "emqx_amd" / "csrc"
ST = ROOT / "emqx_amd" / "study"
k = (CS / "tm_kernels.hip").read_text()
anchor = "template <int MODE, class OT>\n__global__ __launch_bounds__(WV_BLOCK) void k_walk_small("
assert anchor in k
k = k.replace(anchor, '''// study: grid completion flag (HINT_WORDS: one hint word past the product's)
__device__ __forceinline__ void grid_done(const Workspace &ws, uint32_t tag) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        const uint32_t k = atomicAdd(&ws.list_n[LIST_SLOTS], 1u);
        if (k == gridDim.x - 1) {
            ws.list_n[LIST_SLOTS] = 0;
            __threadfence_system();
            __hip_atomic_store(&ws.hint_d[HINT_WORDS], tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
''' + anchor, 1)
a = "    if (s_fail) return;   // (block-uniform)"
assert a in k
k = k.replace(a, "    if (s_fail) { if (MODE == MODE_COUNT) grid_done(ws, tag); return; }   // (block-uniform)", 1)
a = '''        for (uint32_t i = threadIdx.x; i < m; i += WV_BLOCK)
            if (b0 + i < cap) out[b0 + i] = s_vals[i];
    }
}
'''
assert k.count(a) == 1
k = k.replace(a, '''        for (uint32_t i = threadIdx.x; i < m; i += WV_BLOCK)
            if (b0 + i < cap) out[b0 + i] = s_vals[i];
    }
    if (MODE == MODE_COUNT) grid_done(ws, tag);
}
''', 1)
h = (CS / "tm_host.cpp").read_text()
for a, b in (("hipMalloc(&w.list_n, LIST_SLOTS * 4)", "hipMalloc(&w.list_n, (LIST_SLOTS + 1) * 4)"),
             ("hipMemsetAsync(w.list_n, 0, LIST_SLOTS * 4, ln.s)", "hipMemsetAsync(w.list_n, 0, (LIST_SLOTS + 1) * 4, ln.s)"),
             ("hipHostMalloc(&w.hint_h, HINT_WORDS * 4, hipHostMallocMapped)", "hipHostMalloc(&w.hint_h, (HINT_WORDS + 1) * 4, hipHostMallocMapped)"),
             ("std::memset(w.hint_h, 0, HINT_WORDS * 4);", "std::memset(w.hint_h, 0, (HINT_WORDS + 1) * 4);")):
    assert a in h, a
    h = h.replace(a, b, 1)
anchor = "static int retry_or_fail(tm_index *ix, std::unique_lock<std::mutex> &g, Lane &ln, int tries) {"
assert anchor in h
h = h.replace(anchor, '''// study: spin on the small kernel's completion word (bounded), else the stream sync
static hipError_t wait_done(Lane &ln, uint32_t tag, hipStream_t s) {
    volatile uint32_t *f = ln.w.hint_h + HINT_WORDS;
    for (uint32_t i = 0; i < (1u << 20); i++) {
        if (*f == tag) return hipSuccess;
        __builtin_ia32_pause();
    }
    return hipStreamSynchronize(s);
}

''' + anchor, 1)
a = '''                if ((rc = batch_done(ix, ln))) return rc;
                g.unlock();
                if (timing) tt[nt++] = now_us();
                HIPCHK(ix, hipStreamSynchronize(s));'''
assert a in h
h = h.replace(a, '''                if ((rc = batch_done(ix, ln))) return rc;
                g.unlock();
                if (timing) tt[nt++] = now_us();
                if (path == PATH_SMALL && !(sorted && dv)) HIPCHK(ix, wait_done(ln, tag, s));
                else HIPCHK(ix, hipStreamSynchronize(s));''', 1)
a = '''                    if ((rc = batch_done(ix, ln))) return rc;
                    g.unlock();
                    HIPCHK(ix, hipStreamSynchronize(s));
                    if (!batch_failed(ix, ln)) break;'''
assert a in h
h = h.replace(a, '''                    if ((rc = batch_done(ix, ln))) return rc;
                    g.unlock();
                    HIPCHK(ix, wait_done(ln, tag, s));
                    if (!batch_failed(ix, ln)) break;''', 1)
(ST / "spin.hip").write_text(k)
(ST / "spin_host.cpp").write_text(h)
from emqx_amd import build
print(build.build_variant("spin", str(ST / "spin.hip"), force=True, host_src=str(ST / "spin_host.cpp")))
