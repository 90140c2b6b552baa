// store_bench.hip -- calibration: the streaming store ceiling of MI355X for
// the shape k_emit writes (C2: 4 GB of hit-list values per 1M-topic batch,
// each wave writing 1 KiB per store instruction, values read from a small
// L2-resident run table).  The emit's store rate is judged against this.
//
// Kernels (256-thread blocks; each wave owns a contiguous span of the output):
//   fill     16-B stores of a constant (plain / non-temporal)
//   copyrun  16-B loads from a 1,000-value run table (L2 resident) + 16-B stores
// usage: store_bench [GB]   prints mode,blocks,GBps
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void fill(u32x4 *out, uint64_t nq, uint64_t per_wave) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t q0 = wave * per_wave, q1 = q0 + per_wave < nq ? q0 + per_wave : nq;
    const u32x4 v = {(uint32_t)wave, lane, 1u, 2u};
    for (uint64_t q = q0 + lane; q < q1; q += 64) {
        if (NT) __builtin_nontemporal_store(v, out + q);
        else out[q] = v;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void copyrun(u32x4 *out, uint64_t nq, uint64_t per_wave, const uint32_t *run) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t q0 = wave * per_wave, q1 = q0 + per_wave < nq ? q0 + per_wave : nq;
    for (uint64_t q = q0 + lane; q < q1; q += 64) {
        const uint32_t o = (uint32_t)((q * 4) % 996);
        const u32x4 v = *reinterpret_cast<const u32x4 *>(run + (o & ~3u));
        if (NT) __builtin_nontemporal_store(v, out + q);
        else out[q] = v;
    }
}

int main(int argc, char **argv) {
    const uint64_t gb = argc > 1 ? strtoull(argv[1], 0, 10) : 4;
    const uint64_t bytes = gb << 30, nq = bytes / 16;
    u32x4 *out;
    uint32_t *run;
    CHK(hipMalloc(&out, bytes));
    CHK(hipMalloc(&run, 4096 * 4));
    CHK(hipMemset(run, 1, 4096 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    printf("mode,blocks,per_wave_KiB,GBps\n");
    const char *names[4] = {"fill", "fill_nt", "copyrun", "copyrun_nt"};
    // shift: the output starts `shift` bytes into the buffer (16-B aligned but not
    // 128-B aligned, as k_emit's wave spans are) -- modes 0-3 at shift 0, then
    // fill_nt at shifts 16 and 64 and per-wave spans of odd quad counts
    for (int mode = 0; mode < 4; mode++) {
        for (uint64_t blocks : {1024ull, 2048ull, 4096ull, 8192ull, 16384ull}) {
            const uint64_t waves = blocks * 4, per_wave = (nq + waves - 1) / waves;
            auto launch = [&]() {
                switch (mode) {
                    case 0: hipLaunchKernelGGL(fill<false>, dim3(blocks), dim3(256), 0, 0, out, nq, per_wave); break;
                    case 1: hipLaunchKernelGGL(fill<true>, dim3(blocks), dim3(256), 0, 0, out, nq, per_wave); break;
                    case 2: hipLaunchKernelGGL(copyrun<false>, dim3(blocks), dim3(256), 0, 0, out, nq, per_wave, run); break;
                    default: hipLaunchKernelGGL(copyrun<true>, dim3(blocks), dim3(256), 0, 0, out, nq, per_wave, run);
                }
            };
            launch();
            CHK(hipDeviceSynchronize());
            const int reps = 5;
            CHK(hipEventRecord(e0));
            for (int r = 0; r < reps; r++) launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("%s,%lu,%.1f,%.1f\n", names[mode], (unsigned long)blocks, per_wave * 16 / 1024.0,
                   (double)bytes * reps / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    for (uint64_t shift : {16ull, 64ull}) {
        u32x4 *o = reinterpret_cast<u32x4 *>(reinterpret_cast<char *>(out) + shift);
        const uint64_t nq2 = nq - 8, blocks = 4096, waves = blocks * 4;
        for (int odd = 0; odd < 2; odd++) {
            // odd: per-wave spans of an odd number of quads, so every wave starts mid-line
            const uint64_t per_wave = odd ? ((nq2 / waves) | 1) : (nq2 + waves - 1) / waves;
            hipLaunchKernelGGL(fill<true>, dim3(blocks), dim3(256), 0, 0, o, nq2, per_wave);
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(e0));
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fill<true>, dim3(blocks), dim3(256), 0, 0, o, nq2, per_wave);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const uint64_t written = std::min<uint64_t>(nq2, per_wave * waves) * 16;
            printf("fill_nt_shift%lu%s,%lu,%.1f,%.1f\n", (unsigned long)shift, odd ? "_oddspan" : "", (unsigned long)blocks,
                   per_wave * 16 / 1024.0, (double)written * 5 / (ms * 1e-3) / 1e9);
            fflush(stdout);
        }
    }
    return 0;
}
