// gather_bench.hip -- calibration microbenchmark: how many random 64-byte
// lines per second can MI355X serve for a given table footprint?  This is the
// practical ceiling of a pointer-chasing trie walk (each walk step reads one
// random line), which the HBM streaming peak (8 TB/s) overstates.
//
// Modes (one lane = one independent chain, 256-thread blocks, grid fills the chip):
//   chase: each lane follows `steps` dependent random lines (next index from the line)
//   gather: each lane issues `steps` independent random line reads (no dependency)
// Prints lines/s and line-GB/s (64 B per line) per footprint.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void init_lines(uint4 *t, uint64_t nlines, uint64_t seed) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlines) return;
    // full-period LCG over the (power-of-two) line count: every chase walks a
    // permutation cycle, so lanes never merge onto a shrinking set of lines
    uint32_t nxt = (uint32_t)((i * 0x9E3779B1ull + (seed | 1)) & (nlines - 1));
    for (int k = 0; k < 4; k++) t[i * 4 + k] = make_uint4(nxt, (uint32_t)i, k, 0);
}

__global__ __launch_bounds__(256) void chase(const uint4 *t, uint64_t nlines, int steps, uint32_t *sink) {
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cur = (uint32_t)((g * 0x9e3779b97f4a7c15ull) % nlines);
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint4 *p = t + (uint64_t)cur * 4;
        uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc += b.y + c.z + d.w;
        cur = a.x;
    }
    if (acc == 0xFFFFFFFF) sink[0] = cur;
}

__global__ __launch_bounds__(256) void chase16(const uint4 *t, uint64_t nlines, int steps, uint32_t *sink) {
    // one 16-byte read per step (a vocab / fingerprint / edge probe)
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cur = (uint32_t)((g * 0x9e3779b97f4a7c15ull) % nlines);
    for (int s = 0; s < steps; s++) cur = t[(uint64_t)cur * 4].x;
    if (cur == 0xFFFFFFFF) sink[0] = cur;
}

__global__ __launch_bounds__(256) void gather(const uint4 *t, uint64_t nlines, int steps, uint32_t *sink) {
    uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t x = g * 0x9e3779b97f4a7c15ull + 1;
    uint32_t acc = 0;
    for (int s = 0; s < steps; s++) {
        x ^= x >> 31; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27;
        const uint4 *p = t + (x % nlines) * 4;
        uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        acc += a.x + b.y + c.z + d.w;
    }
    if (acc == 0xFFFFFFFF) sink[0] = acc;
}

static const char *NAMES[3] = {"chase", "gather", "chase16"};

// usage: gather_bench            sweep footprints x modes x lane counts
//        gather_bench MB MODE LANES REPS   one configuration (PMC calibration runs)
int main(int argc, char **argv) {
    int steps = 64;
    std::vector<uint64_t> sizes_mb = {8, 64, 256, 512, 1024, 2048, 4096};
    std::vector<int> modes = {0, 1, 2};
    std::vector<uint64_t> lane_set = {(uint64_t)256 * 256 * 8, (uint64_t)256 * 256 * 32};
    int reps = 5;
    if (argc == 5) {
        sizes_mb = {strtoull(argv[1], 0, 10)};
        modes = {atoi(argv[2])};
        lane_set = {strtoull(argv[3], 0, 10)};
        reps = atoi(argv[4]);
    }
    uint32_t *sink;
    CHK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    printf("mode,footprint_MiB,lanes,steps,lines_per_s,GBps_64B,launch_us\n");
    for (uint64_t mb : sizes_mb) {
        uint64_t nlines = mb * 1024 * 1024 / 64;
        uint4 *t;
        CHK(hipMalloc(&t, nlines * 64));
        hipLaunchKernelGGL(init_lines, dim3((nlines + 255) / 256), dim3(256), 0, 0, t, nlines, 12345);
        CHK(hipDeviceSynchronize());
        for (int mode : modes) {
            for (uint64_t lanes : lane_set) {
                dim3 grid(lanes / 256);
                auto k = mode == 0 ? chase : mode == 1 ? gather : chase16;
                hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, t, nlines, steps, sink);
                CHK(hipDeviceSynchronize());
                CHK(hipEventRecord(e0));
                for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, t, nlines, steps, sink);
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                double lines = (double)reps * lanes * steps;
                double lps = lines / (ms * 1e-3);
                printf("%s,%lu,%lu,%d,%.3e,%.1f,%.1f\n", NAMES[mode], mb, lanes, steps, lps, lps * 64 / 1e9,
                       ms * 1e3 / reps);
                fflush(stdout);
            }
        }
        CHK(hipFree(t));
    }
    return 0;
}
