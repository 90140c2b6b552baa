// Study (not product): can the host write device memory directly (fine-grained
// VRAM mapped through the PCIe BAR), and how fast?  If so, a NIF could pack a
// batch's topics straight into HBM and the one-launch kernel would read no
// host memory.
// Build: hipcc --offload-arch=gfx950 -O2 tools/study/bar_probe.hip -o tools/study/bar_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_sum(const uint32_t *p, uint64_t n, unsigned long long *out) {
    unsigned long long s = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) s += p[i];
    atomicAdd(out, s);
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const uint64_t bytes = 64ull << 20, n = bytes / 4;
    uint32_t *d = nullptr;
    CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&d), bytes, hipDeviceMallocFinegrained));
    hipPointerAttribute_t a;
    CK(hipPointerGetAttributes(&a, d));
    printf("fine-grained VRAM: type %d device %d hostPointer %p devicePointer %p\n", (int)a.type, a.device,
           a.hostPointer, a.devicePointer);
    unsigned long long *sum = nullptr;
    CK(hipMalloc(&sum, 8));
    std::vector<uint32_t> h(n);
    for (uint64_t i = 0; i < n; i++) h[i] = (uint32_t)(i * 2654435761u);
    unsigned long long want = 0;
    for (uint64_t i = 0; i < n; i++) want += h[i];
    fflush(stdout);
    // host writes through the pointer itself (faults here if the BAR does not map it)
    for (uint64_t chunk : {4096ull, 147456ull, 1ull << 20, 16ull << 20}) {
        const int reps = (int)std::max<uint64_t>(1, (64ull << 20) / chunk);
        const double t0 = now();
        for (int r = 0; r < reps; r++) std::memcpy(reinterpret_cast<uint8_t *>(d) + (r * chunk) % bytes, h.data(), chunk);
        const double el = now() - t0;
        printf("host memcpy into VRAM: chunk %8llu B  %.2f GB/s  %.2f us per chunk\n", (unsigned long long)chunk,
               chunk * (double)reps / el / 1e9, el / reps * 1e6);
    }
    std::memcpy(d, h.data(), bytes);
    CK(hipMemset(sum, 0, 8));
    CK(hipDeviceSynchronize());
    k_sum<<<1024, 256>>>(d, n, sum);
    unsigned long long got = 0;
    CK(hipMemcpy(&got, sum, 8, hipMemcpyDeviceToHost));
    printf("device sum %s (%llu vs %llu)\n", got == want ? "OK" : "MISMATCH", got, want);
    // host reads back (slow: uncached reads over PCIe)
    const double t0 = now();
    unsigned long long hs = 0;
    for (uint64_t i = 0; i < (1u << 18); i++) hs += d[i];
    printf("host read 1 MiB: %.1f us (%llu)\n", (now() - t0) * 1e6, hs);
    CK(hipFree(d));
    CK(hipFree(sum));
    return 0;
}
