// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes of the
// wavefront renderer's state (SoA planes: 4 B per lane; node / hand-off records: 16 B per lane; scattered
// 4-B stores to chain slots), so that bench.py's roofline `traffic` can be read in bytes.
// MI355X_MICROARCH.md: FETCH_SIZE counts 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read;
// other widths are uncalibrated.  Every kernel here touches a known byte count of a 1 GiB buffer (well past
// the 256 MiB Infinity Cache, so its lines come from HBM):
//   read4    each lane loads 4 B, consecutive lanes consecutive words (256 B per wave-instruction)
//   read16   each lane loads 16 B (1 KB per wave-instruction)
//   write4   each lane stores 4 B, coalesced
//   write16  each lane stores 16 B, coalesced
//   scat4    each lane stores 4 B at a different 128-B line (lane i of wave w -> word (w * 64 + i) * 32 % n):
//            the partial-line stores of k_shade's per-chain-slot SoA writes
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d DIR -o run -- tools/fetch_calib
//        (and a second pass with WRITE_SIZE); tools/fetch_calib.py turns the two passes into ratios.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ __launch_bounds__(256) void read4(const uint32_t *__restrict__ a, size_t n, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= a[i];
    if (acc == 0x9E3779B1u) out[blockIdx.x] = acc;  // (never: keeps the loads live without a store stream)
}
__global__ __launch_bounds__(256) void read16(const uint4 *__restrict__ a, size_t n4, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B1u) out[blockIdx.x] = acc;
}
__global__ __launch_bounds__(256) void write4(uint32_t *a, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (uint32_t)i;
}
__global__ __launch_bounds__(256) void write16(uint4 *a, size_t n4) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
        a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}
__global__ __launch_bounds__(256) void scat4(uint32_t *a, size_t n, size_t nstores) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < nstores; i += (size_t)gridDim.x * 256)
        a[(i * 32) % n + (i * 32) / n] = (uint32_t)i;  // one word per 128-B line, lines visited in order
}

int main() {
    const size_t bytes = (size_t)1 << 30, n = bytes / 4, n4 = bytes / 16, nscat = n / 32;
    uint32_t *a = nullptr, *out = nullptr;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&out, 1 << 20));
    CHECK(hipMemset(a, 1, bytes));
    const dim3 g(4096), b(256);
    for (int rep = 0; rep < 2; ++rep) {  // the second repetition is the one to read (first-touch effects)
        hipLaunchKernelGGL(read4, g, b, 0, 0, a, n, out);
        hipLaunchKernelGGL(read16, g, b, 0, 0, reinterpret_cast<const uint4 *>(a), n4, out);
        hipLaunchKernelGGL(write4, g, b, 0, 0, a, n);
        hipLaunchKernelGGL(write16, g, b, 0, 0, reinterpret_cast<uint4 *>(a), n4);
        hipLaunchKernelGGL(scat4, g, b, 0, 0, a, n, nscat);
        CHECK(hipDeviceSynchronize());
    }
    printf("{\"read4\": %zu, \"read16\": %zu, \"write4\": %zu, \"write16\": %zu, \"scat4_bytes\": %zu, "
           "\"scat4_lines\": %zu}\n", bytes, bytes, bytes, bytes, nscat * 4, nscat);
    CHECK(hipFree(a));
    CHECK(hipFree(out));
    return 0;
}
