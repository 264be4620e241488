// Development microbenchmark: HBM bandwidth of writes/reads of contiguous
// runs of L u64 records at random run-aligned positions (scatter/gather
// efficiency vs run length).  Not part of the library.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t perm(uint64_t r, uint64_t mask) {
    // bijection on [0, mask]: odd multiply + xorshift, masked
    r = (r * 0x9E3779B97F4A7C15ull) & mask;
    r ^= r >> 7;
    return (r * 0xBF58476D1CE4E5B9ull) & mask;
}

__global__ void k_write(uint64_t *out, uint64_t n, int lg, uint64_t runmask) {
    const uint64_t L = 1ull << lg;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t run = i >> lg, off = i & (L - 1);
        out[(perm(run, runmask) << lg) + off] = i;
    }
}
// the same runs, but each run's L records are written by L different waves
// (record i of a block tile of 64 * L records: run i % 64, slot i / 64)
__global__ void k_write_split(uint64_t *out, uint64_t n, int lg, uint64_t runmask) {
    const uint64_t L = 1ull << lg, T = 64 * L;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t tile = i / T, w = i % T;
        const uint64_t run = tile * 64 + (w & 63), off = w >> 6;
        out[(perm(run, runmask) << lg) + off] = i;
    }
}
__global__ void k_read(const uint64_t *in, uint64_t n, int lg, uint64_t runmask, uint64_t *sink) {
    const uint64_t L = 1ull << lg;
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t run = i >> lg, off = i & (L - 1);
        acc += in[(perm(run, runmask) << lg) + off];
    }
    if (acc == 42) sink[0] = acc;
}
__global__ void k_seq(uint64_t *out, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) out[i] = i;
}

int main(int argc, char **argv) {
    const int LGN = argc > 1 ? atoi(argv[1]) : 29;   // 2^LGN records (29 = 4 GiB)
    const uint64_t n = 1ull << LGN;
    uint64_t *buf, *sink;
    CK(hipMalloc(&buf, n * 8));
    CK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 256 * 16, block = 256;
    float ms;
    k_seq<<<grid, block>>>(buf, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; r++) k_seq<<<grid, block>>>(buf, n);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("%.0f GiB buffer, seq write: %.1f GB/s\n", n * 8.0 / (1ull << 30), 3.0 * n * 8 / (ms / 1e3) / 1e9);
    for (int lg = argc > 2 ? atoi(argv[2]) : 0; lg <= 8; lg++) {
        const uint64_t runmask = (1ull << (LGN - lg)) - 1;
        k_write<<<grid, block>>>(buf, n, lg, runmask);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; r++) k_write<<<grid, block>>>(buf, n, lg, runmask);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        const double wgbs = 3.0 * n * 8 / (ms / 1e3) / 1e9;
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; r++) k_read<<<grid, block>>>(buf, n, lg, runmask, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        const double rgbs = 3.0 * n * 8 / (ms / 1e3) / 1e9;
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; r++) k_write_split<<<grid, block>>>(buf, n, lg, runmask);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("run %4d B: write %.1f GB/s  read %.1f GB/s  split-write %.1f GB/s\n", (int)(8 << lg), wgbs, rgbs,
               3.0 * n * 8 / (ms / 1e3) / 1e9);
    }
    return 0;
}
