// Microbenchmark (development): cost of exact h % p on gfx950 -- 64-bit
// Barrett (kh_device.h mod_barrett) vs float64 quotient estimates.
// Every variant is checked against Barrett on the same hashes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include "../khmer_amd/csrc/kh_device.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct P4 { uint64_t p[4], m[4]; double pd[4], inv[4]; };

__device__ __forceinline__ uint64_t hgen(uint64_t x) { return kh::fmix64(x); }

// exact for h < 2^53, p < 2^32
__device__ __forceinline__ uint64_t mod_f64(uint64_t h, double pd, double inv) {
    const double hd = (double)(uint32_t)(h >> 32) * 4294967296.0 + (double)(uint32_t)h;
    const double q = __builtin_floor(hd * inv);
    double r = __builtin_fma(-q, pd, hd);
    r = r < 0 ? r + pd : r;
    r = r >= pd ? r - pd : r;
    return (uint64_t)(uint32_t)r;
}
// general: f64 quotient estimate (+-1), wrapping 64-bit remainder, correction
__device__ __forceinline__ uint64_t mod_f64q(uint64_t h, uint64_t p, double inv) {
    const double hd = (double)(uint32_t)(h >> 32) * 4294967296.0 + (double)(uint32_t)h;
    const uint64_t q = (uint64_t)(hd * inv);
    int64_t r = (int64_t)(h - q * p);
    r = r < 0 ? r + (int64_t)p : r;
    r = r >= (int64_t)p ? r - (int64_t)p : r;
    return (uint64_t)r;
}

template <int V>
__global__ void kmod(P4 P, uint64_t n, uint64_t hmask, uint64_t *out) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = hgen(i) & hmask;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            uint64_t r;
            if (V == 0) r = kh::mod_barrett(h, P.p[t], P.m[t]);
            else if (V == 1) r = mod_f64(h, P.pd[t], P.inv[t]);
            else r = mod_f64q(h, P.p[t], P.inv[t]);
            acc += r * (t + 1);
        }
    }
    atomicAdd((unsigned long long *)out, (unsigned long long)acc);
}

template <int V>
__global__ void kcheck(P4 P, uint64_t n, uint64_t hmask, uint64_t *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t h = hgen(i ^ 0x9e3779b97f4a7c15ull) & hmask;
        if (i < 64) h = hmask - i;   // top of the range
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const uint64_t a = kh::mod_barrett(h, P.p[t], P.m[t]);
            const uint64_t b = V == 1 ? mod_f64(h, P.pd[t], P.inv[t]) : mod_f64q(h, P.p[t], P.inv[t]);
            if (a != b) atomicAdd((unsigned long long *)bad, 1ull);
        }
    }
}

int main() {
    struct Cfg { const char *name; uint64_t p0; uint64_t hmask; bool v1; } cfgs[] = {
        {"C2 k=21 p~1e9", 999999937ull, (1ull << 42) - 1, true},
        {"C3 k=31 p~4e9", 3999999979ull, (1ull << 62) - 1, false},
        {"C4 k=21 p~8e9", 7999999957ull, (1ull << 42) - 1, false},
        {"k=32 p~1e9", 999999937ull, ~0ull, false},
    };
    uint64_t *d;
    CK(hipMalloc(&d, 64));
    const uint64_t n = 1ull << 31;
    for (auto &c : cfgs) {
        P4 P;
        for (int t = 0; t < 4; t++) {
            P.p[t] = c.p0 - 2 * t;
            P.m[t] = kh::barrett_m(P.p[t]);
            P.pd[t] = (double)P.p[t];
            P.inv[t] = 1.0 / (double)P.p[t];
        }
        for (int v = 0; v < 3; v++) {
            if (v == 1 && !c.v1) continue;
            if (v) {
                CK(hipMemset(d, 0, 8));
                if (v == 1) hipLaunchKernelGGL(kcheck<1>, dim3(4096), dim3(256), 0, 0, P, 1ull << 28, c.hmask, d);
                else hipLaunchKernelGGL(kcheck<2>, dim3(4096), dim3(256), 0, 0, P, 1ull << 28, c.hmask, d);
                uint64_t bad;
                CK(hipMemcpy(&bad, d, 8, hipMemcpyDeviceToHost));
                printf("%s V%d mismatches: %llu\n", c.name, v, (unsigned long long)bad);
            }
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            float best = 1e9;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipMemset(d, 0, 8));
                CK(hipEventRecord(e0));
                if (v == 0) hipLaunchKernelGGL(kmod<0>, dim3(8192), dim3(256), 0, 0, P, n, c.hmask, d);
                else if (v == 1) hipLaunchKernelGGL(kmod<1>, dim3(8192), dim3(256), 0, 0, P, n, c.hmask, d);
                else hipLaunchKernelGGL(kmod<2>, dim3(8192), dim3(256), 0, 0, P, n, c.hmask, d);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            uint64_t s;
            CK(hipMemcpy(&s, d, 8, hipMemcpyDeviceToHost));
            printf("%s V%d: %.2f ms for %llu x 4 mods (%.1f Gmod/s) sum %llx\n", c.name, v, best,
                   (unsigned long long)n, n * 4 / best / 1e6, (unsigned long long)s);
        }
    }
    return 0;
}
