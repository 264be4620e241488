// kh_apply.cuh -- region apply, bigcount crossing resolution, finalize.
// Included by kh_engine.hip.
//
// One workgroup owns one region of 2^s0 bins of one table at a time: the
// table slice is read into LDS with 16-byte loads, every record of the region
// bumps its bin's LDS counter and (for bins that were zero before the batch)
// takes the minimum k-mer index (= the first insert in stream order, i.e. the
// reference's is_new winner, storage.hh:578-588), then the saturated values
// are written back with 16-byte stores.
#pragma once
#include "kh_partition.cuh"

namespace kh {

constexpr int APPLY_THREADS = 1024;
constexpr int FIN_THREADS = 256;

struct ApplyArgs {
    const uint64_t *off2;
    const uint64_t *rec;
    uint8_t *tab;
    uint8_t *newf, *fullf;
    uint64_t *cross;
    uint64_t cap_cross;
    uint64_t *ctr;
    uint64_t rprefix[MAXT + 1];   // real-region prefix per table
};

__device__ __forceinline__ void full_add(uint8_t *fullf, uint32_t j) {
    atomicAdd((uint32_t *)(fullf + (j & ~3u)), 1u << (8 * (j & 3u)));
}

__device__ __forceinline__ int region_table(const ApplyArgs &A, int n, uint64_t rr) {
    int i = 0;
    while (i + 1 < n && rr >= A.rprefix[i + 1]) i++;
    return i;
}

// Byte (KIND == BYTE) and Nibble storage: ByteStorage::add / NibbleStorage::add
// (storage.hh:571-624 / 320-359) applied as a batch
template <int KIND>
__global__ void __launch_bounds__(APPLY_THREADS, 2) k_apply_count(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = 1u << P.s0;
    uint32_t *cnt = (uint32_t *)smem;     // [R]
    uint32_t *minj = cnt + R;             // [R]
    uint32_t *chg = minj + R;             // [R/512] changed 16-bin chunks
    uint8_t *c0 = (uint8_t *)(chg + R / 512);  // [R]
    const uint32_t MAXC = KIND == BYTE ? 255u : 15u;
    const bool bigc = KIND == BYTE && P.use_bigcount;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    for (uint64_t rr = blockIdx.x; rr < total; rr += gridDim.x) {
        const int i = region_table(A, P.n, rr);
        const uint64_t lreg = rr - A.rprefix[i];
        const uint64_t region = (P.tbase[i] >> P.s0) + lreg;
        const uint64_t e0 = A.off2[region], e1 = A.off2[region + 1];
        if (e0 == e1) continue;
        const uint64_t bin_lo = lreg << P.s0;
        const uint32_t nb = (uint32_t)min((uint64_t)R, P.p[i] - bin_lo);
        const uint32_t nchunk = (nb + 15) / 16;   // 16 bins per thread-chunk
        uint8_t *tab = A.tab + P.tbyte[i];
        // table slice -> LDS (16-byte loads; the arena pads every table to 256 B)
        if (KIND == BYTE) {
            const uint4 *src = (const uint4 *)(tab + bin_lo);
            for (uint32_t t = threadIdx.x; t < nchunk; t += blockDim.x) ((uint4 *)c0)[t] = src[t];
        } else {
            const uint2 *src = (const uint2 *)(tab + (bin_lo >> 1));
            for (uint32_t t = threadIdx.x; t < nchunk; t += blockDim.x) {
                const uint2 v = src[t];
                uint4 o;
                uint32_t *ow = (uint32_t *)&o;
                const uint32_t w[2] = {v.x, v.y};
#pragma unroll
                for (int h = 0; h < 2; h++) {
#pragma unroll
                    for (int b2 = 0; b2 < 2; b2++) {
                        const uint32_t x = (w[h] >> (16 * b2)) & 0xFFFFu;   // 2 bytes = 4 bins
                        const uint32_t lo = x & 0xFF, hi = x >> 8;
                        ow[2 * h + b2] = (lo >> 4) | ((lo & 15) << 8) | ((hi >> 4) << 16) | ((hi & 15) << 24);
                    }
                }
                ((uint4 *)c0)[t] = o;
            }
        }
        for (uint32_t t = threadIdx.x; t < nchunk * 4; t += blockDim.x) {
            ((uint4 *)cnt)[t] = make_uint4(0, 0, 0, 0);
            ((uint4 *)minj)[t] = make_uint4(NO_J, NO_J, NO_J, NO_J);
        }
        for (uint32_t t = threadIdx.x; t < R / 512; t += blockDim.x) chg[t] = 0;
        __syncthreads();
        // records: four independent loads in flight per thread
        for (uint64_t q0 = e0 + threadIdx.x; q0 < (P.ablate & 2 ? e0 : e1); q0 += 4ull * blockDim.x) {
            uint64_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t q = q0 + (uint64_t)u * blockDim.x;
                v[u] = q < e1 ? A.rec[q] : ~0ull;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (v[u] == ~0ull) continue;
                const uint32_t o = (uint32_t)v[u];
                const uint32_t j = (uint32_t)(v[u] >> 32);
                atomicAdd(&cnt[o], 1u);
                const uint8_t c = c0[o];
                if (c == 0) atomicMin(&minj[o], j);
                if (bigc && c == 255) full_add(A.fullf, j);
            }
        }
        __syncthreads();
        // pass 1 (thread per bin, conflict-free LDS): winners, crossings,
        // saturated value into c0, changed-chunk bitmap
        for (uint32_t o = threadIdx.x; o < nb; o += blockDim.x) {
            const uint32_t n = cnt[o];
            if (!n) continue;
            const uint32_t c = c0[o];
            if (c == 0) {
                if (!(P.ablate & 1)) A.newf[minj[o]] = 1;
                occ += (i == 0);
            }
            const uint32_t v = c + n;
            if (bigc && c < 255 && v >= 255) {
                const uint64_t idx = atomicAdd((unsigned long long *)&A.ctr[CTR_NCROSS], 1ull);
                if (idx < A.cap_cross) A.cross[idx] = ((P.tbase[i] + bin_lo + o) << 8) | c;
                else atomicOr((unsigned long long *)&A.ctr[CTR_ERR], 1ull);
            }
            const uint32_t f = v < MAXC ? v : MAXC;
            if (f != c) {
                c0[o] = (uint8_t)f;
                atomicOr(&chg[o >> 9], 1u << ((o >> 4) & 31));
            }
        }
        __syncthreads();
        // pass 2: write back changed 16-bin chunks
        for (uint32_t t = threadIdx.x; t < nchunk; t += blockDim.x) {
            if (!((chg[t >> 5] >> (t & 31)) & 1) || (P.ablate & 4)) continue;
            const uint4 cv = ((const uint4 *)c0)[t];
            if (KIND == BYTE) {
                ((uint4 *)(tab + bin_lo))[t] = cv;
            } else {
                // even bin -> high nibble (storage.hh:262-272)
                const uint8_t *fin = (const uint8_t *)&cv;
                uint2 o;
                uint32_t *ow = (uint32_t *)&o;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    uint32_t w = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        w |= (uint32_t)((fin[8 * h + 2 * b] << 4) | fin[8 * h + 2 * b + 1]) << (8 * b);
                    ow[h] = w;
                }
                ((uint2 *)(tab + (bin_lo >> 1)))[t] = o;
            }
        }
        __syncthreads();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// Bit storage (Bloom): BitStorage::test_and_set_bits (storage.hh:172-199)
__global__ void __launch_bounds__(APPLY_THREADS, 2) k_apply_bit(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = 1u << P.s0;
    uint32_t *minj = (uint32_t *)smem;          // [R]
    uint32_t *chg = minj + R;                   // [R/4096] changed 128-bin chunks
    uint32_t *bits32 = chg + (R / 4096 < 4 ? 4 : R / 4096);  // [R/32]
    uint8_t *bits = (uint8_t *)bits32;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    for (uint64_t rr = blockIdx.x; rr < total; rr += gridDim.x) {
        const int i = region_table(A, P.n, rr);
        const uint64_t lreg = rr - A.rprefix[i];
        const uint64_t region = (P.tbase[i] >> P.s0) + lreg;
        const uint64_t e0 = A.off2[region], e1 = A.off2[region + 1];
        if (e0 == e1) continue;
        const uint64_t bin_lo = lreg << P.s0;
        const uint32_t nb = (uint32_t)min((uint64_t)R, P.p[i] - bin_lo);
        const uint32_t nchunk = (nb + 127) / 128;   // 16 bytes = 128 bins per chunk
        uint8_t *tab = A.tab + P.tbyte[i] + (bin_lo >> 3);
        for (uint32_t t = threadIdx.x; t < nchunk; t += blockDim.x) ((uint4 *)bits)[t] = ((const uint4 *)tab)[t];
        for (uint32_t t = threadIdx.x; t < nchunk * 32; t += blockDim.x)
            ((uint4 *)minj)[t] = make_uint4(NO_J, NO_J, NO_J, NO_J);
        for (uint32_t t = threadIdx.x; t < 4; t += blockDim.x) chg[t] = 0;
        __syncthreads();
        for (uint64_t q0 = e0 + threadIdx.x; q0 < e1; q0 += 4ull * blockDim.x) {
            uint64_t v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint64_t q = q0 + (uint64_t)u * blockDim.x;
                v[u] = q < e1 ? A.rec[q] : ~0ull;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (v[u] == ~0ull) continue;
                const uint32_t o = (uint32_t)v[u];
                if (!((bits[o >> 3] >> (o & 7)) & 1)) atomicMin(&minj[o], (uint32_t)(v[u] >> 32));
            }
        }
        __syncthreads();
        // pass 1 (thread per bin): winners set their bit
        for (uint32_t o = threadIdx.x; o < nb; o += blockDim.x) {
            const uint32_t mj = minj[o];
            if (mj == NO_J) continue;
            atomicOr(&bits32[o >> 5], 1u << (o & 31));
            atomicOr(&chg[o >> 12], 1u << ((o >> 7) & 31));
            A.newf[mj] = 1;
            occ += (i == 0);
        }
        __syncthreads();
        // pass 2: write back changed 128-bin chunks
        for (uint32_t t = threadIdx.x; t < nchunk; t += blockDim.x)
            if ((chg[t >> 5] >> (t & 31)) & 1) ((uint4 *)tab)[t] = ((const uint4 *)bits)[t];
        __syncthreads();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// ---------------------------------------------------------------------------
// crossing bins (bigcount): inserts with stream rank >= 255 - c0 are "full"
// (ByteStorage::add, storage.hh:590-603).  K-th smallest k-mer index by a
// 4-pass 8-bit radix select over the bin's records.
__global__ void __launch_bounds__(256) k_crossing(Params P, const uint64_t *off2, const uint64_t *rec,
                                                  const uint64_t *cross, const uint64_t *ctr, uint64_t cap_cross,
                                                  uint8_t *fullf) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_sel[2];
    uint64_t ncross = ctr[CTR_NCROSS];
    if (ncross > cap_cross) ncross = cap_cross;
    const uint64_t rmask = (1ull << P.s0) - 1;
    for (uint64_t c = blockIdx.x; c < ncross; c += gridDim.x) {
        const uint64_t G = cross[c] >> 8;
        const uint32_t c0 = (uint32_t)(cross[c] & 0xFF);
        const uint64_t region = G >> P.s0;
        const uint32_t o = (uint32_t)(G & rmask);
        const uint64_t e0 = off2[region], e1 = off2[region + 1];
        uint32_t K = 255 - c0;          // rank of the first full insert
        uint32_t prefix = 0;
        for (int pass = 0; pass < 4; pass++) {
            const int sh = 24 - 8 * pass;
            for (int t = threadIdx.x; t < 256; t += blockDim.x) hist[t] = 0;
            __syncthreads();
            for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
                const uint64_t v = rec[q];
                if ((uint32_t)v != o) continue;
                const uint32_t j = (uint32_t)(v >> 32);
                if (pass > 0 && (j >> (sh + 8)) != (prefix >> (sh + 8))) continue;
                atomicAdd(&hist[(j >> sh) & 0xFF], 1u);
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                uint32_t acc = 0, d = 0;
                for (d = 0; d < 256; d++) {
                    if (acc + hist[d] > K) break;
                    acc += hist[d];
                }
                s_sel[0] = d;
                s_sel[1] = K - acc;
            }
            __syncthreads();
            prefix |= s_sel[0] << sh;
            K = s_sel[1];
            __syncthreads();
        }
        for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
            const uint64_t v = rec[q];
            if ((uint32_t)v != o) continue;
            const uint32_t j = (uint32_t)(v >> 32);
            if (j >= prefix) full_add(fullf, j);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// finalize: n_unique += #new k-mers (16 flags per thread via 16-byte loads);
// k-mers full in every table feed the bigcount map; optional per-k-mer hashes
template <class Src>
__global__ void __launch_bounds__(FIN_THREADS) k_finalize(Params P, Src src, uint64_t nkmers, const uint8_t *newf,
                                                         const uint8_t *fullf, uint64_t *ctr, uint64_t *bc,
                                                         uint64_t cap_bc, uint64_t *out_hash) {
    const bool bigc = P.kind == BYTE && P.use_bigcount;
    const uint64_t nchunk = (nkmers + 15) / 16;
    uint64_t uniq = 0;
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunk;
         c += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 nv = ((const uint4 *)newf)[c];   // bytes are 0/1, zero past nkmers
        uniq += __popc(nv.x) + __popc(nv.y) + __popc(nv.z) + __popc(nv.w);
        if (bigc) {
            const uint4 fv = ((const uint4 *)fullf)[c];
            if (fv.x | fv.y | fv.z | fv.w) {
                const uint8_t *fb = (const uint8_t *)&fv;
                for (int u = 0; u < 16; u++) {
                    const uint64_t j = c * 16 + u;
                    if (j < nkmers && fb[u] == (uint8_t)P.n) {
                        const uint64_t idx = atomicAdd((unsigned long long *)&ctr[CTR_NBC], 1ull);
                        if (idx < cap_bc) bc[idx] = kmer_hash_global(src, j);
                        else atomicOr((unsigned long long *)&ctr[CTR_ERR], 2ull);
                    }
                }
            }
        }
        if (out_hash) {
            for (int u = 0; u < 16; u++) {
                const uint64_t j = c * 16 + u;
                if (j < nkmers) out_hash[j] = kmer_hash_global(src, j);
            }
        }
    }
    uniq = wave_sum(uniq);
    if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
}

}  // namespace kh
