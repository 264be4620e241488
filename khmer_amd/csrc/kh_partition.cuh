// kh_partition.cuh -- two-level partition of insert records (one record per
// (k-mer, table)) into LDS-sized table regions.  Included by kh_engine.hip.
//
// record = (batch k-mer index j << 32) | bin offset   (u64)
//   level 1: offset inside a bucket of 2^(s0+s2) global bins
//   level 2: offset inside a region of 2^s0 bins
// Both scatters stage a tile in LDS sorted by destination (counting sort) and
// write it out in contiguous runs (coalesced), one global cursor bump per
// destination per tile.  Within a destination records are unordered; the
// k-mer index travels with the record, so stream order is recovered exactly
// in the apply step.
#pragma once
#include "kh_src.cuh"

namespace kh {

constexpr int L1_THREADS = 512;
constexpr int L1_MAX_RPT = 8;                      // records per thread per tile
constexpr int L1_TILE_RECS = L1_THREADS * L1_MAX_RPT;
constexpr int L2_THREADS = 1024;
constexpr int L2_RPT = 8;
constexpr int L2_TILE_RECS = L2_THREADS * L2_RPT;  // 8192
constexpr uint32_t NO_J = 0xFFFFFFFFu;

// exclusive scan of hist[0..n) into lstart by one wave (n <= 8192)
__device__ __forceinline__ void wave_exclusive_scan(const uint32_t *hist, uint32_t *lstart, uint32_t n) {
    if (threadIdx.x >= 64) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t per = (n + 63) / 64;
    const uint32_t b0 = lane * per;
    uint32_t sum = 0;
    for (uint32_t t = 0; t < per && b0 + t < n; t++) sum += hist[b0 + t];
    uint32_t incl = sum;
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    uint32_t acc = incl - sum;
    for (uint32_t t = 0; t < per && b0 + t < n; t++) { lstart[b0 + t] = acc; acc += hist[b0 + t]; }
}

// ---------------------------------------------------------------------------
// level 1: bucket histogram over all tables
template <class Src>
__global__ void __launch_bounds__(L1_THREADS) k_count_l1(Params P, Src src, uint64_t nkmers, int tile_kmers,
                                                        uint32_t *cnt1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    uint64_t *s_meta = (uint64_t *)(hist + ((P.F1 + 3) & ~3u));
    uint64_t *s_koff = s_meta + 2;
    const int shift = P.s0 + P.s2;
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x) hist[b] = 0;
    const uint64_t j0 = (uint64_t)blockIdx.x * tile_kmers;
    const uint64_t j1 = min(nkmers, j0 + tile_kmers);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    __syncthreads();
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        const uint64_t h = kmer_hash(src, s_koff, tr, j);
        for (int i = 0; i < P.n; i++) atomicAdd(&hist[global_bin(P, i, h) >> shift], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x)
        if (hist[b]) atomicAdd(&cnt1[b], hist[b]);
}

// block-wide exclusive scan over n u64 values in LDS (blockDim.x == 1024)
__device__ uint64_t block_exclusive_scan(uint64_t *v, uint32_t n, uint64_t *s_part) {
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = threadIdx.x * per;
    uint64_t sum = 0;
    for (uint32_t t = 0; t < per && b0 + t < n; t++) sum += v[b0 + t];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x < 64) {
        // 1024 partials scanned by one wave: 16 per lane
        const uint32_t lane = threadIdx.x;
        uint64_t loc = 0;
        for (int t = 0; t < 16; t++) loc += s_part[lane * 16 + t];
        uint64_t incl = loc;
        for (int d = 1; d < 64; d <<= 1) {
            uint64_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        uint64_t acc = incl - loc;
        for (int t = 0; t < 16; t++) {
            uint64_t x = s_part[lane * 16 + t];
            s_part[lane * 16 + t] = acc;
            acc += x;
        }
        if (lane == 63) s_part[1024] = acc;
    }
    __syncthreads();
    uint64_t acc = s_part[threadIdx.x];
    for (uint32_t t = 0; t < per && b0 + t < n; t++) {
        uint64_t x = v[b0 + t];
        v[b0 + t] = acc;
        acc += x;
    }
    __syncthreads();
    return s_part[1024];
}

// level-1 bucket offsets, their cursors, and the tile prefix of level 2
__global__ void __launch_bounds__(1024) k_scan_l1(uint32_t F1, const uint32_t *cnt1, uint64_t *off1,
                                                  uint64_t *cur1, uint32_t *tile1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *v = (uint64_t *)smem;   // [F1]
    uint64_t *s_part = v + F1;        // [1025]
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) v[b] = cnt1[b];
    __syncthreads();
    const uint64_t total = block_exclusive_scan(v, F1, s_part);
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) { off1[b] = v[b]; cur1[b] = v[b]; }
    if (threadIdx.x == 0) off1[F1] = total;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) v[b] = (cnt1[b] + L2_TILE_RECS - 1) / L2_TILE_RECS;
    __syncthreads();
    const uint64_t tiles = block_exclusive_scan(v, F1, s_part);
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) tile1[b] = (uint32_t)v[b];
    if (threadIdx.x == 0) tile1[F1] = (uint32_t)tiles;
}

// level-1 scatter of tables [t0, t0+nt) (nt <= 8): records are kept in
// registers between the histogram and the placement pass
template <class Src>
__global__ void __launch_bounds__(L1_THREADS) k_scatter_l1(Params P, Src src, uint64_t nkmers, int kpt, int t0,
                                                          int nt, uint64_t *cur1, uint64_t *rec) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    uint64_t *gbase = (uint64_t *)smem;               // [F1]
    uint64_t *stage = gbase + F1a;                    // [L1_TILE_RECS]
    uint32_t *hist = (uint32_t *)(stage + L1_TILE_RECS);  // [F1]
    uint32_t *lstart = hist + F1a;                    // [F1]
    uint16_t *sb = (uint16_t *)(lstart + F1a);        // [L1_TILE_RECS]
    uint64_t *s_meta = (uint64_t *)(sb + L1_TILE_RECS);
    uint64_t *s_koff = s_meta + 2;
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;
    const int tile_kmers = L1_THREADS * kpt;

    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) hist[b] = 0;
    const uint64_t j0 = (uint64_t)blockIdx.x * tile_kmers;
    const uint64_t j1 = min(nkmers, j0 + tile_kmers);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    __syncthreads();

    uint64_t G[L1_MAX_RPT];
    uint32_t rank[L1_MAX_RPT];
    uint32_t jj[L1_MAX_RPT];
    int nr = 0;
#pragma unroll
    for (int q = 0; q < L1_MAX_RPT; q++) { G[q] = 0; rank[q] = 0; jj[q] = 0; }
    // pass A: hash, bins, bucket histogram (ranks within the tile)
    for (int a = 0; a < kpt; a++) {
        const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
        if (j >= j1) break;
        const uint64_t h = kmer_hash(src, s_koff, tr, j);
#pragma unroll
        for (int q = 0; q < L1_MAX_RPT; q++) {
            const int i = q - a * nt;  // table slot of register q for k-mer a
            if (i >= 0 && i < nt) {
                G[q] = global_bin(P, t0 + i, h);
                jj[q] = (uint32_t)j;
                rank[q] = atomicAdd(&hist[(uint32_t)(G[q] >> shift)], 1u);
                nr = q + 1;
            }
        }
    }
    __syncthreads();
    wave_exclusive_scan(hist, lstart, F1);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x)
        if (hist[b]) gbase[b] = atomicAdd((unsigned long long *)&cur1[b], (unsigned long long)hist[b]);
    // pass B: place in LDS in bucket order
#pragma unroll
    for (int q = 0; q < L1_MAX_RPT; q++) {
        if (q < nr) {
            const uint32_t b = (uint32_t)(G[q] >> shift);
            const uint32_t pos = lstart[b] + rank[q];
            stage[pos] = ((uint64_t)jj[q] << 32) | (G[q] & omask);
            sb[pos] = (uint16_t)b;
        }
    }
    __syncthreads();
    // pass C: coalesced runs
    const uint32_t nrec = (P.ablate & 8) ? 0 : (uint32_t)((j1 - j0) * (uint64_t)nt);
    for (uint32_t q = threadIdx.x; q < nrec; q += blockDim.x) {
        const uint32_t b = sb[q];
        rec[gbase[b] + (q - lstart[b])] = stage[q];
    }
}

// ---------------------------------------------------------------------------
// level 2
__device__ __forceinline__ bool l2_tile(uint32_t F1, const uint64_t *off1, const uint32_t *tile1,
                                        uint32_t *bucket, uint64_t *r0, uint64_t *r1) {
    const uint32_t t = blockIdx.x;
    if (t >= tile1[F1]) return false;
    uint32_t lo = 0, hi = F1;  // tile1[lo] <= t < tile1[hi]
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (tile1[mid] <= t) lo = mid; else hi = mid;
    }
    *bucket = lo;
    const uint64_t s = off1[lo] + (uint64_t)(t - tile1[lo]) * L2_TILE_RECS;
    *r0 = s;
    *r1 = min(off1[lo + 1], s + L2_TILE_RECS);
    return true;
}

__global__ void __launch_bounds__(L2_THREADS) k_count_l2(uint32_t F1, int s0, int s2, const uint64_t *off1,
                                                        const uint32_t *tile1, const uint64_t *rec,
                                                        uint32_t *cnt2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    const uint32_t F2 = 1u << s2;
    uint32_t b;
    uint64_t r0, r1;
    if (!l2_tile(F1, off1, tile1, &b, &r0, &r1)) return;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) hist[r] = 0;
    __syncthreads();
    const uint32_t *rec32 = (const uint32_t *)rec;   // low words = offsets
    for (uint64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) atomicAdd(&hist[rec32[2 * q] >> s0], 1u);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x)
        if (hist[r]) atomicAdd(&cnt2[(uint64_t)b * F2 + r], hist[r]);
}

// per bucket: absolute region offsets in the level-2 record array
__global__ void __launch_bounds__(1024) k_scan_l2(int s2, uint32_t F1, const uint64_t *off1, const uint32_t *cnt2,
                                                  uint64_t *off2, uint64_t *cur2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F2 = 1u << s2;
    uint64_t *v = (uint64_t *)smem;   // [F2]
    uint64_t *s_part = v + F2;        // [1025]
    const uint32_t b = blockIdx.x;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) v[r] = cnt2[(uint64_t)b * F2 + r];
    __syncthreads();
    block_exclusive_scan(v, F2, s_part);
    const uint64_t base = off1[b];
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) {
        off2[(uint64_t)b * F2 + r] = base + v[r];
        cur2[(uint64_t)b * F2 + r] = base + v[r];
    }
    if (b == F1 - 1 && threadIdx.x == 0) off2[(uint64_t)F1 * F2] = off1[F1];
}

__global__ void __launch_bounds__(L2_THREADS) k_scatter_l2(uint32_t F1, int s0, int s2, const uint64_t *off1,
                                                          const uint32_t *tile1, uint64_t *cur2,
                                                          const uint64_t *rec_in, uint64_t *rec_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F2 = 1u << s2;
    uint64_t *gbase = (uint64_t *)smem;            // [F2]
    uint64_t *stage = gbase + F2;                  // [L2_TILE_RECS]
    uint32_t *hist = (uint32_t *)(stage + L2_TILE_RECS);  // [F2]
    uint32_t *lstart = hist + F2;                  // [F2]
    uint16_t *sr = (uint16_t *)(lstart + F2);      // [L2_TILE_RECS]
    const uint64_t rmask = (1ull << s0) - 1;
    uint32_t b;
    uint64_t r0, r1;
    if (!l2_tile(F1, off1, tile1, &b, &r0, &r1)) return;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) hist[r] = 0;
    __syncthreads();
    uint64_t v[L2_RPT];
    uint32_t rank[L2_RPT];
#pragma unroll
    for (int q = 0; q < L2_RPT; q++) {
        const uint64_t idx = r0 + (uint64_t)q * L2_THREADS + threadIdx.x;
        v[q] = idx < r1 ? rec_in[idx] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < L2_RPT; q++)
        if (v[q] != ~0ull) rank[q] = atomicAdd(&hist[(uint32_t)v[q] >> s0], 1u);
    __syncthreads();
    wave_exclusive_scan(hist, lstart, F2);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x)
        if (hist[r]) gbase[r] = atomicAdd((unsigned long long *)&cur2[(uint64_t)b * F2 + r],
                                          (unsigned long long)hist[r]);
#pragma unroll
    for (int q = 0; q < L2_RPT; q++) {
        if (v[q] != ~0ull) {
            const uint32_t r = (uint32_t)v[q] >> s0;
            const uint32_t pos = lstart[r] + rank[q];
            stage[pos] = (v[q] & ~0xFFFFFFFFull) | (v[q] & rmask);
            sr[pos] = (uint16_t)r;
        }
    }
    __syncthreads();
    const uint32_t nrec = (uint32_t)(r1 - r0);
    for (uint32_t q = threadIdx.x; q < nrec; q += blockDim.x) {
        const uint32_t r = sr[q];
        rec_out[gbase[r] + (q - lstart[r])] = stage[q];
    }
}

}  // namespace kh
