// kh_engine.hip -- the MI355X hot path of libkhmer_hip.so.
//
// Replaces the reference's per-k-mer loop Hashtable::consume_string ->
// Storage::add (src/oxli/hashtable.cc:280-294, include/oxli/storage.hh:172-199,
// 320-359, 571-624) with a batch pipeline whose results are exactly the
// reference's single-threaded ones:
//
//   1 count_l1    hash every k-mer (2-bit canonical or Murmur), N bins per
//                 k-mer (exact h % p_i by Barrett), histogram of level-1 buckets
//   2 scan_l1     bucket offsets
//   3 scatter_l1  recompute, LDS counting sort per tile, coalesced write of
//                 (bin offset, k-mer index) records into level-1 buckets
//   4 count_l2 / scan_l2 / scatter_l2   split every bucket into regions of
//                 2^s0 bins (one workgroup's LDS)
//   5 apply       one workgroup per region: table slice -> LDS, per-bin counts
//                 and stream-order winners (min k-mer index into a bin that was
//                 zero) with LDS atomics, saturating write-back, per-k-mer
//                 "new" flags, table-0 occupancy, bigcount "full" flags
//   6 crossing    (bigcount only, rare) exact stream-order ranks inside bins
//                 that reach 255 during the batch (radix select of k-mer index)
//   7 finalize    n_unique += #new k-mers; k-mers full in every table -> bigcount
//
// Because a bin's final value depends only on the multiset of its inserts
// (SURVEY.md F4), and the order-dependent counters are derived from exact
// stream ranks, tables AND counters match the single-stream reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kh_internal.h"

namespace kh {

// ---------------------------------------------------------------------------
// tunables
constexpr int L1_THREADS = 512;
constexpr int L1_TILE_RECS = 4096;  // records staged per L1 tile
constexpr int L2_THREADS = 512;
constexpr int L2_TILE_RECS = 4096;  // records per L2 tile
constexpr int APPLY_THREADS = 1024;
constexpr int FIN_THREADS = 256;
constexpr int FIN_TILE = 2048;
constexpr uint32_t NO_J = 0xFFFFFFFFu;

// ---------------------------------------------------------------------------
// k-mer sources
// A batch is a sub-range of a read set: `koff` points at the sub-range's
// k-mer offsets (absolute values), kbase = koff[0], rbase = index of its first
// read in the packed stream (base of read r = koff[r] + r*(k-1)).  Batch-local
// k-mer j is absolute k-mer kbase + j.
struct SrcTwoBit {
    const uint64_t *words;
    const uint64_t *koff;
    uint64_t nreads;
    int k;
    uint64_t kbase, rbase;
    static constexpr bool kReads = true;
    __device__ __forceinline__ uint64_t hash(uint64_t j, uint64_t r) const {
        uint64_t pos = (j + kbase) + (r + rbase) * (uint64_t)(k - 1);
        return canonical2(window2(words, pos, k), k);
    }
};
struct SrcBytes {
    const uint8_t *bytes;
    const uint64_t *koff;
    uint64_t nreads;
    int k;
    uint64_t kbase, rbase;
    static constexpr bool kReads = true;
    __device__ __forceinline__ uint64_t hash(uint64_t j, uint64_t r) const {
        uint64_t pos = (j + kbase) + (r + rbase) * (uint64_t)(k - 1);
        return murmur_canonical(bytes + pos, k);
    }
};
struct SrcHashes {
    const uint64_t *h;
    const uint64_t *koff;
    uint64_t nreads;
    int k;
    uint64_t kbase, rbase;
    static constexpr bool kReads = false;
    __device__ __forceinline__ uint64_t hash(uint64_t j, uint64_t) const { return h[j]; }
};

// LDS window of read offsets covering k-mer tile [j0, j1)
struct TileReads {
    uint64_t rlo;
    uint32_t n;
};

template <class Src>
__device__ __forceinline__ TileReads load_tile_reads(const Src &src, uint64_t j0, uint64_t j1,
                                                     uint64_t *s_koff, uint64_t *s_meta) {
    TileReads tr{0, 0};
    if constexpr (Src::kReads) {
        if (threadIdx.x == 0) {
            const uint64_t ja = j0 + src.kbase;
            uint64_t lo = 0, hi = src.nreads;  // koff[lo] <= ja < koff[hi]
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) >> 1;
                if (src.koff[mid] <= ja) lo = mid; else hi = mid;
            }
            uint64_t cnt = src.nreads - lo;
            if (cnt > j1 - j0) cnt = j1 - j0;
            s_meta[0] = lo;
            s_meta[1] = cnt;
        }
        __syncthreads();
        tr.rlo = s_meta[0];
        tr.n = (uint32_t)s_meta[1];
        for (uint32_t t = threadIdx.x; t <= tr.n; t += blockDim.x) s_koff[t] = src.koff[tr.rlo + t];
        __syncthreads();
    }
    return tr;
}

__device__ __forceinline__ uint64_t find_read(const uint64_t *s_koff, const TileReads &tr, uint64_t j) {
    uint32_t lo = 0, hi = tr.n;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (s_koff[mid] <= j) lo = mid; else hi = mid;
    }
    return tr.rlo + lo;
}

template <class Src>
__device__ __forceinline__ uint64_t kmer_hash(const Src &src, const uint64_t *s_koff, const TileReads &tr,
                                              uint64_t j) {
    uint64_t r = 0;
    if constexpr (Src::kReads) r = find_read(s_koff, tr, j + src.kbase);
    return src.hash(j, r);
}

__device__ __forceinline__ uint64_t global_bin(const Params &P, int i, uint64_t h) {
    return P.tbase[i] + mod_barrett(h, P.p[i], P.m[i]);
}

// ---------------------------------------------------------------------------
// level 1: histogram of buckets
template <class Src>
__global__ void __launch_bounds__(L1_THREADS) k_count_l1(Params P, Src src, uint64_t nkmers, int tile_kmers,
                                                        uint32_t *cnt1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;                       // [F1]
    uint64_t *s_meta = (uint64_t *)(hist + ((P.F1 + 3) & ~3u));
    uint64_t *s_koff = s_meta + 2;
    const int shift = P.s0 + P.s2;
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x) hist[b] = 0;
    uint64_t j0 = (uint64_t)blockIdx.x * tile_kmers;
    uint64_t j1 = min(nkmers, j0 + tile_kmers);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);  // syncs
    if constexpr (!Src::kReads) __syncthreads();
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        uint64_t h = kmer_hash(src, s_koff, tr, j);
        for (int i = 0; i < P.n; i++) atomicAdd(&hist[global_bin(P, i, h) >> shift], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x)
        if (hist[b]) atomicAdd(&cnt1[b], hist[b]);
}

// block-wide exclusive scan helper over up to 8192 u64 values held in `v`
// (in place), returns total.  blockDim.x == 1024.
__device__ uint64_t block_exclusive_scan(uint64_t *v, uint32_t n, uint64_t *s_part) {
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = threadIdx.x * per;
    uint64_t sum = 0;
    for (uint32_t t = 0; t < per && b0 + t < n; t++) sum += v[b0 + t];
    s_part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (uint32_t t = 0; t < blockDim.x; t++) {
            uint64_t x = s_part[t];
            s_part[t] = acc;
            acc += x;
        }
        s_part[blockDim.x] = acc;
    }
    __syncthreads();
    uint64_t acc = s_part[threadIdx.x];
    for (uint32_t t = 0; t < per && b0 + t < n; t++) {
        uint64_t x = v[b0 + t];
        v[b0 + t] = acc;
        acc += x;
    }
    __syncthreads();
    return s_part[blockDim.x];
}

// offsets of level-1 buckets and the tile prefix of the level-2 passes
__global__ void __launch_bounds__(1024) k_scan_l1(uint32_t F1, const uint32_t *cnt1, uint64_t *off1,
                                                  uint64_t *cur1, uint32_t *tile1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *v = (uint64_t *)smem;          // [F1]
    uint64_t *s_part = v + F1;               // [1025]
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) v[b] = cnt1[b];
    __syncthreads();
    uint64_t total = block_exclusive_scan(v, F1, s_part);
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) { off1[b] = v[b]; cur1[b] = v[b]; }
    if (threadIdx.x == 0) off1[F1] = total;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) v[b] = (cnt1[b] + L2_TILE_RECS - 1) / L2_TILE_RECS;
    __syncthreads();
    uint64_t tiles = block_exclusive_scan(v, F1, s_part);
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) tile1[b] = (uint32_t)v[b];
    if (threadIdx.x == 0) tile1[F1] = (uint32_t)tiles;
}

// level 1 scatter: recompute hashes, LDS counting sort of the tile's records
// by bucket, coalesced write-out (one global cursor bump per bucket per tile)
template <class Src>
__global__ void __launch_bounds__(L1_THREADS) k_scatter_l1(Params P, Src src, uint64_t nkmers, int tile_kmers,
                                                          uint64_t *cur1, uint32_t *rec_off, uint32_t *rec_j) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    uint64_t *gbase = (uint64_t *)smem;             // [F1]
    uint32_t *hist = (uint32_t *)(gbase + F1a);     // [F1]
    uint32_t *lstart = hist + F1a;                  // [F1]
    uint32_t *lcur = lstart + F1a;                  // [F1]
    uint32_t *s_off = lcur + F1a;                   // [L1_TILE_RECS]
    uint32_t *s_j = s_off + L1_TILE_RECS;           // [L1_TILE_RECS]
    uint16_t *s_b = (uint16_t *)(s_j + L1_TILE_RECS);  // [L1_TILE_RECS]
    uint64_t *s_meta = (uint64_t *)(s_b + L1_TILE_RECS);
    uint64_t *s_koff = s_meta + 2;
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;

    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) { hist[b] = 0; lcur[b] = 0; }
    uint64_t j0 = (uint64_t)blockIdx.x * tile_kmers;
    uint64_t j1 = min(nkmers, j0 + tile_kmers);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    if constexpr (!Src::kReads) __syncthreads();
    // pass A: histogram
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        uint64_t h = kmer_hash(src, s_koff, tr, j);
        for (int i = 0; i < P.n; i++) atomicAdd(&hist[global_bin(P, i, h) >> shift], 1u);
    }
    __syncthreads();
    // exclusive scan of hist -> lstart (single wave; F1 <= 8192)
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t per = (F1 + 63) / 64;
        const uint32_t b0 = lane * per;
        uint32_t sum = 0;
        for (uint32_t t = 0; t < per && b0 + t < F1; t++) sum += hist[b0 + t];
        uint32_t incl = sum;
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        uint32_t acc = incl - sum;
        for (uint32_t t = 0; t < per && b0 + t < F1; t++) { lstart[b0 + t] = acc; acc += hist[b0 + t]; }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x)
        if (hist[b]) gbase[b] = atomicAdd((unsigned long long *)&cur1[b], (unsigned long long)hist[b]);
    __syncthreads();
    // pass B: recompute, place records in bucket order in LDS
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        uint64_t h = kmer_hash(src, s_koff, tr, j);
        for (int i = 0; i < P.n; i++) {
            uint64_t G = global_bin(P, i, h);
            uint32_t b = (uint32_t)(G >> shift);
            uint32_t pos = lstart[b] + atomicAdd(&lcur[b], 1u);
            s_off[pos] = (uint32_t)(G & omask);
            s_j[pos] = (uint32_t)j;
            s_b[pos] = (uint16_t)b;
        }
    }
    __syncthreads();
    // pass C: coalesced write-out
    const uint32_t nrec = (uint32_t)((j1 - j0) * (uint64_t)P.n);
    for (uint32_t q = threadIdx.x; q < nrec; q += blockDim.x) {
        uint32_t b = s_b[q];
        uint64_t dst = gbase[b] + (q - lstart[b]);
        rec_off[dst] = s_off[q];
        rec_j[dst] = s_j[q];
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
    uint64_t s = off1[lo] + (uint64_t)(t - tile1[lo]) * L2_TILE_RECS;
    *r0 = s;
    *r1 = min(off1[lo + 1], s + L2_TILE_RECS);
    return true;
}

__global__ void __launch_bounds__(L2_THREADS) k_count_l2(uint32_t F1, int s0, int s2, const uint64_t *off1,
                                                        const uint32_t *tile1, const uint32_t *rec_off,
                                                        uint32_t *cnt2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    const uint32_t F2 = 1u << s2;
    uint32_t b;
    uint64_t r0, r1;
    if (!l2_tile(F1, off1, tile1, &b, &r0, &r1)) return;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) hist[r] = 0;
    __syncthreads();
    for (uint64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) atomicAdd(&hist[rec_off[q] >> s0], 1u);
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x)
        if (hist[r]) atomicAdd(&cnt2[(uint64_t)b * F2 + r], hist[r]);
}

// per bucket: region offsets (absolute positions in the record arrays)
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
                                                          const uint32_t *rec_off, const uint32_t *rec_j,
                                                          uint32_t *out_off, uint32_t *out_j) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F2 = 1u << s2;
    uint64_t *gbase = (uint64_t *)smem;           // [F2]
    uint32_t *hist = (uint32_t *)(gbase + F2);    // [F2]
    uint32_t *lstart = hist + F2;                 // [F2]
    uint32_t *lcur = lstart + F2;                 // [F2]
    uint32_t *s_off = lcur + F2;                  // [L2_TILE_RECS]
    uint32_t *s_j = s_off + L2_TILE_RECS;
    uint16_t *s_r = (uint16_t *)(s_j + L2_TILE_RECS);
    const uint32_t rmask = (1u << s0) - 1;
    uint32_t b;
    uint64_t r0, r1;
    if (!l2_tile(F1, off1, tile1, &b, &r0, &r1)) return;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) { hist[r] = 0; lcur[r] = 0; }
    __syncthreads();
    for (uint64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) atomicAdd(&hist[rec_off[q] >> s0], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t per = (F2 + 63) / 64;
        const uint32_t b0 = lane * per;
        uint32_t sum = 0;
        for (uint32_t t = 0; t < per && b0 + t < F2; t++) sum += hist[b0 + t];
        uint32_t incl = sum;
        for (int d = 1; d < 64; d <<= 1) {
            uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        uint32_t acc = incl - sum;
        for (uint32_t t = 0; t < per && b0 + t < F2; t++) { lstart[b0 + t] = acc; acc += hist[b0 + t]; }
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x)
        if (hist[r]) gbase[r] = atomicAdd((unsigned long long *)&cur2[(uint64_t)b * F2 + r],
                                          (unsigned long long)hist[r]);
    __syncthreads();
    for (uint64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) {
        uint32_t o = rec_off[q];
        uint32_t r = o >> s0;
        uint32_t pos = lstart[r] + atomicAdd(&lcur[r], 1u);
        s_off[pos] = o & rmask;
        s_j[pos] = rec_j[q];
        s_r[pos] = (uint16_t)r;
    }
    __syncthreads();
    const uint32_t nrec = (uint32_t)(r1 - r0);
    for (uint32_t q = threadIdx.x; q < nrec; q += blockDim.x) {
        uint32_t r = s_r[q];
        uint64_t dst = gbase[r] + (q - lstart[r]);
        out_off[dst] = s_off[q];
        out_j[dst] = s_j[q];
    }
}

// ---------------------------------------------------------------------------
// apply: one workgroup per region of 2^s0 bins
struct ApplyArgs {
    const uint64_t *off2;
    const uint32_t *rec_off, *rec_j;
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Byte and Nibble storage
template <int KIND>
__global__ void __launch_bounds__(APPLY_THREADS) k_apply_count(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = 1u << P.s0;
    uint32_t *cnt = (uint32_t *)smem;     // [R]
    uint32_t *minj = cnt + R;             // [R]
    uint8_t *c0 = (uint8_t *)(minj + R);  // [R]
    const uint32_t MAXC = KIND == BYTE ? 255u : 15u;
    const bool bigc = KIND == BYTE && P.use_bigcount;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    for (uint64_t rr = blockIdx.x; rr < total; rr += gridDim.x) {
        int i = 0;
        while (rr >= A.rprefix[i + 1]) i++;
        const uint64_t lreg = rr - A.rprefix[i];
        const uint64_t region = (P.tbase[i] >> P.s0) + lreg;
        const uint64_t e0 = A.off2[region], e1 = A.off2[region + 1];
        if (e0 == e1) continue;
        const uint64_t bin_lo = lreg << P.s0;
        const uint32_t nb = (uint32_t)min((uint64_t)R, P.p[i] - bin_lo);
        uint8_t *tab = A.tab + P.tbyte[i];
        // table slice -> LDS
        if (KIND == BYTE) {
            for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) c0[t] = tab[bin_lo + t];
        } else {
            for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) {
                uint64_t bin = bin_lo + t;
                uint8_t byte = tab[bin >> 1];
                c0[t] = (bin & 1) ? (byte & 0x0F) : (byte >> 4);
            }
        }
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) { cnt[t] = 0; minj[t] = NO_J; }
        __syncthreads();
        for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
            const uint32_t o = A.rec_off[q];
            const uint32_t j = A.rec_j[q];
            atomicAdd(&cnt[o], 1u);
            const uint8_t c = c0[o];
            if (c == 0) atomicMin(&minj[o], j);
            if (bigc && c == 255) full_add(A.fullf, j);
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) {
            const uint32_t n = cnt[t];
            if (!n) continue;
            const uint32_t c = c0[t];
            if (c == 0) {
                A.newf[minj[t]] = 1;
                if (i == 0) occ++;
            }
            const uint32_t v = c + n;
            if (bigc && c < 255 && v >= 255) {
                uint64_t idx = atomicAdd((unsigned long long *)&A.ctr[CTR_NCROSS], 1ull);
                if (idx < A.cap_cross) A.cross[idx] = ((P.tbase[i] + bin_lo + t) << 8) | c;
                else atomicOr((unsigned long long *)&A.ctr[CTR_ERR], 1ull);
            }
            cnt[t] = v < MAXC ? v : MAXC;   // final value
        }
        __syncthreads();
        // saturating write-back of touched bins only
        if (KIND == BYTE) {
            for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
                if (cnt[t]) tab[bin_lo + t] = (uint8_t)cnt[t];
        } else {
            // nibble pairs: even bin -> high nibble (storage.hh:262-272)
            const uint32_t npairs = (nb + 1) / 2;
            for (uint32_t t = threadIdx.x; t < npairs; t += blockDim.x) {
                const uint32_t a = 2 * t, bq = 2 * t + 1;
                const bool ta = cnt[a] != 0, tb = bq < nb && cnt[bq] != 0;
                if (!ta && !tb) continue;
                const uint32_t hi = ta ? cnt[a] : c0[a];
                const uint32_t lo = bq < nb ? (tb ? cnt[bq] : c0[bq]) : 0;
                tab[(bin_lo >> 1) + t] = (uint8_t)((hi << 4) | lo);
            }
        }
        __syncthreads();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// Bit storage (Bloom): BitStorage::test_and_set_bits (storage.hh:172-199)
__global__ void __launch_bounds__(APPLY_THREADS) k_apply_bit(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = 1u << P.s0;
    uint32_t *minj = (uint32_t *)smem;          // [R]
    uint8_t *bits = (uint8_t *)(minj + R);      // [R/8]
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    for (uint64_t rr = blockIdx.x; rr < total; rr += gridDim.x) {
        int i = 0;
        while (rr >= A.rprefix[i + 1]) i++;
        const uint64_t lreg = rr - A.rprefix[i];
        const uint64_t region = (P.tbase[i] >> P.s0) + lreg;
        const uint64_t e0 = A.off2[region], e1 = A.off2[region + 1];
        if (e0 == e1) continue;
        const uint64_t bin_lo = lreg << P.s0;
        const uint32_t nb = (uint32_t)min((uint64_t)R, P.p[i] - bin_lo);
        const uint32_t nbytes = (nb + 7) / 8;
        uint8_t *tab = A.tab + P.tbyte[i] + (bin_lo >> 3);
        for (uint32_t t = threadIdx.x; t < nbytes; t += blockDim.x) bits[t] = tab[t];
        for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x) minj[t] = NO_J;
        __syncthreads();
        for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
            const uint32_t o = A.rec_off[q];
            if (!((bits[o >> 3] >> (o & 7)) & 1)) atomicMin(&minj[o], A.rec_j[q]);
        }
        __syncthreads();
        // one thread per output byte
        for (uint32_t t = threadIdx.x; t < nbytes; t += blockDim.x) {
            uint8_t byte = bits[t];
            uint8_t nbyte = byte;
            for (int b = 0; b < 8; b++) {
                const uint32_t o = t * 8 + b;
                if (o >= nb) break;
                const uint32_t mj = minj[o];
                if (mj != NO_J) {
                    nbyte |= (uint8_t)(1u << b);
                    A.newf[mj] = 1;
                    if (i == 0) occ++;
                }
            }
            if (nbyte != byte) tab[t] = nbyte;
        }
        __syncthreads();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// ---------------------------------------------------------------------------
// crossing bins (bigcount): inserts with stream rank >= 255 - c0 are "full"
// (ByteStorage::add, storage.hh:590-603).  K-th smallest k-mer index by a
// 4-pass 8-bit radix select over the bin's records.
__global__ void __launch_bounds__(256) k_crossing(Params P, const uint64_t *off2, const uint32_t *rec_off,
                                                  const uint32_t *rec_j, const uint64_t *cross,
                                                  const uint64_t *ctr, uint64_t cap_cross, uint8_t *fullf) {
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_sel[2];
    uint64_t ncross = ctr[CTR_NCROSS];
    if (ncross > cap_cross) ncross = cap_cross;
    const uint32_t rmask = (1u << P.s0) - 1;
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
                if (rec_off[q] != o) continue;
                const uint32_t j = rec_j[q];
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
        // prefix = the k-mer index of the first full insert
        for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
            if (rec_off[q] != o) continue;
            const uint32_t j = rec_j[q];
            if (j >= prefix) full_add(fullf, j);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// finalize: n_unique, bigcount candidates, optional per-k-mer outputs
template <class Src>
__global__ void __launch_bounds__(FIN_THREADS) k_finalize(Params P, Src src, uint64_t nkmers, const uint8_t *newf,
                                                         const uint8_t *fullf, uint64_t *ctr, uint64_t *bc,
                                                         uint64_t cap_bc, uint8_t *out_new, uint64_t *out_hash) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * FIN_TILE;
    const uint64_t j1 = min(nkmers, j0 + FIN_TILE);
    const bool need_hash = out_hash != nullptr || (P.kind == BYTE && P.use_bigcount);
    TileReads tr{0, 0};
    if (need_hash) tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    uint64_t uniq = 0;
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        const uint8_t nw = newf[j];
        uniq += nw;
        if (out_new) out_new[j] = nw;
        const bool full = P.kind == BYTE && P.use_bigcount && fullf[j] == (uint8_t)P.n;
        if (out_hash || full) {
            const uint64_t h = kmer_hash(src, s_koff, tr, j);
            if (out_hash) out_hash[j] = h;
            if (full) {
                uint64_t idx = atomicAdd((unsigned long long *)&ctr[CTR_NBC], 1ull);
                if (idx < cap_bc) bc[idx] = h;
                else atomicOr((unsigned long long *)&ctr[CTR_ERR], 2ull);
            }
        }
    }
    uniq = wave_sum(uniq);
    if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
}

// ---------------------------------------------------------------------------
// queries: Storage::get_count (storage.hh:206-219, 362-379, 627-649)
__device__ __forceinline__ uint32_t get_count_dev(const Params &P, const uint8_t *tab, uint64_t h,
                                                  const uint64_t *bc_keys, const uint16_t *bc_vals,
                                                  uint64_t bc_n) {
    if (P.kind == BIT) {
        for (int i = 0; i < P.n; i++) {
            const uint64_t bin = mod_barrett(h, P.p[i], P.m[i]);
            if (!((tab[P.tbyte[i] + (bin >> 3)] >> (bin & 7)) & 1)) return 0;
        }
        return 1;
    }
    if (P.kind == NIBBLE) {
        uint32_t mn = 15;
        for (int i = 0; i < P.n; i++) {
            const uint64_t bin = mod_barrett(h, P.p[i], P.m[i]);
            const uint8_t byte = tab[P.tbyte[i] + (bin >> 1)];
            const uint32_t c = (bin & 1) ? (byte & 0x0F) : (byte >> 4);
            mn = c < mn ? c : mn;
        }
        return mn;
    }
    uint32_t mn = 255;
    for (int i = 0; i < P.n; i++) {
        const uint32_t c = tab[P.tbyte[i] + mod_barrett(h, P.p[i], P.m[i])];
        mn = c < mn ? c : mn;
    }
    if (mn == 255 && P.use_bigcount && bc_n) {
        uint64_t lo = 0, hi = bc_n;
        while (lo < hi) {
            uint64_t mid = (lo + hi) >> 1;
            if (bc_keys[mid] < h) lo = mid + 1; else hi = mid;
        }
        if (lo < bc_n && bc_keys[lo] == h) mn = bc_vals[lo];
    }
    return mn;
}

__global__ void k_get_counts(Params P, const uint8_t *tab, const uint64_t *hashes, uint64_t n, uint16_t *out,
                             const uint64_t *bc_keys, const uint16_t *bc_vals, uint64_t bc_n) {
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x)
        out[q] = (uint16_t)get_count_dev(P, tab, hashes[q], bc_keys, bc_vals, bc_n);
}

// hashes of every k-mer of a batch
template <class Src>
__global__ void __launch_bounds__(FIN_THREADS) k_kmer_hashes(Src src, uint64_t nkmers, uint64_t *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * FIN_TILE;
    const uint64_t j1 = min(nkmers, j0 + FIN_TILE);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) out[j] = kmer_hash(src, s_koff, tr, j);
}

// counts of every k-mer of a batch (for get_median_count)
template <class Src>
__global__ void __launch_bounds__(FIN_THREADS) k_kmer_counts(Params P, Src src, uint64_t nkmers, const uint8_t *tab,
                                                            uint16_t *out, const uint64_t *bc_keys,
                                                            const uint16_t *bc_vals, uint64_t bc_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * FIN_TILE;
    const uint64_t j1 = min(nkmers, j0 + FIN_TILE);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x)
        out[j] = (uint16_t)get_count_dev(P, tab, kmer_hash(src, s_koff, tr, j), bc_keys, bc_vals, bc_n);
}

// Correctly rounded float32 division and square root.  The device's native
// f32 sqrt is not correctly rounded (1 ulp), so both start from a double
// estimate and are fixed up against the exact float midpoints: a midpoint has
// 25 significant bits, so midpoint*b (b a float) and midpoint^2 are exact in
// double, and ties cannot occur for these operations.
__device__ __forceinline__ float div_rn_exact(float a, float b) {   // b > 0
    float q = (float)((double)a / (double)b);
    const float dn = nextafterf(q, -INFINITY), up = nextafterf(q, INFINITY);
    const double lo = ((double)q + (double)dn) * 0.5, hi = ((double)q + (double)up) * 0.5;
    const double ad = (double)a, bd = (double)b;
    if (ad < lo * bd) q = dn;
    else if (ad > hi * bd) q = up;
    return q;
}
__device__ __forceinline__ float sqrt_rn_exact(float x) {           // x >= 0
    if (x == 0.f) return x;
    float r = (float)sqrt((double)x);
    const float dn = nextafterf(r, 0.f), up = nextafterf(r, INFINITY);
    const double lo = ((double)r + (double)dn) * 0.5, hi = ((double)r + (double)up) * 0.5;
    const double xd = (double)x;
    if (xd < lo * lo) r = dn;
    else if (xd > hi * hi) r = up;
    return r;
}

// Hashtable::get_median_count (src/oxli/hashtable.cc:299-328): one thread per
// read; float32 in the reference's sequential order with round-to-nearest
// intrinsics (no contraction), IEEE sqrt, median = sorted[n/2].
__global__ void k_median(const uint64_t *koff, uint64_t nreads, uint16_t *counts, uint16_t *med, float *avg,
                         float *sd) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = koff[r], n = koff[r + 1] - a;
        uint16_t *c = counts + a;
        float average = 0.f;
        for (uint64_t t = 0; t < n; t++) average = __fadd_rn(average, (float)c[t]);
        average = div_rn_exact(average, (float)n);
        float s = 0.f;
        for (uint64_t t = 0; t < n; t++) {
            const float d = __fsub_rn((float)c[t], average);
            s = __fadd_rn(s, __fmul_rn(d, d));
        }
        s = div_rn_exact(s, (float)n);
        s = sqrt_rn_exact(s);
        // in-place heapsort of the read's counts, then the middle element
        uint64_t m = n;
        auto sift = [&](uint64_t root, uint64_t end) {
            while (2 * root + 1 < end) {
                uint64_t child = 2 * root + 1;
                if (child + 1 < end && c[child] < c[child + 1]) child++;
                if (c[root] < c[child]) {
                    uint16_t tmp = c[root]; c[root] = c[child]; c[child] = tmp;
                    root = child;
                } else {
                    break;
                }
            }
        };
        for (uint64_t st = m / 2; st-- > 0;) sift(st, m);
        for (uint64_t end = m; end-- > 1;) {
            uint16_t tmp = c[0]; c[0] = c[end]; c[end] = tmp;
            sift(0, end);
        }
        med[r] = c[n / 2];
        avg[r] = average;
        sd[r] = s;
    }
}

// ---------------------------------------------------------------------------
// host side
static size_t lds_count_l1(const Params &P, int tile_kmers) {
    return ((P.F1 + 3) & ~3u) * 4 + 16 + (size_t)(tile_kmers + 2) * 8;
}
static size_t lds_scatter_l1(const Params &P, int tile_kmers) {
    const size_t F1a = (P.F1 + 3) & ~3u;
    return F1a * 8 + F1a * 4 * 3 + (size_t)L1_TILE_RECS * (4 + 4 + 2) + 16 + (size_t)(tile_kmers + 2) * 8;
}
static size_t lds_apply(const Params &P) {
    const size_t R = (size_t)1 << P.s0;
    return P.kind == BIT ? R * 4 + R / 8 : R * 4 * 2 + R;
}

static void ensure(void **p, uint64_t *cap, uint64_t need, size_t elem) {
    if (need <= *cap) return;
    if (*p) KH_HIP(hipFree(*p));
    *p = nullptr;
    uint64_t n = std::max<uint64_t>(need, *cap + *cap / 2);
    KH_HIP(hipMalloc(p, n * elem + 64));
    *cap = n;
}

static void ws_prepare(Graph *g, uint64_t nkmers) {
    Workspace &w = g->ws;
    const uint64_t recs = nkmers * (uint64_t)g->n;
    if (nkmers > w.cap_kmers) {
        uint64_t cap = std::max<uint64_t>(nkmers, w.cap_kmers + w.cap_kmers / 2);
        cap = (cap + 3) & ~3ull;
        if (w.newf) KH_HIP(hipFree(w.newf));
        if (w.fullf) KH_HIP(hipFree(w.fullf));
        KH_HIP(hipMalloc(&w.newf, cap + 64));
        KH_HIP(hipMalloc(&w.fullf, cap + 64));
        w.cap_kmers = cap;
    }
    if (recs > w.cap_recs) {
        uint64_t cap = std::max<uint64_t>(recs, w.cap_recs + w.cap_recs / 2);
        for (uint32_t **pp : {&w.rec1_off, &w.rec1_j, &w.rec2_off, &w.rec2_j}) {
            if (*pp) KH_HIP(hipFree(*pp));
            KH_HIP(hipMalloc((void **)pp, cap * 4 + 64));
        }
        w.cap_recs = cap;
    }
    const uint64_t regions = (uint64_t)g->prm.F1 << g->prm.s2;
    if (regions > w.cap_regions || !w.cnt1) {
        for (void **pp : {(void **)&w.cnt1, (void **)&w.off1, (void **)&w.cur1, (void **)&w.tile1, (void **)&w.cnt2,
                          (void **)&w.off2, (void **)&w.cur2})
            if (*pp) { KH_HIP(hipFree(*pp)); *pp = nullptr; }
        const uint64_t F1 = g->prm.F1;
        KH_HIP(hipMalloc((void **)&w.cnt1, F1 * 4 + 64));
        KH_HIP(hipMalloc((void **)&w.off1, (F1 + 1) * 8 + 64));
        KH_HIP(hipMalloc((void **)&w.cur1, F1 * 8 + 64));
        KH_HIP(hipMalloc((void **)&w.tile1, (F1 + 1) * 4 + 64));
        KH_HIP(hipMalloc((void **)&w.cnt2, regions * 4 + 64));
        KH_HIP(hipMalloc((void **)&w.off2, (regions + 1) * 8 + 64));
        KH_HIP(hipMalloc((void **)&w.cur2, regions * 8 + 64));
        w.cap_regions = regions;
    }
    if (!w.ctr) {
        KH_HIP(hipMalloc((void **)&w.ctr, CTR_N * 8));
        KH_HIP(hipHostMalloc((void **)&w.h_ctr, CTR_N * 8, hipHostMallocDefault));
    }
    if (!w.cross) {
        w.cap_cross = 1 << 20;
        KH_HIP(hipMalloc((void **)&w.cross, w.cap_cross * 8));
    }
    if (!w.bc) {
        w.cap_bc = 1 << 22;
        KH_HIP(hipMalloc((void **)&w.bc, w.cap_bc * 8));
    }
}

void engine_sync_bigcounts(Graph *g) {
    if (!g->bc_dirty) return;
    std::vector<std::pair<uint64_t, uint16_t>> v(g->bigcounts.begin(), g->bigcounts.end());
    std::sort(v.begin(), v.end());
    const uint64_t n = v.size();
    if (n > g->d_bc_cap) {
        if (g->d_bc_keys) KH_HIP(hipFree(g->d_bc_keys));
        if (g->d_bc_vals) KH_HIP(hipFree(g->d_bc_vals));
        g->d_bc_cap = std::max<uint64_t>(n, 1024);
        KH_HIP(hipMalloc((void **)&g->d_bc_keys, g->d_bc_cap * 8));
        KH_HIP(hipMalloc((void **)&g->d_bc_vals, g->d_bc_cap * 2));
    }
    if (n) {
        std::vector<uint64_t> keys(n);
        std::vector<uint16_t> vals(n);
        for (uint64_t i = 0; i < n; i++) { keys[i] = v[i].first; vals[i] = v[i].second; }
        KH_HIP(hipMemcpyAsync(g->d_bc_keys, keys.data(), n * 8, hipMemcpyHostToDevice, g->stream));
        KH_HIP(hipMemcpyAsync(g->d_bc_vals, vals.data(), n * 2, hipMemcpyHostToDevice, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
    }
    g->d_bc_n = n;
    g->bc_dirty = false;
}

// ---- per-kernel HIP-event timing (bench / roofline) ----
static hipEvent_t ev_get(Graph *g) {
    if (g->ev_next == g->ev_pool.size()) {
        hipEvent_t e;
        KH_HIP(hipEventCreate(&e));
        g->ev_pool.push_back(e);
    }
    return g->ev_pool[g->ev_next++];
}
struct KTimer {
    Graph *g;
    const char *name;
    hipEvent_t a = nullptr;
    KTimer(Graph *g_, const char *n) : g(g_), name(n) {
        if (g->profile) { a = ev_get(g); KH_HIP(hipEventRecord(a, g->stream)); }
    }
    ~KTimer() noexcept(false) {
        if (a) {
            hipEvent_t b = ev_get(g);
            KH_HIP(hipEventRecord(b, g->stream));
            g->ev_pending.push_back({name, {a, b}});
        }
    }
};
void engine_collect_events(Graph *g) {
    if (g->ev_pending.empty()) { g->ev_next = 0; return; }
    KH_HIP(hipStreamSynchronize(g->stream));
    for (auto &p : g->ev_pending) {
        float ms = 0;
        KH_HIP(hipEventElapsedTime(&ms, p.second.first, p.second.second));
        auto it = std::find_if(g->kstats.begin(), g->kstats.end(), [&](auto &x) { return x.first == p.first; });
        if (it == g->kstats.end()) { g->kstats.push_back({p.first, Graph::KStat{}}); it = g->kstats.end() - 1; }
        it->second.ms += ms;
        it->second.n += 1;
    }
    g->ev_pending.clear();
    g->ev_next = 0;
}
#define TIMED(name, ...) do { KTimer kt_(g, name); __VA_ARGS__; } while (0)

template <class Src>
static void run_pass(Graph *g, const Src &src, uint64_t nkmers, const PassOut *out) {
    if (nkmers == 0) return;
    if (nkmers > 0xFFFFFFF0ull) fail(KH_EVALUE, "batch too large");
    ws_prepare(g, nkmers);
    Workspace &w = g->ws;
    const Params &P = g->prm;
    hipStream_t st = g->stream;
    const uint64_t F1 = P.F1, F2 = 1ull << P.s2;
    const uint64_t recs = nkmers * (uint64_t)P.n;

    KH_HIP(hipMemsetAsync(w.cnt1, 0, F1 * 4, st));
    KH_HIP(hipMemsetAsync(w.cnt2, 0, F1 * F2 * 4, st));
    KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
    KH_HIP(hipMemsetAsync(w.newf, 0, nkmers, st));
    if (P.kind == BYTE && P.use_bigcount) KH_HIP(hipMemsetAsync(w.fullf, 0, (nkmers + 3) & ~3ull, st));

    int tile_kmers = L1_TILE_RECS / P.n;
    if (tile_kmers < 1) tile_kmers = 1;
    const uint64_t ntiles1 = (nkmers + tile_kmers - 1) / tile_kmers;
    TIMED("count_l1", hipLaunchKernelGGL(k_count_l1<Src>, dim3((unsigned)ntiles1), dim3(L1_THREADS),
                                         lds_count_l1(P, tile_kmers), st, P, src, nkmers, tile_kmers, w.cnt1));
    TIMED("scan_l1", hipLaunchKernelGGL(k_scan_l1, dim3(1), dim3(1024), F1 * 8 + 1025 * 8, st, (uint32_t)F1,
                                        w.cnt1, w.off1, w.cur1, w.tile1));
    TIMED("scatter_l1", hipLaunchKernelGGL(k_scatter_l1<Src>, dim3((unsigned)ntiles1), dim3(L1_THREADS),
                                           lds_scatter_l1(P, tile_kmers), st, P, src, nkmers, tile_kmers, w.cur1,
                                           w.rec1_off, w.rec1_j));
    const uint64_t ntiles2 = (recs + L2_TILE_RECS - 1) / L2_TILE_RECS + F1;
    TIMED("count_l2", hipLaunchKernelGGL(k_count_l2, dim3((unsigned)ntiles2), dim3(L2_THREADS), F2 * 4, st,
                                         (uint32_t)F1, P.s0, P.s2, w.off1, w.tile1, w.rec1_off, w.cnt2));
    TIMED("scan_l2", hipLaunchKernelGGL(k_scan_l2, dim3((unsigned)F1), dim3(1024), F2 * 8 + 1025 * 8, st, P.s2,
                                        (uint32_t)F1, w.off1, w.cnt2, w.off2, w.cur2));
    TIMED("scatter_l2", hipLaunchKernelGGL(k_scatter_l2, dim3((unsigned)ntiles2), dim3(L2_THREADS),
                                           F2 * 8 + F2 * 4 * 3 + L2_TILE_RECS * 10, st, (uint32_t)F1, P.s0, P.s2,
                                           w.off1, w.tile1, w.cur2, w.rec1_off, w.rec1_j, w.rec2_off, w.rec2_j));

    ApplyArgs A;
    A.off2 = w.off2;
    A.rec_off = w.rec2_off;
    A.rec_j = w.rec2_j;
    A.tab = g->d_tab;
    A.newf = w.newf;
    A.fullf = w.fullf;
    A.cross = w.cross;
    A.cap_cross = w.cap_cross;
    A.ctr = w.ctr;
    A.rprefix[0] = 0;
    for (int i = 0; i < P.n; i++)
        A.rprefix[i + 1] = A.rprefix[i] + ((P.p[i] + (1ull << P.s0) - 1) >> P.s0);
    const uint64_t real_regions = A.rprefix[P.n];
    const unsigned agrid = (unsigned)std::min<uint64_t>(real_regions, 256 * 8);
    if (P.kind == BIT)
        TIMED("apply_bit", hipLaunchKernelGGL(k_apply_bit, dim3(agrid), dim3(APPLY_THREADS), lds_apply(P), st, P, A));
    else if (P.kind == NIBBLE)
        TIMED("apply_nibble", hipLaunchKernelGGL(k_apply_count<NIBBLE>, dim3(agrid), dim3(APPLY_THREADS),
                                                 lds_apply(P), st, P, A));
    else
        TIMED("apply_byte", hipLaunchKernelGGL(k_apply_count<BYTE>, dim3(agrid), dim3(APPLY_THREADS), lds_apply(P),
                                               st, P, A));
    if (P.kind == BYTE && P.use_bigcount)
        TIMED("crossing", hipLaunchKernelGGL(k_crossing, dim3(1024), dim3(256), 0, st, P, w.off2, w.rec2_off,
                                             w.rec2_j, w.cross, w.ctr, w.cap_cross, w.fullf));

    uint8_t *d_out_new = nullptr;
    uint64_t *d_out_hash = nullptr;
    if (out && out->h_new) d_out_new = w.newf;   // copied after finalize (read-only there)
    if (out && out->h_hash) {
        uint64_t cap = w.cap_recs;  // reuse rec1 arrays as hash output (8 B per k-mer)
        if (cap * 4 >= nkmers * 8) d_out_hash = (uint64_t *)w.rec1_off;
        else KH_HIP(hipMalloc((void **)&d_out_hash, nkmers * 8));
    }
    const uint64_t fin_tiles = (nkmers + FIN_TILE - 1) / FIN_TILE;
    TIMED("finalize", hipLaunchKernelGGL(k_finalize<Src>, dim3((unsigned)fin_tiles), dim3(FIN_THREADS),
                                         16 + (FIN_TILE + 2) * 8, st, P, src, nkmers, w.newf, w.fullf, w.ctr, w.bc,
                                         w.cap_bc, (uint8_t *)nullptr, d_out_hash));
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(w.h_ctr, w.ctr, CTR_N * 8, hipMemcpyDeviceToHost, st));
    if (d_out_new) KH_HIP(hipMemcpyAsync(out->h_new, d_out_new, nkmers, hipMemcpyDeviceToHost, st));
    if (d_out_hash) KH_HIP(hipMemcpyAsync(out->h_hash, d_out_hash, nkmers * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    engine_collect_events(g);
    if (d_out_hash && d_out_hash != (uint64_t *)w.rec1_off) KH_HIP(hipFree(d_out_hash));
    if (w.h_ctr[CTR_ERR]) fail(KH_EDEVICE, "device overflow of crossing/bigcount buffers");
    g->n_occupied += w.h_ctr[CTR_OCC];
    g->n_unique += w.h_ctr[CTR_UNIQUE];
    const uint64_t nbc = w.h_ctr[CTR_NBC];
    if (nbc) {
        std::vector<uint64_t> hs(nbc);
        KH_HIP(hipMemcpy(hs.data(), w.bc, nbc * 8, hipMemcpyDeviceToHost));
        // ByteStorage::add bigcount update (storage.hh:606-616), merged per hash:
        // absent -> 255 + f, present -> v + f, capped at 65535
        std::sort(hs.begin(), hs.end());
        for (uint64_t a = 0; a < nbc;) {
            uint64_t b = a;
            while (b < nbc && hs[b] == hs[a]) b++;
            auto it = g->bigcounts.find(hs[a]);
            uint64_t base = it == g->bigcounts.end() ? 255 : it->second;
            uint64_t v = base + (b - a);
            g->bigcounts[hs[a]] = (uint16_t)std::min<uint64_t>(v, 65535);
            a = b;
        }
        g->bc_dirty = true;
    }
}

// batch boundaries of a device read set: chunk i starts at the last read whose
// k-mer offset is <= koff[0] + i*B
__global__ void k_chunk_bounds(const uint64_t *koff, uint64_t nreads, uint64_t B, uint64_t nchunks,
                               uint64_t *out_r, uint64_t *out_k) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i <= nchunks;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t r;
        if (i == nchunks) {
            r = nreads;
        } else {
            const uint64_t target = koff[0] + i * B;
            uint64_t lo = 0, hi = nreads;  // koff[lo] <= target
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) >> 1;
                if (koff[mid] <= target) lo = mid; else hi = mid;
            }
            r = lo;
        }
        out_r[i] = r;
        out_k[i] = koff[r];
    }
}

template <class Src>
static void consume_reads_chunked(Graph *g, Src base, const uint64_t *d_koff, uint64_t nreads, uint64_t nkmers,
                                  const PassOut *out) {
    if (nkmers == 0 || nreads == 0) return;
    const uint64_t B = g->batch_kmers;
    if (out || nkmers <= B + (B >> 4)) {   // one pass (koff[0] == 0 by contract)
        Src s = base;
        s.koff = d_koff;
        s.nreads = nreads;
        run_pass(g, s, nkmers, out);
        return;
    }
    const uint64_t nchunks = (nkmers + B - 1) / B;
    std::vector<uint64_t> rr(nchunks + 1), kk(nchunks + 1);
    uint64_t *d = nullptr;
    KH_HIP(hipMalloc((void **)&d, (nchunks + 1) * 16));
    hipLaunchKernelGGL(k_chunk_bounds, dim3((unsigned)std::min<uint64_t>((nchunks + 256) / 256, 4096)), dim3(256), 0,
                       g->stream, d_koff, nreads, B, nchunks, d, d + nchunks + 1);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(rr.data(), d, (nchunks + 1) * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(kk.data(), d + nchunks + 1, (nchunks + 1) * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    KH_HIP(hipFree(d));
    uint64_t done = 0;
    for (uint64_t i = 0; i < nchunks; i++) {
        uint64_t r0 = rr[i], r1 = rr[i + 1];
        if (r1 <= r0) continue;  // a read longer than a batch: merged into the next chunk
        Src s = base;
        s.koff = d_koff + r0;
        s.nreads = r1 - r0;
        s.kbase = kk[i];
        s.rbase = r0;
        run_pass(g, s, kk[i + 1] - kk[i], out);
        done += kk[i + 1] - kk[i];
    }
    if (done != nkmers) fail(KH_EVALUE, "k-mer offsets do not match the k-mer count");
}

void engine_consume_twobit(Graph *g, const uint64_t *d_words, const uint64_t *d_koff, uint64_t nreads,
                           uint64_t nkmers, const PassOut *out) {
    SrcTwoBit s{d_words, d_koff, nreads, g->k, 0, 0};
    consume_reads_chunked(g, s, d_koff, nreads, nkmers, out);
}

void engine_consume_bytes(Graph *g, const uint8_t *d_bytes, const uint64_t *d_koff, uint64_t nreads,
                          uint64_t nkmers, const PassOut *out) {
    SrcBytes s{d_bytes, d_koff, nreads, g->k, 0, 0};
    consume_reads_chunked(g, s, d_koff, nreads, nkmers, out);
}

void engine_consume_hashes(Graph *g, const uint64_t *d_hashes, uint64_t n, const PassOut *out) {
    const uint64_t B = g->batch_kmers;
    if (n > B && out) fail(KH_EVALUE, "per-k-mer outputs need a single device batch");
    for (uint64_t a = 0; a < n; a += B) {
        SrcHashes s{d_hashes + a, nullptr, 0, g->k, 0, 0};
        run_pass(g, s, std::min(B, n - a), out);
    }
}

static void upload_batch(Graph *g, const HostBatch &b) {
    Workspace &w = g->ws;
    const uint64_t nr = b.nreads();
    ensure((void **)&w.d_koff, &w.cap_koff, nr + 1, 8);
    KH_HIP(hipMemcpyAsync(w.d_koff, b.koff.data(), (nr + 1) * 8, hipMemcpyHostToDevice, g->stream));
    if (b.hash == MURMUR) {
        ensure((void **)&w.d_bytes, &w.cap_bytes, b.bytes.size() + 8, 1);
        KH_HIP(hipMemcpyAsync(w.d_bytes, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice, g->stream));
    } else {
        const uint64_t nw = (b.nbases + 31) / 32 + 1;
        ensure((void **)&w.d_words, &w.cap_words, nw, 8);
        KH_HIP(hipMemcpyAsync(w.d_words, b.words.data(), nw * 8, hipMemcpyHostToDevice, g->stream));
    }
}

void engine_consume_host(Graph *g, const HostBatch &b, const PassOut *out) {
    if (b.nkmers() == 0) return;
    upload_batch(g, b);
    if (b.hash == MURMUR) engine_consume_bytes(g, g->ws.d_bytes, g->ws.d_koff, b.nreads(), b.nkmers(), out);
    else engine_consume_twobit(g, g->ws.d_words, g->ws.d_koff, b.nreads(), b.nkmers(), out);
}

void engine_hash_batch(Graph *g, const HostBatch &b, uint64_t *h_out) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nk) return;
    upload_batch(g, b);
    uint64_t *d = nullptr;
    KH_HIP(hipMalloc((void **)&d, nk * 8));
    const uint64_t tiles = (nk + FIN_TILE - 1) / FIN_TILE;
    if (b.hash == MURMUR) {
        SrcBytes s{g->ws.d_bytes, g->ws.d_koff, nr, g->k, 0, 0};
        hipLaunchKernelGGL(k_kmer_hashes<SrcBytes>, dim3((unsigned)tiles), dim3(FIN_THREADS), 16 + (FIN_TILE + 2) * 8,
                           g->stream, s, nk, d);
    } else {
        SrcTwoBit s{g->ws.d_words, g->ws.d_koff, nr, g->k, 0, 0};
        hipLaunchKernelGGL(k_kmer_hashes<SrcTwoBit>, dim3((unsigned)tiles), dim3(FIN_THREADS), 16 + (FIN_TILE + 2) * 8,
                           g->stream, s, nk, d);
    }
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(h_out, d, nk * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    KH_HIP(hipFree(d));
}

void engine_get_counts(Graph *g, const uint64_t *h_hashes, uint64_t n, uint16_t *out) {
    if (!n) return;
    engine_sync_bigcounts(g);
    uint64_t *d_h = nullptr;
    uint16_t *d_o = nullptr;
    KH_HIP(hipMalloc((void **)&d_h, n * 8));
    KH_HIP(hipMalloc((void **)&d_o, n * 2));
    KH_HIP(hipMemcpyAsync(d_h, h_hashes, n * 8, hipMemcpyHostToDevice, g->stream));
    const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(k_get_counts, dim3(grid), dim3(256), 0, g->stream, g->prm, g->d_tab, d_h, n, d_o, g->d_bc_keys,
                       g->d_bc_vals, g->d_bc_n);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(out, d_o, n * 2, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    KH_HIP(hipFree(d_h));
    KH_HIP(hipFree(d_o));
}

void engine_median(Graph *g, const HostBatch &b, uint16_t *med, float *avg, float *sd) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nr) return;
    engine_sync_bigcounts(g);
    upload_batch(g, b);
    uint16_t *d_counts = nullptr, *d_med = nullptr;
    float *d_avg = nullptr, *d_sd = nullptr;
    KH_HIP(hipMalloc((void **)&d_counts, nk * 2 + 64));
    KH_HIP(hipMalloc((void **)&d_med, nr * 2 + 64));
    KH_HIP(hipMalloc((void **)&d_avg, nr * 4 + 64));
    KH_HIP(hipMalloc((void **)&d_sd, nr * 4 + 64));
    const uint64_t tiles = (nk + FIN_TILE - 1) / FIN_TILE;
    if (tiles) {
        if (b.hash == MURMUR) {
            SrcBytes s{g->ws.d_bytes, g->ws.d_koff, nr, g->k, 0, 0};
            hipLaunchKernelGGL(k_kmer_counts<SrcBytes>, dim3((unsigned)tiles), dim3(FIN_THREADS),
                               16 + (FIN_TILE + 2) * 8, g->stream, g->prm, s, nk, g->d_tab, d_counts, g->d_bc_keys,
                               g->d_bc_vals, g->d_bc_n);
        } else {
            SrcTwoBit s{g->ws.d_words, g->ws.d_koff, nr, g->k, 0, 0};
            hipLaunchKernelGGL(k_kmer_counts<SrcTwoBit>, dim3((unsigned)tiles), dim3(FIN_THREADS),
                               16 + (FIN_TILE + 2) * 8, g->stream, g->prm, s, nk, g->d_tab, d_counts, g->d_bc_keys,
                               g->d_bc_vals, g->d_bc_n);
        }
    }
    const unsigned grid = (unsigned)std::min<uint64_t>((nr + 255) / 256, 65536);
    hipLaunchKernelGGL(k_median, dim3(grid), dim3(256), 0, g->stream, g->ws.d_koff, nr, d_counts, d_med, d_avg, d_sd);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(med, d_med, nr * 2, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(avg, d_avg, nr * 4, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(sd, d_sd, nr * 4, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    for (void *p : {(void *)d_counts, (void *)d_med, (void *)d_avg, (void *)d_sd}) KH_HIP(hipFree(p));
}

void engine_download_table(Graph *g, int i, uint8_t *dst) {
    KH_HIP(hipMemcpyAsync(dst, g->d_tab + g->prm.tbyte[i], g->nbytes[(size_t)i], hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

void engine_upload_table(Graph *g, int i, const uint8_t *src) {
    KH_HIP(hipMemcpyAsync(g->d_tab + g->prm.tbyte[i], src, g->nbytes[(size_t)i], hipMemcpyHostToDevice, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}


// ---------------------------------------------------------------------------
// synthetic reads straight into HBM (khmer_amd/synth.py defines the stream):
// word t of read r = mix(seed + (r * 2^20 + t) * golden)
__device__ __forceinline__ uint64_t synth_word(uint64_t seed, uint64_t r, uint64_t t) {
    uint64_t z = seed + ((r << 20) + t) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_synth_packed(uint64_t seed, uint64_t r0, uint64_t nreads, int L, int k, uint64_t *words,
                               uint64_t nwords, uint64_t *koff) {
    const uint64_t nbases = nreads * (uint64_t)L;
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t out = 0;
        uint64_t last_key = ~0ull, src = 0;
        for (int b = 0; b < 32; b++) {
            const uint64_t p = w * 32 + b;
            uint64_t code = 0;
            if (p < nbases) {
                const uint64_t r = p / (uint64_t)L, i = p % (uint64_t)L;
                const uint64_t key = (r << 20) | (i >> 5);
                if (key != last_key) { src = synth_word(seed, r0 + r, i >> 5); last_key = key; }
                code = (src >> (62 - 2 * (i & 31))) & 3;
            }
            out = (out << 2) | code;
        }
        words[w] = out;
    }
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r <= nreads;
         r += (uint64_t)gridDim.x * blockDim.x)
        koff[r] = r * (uint64_t)(L - k + 1);
}

void engine_synth_packed(int device, uint64_t seed, uint64_t r0, uint64_t nreads, int L, int k, uint64_t *d_words,
                         uint64_t *d_koff) {
    KH_HIP(hipSetDevice(device));
    const uint64_t nwords = (nreads * (uint64_t)L + 31) / 32 + 1;
    const unsigned grid = (unsigned)std::min<uint64_t>((nwords + 255) / 256, 1u << 16);
    hipLaunchKernelGGL(k_synth_packed, dim3(grid), dim3(256), 0, 0, seed, r0, nreads, L, k, d_words, nwords, d_koff);
    KH_HIP(hipGetLastError());
    KH_HIP(hipDeviceSynchronize());
}

// ---------------------------------------------------------------------------
// graph creation: table arena + partition geometry
static int ceil_log2(uint64_t x) {
    int s = 0;
    while ((1ull << s) < x) s++;
    return s;
}

void graph_prepare_params(Graph *g) {
    Params &P = g->prm;
    memset(&P, 0, sizeof P);
    P.kind = g->kind;
    P.hash = g->hash;
    P.k = g->k;
    P.n = g->n;
    P.use_bigcount = g->use_bigcount ? 1 : 0;
    P.s0 = g->kind == BIT ? 15 : 14;
    uint64_t maxreg = 1;
    for (int i = 0; i < g->n; i++) maxreg = std::max<uint64_t>(maxreg, (g->sizes[i] + (1ull << P.s0) - 1) >> P.s0);
    P.s2 = std::min(10, ceil_log2(maxreg));
    const uint64_t span = 1ull << (P.s0 + P.s2);
    uint64_t base = 0, byteoff = 0;
    for (int i = 0; i < g->n; i++) {
        P.p[i] = g->sizes[i];
        P.m[i] = barrett_m(g->sizes[i]);
        P.tbase[i] = base;
        base += (g->sizes[i] + span - 1) / span * span;
        P.tbyte[i] = byteoff;
        P.tbytes[i] = g->nbytes[i];
        byteoff += (g->nbytes[i] + 255) / 256 * 256;
    }
    uint64_t F1 = base / span;
    if (F1 > 8192) fail(KH_EVALUE, "tables too large for one device (more than 8192 level-1 buckets)");
    P.F1 = (uint32_t)F1;
}

// allow the large dynamic LDS footprints (gfx950: 160 KiB per workgroup)
static void set_lds_limits() {
    static bool done = false;
    if (done) return;
    done = true;
    const int lim = 160 * 1024;
    (void)hipFuncSetAttribute((const void *)k_apply_count<BYTE>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<NIBBLE>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_bit, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipGetLastError();
}

Graph *graph_create(int kind, int hash, int k, const uint64_t *sizes, int n, int device) {
    if (n < 1 || n > MAXT) fail(KH_EVALUE, "number of tables must be in [1, 32]");
    if (kind != BYTE && kind != BIT && kind != NIBBLE) fail(KH_EVALUE, "unknown storage kind");
    if (hash == TWOBIT && (k < 1 || k > 32)) fail(KH_EVALUE, "k-mer size must be <= 32 for 2-bit hashing");
    if (hash == MURMUR && (k < 1 || k > 127)) fail(KH_EVALUE, "k-mer size must be in [1, 127]");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail(KH_EDEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) fail(KH_EDEVICE, "invalid HIP device");
    std::unique_ptr<Graph> g(new Graph());
    g->kind = kind;
    g->hash = hash;
    g->k = k;
    g->n = n;
    g->device = device;
    for (int i = 0; i < n; i++) {
        if (sizes[i] == 0) fail(KH_EVALUE, "table size must be > 0");
        g->sizes.push_back(sizes[i]);
        // storage.hh:127-140 (bit), 297-310 (nibble), 502-511 (byte)
        g->nbytes.push_back(kind == BIT ? sizes[i] / 8 + 1 : kind == NIBBLE ? sizes[i] / 2 + 1 : sizes[i]);
    }
    KH_HIP(hipSetDevice(device));
    set_lds_limits();
    graph_prepare_params(g.get());
    uint64_t arena = 0;
    for (int i = 0; i < n; i++) arena = g->prm.tbyte[i] + (g->nbytes[(size_t)i] + 255) / 256 * 256;
    g->arena_bytes = arena;
    hipError_t e = hipMalloc((void **)&g->d_tab, arena);
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        fail(KH_ENOMEM, "cannot allocate " + std::to_string(arena) + " bytes of table memory on device");
    }
    KH_HIP(e);
    KH_HIP(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    KH_HIP(hipMemsetAsync(g->d_tab, 0, arena, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    return g.release();
}

Graph::~Graph() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    Workspace &w = ws;
    void *ptrs[] = {d_tab, d_bc_keys, d_bc_vals, w.rec1_off, w.rec1_j, w.rec2_off, w.rec2_j, w.newf, w.fullf,
                    w.bc, w.cnt1, w.off1, w.cur1, w.tile1, w.cnt2, w.off2, w.cur2, w.cross, w.ctr,
                    w.d_words, w.d_koff, w.d_bytes};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (w.h_ctr) (void)hipHostFree(w.h_ctr);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
}

}  // namespace kh
