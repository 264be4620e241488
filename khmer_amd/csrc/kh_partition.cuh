// kh_partition.cuh -- partition of insert records (one per (k-mer, table))
// into LDS-sized table regions, and of winner k-mer indices into k-mer
// windows.  Included by kh_engine.hip.
//
// record = (batch k-mer index j << 32) | bin offset   (u64)
//   level 1: offset inside a bucket of 2^(s0+s2) global bins
//   level 2: offset inside a region of 2^s0 bins
//
// Every partition is a chunked counting sort with NO returning global
// atomics: a histogram kernel writes one count per (destination, chunk) into a
// destination-major matrix, one device-wide exclusive scan (rocPRIM) turns it
// into the exact output offset of every (destination, chunk) pair, and the
// scatter kernel (one workgroup per chunk) keeps its cursors in LDS.  A chunk
// is processed in tiles: each tile is counting-sorted in LDS and written out
// in runs, and since a chunk's records for one destination are contiguous in
// the output, consecutive tiles extend the same lines (write-combining in L2).
// The result is deterministic and keeps the stream order of the k-mers at
// tile granularity; exact stream order is recovered in the apply step from
// the k-mer index carried by every record.
#pragma once
#include "kh_src.cuh"

namespace kh {
__device__ unsigned long long g_dbg[64];   // development phase counters (tools/phase_probe.py)

// Development phase stamps (-DKH_PHASES builds only; tools/phase_probe.py):
// PH_BEGIN starts the clock, PH(i) adds the cycles since the last stamp to
// phase i, PH_END(base) publishes a workgroup's totals at g_dbg[base + i].
#ifdef KH_PHASES
#define PH_BEGIN(n) uint64_t ph_[n] = {}; uint64_t phA_ = __builtin_amdgcn_s_memtime(), phB_
#define PH(i) do { phB_ = __builtin_amdgcn_s_memtime(); ph_[i] += phB_ - phA_; phA_ = phB_; } while (0)
#define PH_END(base, n) do { if (threadIdx.x == 0) for (int z_ = 0; z_ < (n); z_++) atomicAdd(&g_dbg[(base) + z_], (unsigned long long)ph_[z_]); } while (0)
// PH_WG_BEGIN / PH_WG_END(base): a workgroup's wall time (100 MHz clock):
// g_dbg[base] sum, g_dbg[base + 1] max, g_dbg[base + 2] workgroups
#define PH_WG_BEGIN const uint64_t wg0_ = __builtin_amdgcn_s_memrealtime()
#define PH_WG_END(base) do { if (threadIdx.x == 0) { const unsigned long long d_ = __builtin_amdgcn_s_memrealtime() - wg0_; \
    atomicAdd(&g_dbg[(base)], d_); atomicMax(&g_dbg[(base) + 1], d_); atomicAdd(&g_dbg[(base) + 2], 1ull); } } while (0)
#else
#define PH_WG_BEGIN do { } while (0)
#define PH_WG_END(base) do { } while (0)
#define PH_BEGIN(n) do { } while (0)
#define PH(i) do { } while (0)
#define PH_END(base, n) do { } while (0)
#endif

constexpr int L1_THREADS = 512;
constexpr int L1_MAX_RPT = 8;                      // records per thread per tile
constexpr int L1_TILE_RECS = L1_THREADS * L1_MAX_RPT;   // 4096
constexpr int L1_HIST_TILE = 4096;                 // k-mers per histogram tile (window size)
constexpr int PT_THREADS = 1024;                   // level-2 / winner partitions
constexpr int PT_RPT = 8;
constexpr int PT_TILE = PT_THREADS * PT_RPT;       // 8192
constexpr uint64_t L2_CHUNK = 16ull * PT_TILE;     // records per level-2 chunk
constexpr uint32_t NO_J = 0xFFFFFFFFu;

// block-uniform value in a scalar register: loops whose trip count goes
// through this are uniform for the compiler, so the barriers inside them are
// executed by every wave in lock-step (a loop the compiler believes divergent
// is exited through the EXEC mask, which does not order barriers)
__device__ __forceinline__ uint32_t uniform_u32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

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

// exclusive scan of hist[0..n) into lstart by the whole block (n <= 8 *
// blockDim.x): per-thread partial sums, wave scans, wave totals in s_wtot[16].
// The caller synchronises before reading lstart.
__device__ __forceinline__ void block_scan_hist(const uint32_t *hist, uint32_t *lstart, uint32_t n,
                                                uint32_t *s_wtot) {
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = threadIdx.x * per;
    uint32_t v[8];
    uint32_t sum = 0;
#pragma unroll
    for (int u = 0; u < 8; u++) {
        v[u] = ((uint32_t)u < per && b0 + u < n) ? hist[b0 + u] : 0;
        sum += v[u];
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = sum;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_wtot[wave] = incl;
    block_sync();
    uint32_t acc = incl - sum;
    for (uint32_t w = 0; w < wave; w++) acc += s_wtot[w];
#pragma unroll
    for (int u = 0; u < 8; u++) {
        if ((uint32_t)u < per && b0 + u < n) lstart[b0 + u] = acc;
        acc += v[u];
    }
}

// block-wide exclusive scan over n u64 values in LDS (blockDim.x == 1024)
__device__ uint64_t block_exclusive_scan(uint64_t *v, uint32_t n, uint64_t *s_part) {
    const uint32_t per = (n + blockDim.x - 1) / blockDim.x;
    const uint32_t b0 = threadIdx.x * per;
    uint64_t sum = 0;
    for (uint32_t t = 0; t < per && b0 + t < n; t++) sum += v[b0 + t];
    s_part[threadIdx.x] = sum;
    block_sync();
    if (threadIdx.x < 64) {
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
    block_sync();
    uint64_t acc = s_part[threadIdx.x];
    for (uint32_t t = 0; t < per && b0 + t < n; t++) {
        uint64_t x = v[b0 + t];
        v[b0 + t] = acc;
        acc += x;
    }
    block_sync();
    return s_part[1024];
}

// ---------------------------------------------------------------------------
// Tail-buffered emission of a counting-sorted LDS tile.  Destination d's
// records of the tile go to out[lcur[d] ...]; only whole aligned segments of
// SEG records are written, the remainder waits in an LDS tail slot until its
// segment completes or the chunk ends.  Every write is then a full 64-B (or
// 32-B) segment except the first one of each (chunk, destination) run, which
// it shares with the previous chunk.  SEG_ <= 1 writes runs directly.
template <class T, int SEG_>
struct Emit {
    static constexpr bool TAILS = SEG_ > 1;
    static constexpr int SEG = TAILS ? SEG_ : 1;
    uint64_t *lcur;    // [F] next output position
    uint8_t *hskip;    // [F] slots of the head segment owned by the previous chunk
    T *tail;           // [F*SEG]
    uint32_t *hist;    // [F] this tile's count
    uint32_t *lstart;  // [F] this tile's LDS start
    uint64_t *dl;      // [F] output position minus LDS position (prepare())
    uint64_t *lim;     // [F] first output position that goes to the tail (prepare())
    uint16_t *flist;   // [F] destinations whose tail segment completes in this tile (note())
    uint32_t *nflush;  // [1] entries in flist

    __device__ __forceinline__ void init(uint32_t d, uint64_t pos) const {
        lcur[d] = pos;
        if (TAILS) hskip[d] = (uint8_t)(pos & (SEG - 1));
        hist[d] = 0;
    }
    __device__ __forceinline__ uint64_t flush_end(uint64_t e, bool last) const {
        return last ? e : (e & ~(uint64_t)(SEG - 1));
    }
    // phase 1 (after the tile is staged): write tails whose segment completes
    __device__ __forceinline__ void flush_tails(uint32_t F, bool last, T *out) const {
        if (!TAILS) return;
#pragma unroll 4
        for (uint32_t x = threadIdx.x; x < F * SEG; x += blockDim.x) {
            const uint32_t d = x / SEG, sl = x % SEG;
            const uint64_t lc = lcur[d];
            const uint64_t a = lc & ~(uint64_t)(SEG - 1);
            if (lc == a || flush_end(lc + hist[d], last) <= a) continue;
            if (sl >= hskip[d] && a + sl < lc) out[a + sl] = tail[x];
        }
    }
    // after the tile scan: per-destination placement constants for put()
    __device__ __forceinline__ void prepare(uint32_t F, bool last) const {
        for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) {
            const uint64_t lc = lcur[d];
            dl[d] = lc - lstart[d];
            lim[d] = TAILS ? flush_end(lc + hist[d], last) : ~0ull;
        }
    }
    // While ranking a tile: the record whose rank completes destination d's
    // pending tail segment lists d for flush_listed() (not on the chunk's
    // last tile, where every pending tail is flushed)
    __device__ __forceinline__ void note(uint32_t d, uint32_t rank, bool last) const {
        if (!TAILS || last) return;
        const uint32_t need = (0u - (uint32_t)lcur[d]) & (SEG - 1);
        if (need && rank == need - 1) flist[atomicAdd(nflush, 1u)] = (uint16_t)d;
    }
    // flush_tails() over the listed destinations only
    __device__ __forceinline__ void flush_listed(uint32_t F, bool last, T *out) const {
        if (!TAILS) return;
        if (last) {
            flush_tails(F, last, out);
            return;
        }
        const uint32_t n = *nflush * SEG;
        for (uint32_t x = threadIdx.x; x < n; x += blockDim.x) {
            const uint32_t d = flist[x / SEG], sl = x % SEG;
            const uint64_t lc = lcur[d];
            const uint64_t a = lc & ~(uint64_t)(SEG - 1);
            if (sl >= hskip[d] && a + sl < lc) out[a + sl] = tail[d * SEG + sl];
        }
    }
    // phase 2 (after a barrier): staged record q of destination d, from the
    // cursors directly (no prepare())
    __device__ __forceinline__ void put_cur(uint32_t d, uint32_t q, T v, bool last, T *out) const {
        const uint64_t pos = lcur[d] + (q - lstart[d]);
        if (!TAILS || pos < flush_end(lcur[d] + hist[d], last)) out[pos] = v;
        else tail[d * SEG + (uint32_t)(pos & (SEG - 1))] = v;
    }
    // the same with the prepare()d constants
    __device__ __forceinline__ void put(uint32_t d, uint32_t q, T v, T *out) const {
        const uint64_t pos = dl[d] + q;
        if (!TAILS || pos < lim[d]) out[pos] = v;
        else tail[d * SEG + (uint32_t)(pos & (SEG - 1))] = v;
    }
    // register-direct form: record of destination d with tile rank r
    __device__ __forceinline__ void put_rank(uint32_t d, uint32_t r, T v, bool last, T *out) const {
        const uint64_t pos = lcur[d] + r;

        if (!TAILS || pos < flush_end(lcur[d] + hist[d], last)) out[pos] = v;
        else tail[d * SEG + (uint32_t)(pos & (SEG - 1))] = v;
    }
    // phase 3 (after a barrier): advance cursors, clear the tile histogram
    __device__ __forceinline__ void advance(uint32_t F, bool last) const {
        for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) {
            const uint64_t lc = lcur[d], e = lc + hist[d];
            if (TAILS && flush_end(e, last) > (lc & ~(uint64_t)(SEG - 1))) hskip[d] = 0;

            lcur[d] = e;
            hist[d] = 0;
        }
        if (nflush && threadIdx.x == 0) *nflush = 0;
    }
};

// ---------------------------------------------------------------------------
// level 1: per-chunk bucket histogram over all tables -> M1[b * nch1 + chunk]
template <class Src>
__global__ void __launch_bounds__(L1_THREADS) k_hist_l1(Params P, Src src, uint64_t nkmers, uint32_t ck1,
                                                       uint32_t nch1, uint32_t *M1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    uint64_t *s_meta = (uint64_t *)(hist + ((P.F1 + 3) & ~3u));
    uint64_t *s_koff = s_meta + 2;
    const int shift = P.s0 + P.s2;
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x) hist[b] = 0;
    const uint64_t c0 = (uint64_t)blockIdx.x * ck1;
    const uint64_t c1 = min(nkmers, c0 + ck1);
    const uint32_t ntiles = uniform_u32((uint32_t)((c1 - c0 + L1_HIST_TILE - 1) / L1_HIST_TILE));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t j0 = c0 + (uint64_t)ti * L1_HIST_TILE;
        const uint64_t j1 = min(c1, j0 + L1_HIST_TILE);
        block_sync();
        TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
        for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
            const uint64_t h = kmer_hash(src, s_koff, tr, j);
            for (int i = 0; i < P.n; i++) {
                uint64_t G;
                if (local_bin(P, i, h, &G)) atomicAdd(&hist[G >> shift], 1u);
            }
        }
    }
    block_sync();
    for (uint32_t b = threadIdx.x; b < P.F1; b += blockDim.x) M1[(uint64_t)b * nch1 + blockIdx.x] = hist[b];
}

// level-1 bucket offsets (from the scanned matrix) and the level-2 chunk
// prefix: bucket b owns level-2 chunks [ch2[b], ch2[b+1])
__global__ void __launch_bounds__(1024) k_plan_l2(uint32_t F1, uint32_t nch1, const uint64_t *O1, const uint32_t *M1,
                                                  uint64_t *off1, uint32_t *ch2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *v = (uint64_t *)smem;   // [F1]
    uint64_t *s_part = v + F1;        // [1025]
    // records of this pass (only the owned ones when sharded)
    const uint64_t last = (uint64_t)F1 * nch1 - 1;
    const uint64_t total = O1[last] + M1[last];
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) {
        const uint64_t s = O1[(uint64_t)b * nch1];
        const uint64_t e = b + 1 < F1 ? O1[(uint64_t)(b + 1) * nch1] : total;
        off1[b] = s;
        v[b] = (e - s + L2_CHUNK - 1) / L2_CHUNK;
    }
    if (threadIdx.x == 0) off1[F1] = total;
    block_sync();
    const uint64_t chunks = block_exclusive_scan(v, F1, s_part);
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) ch2[b] = (uint32_t)v[b];
    if (threadIdx.x == 0) ch2[F1] = (uint32_t)chunks;
}

// level-1 scatter of tables [t0, t0+nt) (nt <= 8), KPT = 8 / nt k-mers per
// thread per tile, one workgroup per chunk; records stay in registers between
// the tile histogram and the placement.  The chunk's cursors are written back
// so a following table group continues.
//
// PRE: the source yields already-binned records (j << 32) | G (k_own_filter's
// output; one "table", nt == 1): the same tiles, without hashing.
template <class Src, int SEG, int KPT, int RPT = L1_MAX_RPT, bool PRE = false>
__global__ void __launch_bounds__(L1_THREADS) k_scatter_l1(Params P, Src src, uint64_t nkmers, uint32_t ck1,
                                                          uint32_t nch1, int t0, int nt, uint64_t *O1,
                                                          uint64_t *rec, uint32_t jbase, uint32_t bb0) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    uint64_t *lcur = (uint64_t *)smem;                // [F1]
    constexpr int TILE_RECS = L1_THREADS * RPT;
    uint64_t *stage = lcur + F1a;                     // [TILE_RECS]
    uint64_t *tail = stage + TILE_RECS;               // [F1*SEG]
    uint32_t *hist = (uint32_t *)(tail + (SEG > 1 ? F1a * SEG : 0));  // [F1]
    uint32_t *lstart = hist + F1a;                    // [F1]
    uint16_t *sb = (uint16_t *)(lstart + F1a);        // [TILE_RECS]
    uint32_t *s_wtot = (uint32_t *)(sb + TILE_RECS);  // [16]
    uint8_t *hskip = (uint8_t *)(s_wtot + 16);        // [F1]
    uint64_t *s_meta = (uint64_t *)(hskip + ((F1a + 7) & ~7u));
    uint64_t *s_koff = s_meta + 2;
    const Emit<uint64_t, SEG> em{lcur, hskip, tail, hist, lstart, nullptr, nullptr, nullptr, nullptr};
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;
    constexpr int TILE_KMERS = L1_THREADS * KPT;

    // a launch window of buckets [bb0, bb0 + F1) (P's geometry shifted to it):
    // rows bb0 + b of the count matrix
    O1 += (uint64_t)bb0 * nch1;
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) em.init(b, O1[(uint64_t)b * nch1 + blockIdx.x]);
    const uint64_t c0 = (uint64_t)blockIdx.x * ck1;
    const uint64_t c1 = min(nkmers, c0 + ck1);
    PH_BEGIN(6);
    // Without a read-offset window the next tile's input words are loaded a
    // whole tile ahead (fetch) and hashed at the top of the tile (finish):
    // the loads are issued before this tile's stores (loads and stores share
    // one completion counter) and their latency hides behind the tile's work.
    const bool pre = !needs_window(src);
    typename Src::Pend pend[KPT];
    if (pre) {
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = c0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            if (j < min(c1, c0 + TILE_KMERS)) pend[a] = kmer_fetch(src, j);
        }
    }
    const uint32_t ntiles = uniform_u32((uint32_t)((c1 - c0 + TILE_KMERS - 1) / TILE_KMERS));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t j0 = c0 + (uint64_t)ti * TILE_KMERS;
        const uint64_t j1 = min(c1, j0 + TILE_KMERS);
        const bool last = ti + 1 == ntiles;
        block_sync();
        PH(0);
        TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
        uint64_t G[RPT];
        uint32_t rank[RPT];
        uint32_t jj[RPT];
        int nr = 0;
#pragma unroll
        for (int q = 0; q < RPT; q++) { G[q] = ~0ull; rank[q] = 0; jj[q] = 0; }
        // pass A: hashes, bins, tile histogram (ranks)
        uint64_t hh[KPT];
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            hh[a] = j < j1 ? (pre ? src.finish(pend[a]) : kmer_hash(src, s_koff, tr, j)) : 0;
        }
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            const bool ok = j < j1;
#pragma unroll
            for (int q = 0; q < RPT; q++) {
                const int i = q - a * nt;  // table slot of register q for k-mer a
                if (ok && i >= 0 && i < nt) {
                    uint64_t Gq = (uint32_t)hh[a];
                    if (PRE || local_bin(P, t0 + i, hh[a], &Gq)) {   // owned here
                        G[q] = Gq;
                        jj[q] = PRE ? (uint32_t)(hh[a] >> 32) : jbase + (uint32_t)j;
                        rank[q] = atomicAdd(&hist[(uint32_t)(Gq >> shift)], 1u);
                        nr = q + 1;
                    } else {
                        G[q] = ~0ull;
                    }
                }
            }
        }
        block_sync();
        PH(1);
        block_scan_hist(hist, lstart, F1, s_wtot);
        block_sync();
        PH(2);
        // pass B: place in LDS in bucket order
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            if (q < nr && G[q] != ~0ull) {
                const uint32_t b = (uint32_t)(G[q] >> shift);
                const uint32_t pos = lstart[b] + rank[q];
                stage[pos] = ((uint64_t)jj[q] << 32) | (G[q] & omask);
                sb[pos] = (uint16_t)b;
            }
        }
        if (pre) {
            const uint64_t n0 = j0 + TILE_KMERS, n1 = min(c1, n0 + TILE_KMERS);
#pragma unroll
            for (int a = 0; a < KPT; a++) {
                const uint64_t j = n0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                if (j < n1) pend[a] = kmer_fetch(src, j);
            }
        }
        em.flush_tails(F1, last, rec);
        block_sync();
        PH(3);
        // pass C: whole segments at the chunk's cursors
        const uint32_t nrec = lstart[F1 - 1] + hist[F1 - 1];   // records staged (owned ones)
#pragma unroll
        for (int u = 0; u < RPT; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * L1_THREADS;
            if (q < nrec) em.put_cur(sb[q], q, stage[q], last, rec);
        }
        block_sync();
        PH(4);
        em.advance(F1, last);
    }
    PH_END(8, 6);
    if (t0 + nt < P.n) {   // a following table group continues from these cursors
        block_sync();
        for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) O1[(uint64_t)b * nch1 + blockIdx.x] = lcur[b];
    }
}

// ---------------------------------------------------------------------------
// Level 1 into fixed-capacity buckets: the k-mers are hashed once (no
// histogram pass).  Bucket b owns [bkt_base[b], bkt_base[b+1]), sized on the
// host from its expected record count.  A persistent grid: workgroup w takes
// k-mers [w * kpw, (w+1) * kpw) tile by tile; each tile is counting-sorted by
// bucket in LDS as in k_scatter_l1, and its runs are appended to blocks of
// L1F_BLK records that the workgroup reserves with one returning atomic per
// (bucket, tile) on bkt_cur[b] (a block belongs to one workgroup, so runs
// keep their 16-B aligned pairs with 2-record LDS tails).  After its last
// tile a workgroup fills the rest of its partial blocks with the ~0 sentinel;
// bucket b's records are then [bkt_base[b], bkt_cur[b]).  A bucket that runs
// out of capacity sets ctr[CTR_ERR] bit 8 and the host redoes the pass with
// the exact two-pass level 1.
constexpr int L1F_BLK_SH = 8;   // default block: 256 records (KH_L1F_BLK_SH)
// 3 workgroups of 8 waves per CU: <= 80 VGPRs, ~47 KB of LDS at F1 <= 256
#ifndef L1F_WAVES_PER_EU
#define L1F_WAVES_PER_EU 6
#endif

// LDS words per staged tile (TW) and where they live: after the kernel's
// other arrays (lds_scatter_l1f adds 2 * L1F_TW words)
constexpr int L1F_TW = 128;
__host__ __device__ constexpr size_t l1f_tw_offset(size_t F1a, int rpt) {
    // u64 index: 5 F1a u64 arrays, then one u64 slot per
    // record, 5 F1a u32 arrays, s_wtot, s_meta, s_koff (the window, unused
    // for fixed-length reads) rounded to 8 bytes
    return (F1a * 8 * 5 + ((size_t)L1_THREADS * rpt + 2 * F1a) * 8 + F1a * 4 * 5 + 64 + 16 + 7) / 8;
}

template <class Src, int KPT, int RPT_ = L1_MAX_RPT, bool TW_ = false>
__global__ void __launch_bounds__(L1_THREADS, RPT_ == 8 ? L1F_WAVES_PER_EU : 4) k_scatter_l1f(Params P, Src src, uint64_t nkmers, uint64_t kpw, int t0,
                                                           int nt, const uint64_t *bkt_base,
                                                           unsigned long long *bkt_cur, uint64_t *rec,
                                                           uint64_t *ctr, int blk_sh, uint32_t jbase, uint32_t cht) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RPT = RPT_;
    constexpr int TILE_RECS = L1_THREADS * RPT;
    constexpr int TILE_KMERS = L1_THREADS * KPT;
    const uint32_t BLK = 1u << blk_sh;
    PH_WG_BEGIN;
    constexpr uint64_t DEAD = ~0ull;
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    uint64_t *bcur = (uint64_t *)smem;                  // [F1] partially filled block (DEAD: overflowed)
    uint64_t *nbase = bcur + F1a;                       // [F1] blocks reserved for this tile
    uint64_t *dl = nbase + F1a;                         // [F1][2] output - LDS position: current block, new blocks
    uint64_t *tail = dl + 2 * F1a;                      // [F1] a pending odd record
    // stage slots: TILE_RECS records + per bucket at most one leading hole
    // and one trailing pad (every bucket's run starts on an even slot, so
    // stage slot pairs map onto 16-B aligned output record pairs)
    const uint32_t NSLOT = TILE_RECS + 2 * F1a;
    // one 8-byte slot per staged record: (bucket << 16 | k-mer index in the
    // tile) << 32 | bin offset inside the bucket (index SLOT_EMPTY: hole /
    // pad); 16-B aligned (5 F1a u64 arrays before it, F1a a multiple of 4),
    // so a slot pair is one 16-byte LDS read in the write-out
    uint64_t *slot = tail + F1a;                        // [NSLOT]
    uint32_t *cnt = (uint32_t *)(slot + NSLOT);         // [F1] records appended by this workgroup
    uint32_t *hist = cnt + F1a;                         // [F1]
    uint32_t *lstart = hist + F1a;                      // [F1] the bucket's first record slot of the tile
    uint2 *qq = (uint2 *)(lstart + F1a);                // [F1] (first LDS position in the new blocks,
                                                        //       first LDS position left for the tail)
    uint32_t *s_wtot = (uint32_t *)(qq + F1a);          // [16]
    constexpr uint32_t SLOT_EMPTY = 0xFFFFu;
    uint64_t *s_meta = (uint64_t *)(s_wtot + 16);
    uint64_t *s_koff = s_meta + 2;
    // TW: fixed-length 2-bit reads whose tile spans <= L1F_TW words: the
    // tile's packed words are staged in LDS (double-buffered; the next tile's
    // words are loaded one tile ahead, one word per thread) and every k-mer
    // window is read from there -- no per-k-mer global loads, no prefetch
    // registers
    constexpr bool TW = TW_ && std::is_same<Src, SrcTwoBit>::value;
    uint64_t *s_tw = (uint64_t *)smem + l1f_tw_offset(F1a, RPT);   // [2][L1F_TW]
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) {
        bcur[b] = 0;
        cnt[b] = 0;
        hist[b] = 0;
    }
    // Work distribution in chunks of CK k-mers.  Static (cht == 0): one chunk
    // of kpw k-mers per workgroup.  Dynamic (cht > 0): chunks of cht tiles;
    // workgroup w starts with chunks w and w + gridDim.x, and on the first
    // tile of every chunk it takes one more from the queue head
    // ctr[CTR_L1Q] (numbered from 2 * gridDim.x), so the next chunk is always
    // known a chunk ahead (the next tile's words are loaded a tile ahead) and
    // the workgroups finish together instead of waiting for the slowest
    // fixed share (measured: mean 42 vs max 54 ms per launch).
    const uint64_t CK = cht ? (uint64_t)cht * TILE_KMERS : kpw;
    const uint32_t nchunks = (uint32_t)((nkmers + CK - 1) / CK);
    uint32_t cb = cht ? blockIdx.x + gridDim.x : nchunks;   // the chunk after this one (nchunks: none)
    uint64_t j0 = min(nkmers, (uint64_t)blockIdx.x * CK);     // this tile's first k-mer
    uint64_t ce = min(nkmers, j0 + CK);                       // the chunk's end
    bool chunk_top = true;                                    // first tile of a chunk: take one from the queue
    uint32_t *s_q = s_wtot + 15;                              // [1] chunk taken from the queue
    // the run-start scan writes one wave total per wave into s_wtot[0, waves):
    // it must never reach the queue slot (a 1024-thread build once did and hung)
    static_assert(L1_THREADS / 64 < 15, "k_scatter_l1f: the scan's wave totals would overwrite s_q");
    const bool pre = !needs_window(src);
    constexpr int NPEND = TW ? 1 : KPT;
    typename Src::Pend pend[NPEND];
    if (!TW && pre) {
#pragma unroll
        for (int a = 0; a < NPEND; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            if (j < min(ce, j0 + TILE_KMERS)) pend[a] = kmer_fetch(src, j);
        }
    }
    // first word of tile [j0, ..) (TW)
    auto tile_w0 = [&](uint64_t j0) -> uint64_t {
        const uint64_t ja = j0 + src.kbase;
        return ((ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2) >> 6;
    };
    // words [tile_w0(j0), tile_w0(j1 - 1) + 1] hold every window of tile [j0, j1)
    auto tile_nw = [&](uint64_t j0, uint64_t j1) -> uint32_t { return (uint32_t)(tile_w0(j1 - 1) + 2 - tile_w0(j0)); };
    uint64_t tw_next = 0;
    if constexpr (TW) {
        if (ce > j0) {
            const uint64_t e = min(ce, j0 + TILE_KMERS);
            if (threadIdx.x < tile_nw(j0, e)) s_tw[threadIdx.x] = src.words[tile_w0(j0) + threadIdx.x];
        }
    }
    PH_BEGIN(8);
    for (uint32_t ti = 0; j0 < ce; ti++) {
        const uint64_t j1 = min(ce, j0 + TILE_KMERS);
        // the next tile [n0, n1): in this chunk, else the first of chunk cb
        uint64_t n0 = j1, n1 = j1;
        if (j1 < ce) {
            n1 = min(ce, j1 + TILE_KMERS);
        } else if (cb < nchunks) {
            n0 = (uint64_t)cb * CK;
            n1 = min(nkmers, n0 + min(CK, (uint64_t)TILE_KMERS));
        }
        const bool last = n1 == n0;
        unsigned long long qn = 0;
        if (cht && chunk_top && threadIdx.x == 0) qn = atomicAdd((unsigned long long *)&ctr[CTR_L1Q], 1ull);
        block_sync();
        PH(7);
        TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
        const uint64_t *tw_cur = s_tw + (ti & 1) * L1F_TW;
        const uint64_t tw_w0 = TW ? tile_w0(j0) : 0;
        if constexpr (TW) {   // the next tile's words, stored at the end of this tile
            if (!last) {
                if (threadIdx.x < tile_nw(n0, n1)) tw_next = src.words[tile_w0(n0) + threadIdx.x];
            }
        }
        // per record slot q (k-mer a = q / nt of this thread): bin offset
        // inside its bucket (~0: none) and (a << 23 | bucket << 13 | tile
        // rank); the k-mer index is j0 + a * L1_THREADS + thread: 2 VGPRs per record
        uint32_t off[RPT], br[RPT];
#pragma unroll
        for (int q = 0; q < RPT; q++) { off[q] = ~0u; br[q] = 0; }
        uint64_t hh[KPT];
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            if constexpr (TW) {
                uint64_t h = 0;
                if (j < j1) {
                    const uint64_t ja = j + src.kbase;
                    const uint64_t bpos = (ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2;
                    const uint32_t wi = (uint32_t)((bpos >> 6) - tw_w0);
                    h = src.finish(SrcTwoBit::Pend{tw_cur[wi], tw_cur[wi + 1], (uint32_t)(bpos & 63)});
                }
                hh[a] = h;
            } else {
                hh[a] = j < j1 ? (pre ? src.finish(pend[a]) : kmer_hash(src, s_koff, tr, j)) : 0;
            }
            if (KH_ABL(P, 32)) hh[a] = (j * 0x9E3779B97F4A7C15ull) >> 22;   // timing only: no fetch/hash
        }
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            const bool ok = j < j1;
#pragma unroll
            for (int q = 0; q < RPT; q++) {
                const int i = q - a * nt;
                if (ok && i >= 0 && i < nt) {
                    uint64_t Gq;
                    if (local_bin(P, t0 + i, hh[a], &Gq)) {
                        const uint32_t b = (uint32_t)(Gq >> shift);
                        off[q] = (uint32_t)(Gq & omask);
                        br[q] = ((uint32_t)a << 23) | (b << 13) | atomicAdd(&hist[b], 1u);
                    }
                }
            }
        }
        PH(0);
        block_sync();
        PH(1);
        // Block reservations are issued first (thread d owns bucket d and
        // d + L1_THREADS; F1 <= 1024): the returned bases are needed only
        // after the staging below, which hides the atomics' latency.
        uint64_t rsv[2] = {0, 0};
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t d = threadIdx.x + (uint32_t)u * L1_THREADS;
            if (d < F1 && bcur[d] != DEAD) {
                const uint32_t h = hist[d], L0 = cnt[d];
                const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (((L0 + BLK - 1) & ~(BLK - 1)) >> blk_sh);
                if (need) rsv[u] = atomicAdd(&bkt_cur[d], (unsigned long long)need * BLK);
            }
        }
        // stage region of bucket d: an even number of slots, a leading hole
        // when a record of the bucket is pending (its pair partner), the run,
        // a trailing pad when the run ends unpaired.  Region starts: padded
        // run sizes and their exclusive scan by wave 0 alone (<= 16 buckets
        // per lane), one barrier.
        auto run = [&](uint32_t d) -> uint32_t {
            const uint32_t h = hist[d];
            return h ? (h + (cnt[d] & 1u) + 1u) & ~1u : 0u;
        };
        // lstart[d] = the run's first record slot: its region start plus
        // the leading hole (staging then reads one LDS word per record)
        if (F1 > 256) {
            // many buckets: every thread scans two (F1 <= 2 * L1_THREADS),
            // wave totals through s_wtot (one more barrier)
            const uint32_t d0 = 2 * threadIdx.x;
            const uint32_t r0 = d0 < F1 ? run(d0) : 0u, r1 = d0 + 1 < F1 ? run(d0 + 1) : 0u;
            const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            uint32_t incl = r0 + r1;
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t y = __shfl_up(incl, dd, 64);
                if (lane >= (uint32_t)dd) incl += y;
            }
            if (lane == 63) s_wtot[wave] = incl;
            block_sync();
            uint32_t acc = incl - r0 - r1;
            for (uint32_t w = 0; w < wave; w++) acc += s_wtot[w];
            if (d0 < F1) lstart[d0] = acc + (cnt[d0] & 1u);
            if (d0 + 1 < F1) lstart[d0 + 1] = acc + r0 + (cnt[d0 + 1] & 1u);
        } else if (threadIdx.x < 64) {
            // <= 4 buckets a lane, unrolled: the lane's LDS reads issue back
            // to back and the run sizes stay in registers for the writes
            // (four independent row scans over buckets l, 64 + l, ... spilled
            // registers and measured 1 ms/step slower)
            const uint32_t lane = threadIdx.x, per = (F1 + 63) / 64, b0 = lane * per;
            uint32_t rs[4], sum = 0;
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                rs[t] = (t < per && b0 + t < F1) ? run(b0 + t) : 0u;
                sum += rs[t];
            }
            uint32_t incl = sum;
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t y = __shfl_up(incl, dd, 64);
                if (lane >= (uint32_t)dd) incl += y;
            }
            uint32_t acc = incl - sum;
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                if (t < per && b0 + t < F1) lstart[b0 + t] = acc + (cnt[b0 + t] & 1u);
                acc += rs[t];
            }
        }
        block_sync();
        PH(2);
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            if (off[q] != ~0u) {
                const uint32_t b = (br[q] >> 13) & 1023u;
                const uint32_t pos = lstart[b] + (br[q] & 8191u);
                slot[pos] = (uint64_t)((b << 16) | ((br[q] >> 23) * L1_THREADS + threadIdx.x)) << 32 | off[q];
            }
        }
        // The next tile's packed words go to their LDS buffer here, not after
        // the write-out: waiting for that load (vmcnt, which on gfx9 counts
        // loads and stores together, in order) after this tile's stores would
        // drain every store of the tile before the closing barrier.  Buffer
        // (ti + 1) & 1 was last read in tile ti - 1, before this tile's first
        // barrier; tile ti + 1 reads it after this tile's last one.
        if (TW && !last && threadIdx.x < L1F_TW) s_tw[((ti + 1) & 1) * L1F_TW + threadIdx.x] = tw_next;
        PH(3);
        if (!TW && pre) {
#pragma unroll
            for (int a = 0; a < NPEND; a++) {
                const uint64_t j = n0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                if (j < n1 && !(KH_ABL(P, 32))) pend[a] = kmer_fetch(src, j);
            }
        }
        // per bucket: the reserved blocks (past the capacity: overflow), the
        // pending odd record when its pair completes, and the placement
        // constants of this tile's run
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t d = threadIdx.x + (uint32_t)u * L1_THREADS;
            if (d >= F1) continue;
            const uint32_t h = hist[d];
            if (!h && !last) continue;
            const uint32_t L0 = cnt[d];
            const uint32_t split = (L0 + BLK - 1) & ~(BLK - 1);
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (split >> blk_sh);
            uint64_t bc = bcur[d], nb = 0;
            if (bc == DEAD) {
                nb = DEAD;
            } else if (need) {
                nb = rsv[u];
                if (nb + (uint64_t)need * BLK > bkt_base[d + 1]) {
                    atomicOr((unsigned long long *)&ctr[CTR_ERR], 8ull);
                    nb = DEAD;
                }
            }
            const uint32_t e = L0 + h, fe = last ? e : (e & ~1u);
            if ((L0 & 1) && fe > L0 - 1 && bc != DEAD && !(KH_ABL(P, 16))) rec[bc + ((L0 - 1) & (BLK - 1))] = tail[d];   // 16: the tails were never written
            const uint32_t q0 = lstart[d];   // the run's first slot (odd after a hole)
            if (h) {
                if (L0 & 1) slot[q0 - 1] = (uint64_t)((d << 16) | SLOT_EMPTY) << 32;
                if ((q0 + h) & 1) slot[q0 + h] = (uint64_t)((d << 16) | SLOT_EMPTY) << 32;
            }
            const bool dead = bc == DEAD || nb == DEAD;
            nbase[d] = nb;
            dl[2 * d] = bc + (L0 & (BLK - 1)) - q0;
            dl[2 * d + 1] = nb + L0 - split - q0;
            qq[d] = make_uint2(q0 + (split - L0), dead ? 0 : q0 + (fe > L0 ? fe - L0 : 0));
        }
        // the chunk taken from the queue, read after the tile's last barrier
        if (cht && chunk_top && threadIdx.x == 0) *s_q = (uint32_t)min<unsigned long long>(qn + 2ull * gridDim.x, nchunks);
        PH(4);
        block_sync();
        PH(5);
        // write-out by slot pairs: a pair of records is one 16-B store (its
        // output position is even, inside one block); a (hole, record) or
        // (record, pad) pair writes its record alone, or parks it in the
        // bucket's tail when it is the run's unpaired last (not on the last tile)
        {
            const uint32_t dlast = F1 - 1;
            const uint32_t pl = cnt[dlast] & 1u;
            const uint32_t nslot = lstart[dlast] - pl + (hist[dlast] ? (hist[dlast] + pl + 1u) & ~1u : 0u);
            const ulonglong2 *slot2 = (const ulonglong2 *)slot;
            const ulonglong2 *dl2 = (const ulonglong2 *)dl;   // both placement constants in one 16-B read
            auto put_pair = [&](uint32_t m, uint2 bj, uint2 st, uint2 ql, ulonglong2 dd) {
                const uint32_t q = 2 * m;
                const uint32_t d = bj.x >> 16;
                const bool r0 = (bj.x & 0xFFFFu) != SLOT_EMPTY, r1 = (bj.y & 0xFFFFu) != SLOT_EMPTY;
                const uint64_t v0 = ((jbase + j0 + (bj.x & 0xFFFFu)) << 32) | st.x;
                const uint64_t v1 = ((jbase + j0 + (bj.y & 0xFFFFu)) << 32) | st.y;
                if (KH_ABL(P, 16)) return;   // timing only: no run writes
                const uint64_t o = (q >= ql.x ? dd.y : dd.x) + q;   // (qs, qlim): both even
                if (q < ql.y) {
                    if (r0 && r1) *(ulonglong2 *)(rec + o) = make_ulonglong2(v0, v1);
                    else if (r0) rec[o] = v0;
                    else if (r1) rec[o + 1] = v1;
                } else if (r0) {
                    tail[d] = v0;   // the run's unpaired last record
                }
            };
            for (uint32_t m = threadIdx.x; 2 * m < nslot; m += L1_THREADS) {
                const ulonglong2 sp = slot2[m];
                const uint2 bj = make_uint2((uint32_t)(sp.x >> 32), (uint32_t)(sp.y >> 32));
                const uint32_t d = bj.x >> 16;
                put_pair(m, bj, make_uint2((uint32_t)sp.x, (uint32_t)sp.y), qq[d], dl2[d]);
            }
        }
        PH(6);
        block_sync();
        for (uint32_t d = threadIdx.x; d < F1; d += blockDim.x) {
            const uint32_t h = hist[d];
            if (!h) continue;
            const uint32_t L0 = cnt[d];
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - ((L0 + BLK - 1) >> blk_sh);
            if (nbase[d] == DEAD) bcur[d] = DEAD;
            else if (need) bcur[d] = nbase[d] + (uint64_t)(need - 1) * BLK;
            cnt[d] = L0 + h;
            hist[d] = 0;
        }
        // advance: the next tile of this chunk, or the first of chunk cb
        chunk_top = j1 >= ce;
        if (chunk_top) {
            j0 = n0;
            ce = cb < nchunks ? min(nkmers, (uint64_t)cb * CK + CK) : n0;
            cb = cht ? uniform_u32(*s_q) : nchunks;
        } else {
            j0 = j1;
        }
    }
    PH_END(24, 8);
    block_sync();
    for (uint32_t y = threadIdx.x; y < F1 * BLK; y += blockDim.x) {
        const uint32_t d = y >> blk_sh, sl = y & (BLK - 1);
        const uint32_t c = cnt[d] & (BLK - 1);
        if (c == 0 || sl < c || bcur[d] == DEAD) continue;
        rec[bcur[d] + sl] = ~0ull;
    }
    PH_WG_END(40);
}

// ---------------------------------------------------------------------------
// Software-pipelined k_scatter_l1f (round 5) for the hot case: fixed-length
// 2-bit reads whose tile's packed words are staged in LDS, at most 256
// buckets, dynamic chunks of >= 2 tiles.  k_scatter_l1f runs a tile as five
// barrier-separated phases (rank | scan | stage | write-out | advance); here
// a tile takes three, and the write-out of tile t shares its phase with the
// hash + LDS rank of tile t + 1 (two tile histograms), so a wave that is done
// writing moves on to hashing instead of waiting at a barrier, and the
// tile's stores drain while the next tile is hashed:
//   P1: block reservations, run-start scan (tile t)
//   P2: staging, per-bucket placement constants and the bucket state
//       advanced for tile t; the next tile's words into LDS
//   P3: write-out of tile t, then hash + rank of tile t + 1
// Records, blocks, holes and pads are exactly k_scatter_l1f's.
template <int KPT>
__global__ void __launch_bounds__(L1_THREADS, L1F_WAVES_PER_EU) k_scatter_l1p(Params P, SrcTwoBit src, uint64_t nkmers,
                                                                             uint64_t kpw, int t0, int nt,
                                                                             const uint64_t *bkt_base,
                                                                             unsigned long long *bkt_cur, uint64_t *rec,
                                                                             uint64_t *ctr, int blk_sh, uint32_t jbase,
                                                                             uint32_t cht) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RPT = L1_MAX_RPT;
    constexpr int TILE_RECS = L1_THREADS * RPT;
    constexpr int TILE_KMERS = L1_THREADS * KPT;
    constexpr uint32_t SLOT_EMPTY = 0xFFFFu;
    constexpr uint64_t DEAD = ~0ull;
    (void)kpw;
    const uint32_t BLK = 1u << blk_sh;
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    const uint32_t NSLOT = TILE_RECS + 2 * F1a;
    uint64_t *s_tw = (uint64_t *)smem;                  // [2][L1F_TW] packed words of the next tiles
    uint64_t *bcur = s_tw + 2 * L1F_TW;                 // [F1] partially filled block (DEAD: overflowed)
    uint64_t *dl = bcur + F1a;                          // [F1][2] output - LDS position
    uint64_t *tail = dl + 2 * F1a;                      // [F1] a pending odd record
    uint64_t *slot = tail + F1a;                        // [NSLOT] as in k_scatter_l1f
    uint32_t *cnt = (uint32_t *)(slot + NSLOT);         // [F1] records appended by this workgroup
    uint32_t *hist2 = cnt + F1a;                        // [2][F1] the tile histograms (tile parity)
    uint32_t *lstart = hist2 + 2 * F1a;                 // [F1] the bucket's first record slot
    uint2 *qq = (uint2 *)(lstart + F1a);                // [F1]
    uint32_t *s_misc = (uint32_t *)(qq + F1a);          // [0] queue chunk, [1] slots of the staged tile
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) {
        bcur[b] = 0;
        cnt[b] = 0;
        hist2[b] = 0;
        hist2[F1a + b] = 0;
    }
    // the hash stage's tile iterator (k_scatter_l1f's chunk queue: workgroup
    // w starts with chunks w and w + gridDim.x and takes one more from the
    // queue on the first tile of every chunk; with >= 2 tiles a chunk, a
    // queue result is published (P2) before the iterator needs it)
    const uint64_t CK = (uint64_t)cht * TILE_KMERS;
    const uint32_t nchunks = (uint32_t)((nkmers + CK - 1) / CK);
    uint32_t cb = blockIdx.x + gridDim.x;
    uint64_t hj0 = min(nkmers, (uint64_t)blockIdx.x * CK);   // the hashed tile's first k-mer
    uint64_t hce = min(nkmers, hj0 + CK);                      // its chunk's end
    bool htop = true;                                         // the hashed tile starts a chunk
    auto tile_w0 = [&](uint64_t j0) -> uint64_t {
        const uint64_t ja = j0 + src.kbase;
        return ((ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2) >> 6;
    };
    auto tile_nw = [&](uint64_t j0, uint64_t j1) -> uint32_t { return (uint32_t)(tile_w0(j1 - 1) + 2 - tile_w0(j0)); };
    // the tile after the hashed one: [*n0, *n1), empty when there is none
    auto next_tile = [&](uint64_t j1, uint64_t *n0, uint64_t *n1) {
        *n0 = j1;
        *n1 = j1;
        if (j1 < hce) {
            *n1 = min(hce, j1 + TILE_KMERS);
        } else if (cb < nchunks) {
            *n0 = (uint64_t)cb * CK;
            *n1 = min(nkmers, *n0 + (uint64_t)TILE_KMERS);
        }
    };
    uint32_t off[RPT], br[RPT];
    unsigned long long qn = 0;
    uint64_t tw_next = 0;
    // hash + rank of tile [j0, j1) into histogram h (words in s_tw[buf]); the
    // next tile's words (nn0, nn1) are loaded into tw_next
    auto hash_rank = [&](uint64_t j0, uint64_t j1, uint32_t *h, uint32_t buf) {
#pragma unroll
        for (int q = 0; q < RPT; q++) { off[q] = ~0u; br[q] = 0; }
        const uint64_t *tw_cur = s_tw + buf * L1F_TW;
        const uint64_t tw_w0 = tile_w0(j0);
        uint64_t hh[KPT];
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            uint64_t x = 0;
            if (j < j1) {
                const uint64_t ja = j + src.kbase;
                const uint64_t bpos = (ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2;
                const uint32_t wi = (uint32_t)((bpos >> 6) - tw_w0);
                x = src.finish(SrcTwoBit::Pend{tw_cur[wi], tw_cur[wi + 1], (uint32_t)(bpos & 63)});
            }
            hh[a] = x;
        }
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            const bool ok = j < j1;
#pragma unroll
            for (int q = 0; q < RPT; q++) {
                const int i = q - a * nt;
                if (ok && i >= 0 && i < nt) {
                    uint64_t Gq;
                    if (local_bin(P, t0 + i, hh[a], &Gq)) {
                        const uint32_t b = (uint32_t)(Gq >> shift);
                        off[q] = (uint32_t)(Gq & omask);
                        br[q] = ((uint32_t)a << 23) | (b << 13) | atomicAdd(&h[b], 1u);
                    }
                }
            }
        }
    };
    // prologue: the first tile's words, its queue atomic, hash + rank
    uint64_t hj1 = min(hce, hj0 + TILE_KMERS);
    if (hce > hj0 && threadIdx.x < tile_nw(hj0, hj1)) s_tw[threadIdx.x] = src.words[tile_w0(hj0) + threadIdx.x];
    if (hce > hj0 && threadIdx.x == 0) qn = atomicAdd((unsigned long long *)&ctr[CTR_L1Q], 1ull);
    block_sync();
    uint64_t n0, n1;
    next_tile(hj1, &n0, &n1);
    if (hce > hj0) {
        if (n1 > n0 && threadIdx.x < tile_nw(n0, n1)) tw_next = src.words[tile_w0(n0) + threadIdx.x];
        hash_rank(hj0, hj1, hist2, 0);
    }
    block_sync();
    for (uint32_t ti = 0; hce > hj0; ti++) {
        // the staged tile (= the hashed one until P3 moves the iterator on)
        const uint64_t j0 = hj0;
        const bool last = n1 == n0;
        const bool top = htop;
        uint32_t *hist = hist2 + (ti & 1) * F1a;
        // ---- P1: block reservations (thread d owns bucket d), run starts
        uint64_t rsv = 0;
        const uint32_t d = threadIdx.x;
        if (d < F1 && bcur[d] != DEAD) {
            const uint32_t h = hist[d], L0 = cnt[d];
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (((L0 + BLK - 1) & ~(BLK - 1)) >> blk_sh);
            if (need) rsv = atomicAdd(&bkt_cur[d], (unsigned long long)need * BLK);
        }
        if (threadIdx.x < 64) {
            // rows of 64 buckets (conflict-free), four wave scans; lstart =
            // the run's first record slot (region start + leading hole)
            const uint32_t lane = threadIdx.x;
            uint32_t rs[4], incl[4], par[4];
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                const uint32_t b = 64 * t + lane;
                const uint32_t h = b < F1 ? hist[b] : 0u;
                par[t] = b < F1 ? (cnt[b] & 1u) : 0u;
                rs[t] = h ? (h + par[t] + 1u) & ~1u : 0u;
                incl[t] = rs[t];
            }
            for (int dd = 1; dd < 64; dd <<= 1) {
#pragma unroll
                for (uint32_t t = 0; t < 4; t++) {
                    const uint32_t y = __shfl_up(incl[t], dd, 64);
                    if (lane >= (uint32_t)dd) incl[t] += y;
                }
            }
            uint32_t base = 0;
#pragma unroll
            for (uint32_t t = 0; t < 4; t++) {
                const uint32_t b = 64 * t + lane;
                if (b < F1) lstart[b] = base + incl[t] - rs[t] + par[t];
                base += __shfl(incl[t], 63, 64);
            }
            if (lane == 0) s_misc[1] = base;   // slots of the tile (even)
        }
        block_sync();
        // ---- P2: staging; placement constants; bucket state advanced
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            if (off[q] != ~0u) {
                const uint32_t b = (br[q] >> 13) & 1023u;
                const uint32_t pos = lstart[b] + (br[q] & 8191u);
                slot[pos] = (uint64_t)((b << 16) | ((br[q] >> 23) * L1_THREADS + threadIdx.x)) << 32 | off[q];
            }
        }
        if (!last && threadIdx.x < L1F_TW) s_tw[((ti + 1) & 1) * L1F_TW + threadIdx.x] = tw_next;
        if (top && threadIdx.x == 0) s_misc[0] = (uint32_t)min<unsigned long long>(qn + 2ull * gridDim.x, nchunks);
        if (d < F1) {
            const uint32_t h = hist[d];
            if (h || last) {
                const uint32_t L0 = cnt[d];
                const uint32_t split = (L0 + BLK - 1) & ~(BLK - 1);
                const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (split >> blk_sh);
                const uint64_t bc = bcur[d];
                uint64_t nb = 0;
                if (bc == DEAD) {
                    nb = DEAD;
                } else if (need) {
                    nb = rsv;
                    if (nb + (uint64_t)need * BLK > bkt_base[d + 1]) {
                        atomicOr((unsigned long long *)&ctr[CTR_ERR], 8ull);
                        nb = DEAD;
                    }
                }
                const uint32_t e = L0 + h, fe = last ? e : (e & ~1u);
                if ((L0 & 1) && fe > L0 - 1 && bc != DEAD && !(KH_ABL(P, 16))) rec[bc + ((L0 - 1) & (BLK - 1))] = tail[d];   // 16: the tails were never written
                const uint32_t q0 = lstart[d];
                if (h) {
                    if (L0 & 1) slot[q0 - 1] = (uint64_t)((d << 16) | SLOT_EMPTY) << 32;
                    if ((q0 + h) & 1) slot[q0 + h] = (uint64_t)((d << 16) | SLOT_EMPTY) << 32;
                }
                const bool dead = bc == DEAD || nb == DEAD;
                dl[2 * d] = bc + (L0 & (BLK - 1)) - q0;
                dl[2 * d + 1] = nb + L0 - split - q0;
                qq[d] = make_uint2(q0 + (split - L0), dead ? 0 : q0 + (fe > L0 ? fe - L0 : 0));
                // the bucket's state after this tile (the write-out below reads
                // only dl / qq / slot, and tail for unpaired last records)
                if (h) {
                    if (nb == DEAD) bcur[d] = DEAD;
                    else if (need) bcur[d] = nb + (uint64_t)(need - 1) * BLK;
                    cnt[d] = e;
                    hist[d] = 0;
                }
            }
        }
        block_sync();
        // ---- P3: write-out of the staged tile
        {
            const uint32_t nslot = s_misc[1];
            const ulonglong2 *slot2 = (const ulonglong2 *)slot;
            const ulonglong2 *dl2 = (const ulonglong2 *)dl;
            for (uint32_t m = threadIdx.x; 2 * m < nslot; m += L1_THREADS) {
                const ulonglong2 sp = slot2[m];
                const uint32_t bj0 = (uint32_t)(sp.x >> 32), bj1 = (uint32_t)(sp.y >> 32);
                const uint32_t dd = bj0 >> 16;
                const uint2 ql = qq[dd];
                const ulonglong2 dv = dl2[dd];
                const uint32_t q = 2 * m;
                const bool r0 = (bj0 & 0xFFFFu) != SLOT_EMPTY, r1 = (bj1 & 0xFFFFu) != SLOT_EMPTY;
                const uint64_t v0 = ((jbase + j0 + (bj0 & 0xFFFFu)) << 32) | (uint32_t)sp.x;
                const uint64_t v1 = ((jbase + j0 + (bj1 & 0xFFFFu)) << 32) | (uint32_t)sp.y;
                const uint64_t o = (q >= ql.x ? dv.y : dv.x) + q;
                if (KH_ABL(P, 16)) continue;   // timing only: no run writes (as k_scatter_l1f)
                if (q < ql.y) {
                    if (r0 && r1) *(ulonglong2 *)(rec + o) = make_ulonglong2(v0, v1);
                    else if (r0) rec[o] = v0;
                    else if (r1) rec[o + 1] = v1;
                } else if (r0) {
                    tail[dd] = v0;
                }
            }
        }
        // ---- P3: the iterator moves on; hash + rank of the next tile
        if (last) break;
        if (hj1 >= hce) {   // into chunk cb (its successor published in P2 of its predecessor's top tile)
            hce = min(nkmers, (uint64_t)cb * CK + CK);
            cb = uniform_u32(s_misc[0]);
            htop = true;
        } else {
            htop = false;
        }
        hj0 = n0;
        hj1 = n1;
        next_tile(hj1, &n0, &n1);
        if (htop && threadIdx.x == 0) qn = atomicAdd((unsigned long long *)&ctr[CTR_L1Q], 1ull);
        if (n1 > n0 && threadIdx.x < tile_nw(n0, n1)) tw_next = src.words[tile_w0(n0) + threadIdx.x];
        hash_rank(hj0, hj1, hist2 + ((ti + 1) & 1) * F1a, (ti + 1) & 1);
        block_sync();
    }
    block_sync();
    for (uint32_t y = threadIdx.x; y < F1 * BLK; y += blockDim.x) {
        const uint32_t dd = y >> blk_sh, sl = y & (BLK - 1);
        const uint32_t c = cnt[dd] & (BLK - 1);
        if (c == 0 || sl < c || bcur[dd] == DEAD) continue;
        rec[bcur[dd] + sl] = ~0ull;
    }
}
__host__ __device__ constexpr size_t lds_l1p(size_t F1a, int rpt) {
    return 2 * L1F_TW * 8 + F1a * 8 * 4 + ((size_t)L1_THREADS * rpt + 2 * F1a) * 8 + F1a * 4 * 6 + 16;
}

// ---------------------------------------------------------------------------
// Level 1 of a shard ("owned filter").  A shard of a G-rank group owns ~1/G
// of every table's bins but hashes every k-mer of the stream, so with
// k_hist_l1 + k_scatter_l1 it would hash each k-mer twice and run the whole
// tile machinery of scatter_l1 for ~1/G useful records.  k_own_filter hashes
// every k-mer once and keeps only the owned records, (j << 32) | G with the
// local bin id G < 2^32.  They collect in an LDS buffer of OWN_BUF records
// (tile-wide scan for the slots) that is flushed as one contiguous run, so
// one returning global atomic reserves output space per ~OWN_BUF records (a
// per-tile atomic on the single counter serialised at ~12 ns each).  Records
// past `cap` are counted but not written; the host then re-runs the filter
// into a larger buffer.  k_hist_rec and k_scatter_l1<..., PRE> (the level-1
// tiles without hashing) bucket the record stream into the same bucket-major
// level-1 layout, so everything after level 1 is unchanged.
constexpr int OWN_BUF = 8192;
constexpr int OWN_RPT = 16;   // record slots per thread per tile
template <class Src, int KPT>
__global__ void __launch_bounds__(L1_THREADS) k_own_filter(Params P, Src src, uint64_t nkmers, uint32_t ck, int t0,
                                                          int nt, uint64_t cap, uint64_t *out,
                                                          unsigned long long *count) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *buf = (uint64_t *)smem;                     // [OWN_BUF]
    uint32_t *s_wtot = (uint32_t *)(buf + OWN_BUF);       // [2][16] (tile parity)
    unsigned long long *s_base = (unsigned long long *)(s_wtot + 32);
    uint64_t *s_meta = (uint64_t *)(s_base + 1);
    uint64_t *s_koff = s_meta + 2;
    constexpr int TILE_KMERS = L1_THREADS * KPT;
    constexpr int TPK = OWN_RPT / KPT;   // table slots per k-mer
    static_assert(L1_THREADS * OWN_RPT <= OWN_BUF, "a tile must fit the buffer");
    const uint64_t c0 = (uint64_t)blockIdx.x * ck;
    const uint64_t c1 = min(nkmers, c0 + ck);
    const bool pre = !needs_window(src);
    typename Src::Pend pend[KPT];
    if (pre) {
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = c0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            if (j < min(c1, c0 + TILE_KMERS)) pend[a] = kmer_fetch(src, j);
        }
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nwaves = blockDim.x >> 6;
    // buffered records -> out (all threads; nb block-uniform)
    auto flush = [&](uint32_t nb) {
        if (threadIdx.x == 0) *s_base = atomicAdd(count, (unsigned long long)nb);
        block_sync();
        const uint64_t base = *s_base;
        for (uint32_t x = threadIdx.x; x < nb; x += blockDim.x)
            if (base + x < cap) out[base + x] = buf[x];
        block_sync();
    };
    uint32_t nb = 0;   // records in buf
    const uint32_t ntiles = uniform_u32((uint32_t)((c1 - c0 + TILE_KMERS - 1) / TILE_KMERS));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t j0 = c0 + (uint64_t)ti * TILE_KMERS;
        const uint64_t j1 = min(c1, j0 + TILE_KMERS);
        // (no barrier needed here on the fixed-length path: the per-tile
        // wave totals alternate between two slots, and buf is only read by
        // flush(), which synchronises around its reads)
        TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
        uint64_t v[OWN_RPT];
        uint32_t own = 0;   // bit q: record slot q is owned here
        uint64_t hh[KPT];
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            hh[a] = j < j1 ? (pre ? src.finish(pend[a]) : kmer_hash(src, s_koff, tr, j)) : 0;
        }
        if (pre) {
            const uint64_t n0 = j0 + TILE_KMERS, n1 = min(c1, n0 + TILE_KMERS);
#pragma unroll
            for (int a = 0; a < KPT; a++) {
                const uint64_t j = n0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                if (j < n1) pend[a] = kmer_fetch(src, j);
            }
        }
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
#pragma unroll
            for (int i = 0; i < TPK; i++) {
                uint64_t G;
                if (i < nt && j < j1 && !(KH_ABL(P, 128)) && local_bin(P, t0 + i, hh[a], &G)) {
                    v[a * TPK + i] = (j << 32) | G;
                    own |= 1u << (a * TPK + i);
                }
            }
        }
        // tile-wide exclusive scan of the per-thread counts
        uint32_t *wt = s_wtot + (ti & 1) * 16;
        const uint32_t c = __builtin_popcount(own);
        uint32_t incl = c;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        if (lane == 63) wt[wave] = incl;
        block_sync();
        uint32_t tot = 0, pos = incl - c;
        for (uint32_t w = 0; w < nwaves; w++) {
            const uint32_t x = wt[w];
            tot += x;
            if (w < wave) pos += x;
        }
        tot = uniform_u32(tot);
        if (nb + tot > (uint32_t)OWN_BUF) {
            flush(nb);
            nb = 0;
        }
        pos += nb;
#pragma unroll
        for (int q = 0; q < OWN_RPT; q++)
            if ((own >> q) & 1) buf[pos + __builtin_popcount(own & ((1u << q) - 1))] = v[q];
        nb += tot;
    }
    block_sync();
    if (nb) flush(nb);
}

// Level 1 of a shard in one kernel: k_own_filter's owned-record filter feeding
// k_scatter_l1f's fixed-capacity bucket placement.  Each filter tile hashes
// KPT k-mers per thread and appends the owned records (j << 32 | local bin)
// to an LDS buffer; whenever it holds OWN_BATCH records they are
// counting-sorted by bucket in LDS and appended to the workgroup's blocks
// exactly as in k_scatter_l1f (2-record tails, one returning atomic per
// (bucket, batch, new block)).  The owned records never make the round trip
// through HBM that k_own_filter + k_hist_rec + k_scatter_l1<PRE> take.
// records sorted per batch: 2048 keeps the kernel at ~68 KB of LDS at
// F1 = 240 (an 8-way shard), two workgroups per CU (4096: one)
constexpr int OWN_BATCH = L1_THREADS * 4;
constexpr int OWN_FSLOTS = 8;                                  // candidate records per thread per filter tile
constexpr int OWNF_BUF = OWN_BATCH + L1_THREADS * OWN_FSLOTS;  // < OWN_BATCH left + one filter tile
template <class Src, int KPT, bool TW_ = false>
__global__ void __launch_bounds__(L1_THREADS) k_own_l1f(Params P, Src src, uint64_t nkmers, uint64_t kpw, int t0,
                                                       int nt, const uint64_t *bkt_base, unsigned long long *bkt_cur,
                                                       uint64_t *rec, uint64_t *ctr, int blk_sh, uint32_t cht) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RPT = OWN_BATCH / L1_THREADS;
    constexpr int FSLOTS = OWN_FSLOTS;
    constexpr int TPK = FSLOTS / KPT;                  // table slots per k-mer
    constexpr int TILE_KMERS = L1_THREADS * KPT;
    const uint32_t BLK = 1u << blk_sh;
    constexpr uint64_t DEAD = ~0ull;
    const uint32_t F1 = P.F1;
    const uint32_t F1a = (F1 + 3) & ~3u;
    uint64_t *buf = (uint64_t *)smem;                  // [OWNF_BUF] owned records; a batch is its own stage while sorted
    uint64_t *bcur = buf + OWNF_BUF;                   // [F1] partially filled block (DEAD: overflowed)
    uint64_t *nbase = bcur + F1a;                      // [F1] blocks reserved for this batch
    uint64_t *dl = nbase + F1a;                        // [F1][2] output - LDS position: current block, new blocks
    uint64_t *tail = dl + 2 * F1a;                     // [F1] a pending odd record
    uint32_t *cnt = (uint32_t *)(tail + F1a);          // [F1] records appended by this workgroup
    uint32_t *hist = cnt + F1a;                        // [F1]
    uint32_t *lstart = hist + F1a;                     // [F1]
    uint2 *qq = (uint2 *)(lstart + F1a);               // [F1] (first LDS position in the new blocks, first left for the tail)
    uint16_t *sb = (uint16_t *)(qq + F1a);             // [OWN_BATCH] bucket of each stage slot
    uint32_t *s_wtot = (uint32_t *)(sb + OWN_BATCH);   // [3][16]: filter scans (tile parity), batch scan
    // TW: the filter tile's packed words staged in LDS as in k_scatter_l1f
    // (the next tile's words loaded one tile ahead, one word per thread)
    constexpr bool TW = TW_ && std::is_same<Src, SrcTwoBit>::value;
    uint64_t *s_tw = (uint64_t *)(s_wtot + 48);        // [2][L1F_TW] (8-B aligned: F1a and OWN_BATCH are)
    const int shift = P.s0 + P.s2;
    const uint64_t omask = (1ull << shift) - 1;
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) {
        bcur[b] = 0;
        cnt[b] = 0;
        hist[b] = 0;
    }
    // chunks of CK k-mers: a fixed share per workgroup (cht == 0) or chunks of
    // cht tiles from the queue head ctr[CTR_L1Q], as in k_scatter_l1f
    const uint64_t CK = cht ? (uint64_t)cht * TILE_KMERS : kpw;
    const uint32_t nchunks = (uint32_t)((nkmers + CK - 1) / CK);
    uint32_t cb = cht ? blockIdx.x + gridDim.x : nchunks;
    uint64_t j0 = min(nkmers, (uint64_t)blockIdx.x * CK);
    uint64_t ce = min(nkmers, j0 + CK);
    bool chunk_top = true;
    uint32_t *s_q = s_wtot + 47;   // the batch scan uses s_wtot[32, 32 + waves)
    static_assert(L1_THREADS / 64 <= 15, "k_own_l1f: the batch scan's wave totals would overwrite s_q");
    static_assert(L1_THREADS / 64 <= 16, "k_own_l1f: the tile scans use 16 wave-total slots per parity");
    constexpr int NPEND = TW ? 1 : KPT;
    typename Src::Pend pend[NPEND];
    if (!TW) {
#pragma unroll
        for (int a = 0; a < NPEND; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            if (j < min(ce, j0 + TILE_KMERS)) pend[a] = kmer_fetch(src, j);
        }
    }
    auto tile_w0 = [&](uint64_t j0) -> uint64_t {
        const uint64_t ja = j0 + src.kbase;
        return ((ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2) >> 6;
    };
    auto tile_nw = [&](uint64_t j0, uint64_t j1) -> uint32_t { return (uint32_t)(tile_w0(j1 - 1) + 2 - tile_w0(j0)); };
    uint64_t tw_next = 0;
    if constexpr (TW) {
        if (ce > j0) {
            const uint64_t e = min(ce, j0 + TILE_KMERS);
            if (threadIdx.x < tile_nw(j0, e)) s_tw[threadIdx.x] = src.words[tile_w0(j0) + threadIdx.x];
        }
        block_sync();
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nwaves = blockDim.x >> 6;

    // sort buf[o, o + n) by bucket and append it (last: flush every pending tail)
    auto sort_batch = [&](uint32_t o, uint32_t n, bool last) {
        uint64_t *bb = buf + o;
        uint32_t off[RPT], br[RPT], jv[RPT];
#pragma unroll
        for (int u = 0; u < RPT; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * L1_THREADS;
            off[u] = ~0u;
            br[u] = 0;
            jv[u] = 0;
            if (q < n) {
                const uint64_t x = bb[q];
                const uint32_t G = (uint32_t)x, b = G >> shift;
                off[u] = G & (uint32_t)omask;
                jv[u] = (uint32_t)(x >> 32);
                br[u] = (b << 13) | atomicAdd(&hist[b], 1u);
            }
        }
        block_sync();   // every record is in registers: bb[0, n) becomes the stage
        block_scan_hist(hist, lstart, F1, s_wtot + 32);
        block_sync();
#pragma unroll
        for (int u = 0; u < RPT; u++) {
            if (off[u] != ~0u) {
                const uint32_t b = br[u] >> 13;
                const uint32_t pos = lstart[b] + (br[u] & 8191u);
                bb[pos] = ((uint64_t)jv[u] << 32) | off[u];
                sb[pos] = (uint16_t)b;
            }
        }
        for (uint32_t d = threadIdx.x; d < F1; d += blockDim.x) {
            const uint32_t h = hist[d];
            if (!h && !last) continue;
            const uint32_t L0 = cnt[d];
            const uint32_t split = (L0 + BLK - 1) & ~(BLK - 1);
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (split >> blk_sh);
            uint64_t bc = bcur[d], nb = 0;
            if (bc == DEAD) {
                nb = DEAD;
            } else if (need) {
                nb = atomicAdd(&bkt_cur[d], (unsigned long long)need * BLK);
                if (nb + (uint64_t)need * BLK > bkt_base[d + 1]) {
                    atomicOr((unsigned long long *)&ctr[CTR_ERR], 8ull);
                    nb = DEAD;
                }
            }
            const uint32_t e = L0 + h, fe = last ? e : (e & ~1u);
            if ((L0 & 1) && fe > L0 - 1 && bc != DEAD) rec[bc + ((L0 - 1) & (BLK - 1))] = tail[d];
            const uint32_t q0 = lstart[d];
            const bool dead = bc == DEAD || nb == DEAD;
            nbase[d] = nb;
            dl[2 * d] = bc + (L0 & (BLK - 1)) - q0;
            dl[2 * d + 1] = nb + L0 - split - q0;
            qq[d] = make_uint2(q0 + (split - L0), dead ? 0 : q0 + (fe > L0 ? fe - L0 : 0));
        }
        block_sync();
#pragma unroll
        for (int u = 0; u < RPT; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * L1_THREADS;
            if (q >= n) continue;
            const uint32_t d = sb[q];
            const uint64_t v = bb[q];
            const uint2 ql = qq[d];
            if (q < ql.y) rec[dl[2 * d + (q >= ql.x ? 1 : 0)] + q] = v;
            else tail[d] = v;   // the odd last record of the run (not on the last batch)
        }
        block_sync();
        for (uint32_t d = threadIdx.x; d < F1; d += blockDim.x) {
            const uint32_t h = hist[d];
            if (!h) continue;
            const uint32_t L0 = cnt[d];
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - ((L0 + BLK - 1) >> blk_sh);
            if (nbase[d] == DEAD) bcur[d] = DEAD;
            else if (need) bcur[d] = nbase[d] + (uint64_t)(need - 1) * BLK;
            cnt[d] = L0 + h;
            hist[d] = 0;
        }
        block_sync();
    };

    uint32_t nbuf = 0;   // records in buf (block-uniform)
    bool flushed_last = false;
    for (uint32_t ti = 0; j0 < ce; ti++) {
        const uint64_t j1 = min(ce, j0 + TILE_KMERS);
        // the next tile [n0, n1): in this chunk, else the first of chunk cb
        uint64_t n0 = j1, n1 = j1;
        if (j1 < ce) {
            n1 = min(ce, j1 + TILE_KMERS);
        } else if (cb < nchunks) {
            n0 = (uint64_t)cb * CK;
            n1 = min(nkmers, n0 + min(CK, (uint64_t)TILE_KMERS));
        }
        const bool more = n1 > n0;   // a next tile exists
        unsigned long long qn = 0;
        if (cht && chunk_top && threadIdx.x == 0) qn = atomicAdd((unsigned long long *)&ctr[CTR_L1Q], 1ull);
        uint64_t v[FSLOTS];
        uint32_t own = 0;   // bit q: record slot q is owned here
        uint64_t hh[KPT];
        const uint64_t *tw_cur = s_tw + (ti & 1) * L1F_TW;
        if constexpr (TW) {
            const uint64_t tw_w0 = tile_w0(j0);
#pragma unroll
            for (int a = 0; a < KPT; a++) {
                const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                uint64_t h = 0;
                if (j < j1) {
                    const uint64_t ja = j + src.kbase;
                    const uint64_t bpos = (ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2;
                    const uint32_t wi = (uint32_t)((bpos >> 6) - tw_w0);
                    h = src.finish(SrcTwoBit::Pend{tw_cur[wi], tw_cur[wi + 1], (uint32_t)(bpos & 63)});
                }
                hh[a] = h;
            }
            if (more) {   // the next tile's words (stored after this tile's scan barrier)
                if (threadIdx.x < tile_nw(n0, n1)) tw_next = src.words[tile_w0(n0) + threadIdx.x];
            }
        } else {
#pragma unroll
            for (int a = 0; a < KPT; a++) {
                const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                hh[a] = j < j1 ? src.finish(pend[a]) : 0;
            }
#pragma unroll
            for (int a = 0; a < NPEND; a++) {
                const uint64_t j = n0 + (uint64_t)a * L1_THREADS + threadIdx.x;
                if (j < n1) pend[a] = kmer_fetch(src, j);
            }
        }
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
#pragma unroll
            for (int i = 0; i < TPK; i++) {
                uint64_t G;
                if (i < nt && j < j1 && !(KH_ABL(P, 128)) && local_bin(P, t0 + i, hh[a], &G)) {
                    v[a * TPK + i] = (j << 32) | G;
                    own |= 1u << (a * TPK + i);
                }
            }
        }
        // tile-wide exclusive scan of the per-thread counts
        uint32_t *wt = s_wtot + (ti & 1) * 16;
        const uint32_t c = __builtin_popcount(own);
        uint32_t incl = c;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        if (lane == 63) wt[wave] = incl;
        block_sync();
        uint32_t tot = 0, pos = incl - c;
        for (uint32_t w = 0; w < nwaves; w++) {
            const uint32_t x = wt[w];
            tot += x;
            if (w < wave) pos += x;
        }
        tot = uniform_u32(tot);
        pos += nbuf;
#pragma unroll
        for (int q = 0; q < FSLOTS; q++)
            if ((own >> q) & 1) buf[pos + __builtin_popcount(own & ((1u << q) - 1))] = v[q];
        nbuf += tot;
        if (KH_ABL(P, 64)) nbuf = 0;   // timing only: the filter without the bucket placement
        // buffer (ti + 1) & 1 was last read in tile ti - 1, before this tile's scan barrier
        if (TW && more && threadIdx.x < L1F_TW) s_tw[((ti + 1) & 1) * L1F_TW + threadIdx.x] = tw_next;
        // the chunk taken from the queue (after this tile's first barrier:
        // every thread has read the previous value), read after the next one
        if (cht && chunk_top && threadIdx.x == 0) *s_q = (uint32_t)min<unsigned long long>(qn + 2ull * gridDim.x, nchunks);
        block_sync();
        const bool lt = !more;
        uint32_t o = 0;   // batches buf[o, o + OWN_BATCH) in order; the rest (< OWN_BATCH) moves to the front
        while (nbuf - o >= (uint32_t)OWN_BATCH || (lt && !flushed_last)) {
            const uint32_t n = min(nbuf - o, (uint32_t)OWN_BATCH);
            const bool last = lt && nbuf - o == n;
            sort_batch(o, n, last);
            flushed_last = last;
            o += n;
        }
        if (o) {   // the rest is shorter than o: source and destination do not overlap
            for (uint32_t x = threadIdx.x; x < nbuf - o; x += blockDim.x) buf[x] = buf[o + x];
            nbuf -= o;
            block_sync();
        }
        // advance: the next tile of this chunk, or the first of chunk cb
        chunk_top = j1 >= ce;
        if (chunk_top) {
            j0 = n0;
            ce = cb < nchunks ? min(nkmers, (uint64_t)cb * CK + CK) : n0;
            cb = cht ? uniform_u32(*s_q) : nchunks;
        } else {
            j0 = j1;
        }
    }
    block_sync();
    for (uint32_t y = threadIdx.x; y < F1 * BLK; y += blockDim.x) {
        const uint32_t d = y >> blk_sh, sl = y & (BLK - 1);
        const uint32_t c = cnt[d] & (BLK - 1);
        if (c == 0 || sl < c || bcur[d] == DEAD) continue;
        rec[bcur[d] + sl] = ~0ull;
    }
}

// per-chunk bucket histogram of a flat record stream: chunk c = records
// [c * L2_CHUNK, ...), destination (uint32)record >> shift; M[d * nch + c]
__global__ void __launch_bounds__(PT_THREADS) k_hist_rec(const uint64_t *rec, uint64_t n, uint32_t F, int shift,
                                                        uint32_t nch, uint32_t *M) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) hist[d] = 0;
    block_sync();
    const uint64_t r0 = (uint64_t)blockIdx.x * L2_CHUNK, r1 = min(n, r0 + L2_CHUNK);
    const uint32_t *rec32 = (const uint32_t *)rec;   // low words = local bin ids
    for (uint64_t q = r0 + threadIdx.x; q < r1; q += blockDim.x) atomicAdd(&hist[rec32[2 * q] >> shift], 1u);
    block_sync();
    for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) M[(uint64_t)d * nch + blockIdx.x] = hist[d];
}

// ---------------------------------------------------------------------------
// level 2: chunk t of the level-1 output lies in bucket b (ch2[b] <= t < ch2[b+1])
struct L2Chunk {
    uint32_t b, c, nc;
    uint64_t r0, r1;
};

__device__ __forceinline__ bool l2_chunk(uint32_t F1, const uint64_t *off1, const uint32_t *ch2, L2Chunk *k) {
    const uint32_t t = blockIdx.x;
    if (t >= ch2[F1]) return false;
    uint32_t lo = 0, hi = F1;  // largest lo with ch2[lo] <= t (a non-empty bucket)
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (ch2[mid] <= t) lo = mid; else hi = mid;
    }
    k->b = lo;
    k->c = t - ch2[lo];
    k->nc = ch2[lo + 1] - ch2[lo];
    k->r0 = off1[lo] + (uint64_t)k->c * L2_CHUNK;
    k->r1 = min(off1[lo + 1], k->r0 + L2_CHUNK);
    return true;
}

// matrix layout: bucket b, region r, chunk c -> ch2[b]*F2 + r*nc + c; one
// exclusive scan over it gives absolute level-2 offsets (bucket b starts at
// off1[b] automatically)
__global__ void __launch_bounds__(PT_THREADS) k_hist_l2(uint32_t F1, int s0, int s2, const uint64_t *off1,
                                                       const uint32_t *ch2, const uint64_t *rec, uint32_t *M2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *hist = (uint32_t *)smem;
    const uint32_t F2 = 1u << s2;
    L2Chunk k;
    if (!l2_chunk(F1, off1, ch2, &k)) return;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) hist[r] = 0;
    block_sync();
    const uint32_t *rec32 = (const uint32_t *)rec;   // low words = offsets
    for (uint64_t q = k.r0 + threadIdx.x; q < k.r1; q += blockDim.x) atomicAdd(&hist[rec32[2 * q] >> s0], 1u);
    block_sync();
    const uint64_t base = (uint64_t)ch2[k.b] * F2 + k.c;
    for (uint32_t r = threadIdx.x; r < F2; r += blockDim.x) M2[base + (uint64_t)r * k.nc] = hist[r];
}

// region offsets for the apply step
__global__ void k_off2(uint32_t F1, int s2, const uint64_t *off1, const uint32_t *ch2, const uint64_t *O2,
                       uint64_t *off2) {
    const uint32_t F2 = 1u << s2;
    const uint64_t nreg = (uint64_t)F1 * F2;
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < nreg; g += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(g >> s2), r = (uint32_t)(g & (F2 - 1));
        const uint32_t nc = ch2[b + 1] - ch2[b];
        off2[g] = nc ? O2[(uint64_t)ch2[b] * F2 + (uint64_t)r * nc] : off1[b];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) off2[nreg] = off1[F1];
}

// Level-2 scatter, register-direct: no LDS staging; each record goes from
// registers to its region cursor + tile rank.  The records of one region in a
// tile are written together, so L2 completes their lines; only whole aligned
// 128-B segments (SEG = 16 records) are written, remainders wait in LDS tails
// (random 128-B runs stream at ~5 TB/s on MI355X, 64-B runs at ~3 TB/s).
template <int THREADS, int SEG, int RPT>
__global__ void __launch_bounds__(THREADS) k_scatter_l2(uint32_t F1, int s0, int s2, const uint64_t *off1,
                                                        const uint32_t *ch2, const uint64_t *O2,
                                                        const uint64_t *rec_in, uint64_t *rec_out) {
    constexpr int TILE = THREADS * RPT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F2 = 1u << s2;
    uint64_t *lcur = (uint64_t *)smem;             // [F2]
    uint64_t *tail = lcur + F2;                    // [F2*SEG]
    uint32_t *hist = (uint32_t *)(tail + F2 * SEG);  // [F2]
    uint32_t *nflush = hist + F2;                  // [2]
    uint16_t *flist = (uint16_t *)(nflush + 2);    // [F2]
    uint8_t *hskip = (uint8_t *)(flist + ((F2 + 1) & ~1u));  // [F2]
    const Emit<uint64_t, SEG> em{lcur, hskip, tail, hist, nullptr, nullptr, nullptr, flist, nflush};
    const uint64_t rmask = (1ull << s0) - 1;
    L2Chunk k;
    if (!l2_chunk(F1, off1, ch2, &k)) return;
    const uint64_t base = (uint64_t)ch2[k.b] * F2 + k.c;
    for (uint32_t r = threadIdx.x; r < F2; r += THREADS) em.init(r, O2[base + (uint64_t)r * k.nc]);
    if (threadIdx.x == 0) *nflush = 0;
    uint64_t v[RPT];
#pragma unroll
    for (int q = 0; q < RPT; q++) {
        const uint64_t idx = k.r0 + (uint64_t)q * THREADS + threadIdx.x;
        v[q] = idx < min(k.r1, k.r0 + TILE) ? rec_in[idx] : ~0ull;
    }
    const uint32_t ntiles = uniform_u32((uint32_t)((k.r1 - k.r0 + TILE - 1) / TILE));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t t0 = k.r0 + (uint64_t)ti * TILE;
        const bool last = ti + 1 == ntiles;
        block_sync();
        uint32_t rank[RPT];
        uint64_t x[RPT];
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            x[q] = v[q];
            if (x[q] != ~0ull) {
                rank[q] = atomicAdd(&hist[(uint32_t)x[q] >> s0], 1u);
                em.note((uint32_t)x[q] >> s0, rank[q], last);
            }
        }
        {
            const uint64_t n0 = t0 + TILE, n1 = min(k.r1, n0 + TILE);
#pragma unroll
            for (int q = 0; q < RPT; q++) {
                const uint64_t idx = n0 + (uint64_t)q * THREADS + threadIdx.x;
                v[q] = idx < n1 ? rec_in[idx] : ~0ull;
            }
        }
        block_sync();
        em.flush_listed(F2, last, rec_out);
        block_sync();
#pragma unroll
        for (int q = 0; q < RPT; q++)
            if (x[q] != ~0ull)
                em.put_rank((uint32_t)x[q] >> s0, rank[q], (x[q] & ~0xFFFFFFFFull) | (x[q] & rmask), last, rec_out);
        block_sync();
        em.advance(F2, last);
    }
}

// ---------------------------------------------------------------------------
// Level-2 scatter into fixed-capacity regions: no histogram pass over the
// level-1 records.  Region g owns [reg_base[g], reg_base[g+1]), sized on the
// host from its expected record count (+8 sigma and the partial blocks).
// Workgroup (b, p) takes part p of bucket b's level-1 records and appends to
// the bucket's regions in blocks of L2F_BLK records: one returning atomic per
// (region, tile) on reg_cur[g] reserves every block the tile needs, so a
// block is owned by one workgroup and records keep the register-direct
// 128-B segment writes of k_scatter_l2 (partial segments wait in LDS tails).
// After the last tile the rest of each partially filled block is set to the
// ~0 sentinel that every consumer skips; region g's records are then
// [reg_base[g], reg_cur[g]).  A reservation past the region's capacity (a
// skewed input) sets ctr[CTR_ERR] bit 4, writes nothing for that region, and
// the host redoes the pass's level 2 with the exact histogram path.
//
// (Round 5 measured spare blocks reserved one tile ahead -- each thread
// keeping a reserved block of its region in a register so a tile rarely
// waits for its reservation atomic: 93.7 against 90.1 ms/step on one box,
// VGPRs 94 -> 102; not kept)
constexpr int L2F_BLK_SH = 6;   // default block: 64 records (KH_L2F_BLK_SH)
constexpr uint64_t L2F_DEAD = ~0ull;

template <int THREADS, int RPT>
__global__ void __launch_bounds__(THREADS) k_scatter_l2f(uint32_t nbk, int s0, int s2, uint32_t parts,
                                                         const uint64_t *bstart, const uint64_t *bend,
                                                         const uint64_t *reg_base,
                                                         unsigned long long *reg_cur, const uint64_t *rec_in,
                                                         uint64_t *rec_out, uint64_t *ctr, int blk_sh) {
    constexpr int TILE = THREADS * RPT;
    constexpr uint32_t SEG = 16;
    const uint32_t BLK = 1u << blk_sh;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t F2 = 1u << s2;
    uint64_t *bcur = (uint64_t *)smem;              // [F2] base of the partially filled block (DEAD: overflowed)
    uint64_t *nbase = bcur + F2;                    // [F2] base of the blocks reserved for this tile
    uint64_t *tail = nbase + F2;                    // [F2*SEG] pending partial segments
    uint32_t *cnt = (uint32_t *)(tail + F2 * SEG);  // [F2] records appended by this workgroup
    uint32_t *hist = cnt + F2;                      // [F2] this tile's records
    uint32_t *s_nfl = hist + F2;                    // [1] entries of flist (F2 <= THREADS)
    uint16_t *flist = (uint16_t *)(s_nfl + 4);      // [F2] regions whose pending tail completes this tile
    // A level-1 bucket that overflowed (ctr bit 8) left bkt_cur past its
    // capacity with unwritten slots below it: nothing of this pass's level 1
    // may be read; the host redoes the pass on the exact path.
    if (__builtin_amdgcn_readfirstlane((uint32_t)ctr[CTR_ERR]) & 8u) return;
    // segment b: records [bstart[b], bend[b]) of level-1 bucket b % nbk (one
    // segment per bucket, or per (source, bucket) on an exchange-mode owner)
    const uint32_t b = blockIdx.x / parts, p = blockIdx.x % parts;
    const uint64_t b0 = bstart[b], b1 = min(bend[b], bstart[b + 1]);
    // parts of an even length: every tile starts on a 16-B record pair
    // (bucket bases are block-aligned), loaded with one 16-B load per pair
    const uint64_t len = ((b1 - b0 + parts - 1) / parts + 1) & ~1ull;
    const uint64_t r0 = min(b1, b0 + (uint64_t)p * len), r1 = min(b1, r0 + len);
    const uint64_t gb = (uint64_t)(b % nbk) << s2;
    auto load_tile = [&](uint64_t n0, uint64_t *v) {
        const uint64_t n1 = min(r1, n0 + TILE);
#pragma unroll
        for (int q = 0; q < RPT / 2; q++) {
            const uint64_t idx = n0 + 2 * ((uint64_t)q * THREADS + threadIdx.x);
            ulonglong2 x = make_ulonglong2(~0ull, ~0ull);
            if (idx < n1) x = *(const ulonglong2 *)(rec_in + idx);
            v[2 * q] = x.x;
            v[2 * q + 1] = idx + 1 < n1 ? x.y : ~0ull;
        }
    };
    const uint64_t rmask = (1ull << s0) - 1;
    for (uint32_t d = threadIdx.x; d < F2; d += THREADS) {
        bcur[d] = 0;
        cnt[d] = 0;
        hist[d] = 0;
    }
    if (threadIdx.x == 0) *s_nfl = 0;
    // output slot of this workgroup's record number L of region d (this tile)
    auto phys = [&](uint32_t d, uint32_t L) -> uint64_t {
        const uint32_t split = (cnt[d] + BLK - 1) & ~(BLK - 1);
        if (L < split) return bcur[d] == L2F_DEAD ? L2F_DEAD : bcur[d] + (L & (BLK - 1));
        return nbase[d] == L2F_DEAD ? L2F_DEAD : nbase[d] + (L - split);
    };
    uint64_t v[RPT];
    load_tile(r0, v);
    PH_BEGIN(8);
    const uint32_t ntiles = uniform_u32((uint32_t)((r1 - r0 + TILE - 1) / TILE));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t t0 = r0 + (uint64_t)ti * TILE;
        const bool last = ti + 1 == ntiles;
        block_sync();
        PH(7);
        uint32_t rank[RPT];
        uint64_t x[RPT];
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            x[q] = v[q];
            if (x[q] != ~0ull) rank[q] = atomicAdd(&hist[(uint32_t)x[q] >> s0], 1u);
        }
        PH(0);
        load_tile(t0 + TILE, v);
        block_sync();
        PH(1);
        // blocks for this tile (one reservation per region that needs any) and
        // the list of regions whose pending tail segment completes in this
        // tile (every pending one on the last tile); F2 <= THREADS: thread d
        // owns region d
        // The reservations' results go to nbase here.  (-DKH_L2_LATE_NBASE
        // stores them only after the tail flush, to overlap the atomics'
        // latency with it: measured slower, 93.7-95.0 vs 90.2 ms/step, since
        // waiting for the atomic then also waits for the flush stores.)
        uint64_t nb = 0, nlim = ~0ull;
        uint32_t nneed = 0;
        {
            const uint32_t d = threadIdx.x;
            bool fl = false;
            if (d < F2) {
                const uint32_t h = hist[d], c0 = cnt[d];
                const bool dead = bcur[d] == L2F_DEAD;
                if (h) {
                    const uint32_t need = ((c0 + h + BLK - 1) >> blk_sh) - ((c0 + BLK - 1) >> blk_sh);
                    if (dead) {
                        nb = L2F_DEAD;
                    } else if (need) {
                        nb = atomicAdd(&reg_cur[gb + d], (unsigned long long)need * BLK);
                        nlim = reg_base[gb + d + 1];
                        nneed = need;
                    }
                }
#ifndef KH_L2_LATE_NBASE
                if (nneed && nb + (uint64_t)nneed * BLK > nlim) {
                    atomicOr((unsigned long long *)&ctr[CTR_ERR], 4ull);
                    nb = L2F_DEAD;
                }
                nbase[d] = nb;
#endif
                const uint32_t a = c0 & ~(SEG - 1), e = c0 + h;
                fl = !dead && c0 != a && (last ? e : (e & ~(SEG - 1))) > a;
            }
            const uint64_t m = __ballot(fl);
            if (m) {
                uint32_t base = 0;
                if ((threadIdx.x & 63) == 0) base = atomicAdd(s_nfl, (uint32_t)__popcll(m));
                base = __shfl(base, 0, 64);
                if (fl) flist[base + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63)) - 1))] = (uint16_t)d;
            }
        }
        PH(2);
        block_sync();
        PH(3);
        // flush the listed tails: 16 consecutive lanes per 128-B segment (its
        // slots [a, c0) are this workgroup's, inside its current block)
        {
            const uint32_t nfl = *s_nfl;
            for (uint32_t y = threadIdx.x; y < nfl * SEG; y += THREADS) {
                const uint32_t d = flist[y / SEG], sl = y % SEG;
                const uint32_t c0 = cnt[d], a = c0 & ~(SEG - 1);
                if (a + sl < c0) rec_out[bcur[d] + ((a + sl) & (BLK - 1))] = tail[d * SEG + sl];
            }
        }
#ifdef KH_L2_LATE_NBASE
        if (threadIdx.x < F2) {
            if (nneed && nb + (uint64_t)nneed * BLK > nlim) {
                atomicOr((unsigned long long *)&ctr[CTR_ERR], 4ull);
                nb = L2F_DEAD;
            }
            nbase[threadIdx.x] = nb;
        }
#endif
        PH(4);
        block_sync();   // the flushed tail slots are refilled below
        PH(5);
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            if (x[q] == ~0ull) continue;
            const uint32_t d = (uint32_t)x[q] >> s0;
            const uint32_t L = cnt[d] + rank[q];
            const uint32_t e = cnt[d] + hist[d];
            const uint64_t val = (x[q] & ~0xFFFFFFFFull) | (x[q] & rmask);
            if (L < (last ? e : (e & ~(SEG - 1)))) {
                const uint64_t pos = phys(d, L);
                if (pos != L2F_DEAD) rec_out[pos] = val;
            } else {
                tail[d * SEG + (L & (SEG - 1))] = val;
            }
        }
        PH(6);
        block_sync();
        if (threadIdx.x == 0) *s_nfl = 0;
        for (uint32_t d = threadIdx.x; d < F2; d += THREADS) {
            const uint32_t h = hist[d];
            if (!h) continue;
            const uint32_t c0 = cnt[d];
            const uint32_t need = ((c0 + h + BLK - 1) >> blk_sh) - ((c0 + BLK - 1) >> blk_sh);
            if (nbase[d] == L2F_DEAD) bcur[d] = L2F_DEAD;
            else if (need) bcur[d] = nbase[d] + (uint64_t)(need - 1) * BLK;
            cnt[d] = c0 + h;
            hist[d] = 0;
        }
    }
    PH_END(32, 8);
    // the rest of every partially filled block: sentinels
    block_sync();
    for (uint32_t y = threadIdx.x; y < F2 * BLK; y += THREADS) {
        const uint32_t d = y >> blk_sh, sl = y & (BLK - 1);
        const uint32_t c = cnt[d] & (BLK - 1);
        if (c == 0 || sl < c || bcur[d] == L2F_DEAD) continue;
        rec_out[bcur[d] + sl] = ~0ull;
    }
}

// every k-mer's hash of a batch into h[0, nkmers): a Murmur batch on the exact
// (two-pass) level 1 then reads its hashes twice instead of hashing twice
template <class Src>
__global__ void __launch_bounds__(256) k_hash_kmers(Src src, uint64_t nkmers, uint64_t *h) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < nkmers; j += (uint64_t)gridDim.x * blockDim.x)
        h[j] = kmer_hash_global(src, j);
}

// per-pass region cursors start at their region bases
__global__ void k_reg_reset(const uint64_t *reg_base, unsigned long long *reg_cur, uint64_t n) {
    for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x)
        reg_cur[g] = reg_base[g];
}

}  // namespace kh
