// kh_nearprime.cuh -- one level-1 record per k-mer for tables whose sizes are
// nearby primes (included by kh_engine.hip after kh_partition.cuh).
//
// khmer sizes its N tables with get_n_primes_near_x (include/oxli/
// hashtable.hh:99-123): the N largest primes just below x, so they differ by
// a few dozen.  With P the largest and d_i = P - p_i, a hash h = q P + r
// (q = h div P, r = h mod P) gives
//     h mod p_i = (r + q d_i) mod p_i,      r + q d_i < P + q_max d_max,
// and for 2-bit k-mers q_max = (4^k - 1) div P is small (C2: 4398, so every
// table's bin lies within 237,492 bins of r, one subtraction of p_i at most).
// So (r, q) determines all N bins of a k-mer (storage.hh:577's h % p_i for
// every table) and level 1 can bucket each k-mer ONCE, by r:
//
//   level 1 (k_scatter_n1): hash, (q, r) from one double multiply, bucket
//     b = (r >> s0) div R' (R' regions of 2^s0 bins a bucket), one LDS rank
//     atomic, one 8-byte record per k-mer:
//         record = (j - jb) << PB | q << OB | (r - b R' 2^s0)
//     where jb is the k-mer index base of the record's 256-record block
//     (blkj[block], written when the block is reserved; a block's records
//     come from one workgroup's tiles in increasing k-mer order and span less
//     than 2^(64 - PB) indices -- a partial block that would exceed that span
//     is closed with sentinels before the tile that would overflow it).
//   level 2 (k_scatter_n2): per level-1 bucket, expands each record into its
//     N region records (j << 32 | bin offset in its 2^s0-bin region): table
//     i's bins of bucket b lie in its regions [R' b, R' b + R' + E] (E
//     regions of spill, wrapping past p_i into regions 0 .. E), i.e. N x
//     Rloc <= 1024 destinations, the same fan-out as k_scatter_l2f.
//
// Level 1 writes 8 B per k-mer instead of 8 B per (k-mer, table) and does a
// quarter of the LDS rank atomics, staging and run writes at N = 4; level 2
// reads a quarter of the records it writes.  The region records, the apply
// and everything after are unchanged, so the tables and counters are the
// reference's exactly as before (storage.hh:571-624).
#pragma once
#include "kh_partition.cuh"

namespace kh {

constexpr int NP_MAXT = 4;        // tables of the near-prime path
constexpr int NP_KPT = 8;         // k-mers (= records) per thread per level-1 tile
constexpr int NP_TW = 192;        // packed words of a staged 4096-k-mer tile (read length >= ~60)
constexpr int NP_SLOT_B = 55;     // stage slot / register: bucket bits [55, 64)
constexpr int NP_SLOT_K = 42;     // tile index (or rank) bits [42, 55); payload bits [0, 42)
constexpr uint32_t NP_EMPTY = 0x1FFFu;
constexpr uint64_t NP_PAY = (1ull << NP_SLOT_K) - 1;
constexpr uint32_t NP_DEAD = 0xFFFFFFFFu;

// near-prime partition constants (host: np_geometry / np_bkt_plan)
struct NPGeo {
    uint64_t pm;                  // the largest table size P (h = q P + r)
    double ipm;                   // 1 / P
    uint32_t rp;                  // R': regions of 2^s0 bins per level-1 bucket
    uint32_t magic;               // ceil(2^32 / R'): bucket = umulhi(r >> s0, magic)
    uint32_t nb;                  // level-1 buckets
    uint32_t rloc;                // level-2 destinations per table (n * rloc <= 1024)
    int ob, pb;                   // offset bits, payload bits (offset + quotient) of a level-1 record
    uint32_t jlim;                // largest k-mer index span inside one level-1 block (2^(64 - pb) - 1, capped)
    int n, s0;
    int ablate;                   // Params::ablate (KH_ABL: -DKH_ABLATE development builds only)
    uint64_t cap;                 // level-1 records per bucket (a multiple of the block)
    uint64_t d[NP_MAXT];          // P - p_i
    uint64_t p[NP_MAXT];          // p_i
    uint32_t rt[NP_MAXT];         // regions of table i: ceil(p_i / 2^s0)
    uint32_t rbase[NP_MAXT];      // P.tbase[i] >> s0: the global region of table i's region 0
};

// q = h div P and r = h mod P from one double multiply (h < 2^53, q < 2^32):
// the estimate is exact or one off either way (as div_f64 / mod_f64_32)
__device__ __forceinline__ void np_divmod(uint64_t h, const NPGeo &N, uint32_t *q, uint64_t *r) {
    uint32_t qe = (uint32_t)((double)h * N.ipm);
    int64_t re = (int64_t)(h - (uint64_t)qe * N.pm);
    if (re < 0) { re += (int64_t)N.pm; qe--; }
    else if (re >= (int64_t)N.pm) { re -= (int64_t)N.pm; qe++; }
    *q = qe;
    *r = (uint64_t)re;
}

// ---------------------------------------------------------------------------
// Level 1: k_scatter_l1p's software pipeline (3 barrier phases a tile; the
// write-out of tile t shares its phase with the hash + rank of tile t + 1)
// with one record per k-mer and 4096-k-mer tiles.  Buckets have a uniform
// capacity `cap` (bucket d owns [d cap, (d + 1) cap)), so the per-bucket LDS
// positions are 32-bit offsets inside the bucket.  Block reservations, holes,
// pads, tails and the chunk queue are k_scatter_l1p's.
__global__ void __launch_bounds__(L1_THREADS, L1F_WAVES_PER_EU) k_scatter_n1(NPGeo N, SrcTwoBit src, uint64_t nkmers,
                                                                            unsigned long long *bkt_cur, uint64_t *rec,
                                                                            uint32_t *blkj, uint64_t *ctr, int blk_sh,
                                                                            uint32_t jbase, uint32_t cht) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int KPT = NP_KPT;
    constexpr int TILE = L1_THREADS * KPT;   // k-mers = records a tile
    const uint32_t BLK = 1u << blk_sh;
    const uint32_t F1 = N.nb;
    const uint32_t F1a = (F1 + 3) & ~3u;
    const uint32_t NSLOT = TILE + 2 * F1a;
    const uint64_t CAP = N.cap;
    uint64_t *s_tw = (uint64_t *)smem;                  // [2][NP_TW] packed words of the staged / next tile
    uint64_t *tail = s_tw + 2 * NP_TW;                  // [F1] a pending odd record
    uint64_t *slot = tail + F1a;                        // [NSLOT] bucket | tile index | payload
    uint2 *dl2 = (uint2 *)(slot + NSLOT);               // [F1] output - LDS position: current block, new blocks
    uint2 *qq = dl2 + F1a;                              // [F1] first LDS position in the new blocks / left for the tail
    uint32_t *bcur = (uint32_t *)(qq + F1a);            // [F1] partially filled block (bucket-relative; NP_DEAD: overflowed)
    uint32_t *cnt = bcur + F1a;                         // [F1] records appended by this workgroup
    uint32_t *hist2 = cnt + F1a;                        // [2][F1] tile histograms (tile parity)
    uint32_t *lstart = hist2 + 2 * F1a;                 // [F1] the bucket's first record slot of the tile
    uint32_t *bjb = lstart + F1a;                       // [F1] k-mer index base of the partially filled block
    uint32_t *obase = bjb + F1a;                        // [F1] the same, as it was before this tile (write-out)
    uint32_t *s_misc = obase + F1a;                     // [0] queue chunk, [1] slots of the staged tile
    for (uint32_t b = threadIdx.x; b < F1; b += blockDim.x) {
        bcur[b] = 0;
        cnt[b] = 0;
        hist2[b] = 0;
        hist2[F1a + b] = 0;
        bjb[b] = 0;
    }
    const uint64_t CK = (uint64_t)cht * TILE;
    const uint32_t nchunks = (uint32_t)((nkmers + CK - 1) / CK);
    uint32_t cb = blockIdx.x + gridDim.x;
    uint64_t hj0 = min(nkmers, (uint64_t)blockIdx.x * CK);
    uint64_t hce = min(nkmers, hj0 + CK);
    bool htop = true;
    auto tile_w0 = [&](uint64_t j0) -> uint64_t {
        const uint64_t ja = j0 + src.kbase;
        return ((ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2) >> 6;
    };
    auto tile_nw = [&](uint64_t j0, uint64_t j1) -> uint32_t { return (uint32_t)(tile_w0(j1 - 1) + 2 - tile_w0(j0)); };
    auto next_tile = [&](uint64_t j1, uint64_t *n0, uint64_t *n1) {
        *n0 = j1;
        *n1 = j1;
        if (j1 < hce) {
            *n1 = min(hce, j1 + TILE);
        } else if (cb < nchunks) {
            *n0 = (uint64_t)cb * CK;
            *n1 = min(nkmers, *n0 + (uint64_t)TILE);
        }
    };
    const uint32_t S = N.rp << N.s0;     // bins of a bucket
    // per k-mer register: bucket << 55 | tile rank << 42 | payload (~0: none)
    uint64_t rr[KPT];
    unsigned long long qn = 0;
    uint64_t tw_next = 0;
    auto hash_rank = [&](uint64_t j0, uint64_t j1, uint32_t *h, uint32_t buf) {
        const uint64_t *tw_cur = s_tw + buf * NP_TW;
        const uint64_t tw_w0 = tile_w0(j0);
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            const uint64_t j = j0 + (uint64_t)a * L1_THREADS + threadIdx.x;
            rr[a] = ~0ull;
            if (j < j1) {
                const uint64_t ja = j + src.kbase;
                const uint64_t bpos = (ja + src.read_of(ja) * (uint64_t)(src.k - 1)) * 2;
                const uint32_t wi = (uint32_t)((bpos >> 6) - tw_w0);
                const uint64_t x = src.finish(SrcTwoBit::Pend{tw_cur[wi], tw_cur[wi + 1], (uint32_t)(bpos & 63)});
                uint32_t q;
                uint64_t r;
                np_divmod(x, N, &q, &r);
                const uint32_t b = __umulhi((uint32_t)(r >> N.s0), N.magic);
                const uint64_t pay = ((uint64_t)q << N.ob) | (r - (uint64_t)b * S);
                rr[a] = ((uint64_t)b << NP_SLOT_B) | ((uint64_t)atomicAdd(&h[b], 1u) << NP_SLOT_K) | pay;
            }
        }
    };
    uint64_t hj1 = min(hce, hj0 + TILE);
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
        const uint64_t j0 = hj0;
        const bool last = n1 == n0;
        const bool top = htop;
        uint32_t *hist = hist2 + (ti & 1) * F1a;
        const uint32_t tb = jbase + (uint32_t)j0;                        // base of the blocks reserved now
        const uint32_t nhi = last ? tb : jbase + (uint32_t)(n1 - 1);      // the next tile's largest index
        // ---- P1: block reservations (thread d owns bucket d), run starts
        uint64_t rsv = 0;
        const uint32_t d = threadIdx.x;
        if (d < F1 && bcur[d] != NP_DEAD) {
            const uint32_t h = hist[d], L0 = cnt[d];
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (((L0 + BLK - 1) & ~(BLK - 1)) >> blk_sh);
            if (need) rsv = atomicAdd(&bkt_cur[d], (unsigned long long)need * BLK);
        }
        if (threadIdx.x < 64) {
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
            if (lane == 0) s_misc[1] = base;
        }
        block_sync();
        // ---- P2: staging; placement constants; bucket state advanced
#pragma unroll
        for (int a = 0; a < KPT; a++) {
            if (rr[a] != ~0ull) {
                const uint32_t b = (uint32_t)(rr[a] >> NP_SLOT_B);
                const uint32_t pos = lstart[b] + (uint32_t)((rr[a] >> NP_SLOT_K) & NP_EMPTY);
                slot[pos] = ((uint64_t)b << NP_SLOT_B) | ((uint64_t)(a * L1_THREADS + threadIdx.x) << NP_SLOT_K) |
                            (rr[a] & NP_PAY);
            }
        }
        if (!last && threadIdx.x < NP_TW) s_tw[((ti + 1) & 1) * NP_TW + threadIdx.x] = tw_next;
        if (top && threadIdx.x == 0) s_misc[0] = (uint32_t)min<unsigned long long>(qn + 2ull * gridDim.x, nchunks);
        if (d < F1) {
            const uint32_t h = hist[d], L0 = cnt[d];
            const uint32_t split = (L0 + BLK - 1) & ~(BLK - 1);
            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (split >> blk_sh);
            const uint32_t bc = bcur[d];
            const uint32_t e = L0 + h;
            const uint32_t jb_old = bjb[d];
            const uint32_t jb_new = need ? tb : jb_old;   // base of the partially filled block after this tile
            // the next tile's records would not fit the block's index span:
            // close the block after this tile's records
            const bool stale = !last && (e & (BLK - 1)) != 0 && nhi - jb_new > N.jlim;
            if (h || last || stale) {
                uint32_t nb = 0;
                if (bc == NP_DEAD) {
                    nb = NP_DEAD;
                } else if (need) {
                    nb = (uint32_t)(rsv - (uint64_t)d * CAP);
                    if ((uint64_t)nb + (uint64_t)need * BLK > CAP) {
                        atomicOr((unsigned long long *)&ctr[CTR_ERR], 8ull);
                        nb = NP_DEAD;
                    }
                }
                const uint32_t fe = (last || stale) ? e : (e & ~1u);
                if ((L0 & 1) && fe > L0 - 1 && bc != NP_DEAD && !(KH_ABL(N, 16)))   // 16: the tails were never written
                    rec[(uint64_t)d * CAP + bc + ((L0 - 1) & (BLK - 1))] = tail[d];
                const uint32_t q0 = lstart[d];
                if (h) {
                    if (L0 & 1) slot[q0 - 1] = ((uint64_t)d << NP_SLOT_B) | ((uint64_t)NP_EMPTY << NP_SLOT_K);
                    if ((q0 + h) & 1) slot[q0 + h] = ((uint64_t)d << NP_SLOT_B) | ((uint64_t)NP_EMPTY << NP_SLOT_K);
                }
                const bool dead = bc == NP_DEAD || nb == NP_DEAD;
                dl2[d] = make_uint2(bc + (L0 & (BLK - 1)) - q0, nb + L0 - split - q0);
                qq[d] = make_uint2(q0 + (split - L0), dead ? 0 : q0 + (fe > L0 ? fe - L0 : 0));
                obase[d] = jb_old;
                if (h) {
                    if (nb == NP_DEAD) bcur[d] = NP_DEAD;
                    else if (need) bcur[d] = nb + (need - 1) * BLK;
                    cnt[d] = e;
                    hist[d] = 0;
                    bjb[d] = jb_new;
                    if (need && nb != NP_DEAD)
                        for (uint32_t z = 0; z < need; z++) blkj[(((uint64_t)d * CAP + nb) >> blk_sh) + z] = tb;
                }
                if (stale && !dead) {
                    // the rest of the block: sentinels (the write-out below
                    // fills slots below e & (BLK - 1), this loop the ones above)
                    const uint64_t pb0 = (uint64_t)d * CAP + bcur[d];
                    for (uint32_t s = e & (BLK - 1); s < BLK; s++) rec[pb0 + s] = ~0ull;
                    cnt[d] = (e + BLK - 1) & ~(BLK - 1);
                }
            }
        }
        block_sync();
        // ---- P3: write-out of the staged tile
        {
            const uint32_t nslot = s_misc[1];
            const ulonglong2 *slot2 = (const ulonglong2 *)slot;
            for (uint32_t m = threadIdx.x; 2 * m < nslot; m += L1_THREADS) {
                const ulonglong2 sp = slot2[m];
                const uint32_t dd = (uint32_t)(sp.x >> NP_SLOT_B);
                const uint32_t k0 = (uint32_t)(sp.x >> NP_SLOT_K) & NP_EMPTY, k1 = (uint32_t)(sp.y >> NP_SLOT_K) & NP_EMPTY;
                const uint2 ql = qq[dd];
                const uint2 dv = dl2[dd];
                const uint32_t q = 2 * m;
                const bool nw = q >= ql.x;
                const uint32_t base = nw ? tb : obase[dd];
                const bool r0 = k0 != NP_EMPTY, r1 = k1 != NP_EMPTY;
                const uint64_t v0 = ((uint64_t)(tb + k0 - base) << N.pb) | (sp.x & NP_PAY);
                const uint64_t v1 = ((uint64_t)(tb + k1 - base) << N.pb) | (sp.y & NP_PAY);
                const uint64_t o = (uint64_t)dd * CAP + (uint32_t)((nw ? dv.y : dv.x) + q);
                if (KH_ABL(N, 16)) continue;   // timing only: no run writes
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
        if (hj1 >= hce) {
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
        if (c == 0 || sl < c || bcur[dd] == NP_DEAD) continue;
        rec[(uint64_t)dd * CAP + bcur[dd] + sl] = ~0ull;
    }
}
__host__ __device__ constexpr size_t lds_n1(size_t F1a) {
    return 2 * NP_TW * 8 + F1a * 8 + ((size_t)L1_THREADS * NP_KPT + 2 * F1a) * 8 + F1a * 8 * 2 + F1a * 4 * 7 + 16;
}

// ---------------------------------------------------------------------------
// Level 2: k_scatter_l2f's register-direct scatter (fixed-capacity regions,
// 64-record blocks, 128-B segments through LDS tails) over a level-1
// bucket's near-prime records.  Each thread loads IN records (IN / 2 pairs)
// a tile and expands each into its NT region records (IN * NT <= 8 register
// slots, NT = N.n); destination d = i Rloc
// + (region of table i's bin - R' b) (plus table i's regions when the bin
// wrapped past p_i).  The destination rides in bits [16, 32) of the
// register copy of the record and is cleared when it is stored.
template <int THREADS, int NT>
__global__ void __launch_bounds__(THREADS) k_scatter_n2(NPGeo N, uint32_t parts, const unsigned long long *bkt_end,
                                                        const uint32_t *blkj, int blk_sh1, const uint64_t *reg_base,
                                                        unsigned long long *reg_cur, const uint64_t *rec_in,
                                                        uint64_t *rec_out, uint64_t *ctr, int blk_sh) {
#ifndef KH_N2_IN
#define KH_N2_IN 2   // development A/B: level-1 records per thread a tile at 3-4 tables
#endif
    constexpr int IN = NT == 2 ? 2 * KH_N2_IN : KH_N2_IN;   // level-1 records per thread a tile
    constexpr int RPT = IN * NT <= 8 ? 8 : IN * NT;
    constexpr int TILE = THREADS * IN;
    constexpr uint32_t SEG = 16;
    static_assert(NT >= 2 && NT <= NP_MAXT && IN * NT <= RPT, "k_scatter_n2: 2 to 4 tables");
    const uint32_t BLK = 1u << blk_sh;
    const uint32_t F2 = (uint32_t)NT * N.rloc;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *bcur = (uint64_t *)smem;              // [F2]
    uint64_t *nbase = bcur + F2;                    // [F2]
    uint64_t *tail = nbase + F2;                    // [F2*SEG]
    uint32_t *cnt = (uint32_t *)(tail + F2 * SEG);  // [F2]
    uint32_t *hist = cnt + F2;                      // [F2]
    uint32_t *s_nfl = hist + F2;                    // [1]
    uint16_t *flist = (uint16_t *)(s_nfl + 4);      // [F2]
    if (__builtin_amdgcn_readfirstlane((uint32_t)ctr[CTR_ERR]) & 8u) return;
    const uint32_t b = blockIdx.x / parts, p = blockIdx.x % parts;
    const uint64_t b0 = (uint64_t)b * N.cap, b1 = min((uint64_t)bkt_end[b], b0 + N.cap);
    const uint64_t len = ((b1 - b0 + parts - 1) / parts + 1) & ~1ull;
    const uint64_t r0 = min(b1, b0 + (uint64_t)p * len), r1 = min(b1, r0 + len);
    const uint64_t smask = (1ull << N.s0) - 1;
    const uint64_t omask = (1ull << N.ob) - 1;
    const uint64_t bin0 = (uint64_t)b * ((uint64_t)N.rp << N.s0);   // first bin of the bucket (largest table)
    const uint32_t rb = b * N.rp;                                     // its first region
    auto load_tile = [&](uint64_t n0, uint64_t *v, uint32_t *jb) {
        const uint64_t n1 = min(r1, n0 + TILE);
#pragma unroll
        for (int q = 0; q < IN / 2; q++) {
            const uint64_t idx = n0 + 2 * ((uint64_t)q * THREADS + threadIdx.x);
            ulonglong2 x = make_ulonglong2(~0ull, ~0ull);
            uint32_t y = 0;
            if (idx < n1) {
                x = *(const ulonglong2 *)(rec_in + idx);
                y = blkj ? blkj[idx >> blk_sh1] : 0u;   // none: fine records of level 1b (pb = 32)
            }
            v[2 * q] = x.x;
            v[2 * q + 1] = idx + 1 < n1 ? x.y : ~0ull;
            jb[q] = y;
        }
    };
    for (uint32_t d = threadIdx.x; d < F2; d += THREADS) {
        bcur[d] = 0;
        cnt[d] = 0;
        hist[d] = 0;
    }
    if (threadIdx.x == 0) *s_nfl = 0;
    auto phys = [&](uint32_t d, uint32_t L) -> uint64_t {
        const uint32_t split = (cnt[d] + BLK - 1) & ~(BLK - 1);
        if (L < split) return bcur[d] == L2F_DEAD ? L2F_DEAD : bcur[d] + (L & (BLK - 1));
        return nbase[d] == L2F_DEAD ? L2F_DEAD : nbase[d] + (L - split);
    };
    // the global region of destination d (thread d's reservation)
    auto greg = [&](uint32_t d) -> uint64_t {
        const uint32_t i = d / N.rloc;
        uint32_t rho = rb + (d - i * N.rloc);
        if (rho >= N.rt[i]) rho -= N.rt[i];
        return (uint64_t)N.rbase[i] + rho;
    };
    uint64_t v[IN];
    uint32_t jb[IN / 2];
    load_tile(r0, v, jb);
    const uint32_t ntiles = uniform_u32((uint32_t)((r1 - r0 + TILE - 1) / TILE));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t t0 = r0 + (uint64_t)ti * TILE;
        const bool last = ti + 1 == ntiles;
        block_sync();
        // expand: output slot a * NT + i (k-mer a, table i)
        uint64_t x[RPT];
        uint32_t rank[RPT];
#pragma unroll
        for (int q = 0; q < RPT; q++) x[q] = ~0ull;
#pragma unroll
        for (int a = 0; a < IN; a++) {
            if (v[a] == ~0ull) continue;
            const uint64_t jv = (uint64_t)(jb[a >> 1] + (uint32_t)(v[a] >> N.pb)) << 32;
            const uint64_t pay = v[a] & ((1ull << N.pb) - 1);
            const uint64_t qv = pay >> N.ob;
            const uint64_t r = bin0 + (pay & omask);
#pragma unroll
            for (int i = 0; i < NT; i++) {
                uint64_t bin = r + qv * N.d[i];
                if (bin >= N.p[i]) bin -= N.p[i];
                const uint32_t rho = (uint32_t)(bin >> N.s0);
                int32_t loc = (int32_t)(rho - rb);
                if (loc < 0) loc += (int32_t)N.rt[i];
                if ((uint32_t)loc >= N.rloc) {   // outside the bucket's destinations: a host plan error
                    atomicOr((unsigned long long *)&ctr[CTR_ERR], 16ull);
                    continue;
                }
                const uint32_t dst = (uint32_t)i * N.rloc + (uint32_t)loc;
                x[a * NT + i] = jv | ((uint64_t)dst << 16) | (bin & smask);
            }
        }
#pragma unroll
        for (int q = 0; q < RPT; q++)
            if (x[q] != ~0ull) rank[q] = atomicAdd(&hist[((uint32_t)x[q]) >> 16], 1u);
        load_tile(t0 + TILE, v, jb);
        block_sync();
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
                        const uint64_t g = greg(d);
                        nb = atomicAdd(&reg_cur[g], (unsigned long long)need * BLK);
                        nlim = reg_base[g + 1];
                        nneed = need;
                    }
                }
                if (nneed && nb + (uint64_t)nneed * BLK > nlim) {
                    atomicOr((unsigned long long *)&ctr[CTR_ERR], 4ull);
                    nb = L2F_DEAD;
                }
                nbase[d] = nb;
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
        block_sync();
        {
            const uint32_t nfl = *s_nfl;
            for (uint32_t y = threadIdx.x; y < nfl * SEG; y += THREADS) {
                const uint32_t d = flist[y / SEG], sl = y % SEG;
                const uint32_t c0 = cnt[d], a = c0 & ~(SEG - 1);
                if (a + sl < c0) rec_out[bcur[d] + ((a + sl) & (BLK - 1))] = tail[d * SEG + sl];
            }
        }
        block_sync();
#pragma unroll
        for (int q = 0; q < RPT; q++) {
            if (x[q] == ~0ull) continue;
            const uint32_t d = ((uint32_t)x[q]) >> 16;
            const uint32_t L = cnt[d] + rank[q];
            const uint32_t e = cnt[d] + hist[d];
            const uint64_t val = x[q] & 0xFFFFFFFF0000FFFFull;
            if (L < (last ? e : (e & ~(SEG - 1)))) {
                const uint64_t pos = phys(d, L);
                if (pos != L2F_DEAD) rec_out[pos] = val;
            } else {
                tail[d * SEG + (L & (SEG - 1))] = val;
            }
        }
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
    block_sync();
    for (uint32_t y = threadIdx.x; y < F2 * BLK; y += THREADS) {
        const uint32_t d = y >> blk_sh, sl = y & (BLK - 1);
        const uint32_t c = cnt[d] & (BLK - 1);
        if (c == 0 || sl < c || bcur[d] == L2F_DEAD) continue;
        rec_out[bcur[d] + sl] = ~0ull;
    }
}
static size_t lds_scatter_n2(const NPGeo &N) {
    return (size_t)N.n * N.rloc * (8 + 8 + 16 * 8 + 4 + 4 + 2) + 16;
}
using N2Fn = void (*)(NPGeo, uint32_t, const unsigned long long *, const uint32_t *, int, const uint64_t *,
                      unsigned long long *, const uint64_t *, uint64_t *, uint64_t *, int);
static N2Fn n2_kernel(int n) {
    return n == 2 ? k_scatter_n2<PT_THREADS, 2> : n == 3 ? k_scatter_n2<PT_THREADS, 3> : k_scatter_n2<PT_THREADS, 4>;
}

// ---------------------------------------------------------------------------
// Level 1b (three levels: tables too large for <= 256 level-1 buckets of the
// level-2 fan-out, C4's 4 x 8e9): level 1 buckets each k-mer by r into coarse
// buckets of F x R' regions (k_scatter_n1 as above, <= 256 of them), and this
// kernel splits every coarse bucket into its F fine buckets of R' regions,
// still one record per k-mer:
//     fine record = j << 32 | q << ob_f | (r - fine bucket's first bin)
// (absolute pass index j: a fine bucket gathers records of many level-1
// blocks).  A workgroup streams a slice of one coarse bucket in tiles of
// THREADS x 8 records: LDS rank per fine bucket, one returning atomic per
// (tile, fine bucket) reserves a dense run, the tile is staged in LDS in run
// order and written out coalesced.  No blocks, pads or sentinels in the
// output; k_scatter_n2 reads it with pb = 32 and no block bases.
struct NPFine {
    uint32_t F;        // fine buckets per coarse bucket (0: two levels)
    uint32_t rp;       // regions of 2^s0 bins per fine bucket
    uint32_t magic;    // ceil(2^32 / rp)
    int ob;            // offset bits of a fine record
    uint32_t rloc;     // level-2 destinations per table of a fine bucket (rp + spill)
    uint64_t cap;      // records per fine bucket (fine bucket b owns [b cap, (b + 1) cap))
};
constexpr int N1B_THREADS = 256;
constexpr int N1B_IN = 8;          // records per thread a tile
constexpr uint32_t N1B_MAXF = 16;
__global__ void __launch_bounds__(N1B_THREADS) k_scatter_n1b(NPGeo C, NPFine Fi, uint32_t parts,
                                                              const unsigned long long *bkt_end, const uint32_t *blkj,
                                                              int blk_sh1, const uint64_t *rec_in,
                                                              unsigned long long *fcur, uint64_t *rec_out,
                                                              uint64_t *ctr) {
    constexpr int TILE = N1B_THREADS * N1B_IN;
    __shared__ __attribute__((aligned(16))) uint64_t slot[TILE];
    __shared__ uint8_t sf[TILE];
    __shared__ uint32_t hist[N1B_MAXF], lstart[N1B_MAXF + 1];
    __shared__ uint64_t gbase[N1B_MAXF];
    if (__builtin_amdgcn_readfirstlane((uint32_t)ctr[CTR_ERR]) & 8u) return;
    const uint32_t c = blockIdx.x / parts, p = blockIdx.x % parts;
    const uint64_t b0 = (uint64_t)c * C.cap, b1 = min((uint64_t)bkt_end[c], b0 + C.cap);
    const uint64_t len = ((b1 - b0 + parts - 1) / parts + 1) & ~1ull;
    const uint64_t r0 = min(b1, b0 + (uint64_t)p * len), r1 = min(b1, r0 + len);
    const uint64_t pmask = (1ull << C.pb) - 1, omask = (1ull << C.ob) - 1;
    const uint64_t Sf = (uint64_t)Fi.rp << C.s0;   // bins of a fine bucket
    const uint32_t F = Fi.F;
    for (uint64_t t0 = r0; t0 < r1; t0 += TILE) {
        if (threadIdx.x < N1B_MAXF) hist[threadIdx.x] = 0;
        block_sync();
        uint64_t v[N1B_IN];
        uint32_t rk[N1B_IN];
#pragma unroll
        for (int q = 0; q < N1B_IN / 2; q++) {
            const uint64_t idx = t0 + 2 * ((uint64_t)q * N1B_THREADS + threadIdx.x);
            ulonglong2 x = make_ulonglong2(~0ull, ~0ull);
            uint32_t jb = 0;
            if (idx < r1) {
                x = *(const ulonglong2 *)(rec_in + idx);
                jb = blkj[idx >> blk_sh1];
                if (idx + 1 >= r1) x.y = ~0ull;
            }
            v[2 * q] = x.x;
            v[2 * q + 1] = x.y;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint64_t &y = v[2 * q + h];
                if (y == ~0ull) continue;
                const uint64_t j = (uint32_t)(jb + (uint32_t)(y >> C.pb));
                const uint64_t pay = y & pmask;
                const uint64_t off = pay & omask;
                const uint32_t f = __umulhi((uint32_t)(off >> C.s0), Fi.magic);
                y = (j << 32) | ((pay >> C.ob) << Fi.ob) | (off - (uint64_t)f * Sf);
                rk[2 * q + h] = (f << 24) | atomicAdd(&hist[f], 1u);
            }
        }
        block_sync();
        if (threadIdx.x < F) {
            const uint32_t f = threadIdx.x, h = hist[f];
            const uint64_t fb = (uint64_t)c * F + f;
            uint64_t gb = h ? atomicAdd(&fcur[fb], (unsigned long long)h) : 0;
            if (h && gb + h > (fb + 1) * Fi.cap) {
                atomicOr((unsigned long long *)&ctr[CTR_ERR], 8ull);
                gb = ~0ull;
            }
            gbase[f] = gb;
        }
        if (threadIdx.x == 0) {
            uint32_t a = 0;
            for (uint32_t f = 0; f < F; f++) {
                lstart[f] = a;
                a += hist[f];
            }
            lstart[F] = a;
        }
        block_sync();
#pragma unroll
        for (int a = 0; a < N1B_IN; a++) {
            if (v[a] == ~0ull) continue;
            const uint32_t f = rk[a] >> 24;
            const uint32_t s = lstart[f] + (rk[a] & 0xFFFFFFu);
            slot[s] = v[a];
            sf[s] = (uint8_t)f;
        }
        block_sync();
        const uint32_t nv = lstart[F];
        for (uint32_t m = threadIdx.x; m < nv; m += N1B_THREADS) {
            const uint32_t f = sf[m];
            const uint64_t gb = gbase[f];
            if (gb != ~0ull) rec_out[gb + (m - lstart[f])] = slot[m];
        }
    }
}

// level-1 bucket cursors start at d * cap
__global__ void k_np_reset(unsigned long long *cur, uint32_t nb, uint64_t cap) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < nb; d += gridDim.x * blockDim.x)
        cur[d] = (unsigned long long)d * cap;
}

}  // namespace kh
