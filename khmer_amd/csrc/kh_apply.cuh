// kh_apply.cuh -- region apply, winner lists, bigcount crossing resolution,
// finalize.  Included by kh_engine.hip.
//
// One workgroup owns one region of 2^s0 bins of one table at a time: the
// table slice is held in LDS, every record of the region bumps its bin's LDS
// counter and (for bins that were zero before the batch) takes the minimum
// k-mer index (= the first insert in stream order, i.e. the reference's
// is_new winner, storage.hh:578-588); the saturated values are written back
// with 16-byte stores, and the winners are written to the region's own
// segment of the winner list (win[e0 .. e0 + wcnt[rr])), so no global atomics
// are needed.  The next region's table slice and first records are loaded
// into registers while the current region finishes (software pipelining).
#pragma once
#include "kh_partition.cuh"

namespace kh {

constexpr int APPLY_THREADS = 512;
constexpr int APPLY_RECS = 8;          // records in flight per thread
constexpr int FIN_THREADS = 256;
constexpr int W_RPC = 64;              // regions per winner chunk

struct ApplyArgs {
    const uint64_t *rlo, *rhi;   // region g's records: [rlo[g], rhi[g])
    const uint64_t *rec;
    uint8_t *tab;
    uint32_t *win;        // winners of region rr at win[e0(rr) ...]
    uint32_t *wcnt;       // [regions] winners per region
    uint8_t *fullf;
    // crossing bins (bigcount): region rr's entries (offset << 8 | c0) at
    // xent[e0(rr) ...] (a crossing bin holds >= 2 of the region's records, so
    // they fit), one segment descriptor per region with crossings in xseg
    uint32_t *xent;
    uint4 *xseg;
    uint64_t *ctr;
    uint64_t rprefix[MAXT + 1];   // real-region prefix per table
    // coarse-window winners (unsharded passes): instead of per-region lists,
    // every region's winners are counting-sorted in LDS by coarse k-mer
    // window (j >> cjs, <= 64 windows) and appended as runs to that window's
    // range of wco: [cw_cur[c] at the start, its capacity end) -- the capacity
    // is the window's k-mers x tables, a hard bound on its winners
    int coarse, cjs;
    uint32_t *wco;
    unsigned long long *cw_cur;
    // dynamic region order (k_apply_count): workgroup w starts with regions
    // w, w + G and w + 2G (G = gridDim.x) and takes one more per region from
    // the queue head ctr[CTR_APQ] (numbered from 3G); 0: the static stride
    int dyn;
};
constexpr int MAX_CW = 64;

__device__ __forceinline__ void full_add(uint8_t *fullf, uint32_t j) {
    atomicAdd((uint32_t *)(fullf + (j & ~3u)), 1u << (8 * (j & 3u)));
}

struct RegionInfo {
    int i;
    uint32_t nb;
    uint64_t e0, e1, bin_lo;
};

// record range of region rr (in apply order: table by table); loaded one
// region ahead of its prefetch so the prefetch never waits for it
struct Bounds {
    uint64_t e0, e1;
};
__device__ __forceinline__ uint64_t region_index(const Params &P, const ApplyArgs &A, uint64_t rr, int *ti) {
    int i = 0;
    while (i + 1 < P.n && rr >= A.rprefix[i + 1]) i++;
    *ti = i;
    return (P.tbase[i] >> P.s0) + (rr - A.rprefix[i]);
}
__device__ __forceinline__ Bounds load_bounds(const Params &P, const ApplyArgs &A, uint64_t rr, uint64_t total) {
    if (rr >= total) return Bounds{0, 0};
    int i;
    const uint64_t region = region_index(P, A, rr, &i);
    return Bounds{A.rlo[region], A.rhi[region]};
}

// region rr -> table, bins, record range
__device__ __forceinline__ RegionInfo region_info(const Params &P, const ApplyArgs &A, uint64_t rr, Bounds b) {
    RegionInfo ri;
    int i;
    region_index(P, A, rr, &i);
    const uint64_t lreg = rr - A.rprefix[i];
    ri.i = i;
    ri.e0 = b.e0;
    ri.e1 = b.e1;
    ri.bin_lo = lreg << P.s0;
    ri.nb = (uint32_t)min((uint64_t)1 << P.s0, P.lsz[i] - ri.bin_lo);
    return ri;
}

// registers prefetched for one region
struct Prefetch {
    RegionInfo ri;
    uint4 tv;                   // this thread's 16-byte (8-byte nibble) table chunk
    uint64_t v[APPLY_RECS];     // this thread's first records
};

// APPLY_RECS records per thread as APPLY_RECS / 2 16-B pairs: pair p0 + u * TH
// + thread.  Records outside [e0, e1) (the odd ends of an unaligned region,
// the pairs past its end) read as the ~0 sentinel.  One 16-B load per two
// records: apply's record stream is bound by load instructions, not bytes.
template <int TH>
__device__ __forceinline__ void load_recs(const uint64_t *rec, uint64_t p0, uint64_t e0, uint64_t e1, uint64_t *v) {
#pragma unroll
    for (int u = 0; u < APPLY_RECS / 2; u++) {
        const uint64_t r = 2 * (p0 + (uint64_t)u * TH + threadIdx.x);
        ulonglong2 x = make_ulonglong2(~0ull, ~0ull);
        if (r < e1) x = *(const ulonglong2 *)(rec + r);
        v[2 * u] = r >= e0 ? x.x : ~0ull;
        v[2 * u + 1] = r + 1 < e1 ? x.y : ~0ull;
    }
}

template <int KIND, int TH = APPLY_THREADS>
__device__ __forceinline__ void prefetch_region(const Params &P, const ApplyArgs &A, uint64_t rr, uint64_t total,
                                                Bounds b, Prefetch &f) {
    // every field is written on every path (keeps the struct in registers)
    const bool valid = rr < total;
    f.ri = region_info(P, A, valid ? rr : 0, b);
    if (!valid) f.ri.e1 = f.ri.e0;
    f.tv = make_uint4(0, 0, 0, 0);
    const uint32_t t = threadIdx.x;
    const bool any = f.ri.e0 != f.ri.e1;
    const uint8_t *tab = A.tab + P.tbyte[f.ri.i];
    if (KIND == BYTE) {
        if (any && t < (f.ri.nb + 15) / 16) f.tv = ((const uint4 *)(tab + f.ri.bin_lo))[t];
    } else if (KIND == NIBBLE) {
        if (any && t < (f.ri.nb + 15) / 16) {
            const uint2 x = ((const uint2 *)(tab + (f.ri.bin_lo >> 1)))[t];
            f.tv = make_uint4(x.x, x.y, 0, 0);
        }
    } else {
        if (any && t < (f.ri.nb + 127) / 128) f.tv = ((const uint4 *)(tab + (f.ri.bin_lo >> 3)))[t];
    }
    load_recs<TH>(A.rec, f.ri.e0 >> 1, f.ri.e0, f.ri.e1, f.v);
}

// one record of a Byte/Nibble region: two independent fire-and-forget LDS
// atomics (no dependence on the bin's value, so loads and atomics pipeline)
__device__ __forceinline__ void count_record(uint64_t x, uint32_t *cnt, uint32_t *minj) {
    if (x == ~0ull) return;
    const uint32_t o = (uint32_t)x;
    atomicAdd(&cnt[o], 1u);
    atomicMin(&minj[o], (uint32_t)(x >> 32));
}
// one record of a Bit region
__device__ __forceinline__ void bit_record(uint64_t x, uint32_t *minj) {
    if (x == ~0ull) return;
    atomicMin(&minj[(uint32_t)x], (uint32_t)(x >> 32));
}

// winners (held in registers) -> the region's segment of the winner list.
// Called by all threads after a barrier that follows wave_winner_scan.
__device__ __forceinline__ uint32_t wave_winner_scan(uint32_t c, uint32_t *s_wt) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t incl = c;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_wt[threadIdx.x >> 6] = incl;
    return incl - c;
}
__device__ __forceinline__ uint64_t winner_base(const uint32_t *s_wt, uint32_t *total) {
    const uint32_t wave = threadIdx.x >> 6, nwav = blockDim.x >> 6;
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < nwav; w++) {
        const uint32_t x = s_wt[w];
        before += w < wave ? x : 0;
        all += x;
    }
    *total = all;
    return before;
}

// Byte (KIND == BYTE) and Nibble storage: ByteStorage::add / NibbleStorage::add
// (storage.hh:571-624 / 320-359) applied as a batch.  LOS: complement mode of
// the coarse-window runs -- they carry the pass's losers (every record that is
// not its bin's is_new first insert) instead of its winners, for passes where
// most inserts are winners (sparse tables); k_mark_wf counts them per k-mer.
// TH threads, 16 bins per thread: regions of 2^13 (512 threads) or 2^14 bins
// (1024 threads) -- one kernel body for both
template <int KIND, int TH, bool LOS = false>
__global__ void __launch_bounds__(TH, 4) k_apply_count(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BPT = 16;               // bins per thread: R == 16 * TH
    const uint32_t R = 1u << P.s0;
    uint32_t *cnt = (uint32_t *)smem;     // [R]
    uint32_t *minj = cnt + R;             // [R]
    uint32_t *chg = minj + R;             // [R/512] changed 16-bin chunks
    uint32_t *s_wt = chg + R / 512;       // [16] wave winner totals
    uint32_t *full255 = s_wt + 16;        // [R/32] bins at 255 before the batch that got inserts
    uint32_t *s_flag = full255 + R / 32;  // [4]
    uint8_t *c0 = (uint8_t *)(s_flag + 4);  // [R]
    uint8_t *wflag = c0 + R;              // [R/4] winner bits of each 4-bin group
    // coarse-window winners: per-window counts then cursors, first staging
    // slots, output bases (own arrays, cleared with the region's state)
    uint32_t *chist = (uint32_t *)(wflag + R / 4);         // [MAX_CW]
    uint32_t *cst0 = chist + MAX_CW;                        // [MAX_CW]
    unsigned long long *cgb = (unsigned long long *)(cst0 + MAX_CW);   // [MAX_CW]
    uint32_t *ccur = (uint32_t *)(cgb + MAX_CW);           // [MAX_CW] placement cursors
    const uint32_t MAXC = KIND == BYTE ? 255u : 15u;
    const bool bigc = KIND == BYTE && P.use_bigcount;
    PH_WG_BEGIN;
    const uint32_t t = threadIdx.x;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    Prefetch cur, nxt;
    // this workgroup's regions: rr, then r1 (prefetched during rr), then r2
    // (its bounds loaded during rr); the one after r2 is taken during rr
    // (dynamic order) and published through s_q[parity] after a barrier
    const uint64_t G = gridDim.x;
    uint64_t r1 = blockIdx.x + G, r2 = blockIdx.x + 2 * G;
    uint32_t *s_q = (uint32_t *)(ccur + MAX_CW);   // [2]
    uint32_t par = 0;
    prefetch_region<KIND, TH>(P, A, blockIdx.x, total, load_bounds(P, A, blockIdx.x, total), cur);
    Bounds bnext = load_bounds(P, A, r1, total);
    PH_BEGIN(8);
    for (uint64_t rr = blockIdx.x; rr < total;) {
        unsigned long long qn = 0;
        if (A.dyn && t == 0) qn = atomicAdd((unsigned long long *)&A.ctr[CTR_APQ], 1ull);
        // after a barrier of this region: publish the region after r2, and
        // move on (the slot of parity par is rewritten two regions later,
        // after every thread has passed a barrier of the next region)
        auto publish = [&]() {
            if (A.dyn && t == 0) s_q[par] = (uint32_t)min<unsigned long long>(qn + 3 * G, total);
        };
        auto advance = [&]() {
            rr = r1;
            r1 = r2;
            r2 = A.dyn ? (uint64_t)uniform_u32(s_q[par]) : r2 + G;
            par ^= 1;
        };
        const RegionInfo ri = cur.ri;
        if (ri.e0 == ri.e1) {
            if (t == 0) A.wcnt[rr] = 0;
            prefetch_region<KIND, TH>(P, A, r1, total, bnext, cur);
            bnext = load_bounds(P, A, r2, total);
            if (A.dyn) {
                block_sync();
                publish();
                block_sync();
            }
            advance();
            continue;
        }
        const Bounds bafter = load_bounds(P, A, r2, total);
        const uint32_t nb = ri.nb;
        const uint32_t nchunk = (nb + 15) / 16;   // 16 bins per chunk
        uint8_t *tab = A.tab + P.tbyte[ri.i];
        // table chunk (registers) -> LDS; counters and winners reset
        if (t < nchunk) {
            if (KIND == BYTE) {
                ((uint4 *)c0)[t] = cur.tv;
            } else {
                uint4 o;
                uint32_t *ow = (uint32_t *)&o;
                const uint32_t w[2] = {cur.tv.x, cur.tv.y};
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
        for (uint32_t x = t; x < nchunk * 4; x += blockDim.x) {
            ((uint4 *)cnt)[x] = make_uint4(0, 0, 0, 0);
            ((uint4 *)minj)[x] = make_uint4(NO_J, NO_J, NO_J, NO_J);
        }
        if (t < R / 512) chg[t] = 0;
        if (bigc) {
            for (uint32_t x = t; x < R / 32; x += blockDim.x) full255[x] = 0;
            if (t == 0) s_flag[0] = s_flag[1] = 0;
        }
        if (t < MAX_CW) chist[t] = ccur[t] = 0;
        if (LOS && t == 0) s_flag[2] = 0;   // losers listed
        PH(5);
        block_sync();
        PH(0);
        // records: the prefetched batch, then APPLY_RECS loads in flight per thread
        if (!(KH_ABL(P, 2))) {
            // two batches of APPLY_RECS loads in flight: batch k+1 is issued
            // before batch k's atomics, so each wait is for the older batch only
            const uint64_t step = (uint64_t)(APPLY_RECS / 2) * TH;   // pairs
            const uint64_t pend = (ri.e1 + 1) >> 1;
            uint64_t va[APPLY_RECS], vb[APPLY_RECS];
            uint64_t q0 = (ri.e0 >> 1) + step;
            load_recs<TH>(A.rec, q0, ri.e0, ri.e1, va);
#pragma unroll
            for (int u = 0; u < APPLY_RECS; u++) count_record(cur.v[u], cnt, minj);
            for (; q0 < pend; q0 += 2 * step) {
                load_recs<TH>(A.rec, q0 + step, ri.e0, ri.e1, vb);
#pragma unroll
                for (int u = 0; u < APPLY_RECS; u++) count_record(va[u], cnt, minj);
                load_recs<TH>(A.rec, q0 + 2 * step, ri.e0, ri.e1, va);
#pragma unroll
                for (int u = 0; u < APPLY_RECS; u++) count_record(vb[u], cnt, minj);
            }
        }
        block_sync();
        PH(1);
        // pass 1 (thread per bin, conflict-free LDS): winners (bins zero
        // before the batch keep their minimum k-mer index, the others drop
        // it), crossings, bins already full, saturated value into c0, changed
        // chunks
        // pass 1, four consecutive bins per thread and step (one c0 word, one
        // uint4 of counts): saturated values, winners (bins zero before the
        // batch keep their minimum k-mer index; others drop it), crossings,
        // bins already full, changed 16-bin chunks
        uint32_t nw = 0;
        const uint32_t lane = t & 63;
#pragma unroll
        for (int step = 0; step < BPT / 4; step++) {
            const uint32_t g = t + (uint32_t)step * TH;   // 4-bin group
            const uint32_t o = 4 * g;
            const uint4 n4 = ((const uint4 *)cnt)[g];
            const uint32_t cw = ((const uint32_t *)c0)[g];
            const uint32_t na[4] = {n4.x, n4.y, n4.z, n4.w};
            uint32_t fw = cw, win = 0, inval = 0, full = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t n = o + k < nb ? na[k] : 0;
                const uint32_t c = (cw >> (8 * k)) & 0xFFu;
                if (!n) continue;
                const uint32_t v = c + n;
                const uint32_t f = v < MAXC ? v : MAXC;
                fw = (fw & ~(0xFFu << (8 * k))) | (f << (8 * k));
                if (c == 0) win |= 1u << k;
                else inval |= 1u << k;
                if (bigc && c == 255) full |= 1u << k;
                if (bigc && c < 255 && v > 255 && !(KH_ABL(P, 8))) {   // insert r sees c + r: full iff c + r >= 255, r < n
                    const uint32_t idx = atomicAdd(&s_flag[1], 1u);
                    A.xent[ri.e0 + idx] = ((o + k) << 8) | c;
                }
            }
            const bool changed = fw != cw;
            if (changed) ((uint32_t *)c0)[g] = fw;
            if (inval) {
                uint4 m = ((const uint4 *)minj)[g];
                if (inval & 1) m.x = NO_J;
                if (inval & 2) m.y = NO_J;
                if (inval & 4) m.z = NO_J;
                if (inval & 8) m.w = NO_J;
                ((uint4 *)minj)[g] = m;
            }
            wflag[g] = (uint8_t)win;
            const uint32_t pw = __popc(win);
            nw += pw;
            occ += ri.i == 0 ? pw : 0;
            if (full) {
                atomicOr(&full255[o >> 5], full << (o & 31));
                s_flag[0] = 1;
            }
            // changed 16-bin chunks: lanes 4c..4c+3 form chunk (g >> 2); one
            // atomic per wave on chg word (g >> 7), bits (g >> 2) & 31
            uint64_t m = __ballot(changed);
            if (lane == 0 && m) {
                m |= m >> 1;
                m |= m >> 2;
                uint32_t bits = 0;
#pragma unroll
                for (int c4 = 0; c4 < 16; c4++) bits |= (uint32_t)((m >> (4 * c4)) & 1) << c4;
                atomicOr(&chg[g >> 7], bits << ((g >> 2) & 31));
            }
        }
        if (KH_ABL(P, 1)) nw = 0;
        PH(4);
        // changed 16-bin chunks back to the table; the rare full255 re-read
        auto write_back = [&]() {
            // pass 2: write back changed 16-bin chunks; winners to the region's segment
            for (uint32_t x = t; x < nchunk; x += blockDim.x) {
                if (!((chg[x >> 5] >> (x & 31)) & 1) || (KH_ABL(P, 4))) continue;
                const uint4 cv = ((const uint4 *)c0)[x];
                if (KIND == BYTE) {
                    ((uint4 *)(tab + ri.bin_lo))[x] = cv;
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
                    ((uint2 *)(tab + (ri.bin_lo >> 1)))[x] = o;
                }
            }
            if (bigc && s_flag[0]) {
                // bins at 255 before the batch: every insert is "full"
                // (ByteStorage::add, storage.hh:590-603); rare, so the region's
                // records are read again
                for (uint64_t q = ri.e0 + t; q < ri.e1; q += TH) {
                    const uint64_t x = A.rec[q];
                    const uint32_t o = (uint32_t)x;
                    if (x != ~0ull && ((full255[o >> 5] >> (o & 31)) & 1)) full_add(A.fullf, (uint32_t)(x >> 32));
                }
            }
        };
        if (A.coarse) {
            // Coarse-window runs.  The count loop reads only this thread's own
            // pass-1 results (its wflag groups and minj bins), so one barrier
            // publishes the counts and pass 1 (c0, chg, flags) together; every
            // wave then scans the window counts itself (lane c: window c) and
            // places its winners in LDS (the dead count array) without another
            // barrier; wave 0's returning reservation atomics complete
            // meanwhile; consecutive lanes write the runs.
            const int cjs = A.cjs;
            if constexpr (LOS) {
                // complement mode: the region's records again (L2-resident:
                // the count loop just read them), each a loser unless its bin
                // was zero before the pass and its k-mer index is the bin's
                // minimum; losers are counted per coarse window and listed
                // unsorted in the dead count array (a region's records fit its
                // 2^s0 entries: the host's reg_max check)
                block_sync();   // pass 1's wflag / minj of every bin
                const uint32_t lane = t & 63;
                const uint64_t pend = (ri.e1 + 1) >> 1;
                for (uint64_t pr0 = ri.e0 >> 1; pr0 < pend; pr0 += TH) {   // uniform trip count (ballots)
                    const uint64_t pr = pr0 + t, r = 2 * pr;
                    uint64_t xs[2] = {~0ull, ~0ull};
                    if (pr < pend) {
                        const ulonglong2 xx = *(const ulonglong2 *)(A.rec + r);
                        if (r >= ri.e0) xs[0] = xx.x;
                        if (r + 1 < ri.e1) xs[1] = xx.y;
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint64_t x = xs[h];
                        bool lose = false;
                        const uint32_t j = (uint32_t)(x >> 32);
                        if (x != ~0ull) {
                            const uint32_t o = (uint32_t)x;
                            lose = !(((wflag[o >> 2] >> (o & 3)) & 1u) && minj[o] == j);
                        }
                        const uint64_t m = __ballot(lose);
                        if (!m) continue;
                        uint32_t base = 0;
                        if (lane == 0) base = atomicAdd(&s_flag[2], (uint32_t)__popcll(m));
                        base = __shfl(base, 0, 64);
                        if (lose) {
                            cnt[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = j;
                            atomicAdd(&chist[j >> cjs], 1u);
                        }
                    }
                }
            } else if (nw) {
#pragma unroll
                for (int step = 0; step < BPT / 4; step++) {
                    const uint32_t g = t + (uint32_t)step * TH;
                    const uint32_t win = wflag[g];
                    if (!win) continue;
                    const uint4 m = ((const uint4 *)minj)[g];
                    if (win & 1) atomicAdd(&chist[m.x >> cjs], 1u);
                    if (win & 2) atomicAdd(&chist[m.y >> cjs], 1u);
                    if (win & 4) atomicAdd(&chist[m.z >> cjs], 1u);
                    if (win & 8) atomicAdd(&chist[m.w >> cjs], 1u);
                }
            }
            block_sync();
            publish();
            PH(2);
            if (bigc && t == 0 && s_flag[1]) {
                const uint64_t seg = atomicAdd((unsigned long long *)&A.ctr[CTR_NCROSS], 1ull);
                A.xseg[seg] = make_uint4((uint32_t)ri.e0, (uint32_t)(ri.e0 >> 32), (uint32_t)(ri.e1 - ri.e0), s_flag[1]);
            }
            prefetch_region<KIND, TH>(P, A, r1, total, bnext, nxt);
            bnext = bafter;
            write_back();
            PH(6);
            const uint32_t lane = t & 63;
            const uint32_t cc = chist[lane];
            uint32_t incl = cc;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= (uint32_t)d) incl += y;
            }
            const uint32_t st0 = incl - cc;
            const uint32_t wall = __shfl(incl, 63, 64);
            unsigned long long my_gb = 0;
            if (t < 64 && cc && !(KH_ABL(P, 512))) my_gb = atomicAdd(&A.cw_cur[t], (unsigned long long)cc);   // 512: timing only
            PH(7);
            uint32_t *wst = cnt;
            if constexpr (LOS) {
                // the listed losers, counting-sorted by window into the dead
                // min-j array (window starts through LDS, one more barrier)
                if (t < 64) cst0[t] = st0;
                block_sync();
                wst = minj;
                const uint32_t nl = s_flag[2];
                for (uint32_t x = t; x < nl; x += TH) {
                    const uint32_t j = cnt[x], c = j >> cjs;
                    wst[cst0[c] + atomicAdd(&ccur[c], 1u)] = j;
                }
            } else {
#pragma unroll
                for (int step = 0; step < BPT / 4; step++) {
                    const uint32_t g = t + (uint32_t)step * TH;
                    const uint32_t win = wflag[g];
                    if (!__ballot(win != 0)) continue;   // wave-uniform: the shuffles below need every lane
                    const uint4 m = ((const uint4 *)minj)[g];
                    const uint32_t mv[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const bool ok = (win >> k) & 1u;
                        const uint32_t c = ok ? mv[k] >> cjs : 0u;
                        const uint32_t base = __shfl(st0, (int)c, 64);
                        if (ok) wst[base + atomicAdd(&ccur[c], 1u)] = mv[k];
                    }
                }
            }
            if (t == 0) A.wcnt[rr] = wall;
            if (t < 64) {
                cgb[t] = my_gb;
                cst0[t] = st0;
            }
            block_sync();
            for (uint32_t x = t; x < wall; x += TH) {
                const uint32_t v = wst[x], c = v >> cjs;
                A.wco[cgb[c] + (x - cst0[c])] = v;
            }
            block_sync();
            PH(3);
            cur = nxt;
            advance();
            continue;
        }
        const uint32_t wex = wave_winner_scan(nw, s_wt);
        block_sync();
        publish();
        PH(2);
        if (bigc && t == 0 && s_flag[1]) {
            const uint64_t seg = atomicAdd((unsigned long long *)&A.ctr[CTR_NCROSS], 1ull);
            A.xseg[seg] = make_uint4((uint32_t)ri.e0, (uint32_t)(ri.e0 >> 32), (uint32_t)(ri.e1 - ri.e0), s_flag[1]);
        }
        prefetch_region<KIND, TH>(P, A, r1, total, bnext, nxt);
        bnext = bafter;
        write_back();
        uint32_t wall;
        uint32_t pos = winner_base(s_wt, &wall) + wex;
        uint32_t *wst = cnt;
        // winners: staged in LDS in region order (the count array is dead
        // after pass 1), then written to the region's segment by consecutive
        // lanes -- coalesced, where each lane writing its own run directly
        // scatters every store instruction over ~64 lines
        if (nw) {
#pragma unroll
            for (int step = 0; step < BPT / 4; step++) {
                const uint32_t g = t + (uint32_t)step * TH;
                const uint32_t win = wflag[g];
                if (!win) continue;
                const uint4 m = ((const uint4 *)minj)[g];
                if (win & 1) wst[pos++] = m.x;
                if (win & 2) wst[pos++] = m.y;
                if (win & 4) wst[pos++] = m.z;
                if (win & 8) wst[pos++] = m.w;
            }
        }
        if (t == 0) A.wcnt[rr] = wall;
        block_sync();
        for (uint32_t x = t; x < wall; x += TH) A.win[ri.e0 + x] = wst[x];
        block_sync();
        PH(3);
        cur = nxt;
        advance();
    }
    PH_WG_END(43);
    PH_END(16, 8);
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// Record-driven apply for sparse regions (C4 / C5 / C5M: ~6-7K records over
// 2^14 bins; the host takes it when every region's capacity fits the
// APPLY_RECS x 1024 records the workgroup prefetches, so a region's records
// ARE the registers the prefetch filled).  The same batch semantics as
// k_apply_count's coarse path (ByteStorage::add / NibbleStorage::add,
// storage.hh:571-624 / 320-359), but nothing walks the 2^14 bins:
//  - cnt / minj are zero / NO_J between regions: each region resets the bins
//    its records touched (and the staging slots it used) instead of clearing
//    128 KB of LDS;
//  - pass 1 runs per record: the record whose k-mer index is its bin's
//    minimum owns the bin (one record per (k-mer, region): a region is one
//    table) and computes the bin's saturated value, winner (bin zero before
//    the pass), crossing and changed chunk; every record knows whether it is
//    listed (a winner, or in complement mode a loser) and whether its bin was
//    full before the batch (bigcount: full_add directly, no full255 re-read);
//  - the listed k-mer indices go from registers into the coarse-window runs.
// Barriers a region: table chunk + state in, count atomics, per-record reads,
// owner writes + resets, write-back + runs, reset of the staging slots.
template <int KIND, bool LOS>
__global__ void __launch_bounds__(1024, 1) k_apply_sparse(Params P, ApplyArgs A) {
    constexpr int TH = 1024;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t R = 1u << P.s0;
    uint32_t *cnt = (uint32_t *)smem;      // [R] zero between regions; the runs' staging array
    uint32_t *minj = cnt + R;              // [R] NO_J between regions
    uint8_t *c0 = (uint8_t *)(minj + R);   // [R] the region's values
    uint32_t *chg = (uint32_t *)(c0 + R);  // [R/512] changed 16-bin chunks
    uint32_t *s_flag = chg + R / 512;      // [4] [1] crossings
    uint32_t *chist = s_flag + 4;          // [MAX_CW] window counts
    uint32_t *cst0 = chist + MAX_CW;       // [MAX_CW] window's first staging slot
    uint32_t *ccur = cst0 + MAX_CW;        // [MAX_CW] placement cursors
    uint32_t *s_q = ccur + MAX_CW;         // [2] region queue
    unsigned long long *cgb = (unsigned long long *)(s_q + 2);   // [MAX_CW] output bases
    const uint32_t MAXC = KIND == BYTE ? 255u : 15u;
    const bool bigc = KIND == BYTE && P.use_bigcount;
    const uint32_t t = threadIdx.x;
    const int cjs = A.cjs;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    for (uint32_t x = t; x < R / 4; x += TH) {
        ((uint4 *)cnt)[x] = make_uint4(0, 0, 0, 0);
        ((uint4 *)minj)[x] = make_uint4(NO_J, NO_J, NO_J, NO_J);
    }
    Prefetch cur, nxt;
    const uint64_t G = gridDim.x;
    uint64_t r1 = blockIdx.x + G, r2 = blockIdx.x + 2 * G;
    uint32_t par = 0;
    prefetch_region<KIND, TH>(P, A, blockIdx.x, total, load_bounds(P, A, blockIdx.x, total), cur);
    Bounds bnext = load_bounds(P, A, r1, total);
    for (uint64_t rr = blockIdx.x; rr < total;) {
        unsigned long long qn = 0;
        if (A.dyn && t == 0) qn = atomicAdd((unsigned long long *)&A.ctr[CTR_APQ], 1ull);
        auto publish = [&]() {
            if (A.dyn && t == 0) s_q[par] = (uint32_t)min<unsigned long long>(qn + 3 * G, total);
        };
        auto advance = [&]() {
            rr = r1;
            r1 = r2;
            r2 = A.dyn ? (uint64_t)uniform_u32(s_q[par]) : r2 + G;
            par ^= 1;
        };
        const RegionInfo ri = cur.ri;
        if (ri.e0 == ri.e1) {
            if (t == 0) A.wcnt[rr] = 0;
            prefetch_region<KIND, TH>(P, A, r1, total, bnext, cur);
            bnext = load_bounds(P, A, r2, total);
            if (A.dyn) {
                block_sync();
                publish();
                block_sync();
            }
            advance();
            continue;
        }
        const Bounds bafter = load_bounds(P, A, r2, total);
        const uint32_t nb = ri.nb;
        const uint32_t nchunk = (nb + 15) / 16;
        uint8_t *tab = A.tab + P.tbyte[ri.i];
        if (t < nchunk) {
            if (KIND == BYTE) {
                ((uint4 *)c0)[t] = cur.tv;
            } else {
                uint4 o;
                uint32_t *ow = (uint32_t *)&o;
                const uint32_t w[2] = {cur.tv.x, cur.tv.y};
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
        if (t < R / 512) chg[t] = 0;
        if (t < MAX_CW) chist[t] = ccur[t] = 0;
        if (t == 0) s_flag[1] = 0;
        block_sync();
#pragma unroll
        for (int u = 0; u < APPLY_RECS; u++) count_record(cur.v[u], cnt, minj);
        block_sync();
        // per record: owner of its bin?  listed?  (reads only: the owners'
        // writes wait for the barrier below)
        uint32_t lst = 0, own = 0;
        uint32_t fv[APPLY_RECS];
#pragma unroll
        for (int u = 0; u < APPLY_RECS; u++) {
            fv[u] = 0;
            const uint64_t x = cur.v[u];
            if (x == ~0ull) continue;
            const uint32_t o = (uint32_t)x, j = (uint32_t)(x >> 32);
            const uint32_t c = c0[o];
            const bool ow = minj[o] == j;
            const bool win = ow && c == 0;
            if (bigc && c == 255) full_add(A.fullf, j);   // every insert into a bin full before the batch
            if (LOS ? !win : win) {
                lst |= 1u << u;
                atomicAdd(&chist[j >> cjs], 1u);
            }
            if (ow) {
                const uint32_t v = c + cnt[o];
                const uint32_t f = v < MAXC ? v : MAXC;
                if (bigc && c < 255 && v > 255) {   // insert r sees c + r: full iff c + r >= 255, r < n
                    const uint32_t idx = atomicAdd(&s_flag[1], 1u);
                    A.xent[ri.e0 + idx] = (o << 8) | c;
                }
                if (f != c) {
                    own |= 1u << u;
                    fv[u] = f;
                }
                occ += ri.i == 0 && win;
            }
        }
        block_sync();
        // owners write their bins' values; every record resets its bin
#pragma unroll
        for (int u = 0; u < APPLY_RECS; u++) {
            const uint64_t x = cur.v[u];
            if (x == ~0ull) continue;
            const uint32_t o = (uint32_t)x;
            if ((own >> u) & 1u) {
                c0[o] = (uint8_t)fv[u];
                atomicOr(&chg[o >> 9], 1u << ((o >> 4) & 31));
            }
            cnt[o] = 0;
            minj[o] = NO_J;
        }
        publish();
        if (bigc && t == 0 && s_flag[1]) {
            const uint64_t seg = atomicAdd((unsigned long long *)&A.ctr[CTR_NCROSS], 1ull);
            A.xseg[seg] = make_uint4((uint32_t)ri.e0, (uint32_t)(ri.e0 >> 32), (uint32_t)(ri.e1 - ri.e0), s_flag[1]);
        }
        // window bases: every wave scans the window counts itself (lane c:
        // window c); wave 0 reserves the runs
        const uint32_t lane = t & 63;
        const uint32_t cc = chist[lane];
        uint32_t incl = cc;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        const uint32_t st0 = incl - cc;
        const uint32_t wall = __shfl(incl, 63, 64);
        unsigned long long my_gb = 0;
        if (t < 64 && cc) my_gb = atomicAdd(&A.cw_cur[t], (unsigned long long)cc);
        prefetch_region<KIND, TH>(P, A, r1, total, bnext, nxt);
        bnext = bafter;
        block_sync();
        // changed 16-bin chunks back to the table
        for (uint32_t x = t; x < nchunk; x += TH) {
            if (!((chg[x >> 5] >> (x & 31)) & 1)) continue;
            const uint4 cv = ((const uint4 *)c0)[x];
            if (KIND == BYTE) {
                ((uint4 *)(tab + ri.bin_lo))[x] = cv;
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
                ((uint2 *)(tab + (ri.bin_lo >> 1)))[x] = o;
            }
        }
        // listed k-mer indices -> staging (the reset count array) by window
#pragma unroll
        for (int u = 0; u < APPLY_RECS; u++) {
            if (!__ballot((lst >> u) & 1u)) continue;   // wave-uniform: the shuffle needs every lane
            const bool ok = (lst >> u) & 1u;
            const uint32_t j = (uint32_t)(cur.v[u] >> 32);
            const uint32_t c = ok ? j >> cjs : 0u;
            const uint32_t base = __shfl(st0, (int)c, 64);
            if (ok) cnt[base + atomicAdd(&ccur[c], 1u)] = j;
        }
        if (t == 0) A.wcnt[rr] = wall;
        if (t < 64) {
            cgb[t] = my_gb;
            cst0[t] = st0;
        }
        block_sync();
        for (uint32_t x = t; x < wall; x += TH) {
            const uint32_t v = cnt[x], c = v >> cjs;
            A.wco[cgb[c] + (x - cst0[c])] = v;
        }
        block_sync();
        for (uint32_t x = t; x < wall; x += TH) cnt[x] = 0;   // ordered before the next count atomics by its first barrier
        cur = nxt;
        advance();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}
__host__ __device__ constexpr size_t lds_apply_sparse(size_t R) {
    return R * 4 * 2 + (R / 512) * 4 + 16 + MAX_CW * 4 * 3 + 8 + MAX_CW * 8 + R;
}

// Bit storage (Bloom): BitStorage::test_and_set_bits (storage.hh:172-199)
// TH threads over a region of 2^14 bins (BPT bins per thread).  Coarse-window
// winners (A.coarse) are counting-sorted in LDS exactly as in k_apply_count,
// staged in wst[] (BIT has no count array to reuse, so it has its own).
template <int TH>
__global__ void __launch_bounds__(TH, 4) k_apply_bit(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BPT = (1 << 14) / TH;
    const uint32_t R = 1u << P.s0;
    uint32_t *minj = (uint32_t *)smem;          // [R]
    uint32_t *chg = minj + R;                   // [4] changed 128-bin chunks
    uint32_t *s_wt = chg + 4;                   // [16]
    uint32_t *bits32 = s_wt + 16;               // [R/32]
    uint8_t *bits = (uint8_t *)bits32;
    uint32_t *chist = bits32 + R / 32;          // [MAX_CW] coarse windows: counts, then cursors
    uint32_t *cst0 = chist + MAX_CW;            // [MAX_CW] window's first staging slot
    unsigned long long *cgb = (unsigned long long *)(cst0 + MAX_CW);   // [MAX_CW] window's output base
    uint32_t *ccur = (uint32_t *)(cgb + MAX_CW);           // [MAX_CW] placement cursors
    uint32_t *s_q = ccur + MAX_CW;                          // [2] dynamic region order (as k_apply_count)
    uint32_t *wst = s_q + 2;                                // [R] winners in window order (coarse only)
    const uint32_t t = threadIdx.x;
    uint64_t occ = 0;
    const uint64_t total = A.rprefix[P.n];
    Prefetch cur, nxt;
    const uint64_t G = gridDim.x;   // region order as in k_apply_count
    uint64_t r1 = blockIdx.x + G, r2 = blockIdx.x + 2 * G;
    uint32_t par = 0;
    prefetch_region<BIT, TH>(P, A, blockIdx.x, total, load_bounds(P, A, blockIdx.x, total), cur);
    Bounds bnext = load_bounds(P, A, r1, total);
    for (uint64_t rr = blockIdx.x; rr < total;) {
        unsigned long long qn = 0;
        if (A.dyn && t == 0) qn = atomicAdd((unsigned long long *)&A.ctr[CTR_APQ], 1ull);
        auto publish = [&]() {
            if (A.dyn && t == 0) s_q[par] = (uint32_t)min<unsigned long long>(qn + 3 * G, total);
        };
        auto advance = [&]() {
            rr = r1;
            r1 = r2;
            r2 = A.dyn ? (uint64_t)uniform_u32(s_q[par]) : r2 + G;
            par ^= 1;
        };
        const RegionInfo ri = cur.ri;
        if (ri.e0 == ri.e1) {
            if (t == 0) A.wcnt[rr] = 0;
            prefetch_region<BIT, TH>(P, A, r1, total, bnext, cur);
            bnext = load_bounds(P, A, r2, total);
            if (A.dyn) {
                block_sync();
                publish();
                block_sync();
            }
            advance();
            continue;
        }
        const Bounds bafter = load_bounds(P, A, r2, total);
        const uint32_t nb = ri.nb;
        const uint32_t nchunk = (nb + 127) / 128;   // 16 bytes = 128 bins per chunk
        uint8_t *tab = A.tab + P.tbyte[ri.i] + (ri.bin_lo >> 3);
        if (t < nchunk) ((uint4 *)bits)[t] = cur.tv;
        for (uint32_t x = t; x < nchunk * 32; x += blockDim.x) ((uint4 *)minj)[x] = make_uint4(NO_J, NO_J, NO_J, NO_J);
        if (t < 4) chg[t] = 0;
        if (t < MAX_CW) chist[t] = ccur[t] = 0;
        block_sync();
        {
            const uint64_t step = (uint64_t)(APPLY_RECS / 2) * TH;   // pairs
            const uint64_t pend = (ri.e1 + 1) >> 1;
            uint64_t va[APPLY_RECS], vb[APPLY_RECS];
            uint64_t q0 = (ri.e0 >> 1) + step;
            load_recs<TH>(A.rec, q0, ri.e0, ri.e1, va);
#pragma unroll
            for (int u = 0; u < APPLY_RECS; u++) bit_record(cur.v[u], minj);
            for (; q0 < pend; q0 += 2 * step) {
                load_recs<TH>(A.rec, q0 + step, ri.e0, ri.e1, vb);
#pragma unroll
                for (int u = 0; u < APPLY_RECS; u++) bit_record(va[u], minj);
                load_recs<TH>(A.rec, q0 + 2 * step, ri.e0, ri.e1, va);
#pragma unroll
                for (int u = 0; u < APPLY_RECS; u++) bit_record(vb[u], minj);
            }
        }
        block_sync();
        prefetch_region<BIT, TH>(P, A, r1, total, bnext, nxt);
        bnext = bafter;
        // pass 1 (thread per bin): winners set their bit (and, coarse, count
        // per window)
        uint32_t nw = 0;
        const uint32_t lane = t & 63;
        const int cjs = A.cjs;
#pragma unroll 2
        for (int u = 0; u < BPT; u++) {
            const uint32_t o = t + (uint32_t)u * TH;
            bool win = false;
            const uint32_t m = o < nb ? minj[o] : NO_J;
            if (m != NO_J) {
                if ((bits[o >> 3] >> (o & 7)) & 1) {   // bit already set: not new
                    minj[o] = NO_J;
                } else {
                    win = true;
                    nw++;
                    occ += (ri.i == 0);
                    if (A.coarse) atomicAdd(&chist[m >> cjs], 1u);
                }
            }
            // a wave's 64 bins are two 32-bit words of the bit array and one
            // 128-bin write-back chunk
            const uint64_t bm = __ballot(win);
            if (bm) {
                if (lane == 0 && (uint32_t)bm) atomicOr(&bits32[o >> 5], (uint32_t)bm);
                if (lane == 32 && (uint32_t)(bm >> 32)) atomicOr(&bits32[o >> 5], (uint32_t)(bm >> 32));
                if (lane == 0) atomicOr(&chg[o >> 12], 1u << ((o >> 7) & 31));
            }
        }
        const uint32_t wex = wave_winner_scan(nw, s_wt);
        block_sync();
        publish();
        // pass 2: write back changed 128-bin chunks; winners
        for (uint32_t x = t; x < nchunk; x += blockDim.x)
            if ((chg[x >> 5] >> (x & 31)) & 1) ((uint4 *)tab)[x] = ((const uint4 *)bits)[x];
        uint32_t wall;
        uint64_t pos = ri.e0 + winner_base(s_wt, &wall) + wex;
        if (t == 0) A.wcnt[rr] = wall;
        if (A.coarse) {
            // every wave scans the window counts itself (lane c: window c) and
            // places its winners without another barrier (as k_apply_count)
            const uint32_t cc = chist[lane];
            uint32_t incl = cc;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= (uint32_t)d) incl += y;
            }
            const uint32_t st0 = incl - cc;
            unsigned long long my_gb = 0;
            if (t < 64 && cc && !(KH_ABL(P, 512))) my_gb = atomicAdd(&A.cw_cur[t], (unsigned long long)cc);   // 512: timing only
#pragma unroll 2
            for (int u = 0; u < BPT; u++) {
                const uint32_t o = t + (uint32_t)u * TH;
                const uint32_t m = o < nb ? minj[o] : NO_J;
                const bool ok = m != NO_J;
                const uint32_t c = ok ? m >> cjs : 0u;
                const uint32_t base = __shfl(st0, (int)c, 64);
                if (ok) wst[base + atomicAdd(&ccur[c], 1u)] = m;
            }
            if (t < 64) {
                cgb[t] = my_gb;
                cst0[t] = st0;
            }
            block_sync();
            for (uint32_t x = t; x < wall; x += TH) {
                const uint32_t v = wst[x], c = v >> cjs;
                A.wco[cgb[c] + (x - cst0[c])] = v;
            }
        } else if (nw) {
#pragma unroll 2
            for (int u = 0; u < BPT; u++) {
                const uint32_t o = t + (uint32_t)u * TH;
                const uint32_t m = o < nb ? minj[o] : NO_J;
                if (m != NO_J) A.win[pos++] = m;
            }
        }
        block_sync();
        cur = nxt;
        advance();
    }
    occ = wave_sum(occ);
    if ((threadIdx.x & 63) == 0 && occ) atomicAdd((unsigned long long *)&A.ctr[CTR_OCC], (unsigned long long)occ);
}

// ---------------------------------------------------------------------------
// winner lists -> k-mer windows of 2^js (chunks of W_RPC consecutive regions)
__device__ __forceinline__ uint32_t w_chunk_setup(const Params &P, const ApplyArgs &A, uint64_t total,
                                                  uint32_t *s_pre, uint64_t *s_e0) {
    const uint64_t rr0 = (uint64_t)blockIdx.x * W_RPC;
    if (threadIdx.x < W_RPC) {
        const uint64_t rr = rr0 + threadIdx.x;
        const uint32_t c = rr < total ? A.wcnt[rr] : 0;
        s_e0[threadIdx.x] = c ? load_bounds(P, A, rr, A.rprefix[P.n]).e0 : 0;
        const uint32_t lane = threadIdx.x;
        uint32_t incl = c;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= (uint32_t)d) incl += y;
        }
        s_pre[lane + 1] = incl;
        if (lane == 0) s_pre[0] = 0;
    }
    block_sync();
    return s_pre[W_RPC];
}
__device__ __forceinline__ uint32_t w_elem(const ApplyArgs &A, const uint32_t *s_pre, const uint64_t *s_e0,
                                           uint32_t i) {
    uint32_t lo = 0, hi = W_RPC;   // largest lo with s_pre[lo] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_pre[mid] <= i) lo = mid; else hi = mid;
    }
    return A.win[s_e0[lo] + (i - s_pre[lo])];
}

__global__ void __launch_bounds__(PT_THREADS) k_hist_w(Params P, ApplyArgs A, int js, uint32_t FJ, uint32_t nchw,
                                                      uint32_t *M3) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_e0 = (uint64_t *)smem;             // [W_RPC]
    uint32_t *s_pre = (uint32_t *)(s_e0 + W_RPC);  // [W_RPC + 1]
    uint32_t *hist = s_pre + W_RPC + 4;            // [FJ]
    for (uint32_t b = threadIdx.x; b < FJ; b += blockDim.x) hist[b] = 0;
    const uint32_t n = w_chunk_setup(P, A, A.rprefix[P.n], s_pre, s_e0);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[w_elem(A, s_pre, s_e0, i) >> js], 1u);
    block_sync();
    for (uint32_t b = threadIdx.x; b < FJ; b += blockDim.x) M3[(uint64_t)b * nchw + blockIdx.x] = hist[b];
}

template <int THREADS, int SEG>
__global__ void __launch_bounds__(THREADS) k_scatter_w(Params P, ApplyArgs A, int js, uint32_t FJ, uint32_t nchw,
                                                      const uint64_t *O3, uint32_t *wout) {
    constexpr int TILE = THREADS * PT_RPT;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t FJa = (FJ + 3) & ~3u;
    uint64_t *s_e0 = (uint64_t *)smem;             // [W_RPC]
    uint32_t *s_pre = (uint32_t *)(s_e0 + W_RPC);  // [W_RPC + 1]
    uint64_t *lcur = (uint64_t *)(s_pre + W_RPC + 4);  // [FJ]  (W_RPC + 4 keeps 8-B alignment)
    uint32_t *stage = (uint32_t *)(lcur + FJa);    // [TILE]
    uint32_t *tail = stage + TILE;                 // [FJ*SEG]
    uint32_t *hist = tail + (SEG > 1 ? FJa * SEG : 0); // [FJ]
    uint32_t *lstart = hist + FJa;                 // [FJ]
    uint32_t *s_wtot = lstart + FJa;               // [16]
    uint8_t *hskip = (uint8_t *)(s_wtot + 16);     // [FJ]
    const Emit<uint32_t, SEG> em{lcur, hskip, tail, hist, lstart, nullptr, nullptr, nullptr, nullptr};
    for (uint32_t b = threadIdx.x; b < FJ; b += THREADS) em.init(b, O3[(uint64_t)b * nchw + blockIdx.x]);
    const uint32_t n = w_chunk_setup(P, A, A.rprefix[P.n], s_pre, s_e0);
    const uint32_t ntiles = uniform_u32((n + TILE - 1) / TILE);
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint32_t t0 = ti * TILE;
        const uint32_t t1 = min(n, t0 + TILE);
        const bool last = ti + 1 == ntiles;
        block_sync();
        uint32_t v[PT_RPT], rank[PT_RPT];
#pragma unroll
        for (int q = 0; q < PT_RPT; q++) {
            const uint32_t idx = t0 + (uint32_t)q * THREADS + threadIdx.x;
            v[q] = idx < t1 ? w_elem(A, s_pre, s_e0, idx) : NO_J;
        }
#pragma unroll
        for (int q = 0; q < PT_RPT; q++)
            if (v[q] != NO_J) rank[q] = atomicAdd(&hist[v[q] >> js], 1u);
        block_sync();
        block_scan_hist(hist, lstart, FJ, s_wtot);
        block_sync();
#pragma unroll
        for (int q = 0; q < PT_RPT; q++)
            if (v[q] != NO_J) stage[lstart[v[q] >> js] + rank[q]] = v[q];
        em.flush_tails(FJ, last, wout);
        block_sync();
        const uint32_t nrec = t1 - t0;
#pragma unroll
        for (int u = 0; u < PT_RPT; u++) {
            const uint32_t q = threadIdx.x + (uint32_t)u * THREADS;
            if (q < nrec) em.put_cur(stage[q] >> js, q, stage[q], last, wout);
        }
        block_sync();
        em.advance(FJ, last);
    }
}

// one workgroup per window: bitmap of the window's winners in LDS; n_unique +=
// its population; optionally the bitmap is written out (per-k-mer new flags)
__global__ void __launch_bounds__(PT_THREADS) k_mark(const uint32_t *wout, const uint64_t *O3, const uint32_t *M3,
                                                    uint32_t nchw, uint32_t FJ, int js, uint64_t *ctr,
                                                    uint32_t *newbits) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *bits = (uint32_t *)smem;   // [2^js / 32]
    const uint32_t nw = 1u << (js - 5);
    const uint32_t jb = blockIdx.x;
    const uint64_t s = O3[(uint64_t)jb * nchw];
    const uint64_t last = (uint64_t)FJ * nchw - 1;
    const uint64_t e = jb + 1 < FJ ? O3[(uint64_t)(jb + 1) * nchw] : O3[last] + M3[last];
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) ((uint4 *)bits)[t] = make_uint4(0, 0, 0, 0);
    block_sync();
    const uint32_t mask = (1u << js) - 1;
    for (uint64_t q = s + threadIdx.x; q < e; q += blockDim.x) {
        const uint32_t j = wout[q] & mask;
        atomicOr(&bits[j >> 5], 1u << (j & 31));
    }
    block_sync();
    uint64_t uniq = 0;
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) {
        const uint4 x = ((const uint4 *)bits)[t];
        uniq += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        if (newbits) ((uint4 *)(newbits + (uint64_t)jb * nw))[t] = x;
    }
    uniq = wave_sum(uniq);
    if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
}

// ---------------------------------------------------------------------------
// Coarse-window winners -> fine windows of 2^js k-mers -> LDS bitmaps.  A
// chunk is a contiguous slice of one coarse window's winners (host-planned
// from the windows' counts); the count matrix is laid out [coarse][fine][chunk]
// so one exclusive scan gives every (fine window, chunk) its output offset and
// every fine window one contiguous range.
struct WChunk {
    uint64_t start, end;     // winners [start, end) of wco
    uint64_t mbase;          // chunk_prefix(coarse) * fpc
    uint32_t k, nk;          // chunk index inside its coarse window, chunks of that window
};
constexpr int WF_THREADS = 1024;
constexpr int WF_RPT = 8;
constexpr int WF_TILE = WF_THREADS * WF_RPT;
constexpr uint32_t WF_CHUNK = 16 * WF_TILE;   // winners per chunk
constexpr uint32_t FPC_MAX = 256;             // fine windows per coarse window (complement mode: 256)

__global__ void __launch_bounds__(WF_THREADS) k_hist_wf(const uint32_t *wco, const WChunk *chunks, int js,
                                                        uint32_t fpc, uint32_t *M) {
    __shared__ uint32_t hist[FPC_MAX];
    const WChunk ch = chunks[blockIdx.x];
    if (threadIdx.x < FPC_MAX) hist[threadIdx.x] = 0;
    block_sync();
    // eight loads in flight per thread
    for (uint64_t i0 = ch.start; i0 < ch.end; i0 += 8 * WF_THREADS) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint64_t i = i0 + (uint64_t)u * WF_THREADS + threadIdx.x;
            v[u] = i < ch.end ? wco[i] : NO_J;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (v[u] != NO_J) atomicAdd(&hist[(v[u] >> js) & (fpc - 1)], 1u);
    }
    block_sync();
    if (threadIdx.x < fpc) M[ch.mbase + (uint64_t)threadIdx.x * ch.nk + ch.k] = hist[threadIdx.x];
}

__global__ void __launch_bounds__(WF_THREADS) k_scatter_wf(const uint32_t *wco, const WChunk *chunks, int js,
                                                           uint32_t fpc, const uint64_t *O, uint32_t *wout) {
    __shared__ uint32_t stage[WF_TILE];
    __shared__ uint32_t hist[FPC_MAX], lstart[FPC_MAX];
    __shared__ uint64_t cur[FPC_MAX];
    const WChunk ch = chunks[blockIdx.x];
    if (threadIdx.x < fpc) {
        cur[threadIdx.x] = O[ch.mbase + (uint64_t)threadIdx.x * ch.nk + ch.k];
        hist[threadIdx.x] = 0;
    }
    const uint32_t ntiles = uniform_u32((uint32_t)((ch.end - ch.start + WF_TILE - 1) / WF_TILE));
    for (uint32_t ti = 0; ti < ntiles; ti++) {
        const uint64_t t0 = ch.start + (uint64_t)ti * WF_TILE;
        block_sync();
        uint32_t v[WF_RPT], rank[WF_RPT];
#pragma unroll
        for (int q = 0; q < WF_RPT; q++) {
            const uint64_t i = t0 + (uint64_t)q * WF_THREADS + threadIdx.x;
            v[q] = i < ch.end ? wco[i] : NO_J;
            if (v[q] != NO_J) rank[q] = atomicAdd(&hist[(v[q] >> js) & (fpc - 1)], 1u);
        }
        block_sync();
        if (threadIdx.x < 64) {   // lane l: fine windows 4l .. 4l + 3
            const uint32_t l = threadIdx.x;
            uint32_t c4[4], sum = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                c4[k] = 4 * l + k < fpc ? hist[4 * l + k] : 0;
                sum += c4[k];
            }
            uint32_t incl = sum;
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (l >= (uint32_t)d) incl += y;
            }
            uint32_t acc = incl - sum;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (4 * l + k < fpc) lstart[4 * l + k] = acc;
                acc += c4[k];
            }
        }
        block_sync();
#pragma unroll
        for (int q = 0; q < WF_RPT; q++)
            if (v[q] != NO_J) stage[lstart[(v[q] >> js) & (fpc - 1)] + rank[q]] = v[q];
        block_sync();
        const uint32_t n = (uint32_t)min((uint64_t)WF_TILE, ch.end - t0);
        for (uint32_t x = threadIdx.x; x < n; x += WF_THREADS) {
            const uint32_t vv = stage[x], f = (vv >> js) & (fpc - 1);
            wout[cur[f] + (x - lstart[f])] = vv;
        }
        block_sync();
        if (threadIdx.x < fpc) {
            cur[threadIdx.x] += hist[threadIdx.x];
            hist[threadIdx.x] = 0;
        }
    }
}

// one workgroup per fine window: its winners' LDS bitmap -> n_unique (and the
// per-k-mer new flags when asked); range [O[mbase(c) + f*nk_c], next).
// Complement mode (ntab != 0): the range holds losers, one per (k-mer, table)
// the k-mer did not win; a k-mer is new unless it lost in all ntab tables
// (ByteStorage::add's is_new, storage.hh:571-588), so the window counts losers
// per k-mer in 4-bit LDS counters (ntab <= 15) and its k-mers [0, nkmers) with
// a count below ntab are the new ones.
__global__ void __launch_bounds__(PT_THREADS) k_mark_wf(const uint32_t *wout, const uint64_t *O,
                                                        const uint64_t *cmbase, const uint32_t *cnk, uint32_t fpc,
                                                        int js, uint64_t *ctr, uint32_t *newbits, uint32_t ntab,
                                                        uint64_t nkmers) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *bits = (uint32_t *)smem;   // [2^js / 32] (complement mode: [2^js / 8] 4-bit counts)
    const uint32_t nw = 1u << (js - 5);
    const uint32_t fw = blockIdx.x, c = fw / fpc, f = fw % fpc;
    const uint32_t nk = cnk[c];
    uint64_t s = 0, e = 0;
    if (nk) {   // O has one entry past the matrix (the total): (c, f + 1)'s start ends (c, f)
        s = O[cmbase[c] + (uint64_t)f * nk];
        e = O[cmbase[c] + (uint64_t)(f + 1) * nk];
    }
    if (ntab) {
        const uint32_t ncw = 1u << (js - 3);   // count words
        for (uint32_t t = threadIdx.x; t < ncw / 4; t += blockDim.x) ((uint4 *)bits)[t] = make_uint4(0, 0, 0, 0);
        block_sync();
        const uint32_t mask = (1u << js) - 1;
        for (uint64_t q0 = s; q0 < e; q0 += 8 * (uint64_t)blockDim.x) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint64_t q = q0 + (uint64_t)u * blockDim.x + threadIdx.x;
                v[u] = q < e ? wout[q] : NO_J;
            }
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (v[u] != NO_J) {
                    const uint32_t j = v[u] & mask;
                    atomicAdd(&bits[j >> 3], 1u << (4 * (j & 7)));
                }
        }
        block_sync();
        const uint64_t j0 = (uint64_t)fw << js;
        const uint32_t nvalid = (uint32_t)min((uint64_t)1 << js, nkmers - j0);
        uint64_t uniq = 0;
        for (uint32_t t = threadIdx.x; t < nw; t += blockDim.x) {   // 32 k-mers: four count words
            const uint4 x = ((const uint4 *)bits)[t];
            const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
            uint32_t nb = 0;
#pragma unroll
            for (int w4 = 0; w4 < 4; w4++)
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t jl = 32 * t + 8 * w4 + k;
                    if (jl < nvalid && ((xw[w4] >> (4 * k)) & 15u) != ntab) nb |= 1u << (8 * w4 + k);
                }
            uniq += __popc(nb);
            if (newbits) newbits[(uint64_t)fw * nw + t] = nb;
        }
        uniq = wave_sum(uniq);
        if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
        return;
    }
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) ((uint4 *)bits)[t] = make_uint4(0, 0, 0, 0);
    block_sync();
    const uint32_t mask = (1u << js) - 1;
    // eight loads in flight per thread (one per iteration left the window's
    // stream latency-bound at ~2 TB/s)
    for (uint64_t q0 = s; q0 < e; q0 += 8 * (uint64_t)blockDim.x) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const uint64_t q = q0 + (uint64_t)u * blockDim.x + threadIdx.x;
            v[u] = q < e ? wout[q] : NO_J;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (v[u] != NO_J) {
                const uint32_t j = v[u] & mask;
                atomicOr(&bits[j >> 5], 1u << (j & 31));
            }
    }
    block_sync();
    uint64_t uniq = 0;
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) {
        const uint4 x = ((const uint4 *)bits)[t];
        uniq += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
        if (newbits) ((uint4 *)(newbits + (uint64_t)fw * nw))[t] = x;
    }
    uniq = wave_sum(uniq);
    if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
}

// ---------------------------------------------------------------------------
// crossing bins (bigcount): inserts with stream rank >= 255 - c0 are "full"
// (ByteStorage::add, storage.hh:590-603).  One workgroup per region with
// crossings: up to X_GB of its crossing bins at a time get the K-th smallest
// k-mer index of their records by a 4-pass 8-bit radix select, all of them in
// the same sweeps over the region's records (LDS slot map offset -> bin).
constexpr int X_GB = 32;
__global__ void __launch_bounds__(256) k_crossing(Params P, const uint64_t *rec, const uint4 *xseg,
                                                  const uint32_t *xent, const uint64_t *ctr, uint8_t *fullf) {
    __shared__ uint8_t slot[1 << 14];
    __shared__ uint32_t hist[X_GB * 257];    // padded rows: slot s's serial scan stays on its own banks
    __shared__ uint32_t s_pre[X_GB], s_k[X_GB];
    const uint64_t nseg = ctr[CTR_NCROSS];
    const uint32_t R = 1u << P.s0;
    for (uint64_t sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
        const uint4 d = xseg[sg];
        const uint64_t e0 = (uint64_t)d.x | ((uint64_t)d.y << 32), e1 = e0 + d.z;
        const uint32_t m = d.w;
        for (uint32_t g0 = 0; g0 < m; g0 += X_GB) {
            const uint32_t nb = min((uint32_t)X_GB, m - g0);
            for (uint32_t x = threadIdx.x; x < R / 4; x += blockDim.x) ((uint32_t *)slot)[x] = 0xFFFFFFFFu;
            block_sync();
            if (threadIdx.x < nb) {
                const uint32_t e = xent[e0 + g0 + threadIdx.x];
                slot[e >> 8] = (uint8_t)threadIdx.x;
                s_k[threadIdx.x] = 255 - (e & 0xFF);   // rank of the first full insert (< the bin's inserts)
                s_pre[threadIdx.x] = 0;
            }
            block_sync();
            for (int pass = 0; pass < 4; pass++) {
                const int sh = 24 - 8 * pass;
                for (uint32_t x = threadIdx.x; x < nb * 257; x += blockDim.x) hist[x] = 0;
                block_sync();
                for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
                    const uint64_t v = rec[q];
                    if (v == ~0ull) continue;   // fixed-capacity level 2 sentinel
                    const uint32_t sl = slot[(uint32_t)v];
                    if (sl == 0xFF) continue;
                    const uint32_t j = (uint32_t)(v >> 32);
                    if (pass > 0 && (j >> (sh + 8)) != (s_pre[sl] >> (sh + 8))) continue;
                    atomicAdd(&hist[sl * 257 + ((j >> sh) & 0xFF)], 1u);
                }
                block_sync();
                if (threadIdx.x < nb) {
                    const uint32_t sl = threadIdx.x;
                    uint32_t K = s_k[sl], acc = 0, dg = 0;
                    for (dg = 0; dg < 256; dg++) {
                        const uint32_t h = hist[sl * 257 + dg];
                        if (acc + h > K) break;
                        acc += h;
                    }
                    s_pre[sl] |= dg << sh;
                    s_k[sl] = K - acc;
                }
                block_sync();
            }
            for (uint64_t q = e0 + threadIdx.x; q < e1; q += blockDim.x) {
                const uint64_t v = rec[q];
                if (v == ~0ull) continue;
                const uint32_t sl = slot[(uint32_t)v];
                if (sl == 0xFF) continue;
                const uint32_t j = (uint32_t)(v >> 32);
                if (j >= s_pre[sl]) full_add(fullf, j);
            }
            block_sync();
        }
    }
}

// ---------------------------------------------------------------------------
// finalize (bigcount and/or per-k-mer hash output only): k-mers full in every
// table are bigcount events (storage.hh:606-616), aggregated per hash in an
// open-addressing device map (one count per distinct hash; the host merges
// min(65535, base + count), which is order-independent).  A probe run longer
// than BC_PROBES flags CTR_ERR bit 2: the host grows the map and reruns.
constexpr int BC_PROBES = 128;
__device__ __forceinline__ void bc_event(uint64_t *keys, uint32_t *cnt, uint64_t mask, uint64_t *ctr, uint64_t h) {
    if (h == BC_EMPTY) {
        atomicAdd((unsigned long long *)&ctr[CTR_BCFF], 1ull);
        return;
    }
    uint64_t s = fmix64(h) & mask;
    for (int probe = 0; probe < BC_PROBES; probe++, s = (s + 1) & mask) {
        uint64_t k = __atomic_load_n(&keys[s], __ATOMIC_RELAXED);
        if (k == BC_EMPTY) {
            k = atomicCAS((unsigned long long *)&keys[s], (unsigned long long)BC_EMPTY, (unsigned long long)h);
            if (k == BC_EMPTY) {
                atomicAdd((unsigned long long *)&ctr[CTR_NBC], 1ull);
                k = h;
            }
        }
        if (k == h) {
            atomicAdd(&cnt[s], 1u);
            return;
        }
    }
    atomicOr((unsigned long long *)&ctr[CTR_ERR], 2ull);
}

template <class Src>
__global__ void __launch_bounds__(FIN_THREADS) k_finalize(Params P, Src src, uint64_t nkmers, const uint8_t *fullf,
                                                         uint64_t *ctr, uint64_t *bck, uint32_t *bcv, uint64_t bmask,
                                                         uint64_t *out_hash) {
    const bool bigc = P.kind == BYTE && P.use_bigcount && bck;
    const uint64_t nchunk = (nkmers + 15) / 16;
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunk;
         c += (uint64_t)gridDim.x * blockDim.x) {
        if (bigc) {
            const uint4 fv = ((const uint4 *)fullf)[c];
            if (fv.x | fv.y | fv.z | fv.w) {
                const uint8_t *fb = (const uint8_t *)&fv;
                for (int u = 0; u < 16; u++) {
                    const uint64_t j = c * 16 + u;
                    if (j < nkmers && fb[u] == (uint8_t)P.n) bc_event(bck, bcv, bmask, ctr, kmer_hash_global(src, j));
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
}

// occupied map slots -> (keys, counts) for the host merge
__global__ void k_bc_compact(const uint64_t *bck, const uint32_t *bcv, uint64_t cap, uint64_t *ctr, uint64_t *keys,
                             uint32_t *cnts) {
    for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = bck[s];
        if (k == BC_EMPTY) continue;
        const uint64_t i = atomicAdd((unsigned long long *)&ctr[CTR_BCOUT], 1ull);
        keys[i] = k;
        cnts[i] = bcv[s];
    }
}

// ---------------------------------------------------------------------------
// Small passes (a single add(), one short consume()): the reference's
// per-k-mer Storage::add (storage.hh:172-199, 320-359, 571-624) in stream
// order by one wavefront, lane i owning table i, instead of the partition
// pipeline whose fixed cost grows with the table size.  flags[j]: bit 0
// is_new, bit 1 table-0 first touch (n_occupied), bit 2 full in every table
// (a bigcount event); hashes[j] the k-mer's hash.  Not for shards.
template <class Src>
__global__ void __launch_bounds__(64) k_small_pass(Params P, Src src, uint64_t nkmers, uint8_t *tab, uint8_t *flags,
                                                   uint64_t *hashes) {
    __shared__ uint64_t sh[64];
    const uint32_t lane = threadIdx.x;
    const uint64_t nmask = P.n >= 64 ? ~0ull : ((1ull << P.n) - 1);
    for (uint64_t j0 = 0; j0 < nkmers; j0 += 64) {
        const uint64_t j = j0 + lane;
        if (j < nkmers) {
            const uint64_t h = kmer_hash_global(src, j);
            sh[lane] = h;
            hashes[j] = h;
        }
        block_sync();
        const uint32_t m = (uint32_t)min<uint64_t>(64, nkmers - j0);
        for (uint32_t u = 0; u < m; u++) {
            const uint64_t h = sh[u];
            bool zero = false, full = false;
            if ((int)lane < P.n) {
                const uint64_t bin = mod_barrett(h, P.p[lane], P.m[lane]);
                uint8_t *t = tab + P.tbyte[lane];
                if (P.kind == BIT) {
                    const uint8_t bit = (uint8_t)(1u << (bin & 7));
                    const uint8_t v = t[bin >> 3];
                    zero = !(v & bit);
                    t[bin >> 3] = v | bit;
                } else if (P.kind == NIBBLE) {   // even bin -> high nibble (storage.hh:262-272)
                    const int sh4 = (bin & 1) ? 0 : 4;
                    const uint8_t v = t[bin >> 1];
                    const uint32_t cur = (v >> sh4) & 15u;
                    zero = cur == 0;
                    if (cur < 15) t[bin >> 1] = (uint8_t)((v & ~(15u << sh4)) | ((cur + 1) << sh4));
                } else {
                    const uint32_t cur = t[bin];
                    zero = cur == 0;
                    if (cur < 255) t[bin] = (uint8_t)(cur + 1);
                    else full = true;
                }
            }
            const uint64_t zb = __ballot(zero) & nmask, fb = __ballot(full) & nmask;
            if (lane == 0)
                flags[j0 + u] = (uint8_t)((zb ? 1 : 0) | ((zb & 1) ? 2 : 0) |
                                          (P.kind == BYTE && P.use_bigcount && fb == nmask ? 4 : 0));
        }
        block_sync();
    }
}

// ---------------------------------------------------------------------------
// sharded groups (kh_engine.hip group_*): winners of every shard are routed to
// the rank owning their k-mer window; full events are merged on every rank

// window start offsets of the partitioned winner list (FJ + 1 entries)
__global__ void k_window_starts(const uint64_t *O3, const uint32_t *M3, uint32_t nchw, uint32_t FJ, uint64_t *ws) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= FJ; w += gridDim.x * blockDim.x) {
        const uint64_t last = (uint64_t)FJ * nchw - 1;
        ws[w] = w < FJ ? O3[(uint64_t)w * nchw] : O3[last] + M3[last];
    }
}

// the same from the coarse-window path's [coarse][fine][chunk] matrix
// (k_hist_wf / k_scatter_wf): fine window w = c * fpc + f starts at
// O[cmbase[c] + f * cnk[c]]; a coarse window without chunks, and every window
// past the last winner, starts at the running total (O has one entry past
// the matrix, and cmbase[c] = that entry for c >= the pass's coarse windows)
__global__ void k_window_starts_cw(const uint64_t *O, const uint64_t *cmbase, const uint32_t *cnk, uint32_t fpc,
                                   uint32_t FJ, uint64_t *ws) {
    for (uint32_t w = blockIdx.x * blockDim.x + threadIdx.x; w <= FJ; w += gridDim.x * blockDim.x) {
        const uint32_t c = w / fpc, f = w % fpc;
        ws[w] = c < MAX_CW ? O[cmbase[c] + (uint64_t)f * cnk[c]] : O[cmbase[MAX_CW]];
    }
}

// k_mark over windows [wlo, wlo + gridDim.x) whose winners arrived from G
// shards: source s's part of window w is recv[roff[s] + ws_s[w] - ws_s[wlo] ...)
__global__ void __launch_bounds__(PT_THREADS) k_mark_multi(const uint32_t *recv, const uint64_t *ws_all,
                                                          const uint64_t *roff, int G, uint32_t FJ, uint32_t wlo,
                                                          int js, uint64_t *ctr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t *bits = (uint32_t *)smem;   // [2^js / 32]
    const uint32_t nw = 1u << (js - 5);
    const uint32_t w = wlo + blockIdx.x;
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) ((uint4 *)bits)[t] = make_uint4(0, 0, 0, 0);
    block_sync();
    const uint32_t mask = (1u << js) - 1;
    for (int s = 0; s < G; s++) {
        const uint64_t *ws = ws_all + (uint64_t)s * (FJ + 1);
        const uint64_t b = roff[s] + (ws[w] - ws[wlo]);
        const uint64_t n = ws[w + 1] - ws[w];
        for (uint64_t q = threadIdx.x; q < n; q += blockDim.x) {
            const uint32_t j = recv[b + q] & mask;
            atomicOr(&bits[j >> 5], 1u << (j & 31));
        }
    }
    block_sync();
    uint64_t uniq = 0;
    for (uint32_t t = threadIdx.x; t < nw / 4; t += blockDim.x) {
        const uint4 x = ((const uint4 *)bits)[t];
        uniq += __popc(x.x) + __popc(x.y) + __popc(x.z) + __popc(x.w);
    }
    uniq = wave_sum(uniq);
    if ((threadIdx.x & 63) == 0 && uniq) atomicAdd((unsigned long long *)&ctr[CTR_UNIQUE], (unsigned long long)uniq);
}

// nonzero per-k-mer full tallies -> (j << 8 | tally) list (rare events)
__global__ void k_full_compact(const uint8_t *fullf, uint64_t nkmers, uint64_t *list, uint64_t cap, uint64_t *ctr) {
    // one counter atomic per wave (a saturated stream makes most k-mers full)
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n_iter = (nkmers + stride - 1) / stride;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t it = 0; it < n_iter; it++) {
        const uint64_t j = it * stride + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
        const uint32_t f = j < nkmers ? fullf[j] : 0u;
        const uint64_t m = __ballot(f != 0);
        if (!m) continue;
        uint64_t base = 0;
        if (lane == 0) base = atomicAdd((unsigned long long *)&ctr[CTR_NFULL], (unsigned long long)__popcll(m));
        base = __shfl(base, 0, 64);
        const uint64_t idx = base + (uint64_t)__popcll(m & ((1ull << lane) - 1));
        if (f && idx < cap) list[idx] = (j << 8) | f;   // overflow: the host sees NFULL > cap
    }
}

// dst += src bytewise over n bytes (16-B aligned, n a multiple of 16); the
// per-k-mer full tallies of all shards sum to at most N < 256, so no carries
__global__ void k_add_bytes(uint8_t *dst, const uint8_t *src, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n / 16; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 d = ((uint4 *)dst)[i];
        const uint4 s = ((const uint4 *)src)[i];
        d.x += s.x;
        d.y += s.y;
        d.z += s.z;
        d.w += s.w;
        ((uint4 *)dst)[i] = d;
    }
}

// add merged full tallies back into fullf (entries ~0 are padding)
__global__ void k_full_scatter(const uint64_t *list, uint64_t n, uint8_t *fullf) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t e = list[i];
        if (e == ~0ull) continue;
        const uint32_t j = (uint32_t)(e >> 8);
        atomicAdd((uint32_t *)(fullf + (j & ~3u)), (uint32_t)(e & 0xFF) << (8 * (j & 3u)));
    }
}


// ---------------------------------------------------------------------------
// Delta mode (group mode KH_GROUP_DELTA, kh_engine.hip group_consume_delta).
// Every rank partitions its own chunk in the unsharded geometry, and
// k_apply_delta writes the table that chunk ALONE would produce from empty
// tables -- min(cap, inserts) per bin, in the storage's own layout (Byte: 1
// B per bin; Nibble: even bin -> high nibble, storage.hh:262-272; Bit: bin b
// -> bit b % 8 of byte b / 8, storage.hh:172-199) -- into the view's table
// arena.  No k-mer index is needed: the table value of a bin is order-free
// (SURVEY F4).  One workgroup of TH threads per region of R = 16 * TH bins
// (every region is written, empty ones as zeros, so the arena needs no
// clearing).
template <int KIND, int TH>
__global__ void __launch_bounds__(TH) k_apply_delta(Params P, ApplyArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int BPT = 16;
    const uint32_t R = 1u << P.s0;
    uint32_t *cnt = (uint32_t *)smem;   // [R]
    const uint32_t t = threadIdx.x;
    const uint32_t cap = KIND == BYTE ? 255u : KIND == NIBBLE ? 15u : 1u;
    const uint64_t total = A.rprefix[P.n];
    for (uint64_t rr = blockIdx.x; rr < total; rr += gridDim.x) {
        const RegionInfo ri = region_info(P, A, rr, load_bounds(P, A, rr, total));
        const bool any = ri.e0 != ri.e1;
        if (any) {
            for (uint32_t x = t; x < R / 4; x += TH) ((uint4 *)cnt)[x] = make_uint4(0, 0, 0, 0);
            block_sync();
            // 16-B record pairs, APPLY_RECS records per thread in flight
            const uint64_t step = (uint64_t)(APPLY_RECS / 2) * TH;
            for (uint64_t q0 = ri.e0 >> 1; 2 * q0 < ri.e1; q0 += step) {
                uint64_t v[APPLY_RECS];
                load_recs<TH>(A.rec, q0, ri.e0, ri.e1, v);
#pragma unroll
                for (int u = 0; u < APPLY_RECS; u++)
                    if (v[u] != ~0ull) atomicAdd(&cnt[(uint32_t)v[u]], 1u);
            }
            block_sync();
        }
        // this thread's 16 bins -> their bytes of the region
        const uint32_t b0 = BPT * t;
        if (b0 < ri.nb) {
            uint32_t c[BPT];
            if (any) {
#pragma unroll
                for (int q = 0; q < BPT / 4; q++) {
                    const uint4 n4 = ((const uint4 *)cnt)[4 * t + q];
                    c[4 * q] = min(n4.x, cap);
                    c[4 * q + 1] = min(n4.y, cap);
                    c[4 * q + 2] = min(n4.z, cap);
                    c[4 * q + 3] = min(n4.w, cap);
                }
            } else {
#pragma unroll
                for (int q = 0; q < BPT; q++) c[q] = 0;
            }
            // the chunk's bytes (16 / 8 / 2) in o; a chunk that runs past the
            // table's last byte (the arena pads tables to 256 B, and the
            // padding may be shorter than a chunk) is written byte by byte
            uint8_t *tab = A.tab + P.tbyte[ri.i];
            uint32_t o[4] = {0, 0, 0, 0};
            uint64_t at;
            int nby;
            if (KIND == BYTE) {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    o[q] = c[4 * q] | c[4 * q + 1] << 8 | c[4 * q + 2] << 16 | c[4 * q + 3] << 24;
                at = ri.bin_lo + b0;
                nby = 16;
            } else if (KIND == NIBBLE) {
#pragma unroll
                for (int q = 0; q < 2; q++)
                    o[q] = (c[8 * q] << 4 | c[8 * q + 1]) | (c[8 * q + 2] << 4 | c[8 * q + 3]) << 8 |
                           (c[8 * q + 4] << 4 | c[8 * q + 5]) << 16 | (c[8 * q + 6] << 4 | c[8 * q + 7]) << 24;
                at = (ri.bin_lo + b0) >> 1;
                nby = 8;
            } else {
#pragma unroll
                for (int q = 0; q < BPT; q++) o[0] |= c[q] << q;
                at = (ri.bin_lo + b0) >> 3;
                nby = 2;
            }
            if (at + nby <= P.tbytes[ri.i]) {
                if (KIND == BYTE) *(uint4 *)(tab + at) = make_uint4(o[0], o[1], o[2], o[3]);
                else if (KIND == NIBBLE) *(uint2 *)(tab + at) = make_uint2(o[0], o[1]);
                else *(uint16_t *)(tab + at) = (uint16_t)o[0];
            } else {
                for (int q = 0; q < nby && at + q < P.tbytes[ri.i]; q++) tab[at + q] = (uint8_t)(o[q >> 2] >> (8 * (q & 3)));
            }
        }
        if (any) block_sync();   // cnt is reused by the next region
    }
}

// The owner's prefix over ranks (delta mode): for every byte x of its slice,
// the table value before the pass t = T[x]; rank r's chunk sees
// P_r = t + D_0 + ... + D_{r-1} (saturating, in the storage's layout) and
// T[x] becomes t + D_0 + ... + D_{W-1}.  buf[r * stride + x] holds D_r on
// entry and P_r on exit.  Exact because min(cap, a + min(cap, b)) =
// min(cap, a + b) (storage.hh:320-359, 571-624 saturate; bits OR).
template <int KIND>
__device__ __forceinline__ uint32_t sat_add4(uint32_t a, uint32_t b) {
    if (KIND == BIT) return a | b;
    uint32_t o = 0;
    if (KIND == BYTE) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t s = ((a >> (8 * k)) & 0xFF) + ((b >> (8 * k)) & 0xFF);
            o |= min(s, 255u) << (8 * k);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t s = ((a >> (4 * k)) & 0xF) + ((b >> (4 * k)) & 0xF);
            o |= min(s, 15u) << (4 * k);
        }
    }
    return o;
}
template <int KIND>
__global__ void k_delta_prefix(uint8_t *T, uint8_t *buf, uint64_t nbytes, uint64_t stride, int W) {
    const uint64_t n16 = nbytes / 16;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (nbytes + 15) / 16;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (i < n16) {
            uint4 tv = ((const uint4 *)T)[i];
            for (int r = 0; r < W; r++) {
                uint4 *p = (uint4 *)(buf + (uint64_t)r * stride) + i;
                const uint4 d = *p;
                *p = tv;
                tv = make_uint4(sat_add4<KIND>(tv.x, d.x), sat_add4<KIND>(tv.y, d.y), sat_add4<KIND>(tv.z, d.z),
                                sat_add4<KIND>(tv.w, d.w));
            }
            ((uint4 *)T)[i] = tv;
        } else {   // the slice's last < 16 bytes
            for (uint64_t x = 16 * i; x < nbytes; x++) {
                uint32_t tv = T[x];
                for (int r = 0; r < W; r++) {
                    uint8_t *p = buf + (uint64_t)r * stride + x;
                    const uint32_t d = *p;
                    *p = (uint8_t)tv;
                    tv = sat_add4<KIND>(tv, d) & 0xFF;
                }
                T[x] = (uint8_t)tv;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Sparse delta pieces (delta mode's table exchange, kh_engine.hip
// delta_exchange): a byte range of nb bytes travels as a bitmap of its
// nonzero bytes (a u16 mask per 16 bytes, nb / 8 bytes) followed by the
// nonzero bytes in order.  A workgroup of 256 threads codes one 4096-byte
// chunk (16 bytes a thread); chunk payload offsets come from an exclusive
// scan of the per-chunk counts (sender: from the bytes, receiver: from the
// bitmap).  The ranges are 16-byte aligned (the host checks).
constexpr uint32_t SP_CHUNK = 4096;
constexpr int SP_THREADS = 256;
__device__ __forceinline__ uint32_t sp_mask16(uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int b = 0; b < 4; b++) m |= (((w[q] >> (8 * b)) & 0xFFu) != 0u ? 1u : 0u) << (4 * q + b);
    return m;
}
// this thread's 16 bytes (zero past nb)
__device__ __forceinline__ uint4 sp_load16(const uint8_t *src, uint64_t x0, uint64_t nb) {
    if (x0 + 16 <= nb) return *(const uint4 *)(src + x0);
    uint4 v = make_uint4(0, 0, 0, 0);
    uint8_t *b = (uint8_t *)&v;
    for (uint64_t x = x0; x < nb; x++) b[x - x0] = src[x];
    return v;
}
// block-wide exclusive prefix of n (256 threads), total in *tot
__device__ __forceinline__ uint32_t sp_block_prefix(uint32_t n, uint32_t *s_w, uint32_t *tot) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = n;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t q = 0; q < SP_THREADS / 64; q++) {
        before += q < wv ? s_w[q] : 0u;
        all += s_w[q];
    }
    *tot = all;
    return before + incl - n;
}
// per-chunk nonzero counts, from the bytes (bm == null) or from the bitmap;
// cnt[nchunks] = 0 (the scan's last value is then the total)
__global__ void __launch_bounds__(SP_THREADS) k_sp_count(const uint8_t *src, const uint16_t *bm, uint64_t nb,
                                                         uint32_t *cnt) {
    __shared__ uint32_t s_w[SP_THREADS / 64];
    const uint64_t c = blockIdx.x;
    const uint64_t x0 = c * SP_CHUNK + 16ull * threadIdx.x;
    uint32_t n = 0;
    if (x0 < nb) n = __popc(bm ? (uint32_t)bm[x0 / 16] : sp_mask16(sp_load16(src, x0, nb)));
    uint32_t tot;
    (void)sp_block_prefix(n, s_w, &tot);
    if (threadIdx.x == 0) {
        cnt[c] = tot;
        if (c + 1 == gridDim.x) cnt[c + 1] = 0;
    }
}
__global__ void __launch_bounds__(SP_THREADS) k_sp_pack(const uint8_t *src, uint64_t nb, const uint64_t *off,
                                                        uint16_t *bm, uint8_t *pay) {
    __shared__ uint32_t s_w[SP_THREADS / 64];
    const uint64_t c = blockIdx.x;
    const uint64_t x0 = c * SP_CHUNK + 16ull * threadIdx.x;
    uint4 v = make_uint4(0, 0, 0, 0);
    uint32_t m = 0;
    if (x0 < nb) {
        v = sp_load16(src, x0, nb);
        m = sp_mask16(v);
        bm[x0 / 16] = (uint16_t)m;
    }
    uint32_t tot;
    uint64_t pos = off[c] + sp_block_prefix((uint32_t)__popc(m), s_w, &tot);
    const uint8_t *b = (const uint8_t *)&v;
#pragma unroll
    for (int q = 0; q < 16; q++)
        if ((m >> q) & 1u) pay[pos++] = b[q];
}
__global__ void __launch_bounds__(SP_THREADS) k_sp_unpack(const uint16_t *bm, const uint8_t *pay, const uint64_t *off,
                                                          uint64_t nb, uint8_t *dst) {
    __shared__ uint32_t s_w[SP_THREADS / 64];
    const uint64_t c = blockIdx.x;
    const uint64_t x0 = c * SP_CHUNK + 16ull * threadIdx.x;
    const uint32_t m = x0 < nb ? (uint32_t)bm[x0 / 16] : 0u;
    uint32_t tot;
    uint64_t pos = off[c] + sp_block_prefix((uint32_t)__popc(m), s_w, &tot);
    if (x0 >= nb) return;
    uint4 v = make_uint4(0, 0, 0, 0);
    uint8_t *b = (uint8_t *)&v;
#pragma unroll
    for (int q = 0; q < 16; q++)
        if ((m >> q) & 1u) b[q] = pay[pos++];
    if (x0 + 16 <= nb) {
        *(uint4 *)(dst + x0) = v;
    } else {
        for (uint64_t x = x0; x < nb; x++) dst[x] = b[x - x0];
    }
}

}  // namespace kh
