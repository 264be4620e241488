// kh_engine.hip -- the MI355X hot path of libkhmer_hip.so (host orchestration).
//
// Replaces the reference's per-k-mer loop Hashtable::consume_string ->
// Storage::add (src/oxli/hashtable.cc:280-294, include/oxli/storage.hh:172-199,
// 320-359, 571-624) with a batch pipeline whose results equal the reference's
// single-threaded ones, tables and counters alike:
//
//   count_l1 / scan_l1 / scatter_l1   hash every k-mer (2-bit canonical or
//       Murmur), N exact bins (Barrett), records into level-1 buckets
//   count_l2 / scan_l2 / scatter_l2   buckets -> LDS-sized regions
//   apply      one workgroup per region: counts, stream-order winners,
//              saturating write-back, table-0 occupancy, bigcount "full" flags
//   crossing   (bigcount, rare) exact ranks inside bins reaching 255
//   finalize   n_unique, bigcount candidates
//
// Kernels: kh_partition.cuh, kh_apply.cuh, kh_query.cuh.  A bin's final value
// depends only on the multiset of its inserts; the order-
// dependent counters come from the k-mer index carried by every record.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include "kh_apply.cuh"
#include "kh_internal.h"
#include "kh_nearprime.cuh"
#include "kh_query.cuh"

namespace kh {

// ---------------------------------------------------------------------------
// workspace
static void ensure(void **p, uint64_t *cap, uint64_t need, size_t elem) {
    if (need <= *cap) return;
    if (*p) KH_HIP(hipFree(*p));
    *p = nullptr;
    uint64_t n = std::max<uint64_t>(need, *cap + *cap / 2);
    KH_HIP(hipMalloc(p, n * elem + 64));
    *cap = n;
}


// Device fill with 16-byte stores and 64-bit indices, for every range that
// can be large (tables, record buffers, per-k-mer flags); hipMemsetAsync
// only below 1 MiB.  Round 5's `bench.py --ablate 16` run faulted ("illegal
// memory access") in its first pass after a hipMemsetAsync of the whole
// level-1 buffer (~1.35e11 bytes) -- the only difference from the clean
// --ablate 0 run of the same build; no memset that large remains
// (DESIGN.md §5.3).
__global__ void k_fill16(uint4 *p, uint64_t n, uint4 v) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}
void dev_fill(void *p, int v, uint64_t bytes, hipStream_t st) {
    uint8_t *b = (uint8_t *)p;
    if (bytes < (1u << 20)) {
        if (bytes) KH_HIP(hipMemsetAsync(p, v, bytes, st));
        return;
    }
    const uint64_t head = (16 - ((uintptr_t)b & 15)) & 15;
    if (head) {
        KH_HIP(hipMemsetAsync(b, v, head, st));
        b += head;
        bytes -= head;
    }
    const uint64_t n = bytes / 16;
    const uint32_t w = (uint32_t)(uint8_t)v * 0x01010101u;
    const unsigned grid = (unsigned)std::min<uint64_t>(n / 256 + 1, 16384);
    hipLaunchKernelGGL(k_fill16, dim3(grid), dim3(256), 0, st, (uint4 *)b, n, make_uint4(w, w, w, w));
    KH_HIP(hipGetLastError());
    if (bytes & 15) KH_HIP(hipMemsetAsync(b + n * 16, v, bytes & 15, st));
}

static int ceil_log2(uint64_t x) {
    int s = 0;
    while ((1ull << s) < x) s++;
    return s;
}

// geometry of one device pass (all partitions are chunked counting sorts)
struct PassGeo {
    uint64_t nkmers, recs;
    uint32_t ck1, nch1;        // level-1 chunk (k-mers) and chunk count
    uint64_t nch2max;          // level-2 chunk bound
    int js;                    // winner window = 2^js k-mers
    uint32_t FJ, nchw;         // windows, winner chunks (W_RPC regions each)
    uint64_t regions;          // table regions (apply order)
    uint64_t mcnt;             // count-matrix entries (max over the three sorts)
};

static PassGeo pass_geo(const Params &P, uint64_t nkmers) {
    PassGeo q;
    q.nkmers = nkmers;
    q.recs = nkmers * (uint64_t)P.n;
    q.ck1 = 32768u * ((P.F1 + 1023) / 1024);
    q.nch1 = (uint32_t)((nkmers + q.ck1 - 1) / q.ck1);
    q.nch2max = q.recs / L2_CHUNK + P.F1 + 1;
    q.js = std::min(20, std::max(17, ceil_log2(nkmers) - 11));   // <= 3200 windows of <= 2^20 k-mers
    q.FJ = (uint32_t)((nkmers + (1ull << q.js) - 1) >> q.js);
    q.regions = 0;
    for (int i = 0; i < P.n; i++) q.regions += (P.lsz[i] + (1ull << P.s0) - 1) >> P.s0;
    q.nchw = (uint32_t)((q.regions + W_RPC - 1) / W_RPC);
    const uint64_t F2 = 1ull << P.s2;
    q.mcnt = std::max<uint64_t>({(uint64_t)P.F1 * q.nch1, F2 * q.nch2max, (uint64_t)q.FJ * q.nchw});
    return q;
}

static void bcmap_alloc(Workspace &w, uint64_t cap);
static void bcmap_clear(Workspace &w, hipStream_t st);

static void ws_prepare(Graph *g, const PassGeo &q) {
    Workspace &w = g->ws;
    if (q.nkmers > w.cap_kmers) {
        uint64_t cap = std::max<uint64_t>(q.nkmers, w.cap_kmers + w.cap_kmers / 2);
        cap = (cap + 15) & ~15ull;
        if (w.fullf) KH_HIP(hipFree(w.fullf));
        w.fullf = nullptr;
        KH_HIP(hipMalloc((void **)&w.fullf, cap + 64));
        w.cap_kmers = cap;
    }
    ensure((void **)&w.mcnt, &w.cap_m, q.mcnt, 4);
    ensure((void **)&w.moff, &w.cap_moff, q.mcnt, 8);
    ensure((void **)&w.wcnt, &w.cap_wcnt, q.regions, 4);
    ensure((void **)&w.newbits, &w.cap_newbits, ((uint64_t)q.FJ << q.js) / 32, 4);
    const uint64_t regions = (uint64_t)g->prm.F1 << g->prm.s2;
    if (regions > w.cap_regions || !w.off1) {
        for (void **pp : {(void **)&w.off1, (void **)&w.ch2, (void **)&w.off2})
            if (*pp) { KH_HIP(hipFree(*pp)); *pp = nullptr; }
        const uint64_t F1 = g->prm.F1;
        KH_HIP(hipMalloc((void **)&w.off1, (F1 + 1) * 8 + 64));
        KH_HIP(hipMalloc((void **)&w.ch2, (F1 + 1) * 4 + 64));
        KH_HIP(hipMalloc((void **)&w.off2, (regions + 1) * 8 + 64));
        w.cap_regions = regions;
    }
    ensure((void **)&w.xseg, &w.cap_xseg, regions + 1, sizeof(uint4));
    if (!w.ctr) {
        KH_HIP(hipMalloc((void **)&w.ctr, CTR_N * 8));
        KH_HIP(hipHostMalloc((void **)&w.h_ctr, CTR_N * 8, hipHostMallocDefault));
    }
    if (g->kind == BYTE && g->use_bigcount && !w.bck) bcmap_alloc(w, 1ull << 20);
}

// ---- per-pass bigcount map (k_finalize) ----
static void bcmap_alloc(Workspace &w, uint64_t cap) {
    for (void **pp : {(void **)&w.bck, (void **)&w.bcv, (void **)&w.bc, (void **)&w.bcn})
        if (*pp) { KH_HIP(hipFree(*pp)); *pp = nullptr; }
    KH_HIP(hipMalloc((void **)&w.bck, cap * 8));
    KH_HIP(hipMalloc((void **)&w.bcv, cap * 4));
    KH_HIP(hipMalloc((void **)&w.bc, cap * 8));
    KH_HIP(hipMalloc((void **)&w.bcn, cap * 4));
    w.cap_bcmap = cap;
}

static void bcmap_clear(Workspace &w, hipStream_t st) {
    KH_HIP(hipMemsetAsync(w.bck, 0xFF, w.cap_bcmap * 8, st));
    KH_HIP(hipMemsetAsync(w.bcv, 0, w.cap_bcmap * 4, st));
}

// ByteStorage::add's bigcount update (storage.hh:606-616) for a whole pass:
// f full inserts of hash h give bc[h] = min(65535, base + f), base = bc[h] if
// present else 255 -- the same value as f sequential updates.
static void bcmap_merge(Graph *g, uint64_t nkeys, uint64_t n_ff) {
    Workspace &w = g->ws;
    auto bump = [&](uint64_t h, uint64_t f) {
        auto it = g->bigcounts.find(h);
        const uint64_t base = it == g->bigcounts.end() ? 255 : it->second;
        g->bigcounts[h] = (uint16_t)std::min<uint64_t>(base + f, 65535);
    };
    if (n_ff) bump(BC_EMPTY, n_ff);
    if (nkeys) {
        const unsigned grid = (unsigned)std::min<uint64_t>((w.cap_bcmap + 255) / 256, 8192);
        hipLaunchKernelGGL(k_bc_compact, dim3(grid), dim3(256), 0, g->stream, w.bck, w.bcv, w.cap_bcmap, w.ctr, w.bc,
                           w.bcn);
        KH_HIP(hipGetLastError());
        std::vector<uint64_t> keys(nkeys);
        std::vector<uint32_t> cnts(nkeys);
        KH_HIP(hipMemcpyAsync(keys.data(), w.bc, nkeys * 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipMemcpyAsync(cnts.data(), w.bcn, nkeys * 4, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        g->bigcounts.reserve(g->bigcounts.size() + nkeys);
        for (uint64_t i = 0; i < nkeys; i++) bump(keys[i], cnts[i]);
    }
    if (nkeys || n_ff) g->bc_dirty = true;
}

// record buffers for a pass holding `recs` records (level-1 out / level-2 out;
// the dead level-1 buffer later holds the winner lists).  Sized from the
// device's exact count, so a shard only holds the records it owns.
static void ensure_recs(Graph *g, uint64_t recs, bool level2 = true) {
    Workspace &w = g->ws;
    if (recs <= w.cap_recs && w.rec1) return;
    // grow by half (fewer reallocations) while that fits next to everything
    // else on the device; the exact need otherwise
    uint64_t grow = w.cap_recs + w.cap_recs / 2;
    size_t freeb = 0, total = 0;
    if (hipMemGetInfo(&freeb, &total) == hipSuccess) {
        const double per = level2 ? 16.0 : 8.0;   // bytes per record of capacity (one or two buffers)
        const double fit = ((double)freeb + per * (double)w.cap_recs) * 0.95 / per - 64.0;
        grow = std::min<uint64_t>(grow, fit > 0 ? (uint64_t)fit : 0);
    } else {
        (void)hipGetLastError();
    }
    uint64_t cap = std::max<uint64_t>(recs, grow);
    cap = std::max<uint64_t>(cap, 1024);
    for (uint64_t **pp : {&w.rec1, &w.rec2}) {
        if (*pp) KH_HIP(hipFree(*pp));
        *pp = nullptr;
        if (!level2 && pp == &w.rec2) continue;   // level-1 only (an exchange-mode view)
        // KH_REC_MALLOC_FLAGS: development knob, hipExtMallocWithFlags flags for
        // the record buffers (placement experiments); plain hipMalloc otherwise
        static const char *fl = dev_getenv("KH_REC_MALLOC_FLAGS");
        if (fl && atoi(fl) &&
            hipExtMallocWithFlags((void **)pp, cap * 8 + 64, (unsigned)atoi(fl)) == hipSuccess)
            continue;
        (void)hipGetLastError();
        KH_HIP(hipMalloc((void **)pp, cap * 8 + 64));
    }
    w.cap_recs = cap;
}

// ---- fixed-capacity level 2 (k_scatter_l2f) ----
// Workgroups per level-1 bucket: enough for ~2048 in the grid.
static int env_seg(const char *name, int dflt);
static int l1f_blk_sh() { static const int v = env_seg("KH_L1F_BLK_SH", L1F_BLK_SH); return v; }
static int l2f_blk_sh() { static const int v = env_seg("KH_L2F_BLK_SH", L2F_BLK_SH); return v; }
static uint32_t l2f_parts(uint32_t F1) {
    static const int v = env_seg("KH_L2F_PARTS", 0);   // development: workgroups per bucket
    if (v > 0) return (uint32_t)v;
    // ~8K workgroups, at most 16 per bucket: few buckets' regions are written
    // at once (round 3: 32 per bucket at C2 beat 8 by 3 ms/step); round 5 at
    // C2 (240 buckets; profiles/r5/ab_l2_parts.txt, 2 rounds): 16 -> 237.9,
    // 32 -> 239.6-239.9, 24 -> 240.6-240.8, 12 -> 242.2 ms/step -- 16 and
    // 32 fill whole waves of one workgroup a CU (3840 / 7680 workgroups on
    // 256 CUs) and 16 leaves fewer partial blocks
    return std::max<uint32_t>(1, std::min<uint32_t>(16, (8192 + F1 - 1) / F1));
}
static size_t lds_scatter_l2f(const Params &P) { return ((size_t)1 << P.s2) * (8 + 8 + 16 * 8 + 4 + 4 + 2) + 16; }
// The fixed-capacity path is used when a full region expects >= 512 records
// per pass (the capacity slack is then a few percent); KH_L2_EXACT=1 forces
// the histogram path (development).
static bool l2f_wanted(const Graph *g, uint64_t nkmers) {
    static const bool off = [] { const char *e = dev_getenv("KH_L2_EXACT"); return e && atoi(e); }();
    if (off || g->l2_cool > 0) return false;
    const Params &P = g->prm;
    if ((1u << P.s2) > 1024) return false;
    for (int i = 0; i < P.n; i++)
        if ((double)nkmers * (double)(1ull << P.s0) / (double)P.p[i] < 512.0) return false;
    return true;
}

// Region capacities for passes of `nkmers` k-mers: expected records (a table
// gets one record per k-mer, spread over its p_i bins) + 8 sigma + the
// partially filled blocks of every workgroup; uploaded once per pass size.
// Returns the total capacity in records.
// A region is written by the level-2 workgroups of one level-1 bucket (the
// near-prime level 2, `np`: of two, the spill of the previous bucket's range).
// np2 (near-prime level 2, kh_nearprime.cuh): a region's first E + 1
// regions of each bucket range also take the previous bucket's spill, so
// twice the writing workgroups may leave a partial block there
static uint64_t reg_plan(Graph *g, uint64_t nkmers, const NPGeo *np2 = nullptr) {
    Workspace &w = g->ws;
    const Params &P = g->prm;
    const uint32_t nparts = np2 ? l2f_parts(np2->nb) : 0;
    const uint64_t npkey = np2 ? ((uint64_t)np2->rp << 40 | (uint64_t)np2->rloc << 20 | nparts) : 0;
    if (w.reg_base && w.reg_nkmers == nkmers && w.reg_sigma == g->cap_sigma && w.reg_np == npkey) return w.reg_total;
    const uint64_t nreg = (uint64_t)P.F1 << P.s2;
    const uint64_t R = 1ull << P.s0;
    const uint64_t blk = 1ull << l2f_blk_sh();
    const uint64_t slack1 = np2 ? (uint64_t)(nparts + 1) * blk + 16 : (uint64_t)(l2f_parts(P.F1) + 1) * blk + 16;
    const uint64_t slack2 = np2 ? (uint64_t)(2 * nparts + 1) * blk + 16 : slack1;
    const uint64_t E = np2 ? np2->rloc - np2->rp - 1 : 0;
    std::vector<uint64_t> base(nreg + 1, 0);
    uint64_t acc = 0, cmax = 0;
    int i = 0;
    for (uint64_t gi = 0; gi < nreg; gi++) {
        base[gi] = acc;
        const uint64_t lo = gi * R;
        while (i + 1 < P.n && lo >= P.tbase[i + 1]) i++;
        if (lo >= P.tbase[i] + P.lsz[i]) continue;   // padding up to the next bucket boundary
        const uint64_t nb = std::min<uint64_t>(R, P.tbase[i] + P.lsz[i] - lo);
        const double mean = (double)nkmers * (double)nb / (double)P.p[i];
        const uint64_t rho = (lo - P.tbase[i]) >> P.s0;
        const uint64_t slack = np2 && rho % np2->rp <= E ? slack2 : slack1;
        uint64_t c = (uint64_t)(mean + g->cap_sigma * sqrt(mean)) + slack;
        acc += (c + 15) & ~15ull;
        cmax = std::max<uint64_t>(cmax, (c + 15) & ~15ull);
    }
    base[nreg] = acc;
    ensure((void **)&w.reg_base, &w.cap_reg, nreg + 1, 8);
    uint64_t cap_cur = 0;
    if (w.reg_cur) KH_HIP(hipFree(w.reg_cur));
    w.reg_cur = nullptr;
    ensure((void **)&w.reg_cur, &cap_cur, nreg, 8);
    KH_HIP(hipMemcpy(w.reg_base, base.data(), (nreg + 1) * 8, hipMemcpyHostToDevice));
    w.reg_nkmers = nkmers;
    w.reg_sigma = g->cap_sigma;
    w.reg_np = npkey;
    w.reg_total = acc;
    w.reg_max = cmax;
    return acc;
}

// ---- fixed-capacity level 1 (k_scatter_l1f) ----
// up to 1024 buckets (the per-bucket LDS state), hashed sources with <= 8
// tables per launch; not for shards using the owned-record filter
static int env_seg(const char *name, int dflt) {   // development knobs: -DKH_DEV builds only
    const char *e = dev_getenv(name);
    return e && *e ? atoi(e) : dflt;
}
static int test_env_int(const char *name, int dflt) {   // read in every build: the tests set it
    const char *e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}
static bool use_own_filter(const Graph *g);
static size_t lds_window(bool window, int tile_kmers);
static int l1f_tables_per_launch();

// Level-1 launch windows.  k_scatter_l1f keeps per-bucket state in LDS for at
// most 1024 buckets; a geometry with more (C4 / C5: 4 x 8e9 bins = 1908
// buckets of 2^24 bins) runs one launch per group of consecutive tables whose
// buckets [bb0, bb0 + nb) number at most l1f_win_max() (512).  Every
// table starts on a bucket boundary (graph_prepare_params), so a group's
// buckets are contiguous and each launch fills its own range of the bucket
// buffer; the launch sees them as buckets 0 .. nb - 1 through a Params copy
// whose table bases are shifted down by bb0 buckets (win_params).  Each
// launch re-reads and re-hashes the k-mers (the 2-bit hash is ~3 % of level
// 1; Murmur sources are hashed once into a u64 array first, pass_stage_a).
struct L1Win {
    int t0, nt;
    uint32_t bb0, nb;
};
// Measured (C4 / C5 / C5M on one MI355X, profiles/r4_a): with the k-mers
// of a 2-bit source re-hashed per launch, windows of 954 or 477 buckets take
// 280 / 290 ms per step of level 1 against 195 for the exact two-pass level 1
// (k_hist_l1 + k_scatter_l1), so multi-window level 1 is used only for
// hashed-once sources (Murmur: 136 vs 151 ms at 477-bucket windows, 206 at
// 954) and the exact path keeps the rest.  Windows of at most 512 buckets:
// one table per launch at C4 / C5 / C5M.
static uint32_t l1f_win_max() {
    static const int v = [] {
        const char *e = dev_getenv("KH_L1_WIN");   // development A/B: buckets per launch
        const int x = e && *e ? atoi(e) : 512;
        return std::max(1, std::min(1024, x));
    }();
    return (uint32_t)v;
}
static std::vector<L1Win> l1f_windows(const Params &P, int tpl) {
    const int shift = P.s0 + P.s2;
    const uint32_t wmax = l1f_win_max();
    auto bs = [&](int i) -> uint32_t { return (uint32_t)(P.tbase[i] >> shift); };
    auto be = [&](int i) -> uint32_t { return i + 1 < P.n ? bs(i + 1) : P.F1; };
    std::vector<L1Win> v;
    if (P.F1 <= 1024 && P.n <= tpl) {   // one launch (C2: 240 buckets, C3: 956)
        v.push_back({0, P.n, 0, P.F1});
        return v;
    }
    for (int t0 = 0; t0 < P.n;) {
        if (be(t0) - bs(t0) > 1024) return {};   // one table alone is too large
        int nt = 1;
        while (t0 + nt < P.n && nt < tpl && be(t0 + nt) - bs(t0) <= wmax) nt++;
        v.push_back({t0, nt, bs(t0), std::max<uint32_t>(1, be(t0 + nt - 1) - bs(t0))});
        t0 += nt;
    }
    return v;
}
static Params win_params(const Params &P, const L1Win &w) {
    Params Q = P;
    Q.F1 = w.nb;
    const uint64_t sh = (uint64_t)w.bb0 << (P.s0 + P.s2);
    for (int i = w.t0; i < w.t0 + w.nt; i++) Q.tbase[i] -= sh;
    return Q;
}
static bool l1f_ok(const Graph *g) {
    static const bool off = [] { const char *e = dev_getenv("KH_L1_EXACT"); return e && atoi(e); }();
    return !off && !use_own_filter(g) && !l1f_windows(g->prm, l1f_tables_per_launch()).empty();
}
static uint32_t device_cus(const Graph *g) {
    static int cus[64] = {0};
    const int d = g->device & 63;
    if (!cus[d]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || v <= 0) v = 256;
        cus[d] = v;
    }
    return (uint32_t)cus[d];
}
// a persistent grid: two workgroups per CU (the kernel's LDS allows two at up
// to ~512 buckets), fewer for small passes
// records per thread and tile: 8 (3 workgroups per CU; 16 records with 2
// workgroups per CU measured slower, 117 vs 112 ms/step, round 2)
static int l1f_rpt() { return L1_MAX_RPT; }
// tiles per dynamically scheduled k_scatter_l1f chunk (0: one fixed share
// per workgroup); KH_L1_CHUNK overrides (development)
static uint32_t l1f_chunk_tiles(const Graph *g) {
    static const int v = env_seg("KH_L1_CHUNK", 32);
    return (uint32_t)std::max(0, g->l1_chunk >= 0 ? g->l1_chunk : v);
}
// dynamic region order in k_apply_count (KH_APPLY_DYN=0: the static stride; development)
static bool apply_dynamic(const Graph *g) {
    static const bool v = env_seg("KH_APPLY_DYN", 1) != 0;
    return g->apply_dyn >= 0 ? g->apply_dyn != 0 : v;
}
// tables per k_scatter_l1f launch (development A/B: fewer tables per launch
// means fewer live buckets and longer runs per tile, at one k-mer hash per launch)
static int l1f_tables_per_launch() {
    static const int v = std::max(1, std::min(L1_MAX_RPT, env_seg("KH_L1_NT", L1_MAX_RPT)));
    return v;
}
static size_t lds_scatter_l1f(const Params &P, bool window, int tile_kmers) {
    const size_t F1a = (P.F1 + 3) & ~3u;
    const size_t tile = (size_t)L1_THREADS * l1f_rpt();
    return F1a * 8 * 5 + (tile + 2 * F1a) * 4 + F1a * 4 * 5 + (tile + 2 * F1a) * 4 + 64 +
           lds_window(window, tile_kmers) + 2 * L1F_TW * 8;
}
// as many workgroups per CU as the LDS allows, up to the kernel's register
// budget (3 at 8 records per thread, 2 at 16); KH_L1F_WPC overrides (development)
static uint32_t l1f_wpc(const Params &P) {
    static const int v = env_seg("KH_L1F_WPC", 0);
    if (v > 0) return (uint32_t)v;
    const size_t lds = lds_scatter_l1f(P, false, L1_THREADS * l1f_rpt());
    const size_t regs = L1F_WAVES_PER_EU * 4 / (L1_THREADS / 64);
    return (uint32_t)std::max<size_t>(1, std::min<size_t>(regs, 163840 / lds));
}
// A 2-bit (or ASCII) source's level 1 in one k_scatter_l1f launch needs
// all F1 buckets' LDS arrays: beyond ~590 buckets only one workgroup fits a
// CU, and the exact two-pass level 1 is faster there (C3, 956 buckets: 404
// against 475 ms/step, profiles/r4/c3_level1.txt).  KH_L1F_ONE_WG=1 keeps the
// one-workgroup launch (development A/B).
static bool l1f_direct(const Params &P) {
    static const bool one = env_seg("KH_L1F_ONE_WG", 0) != 0;
    return P.F1 <= 1024 && (one || l1f_wpc(P) >= 2);
}
static bool use_own_filter(const Graph *g);
// workgroups of one level-1 launch over window geometry Q
static uint32_t l1f_workgroups_q(const Graph *g, const Params &Q, uint64_t nkmers) {
    const uint64_t tiles = (nkmers + L1_THREADS - 1) / L1_THREADS;
    const uint64_t wpc = use_own_filter(g) ? 2 : l1f_wpc(Q);   // k_own_l1f: ~75 KB of LDS
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles / 8 + 1, wpc * device_cus(g)));
}
// the most workgroups any level-1 launch of the pass has (each leaves at most
// one partial block per bucket it fills: bkt_plan's slack)
static uint32_t l1f_workgroups(const Graph *g, uint64_t nkmers) {
    if (use_own_filter(g)) return l1f_workgroups_q(g, g->prm, nkmers);
    uint32_t m = 1;
    for (const L1Win &w : l1f_windows(g->prm, l1f_tables_per_launch()))
        m = std::max(m, l1f_workgroups_q(g, win_params(g->prm, w), nkmers));
    return m;
}
static size_t lds_own_l1f(const Params &P) {
    const size_t F1a = (P.F1 + 3) & ~3u;
    return (size_t)OWNF_BUF * 8 + F1a * 60 + (size_t)OWN_BATCH * 2 + 48 * 4 + 2 * L1F_TW * 8;
}
// a shard's level 1 in one kernel (k_own_l1f) for fixed-length reads;
// KH_OWN_L1F=0 falls back to k_own_filter + k_scatter_l1<PRE> (development)
static bool own_l1f_on() { static const bool v = env_seg("KH_OWN_L1F", 1) != 0; return v; }
template <class Src>
using OwnL1FFn = void (*)(Params, Src, uint64_t, uint64_t, int, int, const uint64_t *, unsigned long long *,
                          uint64_t *, uint64_t *, int, uint32_t);
template <class Src>
static OwnL1FFn<Src> own_l1f_kernel(int kpt, bool tw) {
    if constexpr (std::is_same<Src, SrcTwoBit>::value) {
        if (tw) {
            switch (kpt) {
                case 1: return k_own_l1f<Src, 1, true>;
                case 2: return k_own_l1f<Src, 2, true>;
                case 4: return k_own_l1f<Src, 4, true>;
                default: return k_own_l1f<Src, 8, true>;
            }
        }
    }
    switch (kpt) {
        case 1: return k_own_l1f<Src, 1>;
        case 2: return k_own_l1f<Src, 2>;
        case 4: return k_own_l1f<Src, 4>;
        default: return k_own_l1f<Src, 8>;
    }
}
template <class Src>
using L1FFn = void (*)(Params, Src, uint64_t, uint64_t, int, int, const uint64_t *, unsigned long long *, uint64_t *,
                       uint64_t *, int, uint32_t, uint32_t);
// fixed-length 2-bit reads whose tiles span at most L1F_TW packed words take
// the LDS-staged variant (k_scatter_l1f<..., TW = true>)
template <class Src>
static bool l1f_tw(const Src &src, int kpt) {
    if constexpr (!std::is_same<Src, SrcTwoBit>::value) return false;
    else {
        static const bool off = env_seg("KH_L1F_TW", 1) == 0;   // development
        if (off || !src.kpr) return false;
        const uint64_t T = (uint64_t)L1_THREADS * kpt;
        const uint64_t reads = (T + src.kpr - 1) / src.kpr + 1;
        const uint64_t span = T + reads * (uint64_t)(src.k - 1) + (uint64_t)src.k;
        return span / 32 + 3 <= (uint64_t)L1F_TW;
    }
}
template <class Src>
static L1FFn<Src> l1f_kernel(int kpt, int rpt, bool tw = false) {
    (void)rpt;
    if constexpr (std::is_same<Src, SrcTwoBit>::value) {
        if (tw) {
            switch (kpt) {
                case 1: return k_scatter_l1f<Src, 1, 8, true>;
                case 2: return k_scatter_l1f<Src, 2, 8, true>;
                case 4: return k_scatter_l1f<Src, 4, 8, true>;
                default: return k_scatter_l1f<Src, 8, 8, true>;
            }
        }
    }
    switch (kpt) {
        case 1: return k_scatter_l1f<Src, 1>;
        case 2: return k_scatter_l1f<Src, 2>;
        case 4: return k_scatter_l1f<Src, 4>;
        default: return k_scatter_l1f<Src, 8>;
    }
}

// Bucket capacities for passes of `nkmers` k-mers: expected records + 8 sigma
// + one partial block per workgroup.  Returns the total capacity in records.
static uint64_t bkt_plan(Graph *g, uint64_t nkmers) {
    Workspace &w = g->ws;
    const Params &P = g->prm;
    if (w.bkt_base && w.bkt_nkmers == nkmers && w.bkt_sigma == g->cap_sigma) return w.bkt_total;
    const uint64_t F1 = P.F1, span = 1ull << (P.s0 + P.s2);
    const uint64_t slack = (uint64_t)l1f_workgroups(g, nkmers) * (1ull << l1f_blk_sh()) + 16;
    std::vector<uint64_t> base(F1 + 1, 0);
    uint64_t acc = 0;
    for (uint64_t b = 0; b < F1; b++) {
        base[b] = acc;
        const uint64_t lo = b * span, hi = lo + span;
        double mean = 0;   // a paired bucket may hold the end of one table and the start of the next
        for (int i = 0; i < P.n; i++) {
            const uint64_t a = std::max(lo, P.tbase[i]), e = std::min(hi, P.tbase[i] + P.lsz[i]);
            if (e > a) mean += (double)nkmers * (double)(e - a) / (double)P.p[i];
        }
        if (mean == 0) continue;
        const uint64_t c = (uint64_t)(mean + g->cap_sigma * sqrt(mean)) + slack;
        acc += (c + 15) & ~15ull;
    }
    base[F1] = acc;
    uint64_t cap = 0;
    for (void **pp : {(void **)&w.bkt_base, (void **)&w.bkt_cur})
        if (*pp) { KH_HIP(hipFree(*pp)); *pp = nullptr; }
    ensure((void **)&w.bkt_base, &cap, F1 + 1, 8);
    cap = 0;
    ensure((void **)&w.bkt_cur, &cap, F1 + 1, 8);
    KH_HIP(hipMemcpy(w.bkt_base, base.data(), (F1 + 1) * 8, hipMemcpyHostToDevice));
    w.bkt_nkmers = nkmers;
    w.bkt_sigma = g->cap_sigma;
    w.bkt_total = acc;
    return acc;
}

// ---- near-prime level 1 / level 2 (kh_nearprime.cuh) ----
// Taken for 2-bit fixed-length reads into 2-4 unsharded tables whose sizes
// are close enough that every k-mer's bins lie within a few regions of its
// bin in the largest table (khmer's get_n_primes_near_x sizes at C2 / C4
// scale); KH_NEAR_PRIME=0 keeps the per-table level 1 (read in every build:
// the tests compare both paths).
static bool np_enabled() { return test_env_int("KH_NEAR_PRIME", 1) != 0; }
// magic division check: (rho * magic) >> 32 == rho / d for every rho < n
static bool np_magic_ok(uint64_t n, uint32_t d, uint32_t magic) {
    for (uint64_t rho = 0; rho < n; rho++)
        if ((uint32_t)((rho * magic) >> 32) != rho / d) return false;
    return true;
}
// *fine: F = 0 for two levels; otherwise the level-1b split of each of the
// out->nb coarse buckets (out->rp = F x fine R') into F fine buckets, taken
// when the two-level geometry needs more than 256 level-1 buckets (C4) and a
// fine record (j << 32 | q << ob_f | offset) fits 64 bits.  KH_NP_L1MAX
// (tests) lowers the 256, so small tables take three levels too.
static bool np_geometry(const Graph *g, NPGeo *out, NPFine *fine) {
    const Params &P = g->prm;
    *fine = NPFine{};
    if (!np_enabled() || g->hash != TWOBIT || P.n < 2 || P.n > NP_MAXT || g->k > 26 || use_own_filter(g)) return false;
    for (int i = 0; i < P.n; i++)
        if (P.lo[i] != 0 || P.lsz[i] != P.p[i]) return false;
    NPGeo N{};
    N.n = P.n;
    N.s0 = P.s0;
    N.ablate = P.ablate;
    const uint64_t R = 1ull << P.s0;
    uint64_t pm = 0, dmax = 0;
    for (int i = 0; i < P.n; i++) pm = std::max<uint64_t>(pm, P.p[i]);
    for (int i = 0; i < P.n; i++) {
        N.d[i] = pm - P.p[i];
        N.p[i] = P.p[i];
        N.rt[i] = (uint32_t)((P.p[i] + R - 1) >> P.s0);
        N.rbase[i] = (uint32_t)(P.tbase[i] >> P.s0);
        dmax = std::max<uint64_t>(dmax, N.d[i]);
        if ((P.tbase[i] & (R - 1)) || (P.tbase[i] >> P.s0) >= (1ull << 32)) return false;
    }
    // h < 4^k: the quotient by P, and the farthest a bin lies past r
    const uint64_t qmax = ((1ull << (2 * g->k)) - 1) / pm;
    if (qmax >= (1ull << 31)) return false;
    const unsigned __int128 maxoff = (unsigned __int128)qmax * dmax;
    if (maxoff + 2 * (unsigned __int128)dmax >= pm) return false;   // r + q d_i < 2 p_i: one subtraction
    N.rloc = 1024u / (uint32_t)P.n;
    const uint64_t E = (uint64_t)((maxoff + R - 1) >> P.s0);   // regions of spill past a bucket's range
    if (E + 1 >= N.rloc / 2) return false;
    const uint32_t rpf = N.rloc - (uint32_t)E - 1;   // + 1: a wrapped bin's region index can round up by one
    const uint64_t Rm = (pm + R - 1) >> P.s0;
    const uint64_t lim = (uint64_t)std::max(1, std::min(256, test_env_int("KH_NP_L1MAX", 256)));
    uint64_t F = 1, rp = rpf;
    if ((Rm + rpf - 1) / rpf > lim) {   // three levels
        // fine buckets small enough that q << ob_f | offset fits 32 bits
        const int qb = ceil_log2(qmax + 1);
        if (qb + P.s0 + 1 > 32) return false;
        rp = std::min<uint64_t>(rpf, ((1ull << (32 - qb)) - 1) / R);
        F = (Rm + rp * lim - 1) / (rp * lim);
        const int obf = ceil_log2(rp * R + 1);
        if (F > N1B_MAXF || obf + qb > 32) return false;
        const uint32_t mf = (uint32_t)(((1ull << 32) + rp - 1) / rp);
        if (!np_magic_ok(rp * F, (uint32_t)rp, mf)) return false;
        fine->F = (uint32_t)F;
        fine->rp = (uint32_t)rp;
        fine->magic = mf;
        fine->ob = obf;
        fine->rloc = (uint32_t)(rp + E + 1);   // level-2 destinations per table
    }
    N.rp = (uint32_t)(rp * F);
    const uint64_t nb = (Rm + N.rp - 1) / N.rp;
    if (nb == 0 || nb > lim) return false;   // k_scatter_n1's per-bucket state (one row scan of 4 x 64)
    N.nb = (uint32_t)nb;
    N.ob = ceil_log2((uint64_t)N.rp * R + 1);   // an offset is never all ones (the ~0 sentinel)
    N.pb = N.ob + ceil_log2(qmax + 1);
    if (N.pb > NP_SLOT_K || 64 - N.pb < 26) return false;
    N.jlim = 64 - N.pb >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << (64 - N.pb)) - 1);
    // KH_NP_JLIM (tests): a smaller block index span, so blocks are closed
    // early and often (np_bkt_plan then allows a closed block per tile)
    const int jl = test_env_int("KH_NP_JLIM", 0);
    if (jl >= L1_THREADS * NP_KPT) N.jlim = std::min<uint32_t>(N.jlim, (uint32_t)jl);
    N.magic = (uint32_t)(((1ull << 32) + N.rp - 1) / N.rp);
    if (!np_magic_ok(Rm, N.rp, N.magic)) return false;
    N.pm = pm;
    N.ipm = 1.0 / (double)pm;
    *out = N;
    return true;
}
// the level-2 view of a three-level partition: fine buckets, fine records
static NPGeo np_fine_geo(const NPGeo &C, const NPFine &Fi) {
    NPGeo N = C;
    N.rp = Fi.rp;
    N.magic = Fi.magic;
    N.nb = C.nb * Fi.F;
    N.ob = Fi.ob;
    N.pb = 32;
    N.cap = Fi.cap;
    N.rloc = Fi.rloc;
    return N;
}
// fine bucket capacity (dense runs: the mean + the margin) and cursors;
// returns the records of all fine buckets
static uint64_t np_fine_plan(Graph *g, const NPGeo &C, NPFine &Fi, uint64_t nkmers) {
    Workspace &w = g->ws;
    const double mean = (double)nkmers * (double)((uint64_t)Fi.rp << C.s0) / (double)C.pm;
    Fi.cap = ((uint64_t)(mean + g->cap_sigma * sqrt(mean)) + 64 + 1) & ~1ull;   // even: 16-B pair loads
    const uint64_t nbf = (uint64_t)C.nb * Fi.F;
    ensure((void **)&w.np_fcur, &w.cap_npfcur, nbf + 1, 8);
    return Fi.cap * nbf;
}
// fixed-length 2-bit reads whose 4096-k-mer tile spans at most NP_TW packed words
template <class Src>
static bool np_source(const Src &src) {
    if constexpr (!std::is_same<Src, SrcTwoBit>::value) return false;
    else {
        if (!src.kpr) return false;
        const uint64_t T = (uint64_t)L1_THREADS * NP_KPT;
        const uint64_t reads = (T + src.kpr - 1) / src.kpr + 1;
        const uint64_t span = T + reads * (uint64_t)(src.k - 1) + (uint64_t)src.k;
        return span / 32 + 3 <= (uint64_t)NP_TW;
    }
}
static uint32_t np_workgroups(const Graph *g, uint64_t nkmers, uint32_t nb) {
    const uint64_t tiles = (nkmers + (uint64_t)L1_THREADS * NP_KPT - 1) / ((uint64_t)L1_THREADS * NP_KPT);
    const uint64_t wpc = std::max<uint64_t>(1, std::min<uint64_t>(L1F_WAVES_PER_EU * 4 / (L1_THREADS / 64),
                                                                   163840 / lds_n1((nb + 3) & ~3u)));
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(tiles / 4 + 1, wpc * device_cus(g)));
}
// tiles of a k_scatter_n1 chunk: the k-mers of a k_scatter_l1p chunk
static uint32_t np_chunk_tiles(const Graph *g) { return std::max<uint32_t>(1, l1f_chunk_tiles(g) / 4); }
// uniform bucket capacity: a full bucket's expected records + the margin + a
// partial block per workgroup; returns the records of all buckets
static uint64_t np_bkt_plan(Graph *g, NPGeo &N, uint64_t nkmers, uint32_t nwg) {
    Workspace &w = g->ws;
    const uint64_t BLK = 1ull << l1f_blk_sh();
    const double mean = (double)nkmers * (double)((uint64_t)N.rp << N.s0) / (double)N.pm;
    uint64_t cap = (uint64_t)(mean + g->cap_sigma * sqrt(mean)) + (uint64_t)(nwg + 1) * BLK;
    if (test_env_int("KH_NP_JLIM", 0) > 0)   // at most one closed block per (bucket, tile)
        cap += (nkmers + L1_THREADS * NP_KPT - 1) / (L1_THREADS * NP_KPT) * BLK;
    cap = (cap + BLK - 1) / BLK * BLK;
    N.cap = cap;
    ensure((void **)&w.np_cur, &w.cap_npcur, N.nb + 1, 8);
    ensure((void **)&w.np_blkj, &w.cap_blkj, cap / BLK * N.nb + 1, 4);
    return cap * N.nb;
}

// KH_CHECK (development): record buffers pre-filled with a sentinel; after
// each scatter the slots still holding it (holes) are counted
static bool check_mode() {
    static bool v = [] { const char *e = dev_getenv("KH_CHECK"); return e && atoi(e); }();
    return v;
}
__global__ void k_count_sentinel(const uint64_t *r, uint64_t n, unsigned long long *out) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        c += r[i] == ~0ull;
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}
static void check_holes(Graph *g, const uint64_t *r, uint64_t n, const char *what) {
    unsigned long long *d = nullptr, h = 0;
    KH_HIP(hipMalloc((void **)&d, 8));
    KH_HIP(hipMemsetAsync(d, 0, 8, g->stream));
    hipLaunchKernelGGL(k_count_sentinel, dim3(4096), dim3(256), 0, g->stream, r, n, d);
    KH_HIP(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    KH_HIP(hipFree(d));
    if (h) {
        fprintf(stderr, "KH_CHECK: %llu holes after %s (of %llu)\n", h, what, (unsigned long long)n);
        std::vector<uint64_t> v(n);
        KH_HIP(hipMemcpy(v.data(), r, n * 8, hipMemcpyDeviceToHost));
        int shown = 0;
        uint64_t run0 = 0, prev = ~0ull, runs = 0;
        for (uint64_t i = 0; i < n; i++) {
            if (v[i] != ~0ull) continue;
            if (i != prev + 1) {
                if (shown < 12 && prev != ~0ull)
                    fprintf(stderr, "  hole run [%llu, %llu) len %llu\n", (unsigned long long)run0,
                            (unsigned long long)prev + 1, (unsigned long long)(prev + 1 - run0)), shown++;
                run0 = i;
                runs++;
            }
            prev = i;
        }
        fprintf(stderr, "  last run [%llu, %llu), %llu runs\n", (unsigned long long)run0, (unsigned long long)prev + 1,
                (unsigned long long)runs);
    }
}

// exclusive scan of n u32 counts into u64 offsets (rocPRIM decoupled look-back)
static void scan_counts(Graph *g, const uint32_t *in, uint64_t *out, uint64_t n) {
    Workspace &w = g->ws;
    size_t bytes = 0;
    KH_HIP(rocprim::exclusive_scan(nullptr, bytes, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(),
                                   g->stream));
    ensure(&w.scan_tmp, &w.cap_scan, bytes, 1);
    bytes = w.cap_scan;
    KH_HIP(rocprim::exclusive_scan(w.scan_tmp, bytes, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(),
                                   g->stream));
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
#define TIMED_G(gr, name, ...) do { KTimer kt_(gr, name); __VA_ARGS__; } while (0)
// an exchange-mode view's kernel timings go to its shard's statistics
static void move_kstats(Graph *dst, Graph *src) {
    engine_collect_events(src);
    for (auto &p : src->kstats) {
        auto it = std::find_if(dst->kstats.begin(), dst->kstats.end(), [&](auto &x) { return x.first == p.first; });
        if (it == dst->kstats.end()) { dst->kstats.push_back({p.first, Graph::KStat{}}); it = dst->kstats.end() - 1; }
        it->second.ms += p.second.ms;
        it->second.n += p.second.n;
    }
    src->kstats.clear();
}

// level-1 scatter instance for a tail mode and k-mers per thread (8 / nt)
template <class Src>
using L1Fn = void (*)(Params, Src, uint64_t, uint32_t, uint32_t, int, int, uint64_t *, uint64_t *, uint32_t, uint32_t);
template <class Src>
static L1Fn<Src> l1_kernel(bool seg, int kpt) {
    switch (kpt) {
        case 8: return seg ? k_scatter_l1<Src, 2, 8> : k_scatter_l1<Src, 0, 8>;
        case 4: return seg ? k_scatter_l1<Src, 2, 4> : k_scatter_l1<Src, 0, 4>;
        case 2: return seg ? k_scatter_l1<Src, 2, 2> : k_scatter_l1<Src, 0, 2>;
        default: return seg ? k_scatter_l1<Src, 2, 1> : k_scatter_l1<Src, 0, 1>;
    }
}

static size_t lds_window(bool window, int tile_kmers) { return 16 + (window ? (size_t)(tile_kmers + 2) * 8 : 0); }

// LDS footprints
static size_t lds_hist_l1(const Params &P, bool window) {
    return (size_t)((P.F1 + 3) & ~3u) * 4 + lds_window(window, L1_HIST_TILE);
}
// level-1 tails of 2 records (16-B aligned runs) when they fit next to the
// tile.  Measured on C2 (scatter_l1 ms/step): no tails 128, 2 records 108,
// 4 records 114, 8 records 122 -- every tile flushes nearly every bucket's
// tail, so smaller tails mean fewer LDS slot scans per tile.
static int l1_seg(const Params &P) {
    static const int v = env_seg("KH_L1_SEG", -1);   // development A/B: 0 or 2 at any F1
    if (v == 0 || v == 2) return v;
    return P.F1 <= 1024 ? 2 : 0;
}
static size_t lds_scatter_l1(const Params &P, bool window, int tile_kmers) {
    const size_t F1a = (P.F1 + 3) & ~3u;
    const int seg = l1_seg(P);
    const size_t tile = (size_t)L1_THREADS * L1_MAX_RPT;
    return F1a * 8 + tile * 8 + F1a * 8 * seg + F1a * 4 * 2 + tile * 2 + 64 + ((F1a + 7) & ~7u) +
           lds_window(window, tile_kmers);
}

constexpr int L2_SEG = 16;   // 128-B level-2 write segments
constexpr int L2_RPT = 8;    // level-2 records per thread per tile
static int l2_seg() { return L2_SEG; }
static int w_seg() { return 2; }   // winner tails of 2 (measured: 8 -> 26.8, 2 -> 25.5 ms/step, round 1)
static size_t lds_scatter_l2(const Params &P) {
    const size_t F2 = (size_t)1 << P.s2;
    return F2 * 8 + F2 * 8 * l2_seg() + F2 * 4 + 8 + ((F2 + 1) & ~(size_t)1) * 2 + F2;
}
using L2Fn = void (*)(uint32_t, int, int, const uint64_t *, const uint32_t *, const uint64_t *, const uint64_t *,
                      uint64_t *);
static L2Fn l2_kernel() { return k_scatter_l2<PT_THREADS, L2_SEG, L2_RPT>; }
using WFn = void (*)(Params, ApplyArgs, int, uint32_t, uint32_t, const uint64_t *, uint32_t *);
static WFn w_kernel() { return k_scatter_w<PT_THREADS, 2>; }
static size_t lds_scatter_w(uint32_t FJ) {
    const size_t FJa = (FJ + 3) & ~3u;
    return W_RPC * 8 + (W_RPC + 4) * 4 + FJa * 8 + (size_t)PT_TILE * 4 + FJa * 4 * w_seg() + FJa * 4 * 2 + 64 + FJa;
}
static int apply_count_threads(const Params &P) { return (1 << P.s0) / 16; }
template <int KIND>
static void (*apply_count_kernel(const Params &P, bool losers = false))(Params, ApplyArgs) {
    if (losers) return P.s0 == 14 ? k_apply_count<KIND, 1024, true> : k_apply_count<KIND, 512, true>;
    return P.s0 == 14 ? k_apply_count<KIND, 1024> : k_apply_count<KIND, 512>;
}
// one 1024-thread workgroup per CU fits the 2^14-bin LDS footprint; two of 512
static unsigned agrid_count(const Graph *g, const PassGeo &q) {
    const uint64_t per_cu = g->prm.s0 == 14 ? 1 : 2;
    return (unsigned)std::min<uint64_t>(q.regions, per_cu * device_cus(g));
}
static size_t lds_apply(const Params &P, bool coarse = false) {
    const size_t R = (size_t)1 << P.s0;
    if (P.kind == BIT)   // coarse-window winners: window arrays + a winner staging array
        return R * 4 + 16 + 64 + R / 8 + MAX_CW * 20 + 8 + (coarse ? R * 4 : 0);
    return R * 4 * 2 + (R / 512) * 4 + 64 + R / 8 + 16 + R + R / 4 + MAX_CW * 20 + 8;   // + s_q[2]
}

// A shard's level 1 through k_own_filter (kh_partition.cuh) when it owns a
// small share of the bins: a group of >= KH_OWN_FILTER_MIN ranks (default 3;
// 0 disables), local bin ids below 2^32 and at most 1024 level-1 buckets.
static bool use_own_filter(const Graph *g) {
    const char *e = getenv("KH_OWN_FILTER_MIN");
    const int min_world = e && *e ? atoi(e) : 3;
    const Params &P = g->prm;
    return min_world > 0 && g->world >= min_world && P.F1 <= 1024 &&
           ((uint64_t)P.F1 << (P.s0 + P.s2)) <= (1ull << 32);
}
template <class Src, int KPT>
static void launch_own_filter(Graph *g, const Src &src, uint64_t nkmers, bool window, int t0, int nt) {
    constexpr uint32_t CK = 32768;
    const uint32_t nch = (uint32_t)((nkmers + CK - 1) / CK);
    const size_t lds = (size_t)OWN_BUF * 8 + 32 * 4 + 8 + lds_window(window, L1_THREADS * KPT);
    hipLaunchKernelGGL((k_own_filter<Src, KPT>), dim3(nch), dim3(L1_THREADS), lds, g->stream, g->prm, src, nkmers,
                       CK, t0, nt, g->ws.cap_frec, g->ws.frec, g->ws.fcount);
}
// owned records of the pass into ws.frec (grown and re-run when the estimate
// was short); returns their number
template <class Src>
static uint64_t own_filter(Graph *g, const Src &src, uint64_t nkmers, bool window) {
    const Params &P = g->prm;
    Workspace &w = g->ws;
    double expect = 0;
    for (int i = 0; i < P.n; i++) expect += (double)nkmers * (double)P.lsz[i] / (double)P.p[i];
    // first buffer: the expectation + 5 % (KH_OWN_FILTER_FRAC overrides the
    // factor; below 1 it forces the re-run path, for tests)
    const char *fe = getenv("KH_OWN_FILTER_FRAC");
    const double frac = fe && *fe ? atof(fe) : 1.05;
    const uint64_t want = (uint64_t)(expect * frac) + (frac < 1 ? 0 : (1u << 20));
    ensure((void **)&w.frec, &w.cap_frec, want, 8);
    if (!w.fcount) KH_HIP(hipMalloc((void **)&w.fcount, 64));
    for (int attempt = 0;; attempt++) {
        KH_HIP(hipMemsetAsync(w.fcount, 0, 8, g->stream));
        for (int t0 = 0; t0 < P.n; t0 += OWN_RPT) {
            const int nt = std::min(OWN_RPT, P.n - t0);
            int kpt = 1;
            while (kpt * 2 * nt <= OWN_RPT) kpt *= 2;
            TIMED("own_filter", switch (kpt) {
                case 16: launch_own_filter<Src, 16>(g, src, nkmers, window, t0, nt); break;
                case 8: launch_own_filter<Src, 8>(g, src, nkmers, window, t0, nt); break;
                case 4: launch_own_filter<Src, 4>(g, src, nkmers, window, t0, nt); break;
                case 2: launch_own_filter<Src, 2>(g, src, nkmers, window, t0, nt); break;
                default: launch_own_filter<Src, 1>(g, src, nkmers, window, t0, nt); break;
            });
        }
        unsigned long long cnt = 0;
        KH_HIP(hipMemcpyAsync(&cnt, w.fcount, 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        if (cnt <= w.cap_frec) return cnt;
        if (attempt) fail(KH_EDEVICE, "owned-record filter overflowed twice");
        ensure((void **)&w.frec, &w.cap_frec, cnt, 8);
    }
}

// k_scatter_l1f over every level-1 window (l1f_windows) of graph g's
// geometry: records of k-mer j carry index jbase + j
// the software-pipelined level 1 (k_scatter_l1p) for fixed-length 2-bit
// reads at <= 256 buckets: 240.6 against 242.2 ms/step (k_scatter_l1f with
// the same fused stage slots) and 243.4 (round 4's kernel), same box,
// profiles/r5/ab_3way_b.txt; KH_L1F=1 keeps k_scatter_l1f (development)
static bool l1p_on() {
    static const bool off = env_seg("KH_L1F", 0) != 0;
    return !off;
}
template <class Src>
static void launch_l1f(Graph *g, const Src &src, uint64_t nkmers, bool window, uint32_t jbase) {
    Workspace &w = g->ws;
    const int rpt = l1f_rpt();
    for (const L1Win &wn : l1f_windows(g->prm, l1f_tables_per_launch())) {
        const Params Q = win_params(g->prm, wn);
        const uint32_t nwg = l1f_workgroups_q(g, Q, nkmers);
        int kpt = 1;
        while (kpt * 2 * wn.nt <= rpt) kpt *= 2;
        const uint64_t tk = (uint64_t)L1_THREADS * kpt;
        const uint64_t kpw = (nkmers + (uint64_t)nwg * tk - 1) / ((uint64_t)nwg * tk) * tk;
        KH_HIP(hipMemsetAsync(w.ctr + CTR_L1Q, 0, 8, g->stream));   // the chunk queue's head
        if constexpr (std::is_same<Src, SrcTwoBit>::value) {
            if (l1p_on() && !window && l1f_tw(src, kpt) && Q.F1 <= 256 && l1f_chunk_tiles(g) >= 1 && kpt == 2 &&
                rpt == L1_MAX_RPT) {
                const size_t lds = lds_l1p((Q.F1 + 3) & ~3u, rpt);
                TIMED("scatter_l1", hipLaunchKernelGGL(k_scatter_l1p<2>, dim3(nwg), dim3(L1_THREADS), lds, g->stream, Q,
                                                       src, nkmers, kpw, wn.t0, wn.nt, w.bkt_base + wn.bb0,
                                                       (unsigned long long *)w.bkt_cur + wn.bb0, w.rec1, w.ctr,
                                                       l1f_blk_sh(), jbase, l1f_chunk_tiles(g)));
                continue;
            }
        }
        TIMED("scatter_l1", hipLaunchKernelGGL(l1f_kernel<Src>(kpt, rpt, !window && l1f_tw(src, kpt)), dim3(nwg),
                                               dim3(L1_THREADS), lds_scatter_l1f(Q, window, (int)tk), g->stream, Q,
                                               src, nkmers, kpw, wn.t0, wn.nt, w.bkt_base + wn.bb0,
                                               (unsigned long long *)w.bkt_cur + wn.bb0, w.rec1, w.ctr, l1f_blk_sh(),
                                               jbase, l1f_chunk_tiles(g)));
    }
}

// Would the record buffers of a pass of nkmers k-mers, planned with capacity
// margin `sigma`, fit in the device memory left (the current buffers are
// freed and reallocated)?  Estimate: the expected records plus the margin
// over every region, twice (level-1 and level-2 buffers, 8 B a record).
static bool recs_fit(Graph *g, uint64_t nkmers, double sigma) {
    const Params &P = g->prm;
    const double R = (double)(1ull << P.s0);
    double recs = 0;
    for (int i = 0; i < P.n; i++) {
        const double regions = (double)P.lsz[i] / R, mean = (double)nkmers * R / (double)P.p[i];
        recs += regions * (mean + sigma * sqrt(mean) + (double)((l2f_parts(P.F1) + 1) << l2f_blk_sh()));
    }
    size_t freeb = 0, total = 0;
    if (hipMemGetInfo(&freeb, &total) != hipSuccess) return false;
    const double have = (double)freeb + 16.0 * (double)g->ws.cap_recs;
    return 16.0 * recs * 1.05 < have * 0.95;
}

// ---------------------------------------------------------------------------
// one device pass over a batch of <= 2^32 - 16 k-mers
// A pass runs in three stages so a sharded group can exchange data between
// them: (A) partition, apply, winner lists partitioned by k-mer window;
// (B) mark: n_unique from the winners (+ per-k-mer new flags); (C) bigcount
// candidates, per-k-mer outputs, counters.
struct PassState {
    PassGeo q;
    uint64_t nkmers = 0;
    bool bigc = false;
    ApplyArgs A;
    uint32_t *win = nullptr, *wout = nullptr;
    // coarse-window winner path
    bool coarse = false;
    uint32_t ncw = 0, fpc = 0;
    // complement mode (losers in the runs, counted per k-mer by k_mark_wf)
    // and the fine windows of 2^js k-mers (FJ of them) the runs are split into
    bool losers = false;
    int js = 0;
    uint32_t FJ = 0;
};

// Complement mode for a pass of the coarse path: the runs carry the records
// that are not their bin's is_new first insert, when those are the fewer --
// sparse tables, where nearly every insert is a winner (C4 / C5; C2 keeps the
// winners).  The winner share of a table's inserts is estimated from table 0's
// zero bins Z before the pass: Z (1 - e^(-m/p)) / m for m inserts into p bins
// (exactness does not depend on it).  Needs the region's records (<= its
// l2f capacity) to fit the LDS staging array (2^s0 entries) and at most 15
// tables (k_mark_wf's 4-bit loser counts); KH_LOSERS=0 / 1 forces it off / on
// where it applies (development).
static bool complement_mode(const Graph *g, uint64_t nkmers, bool l2f) {
    const Params &P = g->prm;
    static const int force = env_seg("KH_LOSERS", -1);
    if (force == 0 || g->grouped || P.kind == BIT || P.n > 15 || !l2f || nkmers == 0) return false;
    if (g->ws.reg_max > (1ull << P.s0)) return false;
    if (force == 1) return true;
    const double p0 = (double)P.p[0], m = (double)nkmers;
    const double occ = g->occ_hint >= 0 ? (double)g->occ_hint : (double)g->n_occupied;
    const double z = std::max(0.0, p0 - occ);
    return z * (1.0 - std::exp(-m / p0)) > 0.6 * m;
}

// The coarse-window winner path (k_apply_count with A.coarse, k_hist_wf,
// k_scatter_wf, k_mark_wf); KH_WINNERS=1 keeps the per-region winner lists
// (development).  Sharded groups route the fine windows of either layout
// (group_route_winners: k_window_starts / k_window_starts_cw); pass_apply
// decides per pass whether the coarse layout fits a shard's buffer.
static bool coarse_winners(const Graph *g) {
    static const bool off = env_seg("KH_WINNERS", 0) == 1;
    (void)g;
    return !off;
}

// coarse-window runs -> fine windows: the windows' counts (one small copy),
// chunks of WF_CHUNK winners per coarse window, a [coarse][fine][chunk] count
// matrix (one extra zero entry: its scan's last value is the total), then
// the 64-way scatter into the fine windows' contiguous ranges of wout
static void winners_fine(Graph *g, PassState &ps) {
    Workspace &w = g->ws;
    hipStream_t st = g->stream;
    const ApplyArgs &A = ps.A;
    std::vector<unsigned long long> cur(MAX_CW), base(MAX_CW, 0);
    KH_HIP(hipMemcpyAsync(cur.data(), w.cw_cur, MAX_CW * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    uint64_t acc = 0;
    for (uint32_t c = 0; c < ps.ncw; c++) {
        base[c] = acc;
        acc += std::min<uint64_t>(1ull << A.cjs, ps.nkmers - ((uint64_t)c << A.cjs)) * (uint64_t)g->prm.n;
    }
    std::vector<WChunk> ch;
    std::vector<uint64_t> cmbase(MAX_CW + 1, 0);
    std::vector<uint32_t> cnk(MAX_CW, 0);
    uint64_t m = 0;
    for (uint32_t c = 0; c < ps.ncw; c++) {
        const uint64_t n = cur[c] - base[c];
        const uint32_t nk = (uint32_t)((n + WF_CHUNK - 1) / WF_CHUNK);
        cmbase[c] = m;
        cnk[c] = nk;
        for (uint32_t k = 0; k < nk; k++)
            ch.push_back(WChunk{base[c] + (uint64_t)k * WF_CHUNK, std::min<uint64_t>(cur[c], base[c] + (uint64_t)(k + 1) * WF_CHUNK),
                                m, k, nk});
        m += (uint64_t)nk * ps.fpc;
    }
    for (uint32_t c = ps.ncw; c <= MAX_CW; c++) cmbase[c] = m;
    ensure(&w.wch, &w.cap_wch, std::max<size_t>(ch.size(), 1), sizeof(WChunk));
    ensure((void **)&w.mcnt, &w.cap_m, m + 1, 4);
    ensure((void **)&w.moff, &w.cap_moff, m + 1, 8);
    if (!ch.empty()) KH_HIP(hipMemcpyAsync(w.wch, ch.data(), ch.size() * sizeof(WChunk), hipMemcpyHostToDevice, st));
    KH_HIP(hipMemcpyAsync(w.cmbase, cmbase.data(), (MAX_CW + 1) * 8, hipMemcpyHostToDevice, st));
    KH_HIP(hipMemcpyAsync(w.cnk, cnk.data(), MAX_CW * 4, hipMemcpyHostToDevice, st));
    KH_HIP(hipMemsetAsync(w.mcnt + m, 0, 4, st));
    const int js = ps.js;
    if (!ch.empty())
        TIMED("hist_w", hipLaunchKernelGGL(k_hist_wf, dim3((unsigned)ch.size()), dim3(WF_THREADS), 0, st, A.wco,
                                           (const WChunk *)w.wch, js, ps.fpc, w.mcnt));
    TIMED("scan", scan_counts(g, w.mcnt, w.moff, m + 1));
    if (!ch.empty())
        TIMED("scatter_w", hipLaunchKernelGGL(k_scatter_wf, dim3((unsigned)ch.size()), dim3(WF_THREADS), 0, st, A.wco,
                                              (const WChunk *)w.wch, js, ps.fpc, w.moff, ps.wout));
    KH_HIP(hipGetLastError());
}

// apply, crossing bins and the winner partition of a pass whose level-2
// records are in place (fixed-capacity regions when l2f, else the exact
// offsets off2)
// The record-driven apply (k_apply_sparse) for the coarse-window path when
// every region's capacity fits the APPLY_RECS records per thread of its 1024
// threads (C4 / C5 / C5M regions: ~6-7K records); KH_SPARSE_APPLY=0 keeps
// k_apply_count (read in every build: the tests compare both).  A Bit
// variant (16 records a thread, C3's ~12K a region) measured slower than
// k_apply_bit (142 vs 115 ms/step) and was removed.
static bool sparse_apply(const Graph *g, const PassState &ps, bool l2f) {
    const bool on = test_env_int("KH_SPARSE_APPLY", 1) != 0;   // per pass: the tests toggle it
    const Params &P = g->prm;
    return on && ps.coarse && l2f && P.s0 == 14 && (P.kind == BYTE || P.kind == NIBBLE) &&
           g->ws.reg_max + 2 <= (uint64_t)1024 * APPLY_RECS;
}
static void pass_apply(Graph *g, PassState &ps, bool l2f) {
    const Params &P = g->prm;
    Workspace &w = g->ws;
    hipStream_t st = g->stream;
    const PassGeo &q = ps.q;
    const uint64_t nkmers = ps.nkmers;
    const bool bigc = ps.bigc;
    // apply (winner segments -> first half of the dead level-1 buffer)
    uint32_t *win = (uint32_t *)w.rec1;
    uint32_t *wout = win + w.cap_recs;
    ps.win = win;
    ps.wout = wout;
    ApplyArgs &A = ps.A;
    A.rlo = l2f ? w.reg_base : w.off2;
    A.rhi = l2f ? w.reg_cur : w.off2 + 1;
    A.rec = w.rec2;
    A.tab = g->d_tab;
    A.win = win;
    A.wcnt = w.wcnt;
    A.fullf = w.fullf;
    A.xent = wout;       // free until scatter_w: crossing entries live there meanwhile
    A.xseg = w.xseg;
    A.ctr = w.ctr;
    A.rprefix[0] = 0;
    for (int i = 0; i < P.n; i++)
        A.rprefix[i + 1] = A.rprefix[i] + ((P.lsz[i] + (1ull << P.s0) - 1) >> P.s0);
    // coarse windows of 2^cjs k-mers (<= 64), each a fine window multiple;
    // window c may hold (its k-mers) x (tables) winners, the capacity of its
    // range of the winner array (the dead level-1 records)
    A.cjs = std::max(q.js, ceil_log2(nkmers) - 6);
    // A coarse window's range of the winner array holds (its k-mers) x
    // (tables) winners, a hard bound that sums to the pass's k-mers x tables:
    // an unsharded pass's record count, which the dead level-1 buffer holds.
    // A shard (or an exchange-mode owner) holds ~1/G of the records, so it
    // takes the coarse path only when that bound still fits its buffer, and
    // the per-region lists otherwise (their capacity is the region's records).
    ps.coarse = coarse_winners(g) && (!g->grouped || nkmers * (uint64_t)P.n <= w.cap_recs);
    A.coarse = ps.coarse ? 1 : 0;
    A.wco = win;
    A.cw_cur = nullptr;
    A.dyn = apply_dynamic(g) ? 1 : 0;
    // complement mode: fine windows of 2^(cjs - 8) k-mers (<= 256 a coarse
    // window; 4-bit counts of 2^17 k-mers fill k_mark_wf's 128 KB of LDS)
    ps.losers = ps.coarse && complement_mode(g, nkmers, l2f);
    ps.js = ps.losers ? A.cjs - 8 : q.js;
    ps.FJ = (uint32_t)((nkmers + (1ull << ps.js) - 1) >> ps.js);
    if (ps.coarse) {
        ps.ncw = (uint32_t)((nkmers + (1ull << A.cjs) - 1) >> A.cjs);
        ps.fpc = 1u << (A.cjs - ps.js);
        if (!w.cw_cur) {
            KH_HIP(hipMalloc((void **)&w.cw_cur, MAX_CW * 8));
            KH_HIP(hipMalloc((void **)&w.cmbase, (MAX_CW + 1) * 8));
            KH_HIP(hipMalloc((void **)&w.cnk, MAX_CW * 4));
        }
        std::vector<unsigned long long> cb(MAX_CW, 0);
        uint64_t acc = 0;
        for (uint32_t c = 0; c < ps.ncw; c++) {
            cb[c] = acc;
            acc += std::min<uint64_t>(1ull << A.cjs, nkmers - ((uint64_t)c << A.cjs)) * (uint64_t)P.n;
        }
        if (acc > w.cap_recs) fail(KH_EDEVICE, "winner capacity exceeds the record buffer");
        KH_HIP(hipMemcpyAsync(w.cw_cur, cb.data(), MAX_CW * 8, hipMemcpyHostToDevice, st));
        A.cw_cur = w.cw_cur;
    }
    const unsigned agrid = (unsigned)std::min<uint64_t>(q.regions, 256 * 2);
    KH_HIP(hipMemsetAsync(w.ctr + CTR_APQ, 0, 8, st));   // the region queue's head (k_apply_*)
    if (P.kind == BIT && ps.coarse)   // one 1024-thread workgroup per CU (the staging array), else two of 512
        TIMED("apply_bit", hipLaunchKernelGGL(k_apply_bit<1024>, dim3((unsigned)std::min<uint64_t>(q.regions, device_cus(g))),
                                              dim3(1024), lds_apply(P, true), st, P, A));
    else if (P.kind == BIT)
        TIMED("apply_bit", hipLaunchKernelGGL(k_apply_bit<APPLY_THREADS>, dim3(agrid), dim3(APPLY_THREADS),
                                              lds_apply(P), st, P, A));
    else if (sparse_apply(g, ps, l2f)) {
        // record-driven apply: every region's records fit the prefetch registers
        const unsigned grid = (unsigned)std::min<uint64_t>(q.regions, device_cus(g));
        const size_t lds = lds_apply_sparse((size_t)1 << P.s0);
        using SpFn = void (*)(Params, ApplyArgs);
        SpFn kn = ps.losers ? k_apply_sparse<NIBBLE, true> : k_apply_sparse<NIBBLE, false>;
        SpFn kb = ps.losers ? k_apply_sparse<BYTE, true> : k_apply_sparse<BYTE, false>;
        if (P.kind == NIBBLE)
            TIMED("apply_nibble", hipLaunchKernelGGL(kn, dim3(grid), dim3(1024), lds, st, P, A));
        else
            TIMED("apply_byte", hipLaunchKernelGGL(kb, dim3(grid), dim3(1024), lds, st, P, A));
    } else if (P.kind == NIBBLE) {
        TIMED("apply_nibble", hipLaunchKernelGGL(apply_count_kernel<NIBBLE>(P, ps.losers), dim3(agrid_count(g, q)),
                                                 dim3(apply_count_threads(P)), lds_apply(P), st, P, A));
    } else {
        TIMED("apply_byte", hipLaunchKernelGGL(apply_count_kernel<BYTE>(P, ps.losers), dim3(agrid_count(g, q)),
                                               dim3(apply_count_threads(P)), lds_apply(P), st, P, A));
    }
    if (bigc)
        TIMED("crossing", hipLaunchKernelGGL(k_crossing, dim3(1024), dim3(256), 0, st, P, w.rec2, w.xseg, wout,
                                             w.ctr, w.fullf));

    if (ps.coarse) {
        winners_fine(g, ps);
        return;
    }
    // winners -> k-mer windows
    const size_t wmeta = W_RPC * 8 + (W_RPC + 4) * 4;
    TIMED("hist_w", hipLaunchKernelGGL(k_hist_w, dim3(q.nchw), dim3(PT_THREADS), wmeta + (size_t)q.FJ * 4, st, P, A,
                                       q.js, q.FJ, q.nchw, w.mcnt));
    TIMED("scan", scan_counts(g, w.mcnt, w.moff, (uint64_t)q.FJ * q.nchw));
    TIMED("scatter_w", hipLaunchKernelGGL(w_kernel(), dim3(q.nchw), dim3(PT_THREADS),
                                          lds_scatter_w(q.FJ), st, P, A, q.js, q.FJ, q.nchw, w.moff, wout));
}

template <class Src>
static PassState pass_stage_a(Graph *g, const Src &src, uint64_t nkmers, bool apply = true, bool *fast_out = nullptr) {
    if (nkmers > MAX_PASS_KMERS) fail(KH_EVALUE, "device batch too large (more than 3200 * 2^20 k-mers)");
    if constexpr (std::is_same<Src, SrcBytes>::value || std::is_same<Src, SrcTwoBit>::value) {
        // Murmur (the costly hash) over more than one level-1 window (or the
        // exact level 1, which hashes every k-mer twice: histogram, scatter):
        // hash once into a u64 array and run the partition over that.
        // KH_HASH_ONCE=0 keeps the repeated hashing, =2 also hashes 2-bit
        // sources once (development A/B).
        static const int once = env_seg("KH_HASH_ONCE", 1);
        const bool want = std::is_same<Src, SrcBytes>::value ? once != 0 : once == 2;
        const bool multi = !l1f_ok(g) || l1f_windows(g->prm, l1f_tables_per_launch()).size() > 1;
        if (want && multi && !use_own_filter(g)) {
            Workspace &w = g->ws;
            ensure((void **)&w.frec, &w.cap_frec, nkmers, 8);
            const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nkmers + 255) / 256, 4096));
            TIMED("hash", hipLaunchKernelGGL(k_hash_kmers<Src>, dim3(grid), dim3(256), 0, g->stream, src, nkmers,
                                             w.frec));
            KH_HIP(hipGetLastError());
            SrcHashes hs{};
            static_cast<SrcCommon &>(hs) = static_cast<const SrcCommon &>(src);
            hs.koff = nullptr;
            hs.kpr = 0;
            hs.kbase = 0;
            hs.h = w.frec;
            return pass_stage_a(g, hs, nkmers, apply, fast_out);
        }
    }
    const Params &P = g->prm;
    PassState ps;
    ps.q = pass_geo(P, nkmers);
    ps.nkmers = nkmers;
    const PassGeo &q = ps.q;
    ws_prepare(g, q);
    Workspace &w = g->ws;
    hipStream_t st = g->stream;
    const uint64_t F1 = P.F1, F2 = 1ull << P.s2;
    const bool bigc = P.kind == BYTE && P.use_bigcount;
    ps.bigc = bigc;
    const bool window = [&] {
        if constexpr (!Src::kReads) return false;
        else return src.kpr == 0;
    }();
    const uint64_t flag_bytes = (nkmers + 15) & ~15ull;

    const bool l2f_try = l2f_wanted(g, nkmers);
    // near-prime partition: one level-1 record per k-mer (kh_nearprime.cuh)
    NPGeo npg{};
    NPFine npf{};
    bool np = false;
    if constexpr (std::is_same<Src, SrcTwoBit>::value)
        np = l2f_try && np_source(src) && l1f_chunk_tiles(g) >= 1 && np_geometry(g, &npg, &npf);
    const NPGeo np2 = npf.F ? np_fine_geo(npg, npf) : npg;   // the level-2 view (buckets, destinations)
    uint64_t cap2 = l2f_try ? reg_plan(g, nkmers, np ? &np2 : nullptr) : 0;   // level-2 capacity (records)
    KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
    if (bigc) {
        dev_fill(w.fullf, 0, flag_bytes, st);
        bcmap_clear(w, st);
    }

    // Partition: the fast path hashes every k-mer once into fixed-capacity
    // level-1 buckets (k_scatter_l1f) and makes one pass over them into
    // fixed-capacity level-2 regions (k_scatter_l2f); the exact path counts
    // first (histogram + scan) at both levels.  Capacities hold for any input
    // that is not heavily skewed; an overflow redoes the pass exactly (the
    // tables are untouched until apply) and keeps the next few passes exact.
    bool fast = l2f_try;
    bool l1f = false;
    uint64_t nrec = 0;   // records this pass writes (exact level 1 only)
    for (;;) {
        np = np && fast;
        l1f = !np && fast && l1f_ok(g) && (std::is_same<Src, SrcHashes>::value || l1f_direct(P));
        const bool ownf = !np && fast && !window && use_own_filter(g) && own_l1f_on();
        const uint64_t cap1 = (l1f || ownf) ? bkt_plan(g, nkmers) : 0;
        // level 1
        if (np) {
            if constexpr (std::is_same<Src, SrcTwoBit>::value) {
                const uint32_t nwg = np_workgroups(g, nkmers, npg.nb);
                const uint64_t capn = np_bkt_plan(g, npg, nkmers, nwg);
                // three levels: the fine records follow the coarse ones in rec1
                const uint64_t fofs = (capn + 63) & ~63ull;
                const uint64_t capf = npf.F ? np_fine_plan(g, npg, npf, nkmers) : 0;
                ensure_recs(g, std::max(fofs + capf, cap2));
                if (KH_ABL(P, 16)) dev_fill(w.rec1, 0xFF, capn * 8, st);   // timing only: level 2 sees sentinels
                hipLaunchKernelGGL(k_np_reset, dim3(1), dim3(256), 0, st, w.np_cur, npg.nb, npg.cap);
                KH_HIP(hipMemsetAsync(w.ctr + CTR_L1Q, 0, 8, st));   // the chunk queue's head
                TIMED("scatter_n1", hipLaunchKernelGGL(k_scatter_n1, dim3(nwg), dim3(L1_THREADS),
                                                       lds_n1((npg.nb + 3) & ~3u), st, npg, src, nkmers, w.np_cur,
                                                       w.rec1, w.np_blkj, w.ctr, l1f_blk_sh(), 0u,
                                                       np_chunk_tiles(g)));
                if (npf.F) {
                    const uint32_t nbf = npg.nb * npf.F;
                    hipLaunchKernelGGL(k_np_reset, dim3((nbf + 255) / 256), dim3(256), 0, st, w.np_fcur, nbf,
                                       npf.cap);
                    const uint32_t pb = (uint32_t)std::max<uint64_t>(1, 4096 / npg.nb);
                    TIMED("scatter_n1b", hipLaunchKernelGGL(k_scatter_n1b, dim3(npg.nb * pb), dim3(N1B_THREADS), 0, st,
                                                            npg, npf, pb, w.np_cur, w.np_blkj, l1f_blk_sh(),
                                                            w.rec1, w.np_fcur, w.rec1 + fofs, w.ctr));
                }
            }
        } else if (ownf) {
            ensure_recs(g, std::max(cap1, cap2));
            hipLaunchKernelGGL(k_reg_reset, dim3((unsigned)((F1 + 255) / 256)), dim3(256), 0, st, w.bkt_base,
                               (unsigned long long *)w.bkt_cur, (uint64_t)F1);
            const uint32_t nwg = l1f_workgroups(g, nkmers);
            for (int t0 = 0; t0 < P.n; t0 += 8) {
                const int nt = std::min(8, P.n - t0);
                int kpt = 1;
                while (kpt * 2 * nt <= 8) kpt *= 2;
                const uint64_t tk = (uint64_t)L1_THREADS * kpt;
                const uint64_t kpw = (nkmers + (uint64_t)nwg * tk - 1) / ((uint64_t)nwg * tk) * tk;
                KH_HIP(hipMemsetAsync(w.ctr + CTR_L1Q, 0, 8, st));   // the chunk queue's head
                TIMED("own_l1f", hipLaunchKernelGGL(own_l1f_kernel<Src>(kpt, l1f_tw(src, kpt)), dim3(nwg), dim3(L1_THREADS),
                                                    lds_own_l1f(P), st, P, src, nkmers, kpw, t0, nt, w.bkt_base,
                                                    (unsigned long long *)w.bkt_cur, w.rec1, w.ctr, l1f_blk_sh(),
                                                    l1f_chunk_tiles(g)));
            }
        } else if (l1f) {
            ensure_recs(g, std::max(cap1, cap2));
            if (KH_ABL(P, 16)) dev_fill(w.rec1, 0xFF, w.cap_recs * 8, st);   // timing only
            hipLaunchKernelGGL(k_reg_reset, dim3((unsigned)((F1 + 255) / 256)), dim3(256), 0, st, w.bkt_base,
                               (unsigned long long *)w.bkt_cur, (uint64_t)F1);
            launch_l1f(g, src, nkmers, window, 0u);
        } else if (use_own_filter(g)) {
            nrec = own_filter(g, src, nkmers, window);
            const uint32_t nch = (uint32_t)std::max<uint64_t>(1, (nrec + L2_CHUNK - 1) / L2_CHUNK);
            ensure((void **)&w.mcnt, &w.cap_m, F1 * nch, 4);
            ensure((void **)&w.moff, &w.cap_moff, F1 * nch, 8);
            const int shift = P.s0 + P.s2;
            TIMED("hist_rec", hipLaunchKernelGGL(k_hist_rec, dim3(nch), dim3(PT_THREADS), F1 * 4, st, w.frec, nrec,
                                                 (uint32_t)F1, shift, nch, w.mcnt));
            TIMED("scan", scan_counts(g, w.mcnt, w.moff, F1 * nch));
            TIMED("plan_l2", hipLaunchKernelGGL(k_plan_l2, dim3(1), dim3(1024), F1 * 8 + 1025 * 8, st, (uint32_t)F1,
                                                nch, w.moff, w.mcnt, w.off1, w.ch2));
            ensure_recs(g, std::max(nrec, cap2));
            if (check_mode()) {
                dev_fill(w.rec1, 0xFF, nrec * 8, st);
                dev_fill(w.rec2, 0xFF, nrec * 8, st);
            }
            SrcHashes rs{};
            rs.h = w.frec;
            rs.k = P.k;
            TIMED("scatter_l1", hipLaunchKernelGGL((k_scatter_l1<SrcHashes, 2, L1_MAX_RPT, L1_MAX_RPT, true>),
                                                   dim3(nch), dim3(L1_THREADS),
                                                   lds_scatter_l1(P, false, L1_THREADS * L1_MAX_RPT), st, P, rs, nrec,
                                                   (uint32_t)L2_CHUNK, nch, 0, 1, w.moff, w.rec1, 0u, 0u));
        } else {
            TIMED("hist_l1", hipLaunchKernelGGL(k_hist_l1<Src>, dim3(q.nch1), dim3(L1_THREADS), lds_hist_l1(P, window),
                                                st, P, src, nkmers, q.ck1, q.nch1, w.mcnt));
            TIMED("scan", scan_counts(g, w.mcnt, w.moff, F1 * q.nch1));
            TIMED("plan_l2", hipLaunchKernelGGL(k_plan_l2, dim3(1), dim3(1024), F1 * 8 + 1025 * 8, st, (uint32_t)F1,
                                                q.nch1, w.moff, w.mcnt, w.off1, w.ch2));
            KH_HIP(hipMemcpyAsync(&nrec, w.off1 + F1, 8, hipMemcpyDeviceToHost, st));
            KH_HIP(hipStreamSynchronize(st));
            ensure_recs(g, std::max(nrec, cap2));
            if (check_mode()) {
                dev_fill(w.rec1, 0xFF, nrec * 8, st);
                dev_fill(w.rec2, 0xFF, nrec * 8, st);
            }
            // Table groups of up to 8 per launch.  Above 1024 buckets (C4, C5:
            // 1908), each launch takes the tables whose buckets fit 1024 and
            // holds only those in LDS: the 2-record tails then fit beside the
            // tile at two workgroups a CU, for one more hash of each k-mer
            // (measured C4 570.1 -> 563.5, C5 516.7 -> 505.9 ms/step,
            // profiles/r5/ab_l1_exact_windows.txt).  KH_L1X_NT fixes the
            // tables per launch (development A/B).
            static const int xnt = env_seg("KH_L1X_NT", 0);
            const int shift = P.s0 + P.s2;
            auto bstart = [&](int i) { return i < P.n ? (uint32_t)(P.tbase[i] >> shift) : P.F1; };
            for (int t0 = 0, nt = 0; t0 < P.n; t0 += nt) {
                if (xnt > 0) {
                    nt = std::min({xnt, L1_MAX_RPT, P.n - t0});
                } else if (P.F1 <= 1024) {
                    nt = std::min(L1_MAX_RPT, P.n - t0);
                } else {
                    nt = 1;
                    while (t0 + nt < P.n && nt < L1_MAX_RPT && bstart(t0 + nt + 1) - bstart(t0) <= 1024) nt++;
                }
                const int kpt = std::max(1, L1_MAX_RPT / nt);
                const int tile_kmers = L1_THREADS * kpt;
                Params Q = P;
                uint32_t bb0 = 0;
                if (nt < P.n) {   // window: the buckets of tables [t0, t0 + nt)
                    bb0 = bstart(t0);
                    Q = win_params(P, L1Win{t0, nt, bb0, bstart(t0 + nt) - bb0});
                }
                TIMED("scatter_l1", hipLaunchKernelGGL(l1_kernel<Src>(l1_seg(Q) != 0, kpt), dim3(q.nch1),
                                                       dim3(L1_THREADS), lds_scatter_l1(Q, window, tile_kmers), st, Q,
                                                       src, nkmers, q.ck1, q.nch1, t0, nt, w.moff, w.rec1, 0u, bb0));
            }
        }
        if (check_mode() && !l1f && !ownf) check_holes(g, w.rec1, nrec, "scatter_l1");
        // level 2
        if (fast) {
            const uint64_t nreg = F1 * F2;
            const uint32_t parts = l2f_parts((uint32_t)F1);
            hipLaunchKernelGGL(k_reg_reset, dim3((unsigned)std::min<uint64_t>((nreg + 255) / 256, 4096)), dim3(256), 0,
                               st, w.reg_base, (unsigned long long *)w.reg_cur, nreg);
            const bool bkt = l1f || ownf;   // level 1 went into fixed-capacity buckets
            const uint64_t *bs = bkt ? w.bkt_base : w.off1;
            const uint64_t *be = bkt ? w.bkt_cur : w.off1 + 1;
            if (np && npf.F) {   // level 2 over the fine buckets of level 1b
                const NPGeo fg = np_fine_geo(npg, npf);
                const uint32_t nparts = l2f_parts(fg.nb);
                const uint64_t fofs = (npg.cap * npg.nb + 63) & ~63ull;
                TIMED("scatter_n2", hipLaunchKernelGGL(n2_kernel(fg.n), dim3(fg.nb * nparts), dim3(PT_THREADS),
                                                       lds_scatter_n2(fg), st, fg, nparts, w.np_fcur, nullptr,
                                                       l1f_blk_sh(), w.reg_base, (unsigned long long *)w.reg_cur,
                                                       w.rec1 + fofs, w.rec2, w.ctr, l2f_blk_sh()));
            } else if (np) {
                const uint32_t nparts = l2f_parts(npg.nb);
                TIMED("scatter_n2", hipLaunchKernelGGL(n2_kernel(npg.n), dim3(npg.nb * nparts), dim3(PT_THREADS),
                                                       lds_scatter_n2(npg), st, npg, nparts, w.np_cur, w.np_blkj,
                                                       l1f_blk_sh(), w.reg_base, (unsigned long long *)w.reg_cur,
                                                       w.rec1, w.rec2, w.ctr, l2f_blk_sh()));
            } else {
                TIMED("scatter_l2", hipLaunchKernelGGL((k_scatter_l2f<PT_THREADS, L2_RPT>), dim3((unsigned)(F1 * parts)),
                                                       dim3(PT_THREADS), lds_scatter_l2f(P), st, (uint32_t)F1, P.s0,
                                                       P.s2, parts, bs, be, w.reg_base, (unsigned long long *)w.reg_cur,
                                                       w.rec1, w.rec2, w.ctr, l2f_blk_sh()));
            }
            uint64_t err = 0;
            KH_HIP(hipMemcpyAsync(&err, w.ctr + CTR_ERR, 8, hipMemcpyDeviceToHost, st));
            KH_HIP(hipStreamSynchronize(st));
            if (err & 16) fail(KH_EDEVICE, "near-prime level 2: a bin outside its bucket's regions");
            if (err & 12) {   // a bucket or region overflowed (the tables are untouched until apply)
                KH_HIP(hipMemsetAsync(w.ctr + CTR_ERR, 0, 8, st));
                // redo the pass on the fast path with 3x the capacity margin
                // while the larger record buffers fit the device; beyond that,
                // exactly (histogram path), and the next 8 passes too
                if (g->cap_sigma < 72.0 && recs_fit(g, nkmers, g->cap_sigma * 3.0)) {
                    g->cap_sigma *= 3.0;
                    cap2 = reg_plan(g, nkmers, np ? &np2 : nullptr);
                    continue;
                }
                fast = false;
                g->l2_cool = 8;
                continue;
            }
        } else {
            if (g->l2_cool > 0) g->l2_cool--;
            const unsigned g2 = (unsigned)q.nch2max;
            TIMED("hist_l2", hipLaunchKernelGGL(k_hist_l2, dim3(g2), dim3(PT_THREADS), F2 * 4, st, (uint32_t)F1, P.s0,
                                                P.s2, w.off1, w.ch2, w.rec1, w.mcnt));
            TIMED("scan", scan_counts(g, w.mcnt, w.moff, F2 * q.nch2max));
            TIMED("off2", hipLaunchKernelGGL(k_off2, dim3((unsigned)std::min<uint64_t>((F1 * F2 + 255) / 256, 8192)),
                                             dim3(256), 0, st, (uint32_t)F1, P.s2, w.off1, w.ch2, w.moff, w.off2));
            TIMED("scatter_l2", hipLaunchKernelGGL(l2_kernel(), dim3(g2), dim3(PT_THREADS), lds_scatter_l2(P), st,
                                                   (uint32_t)F1, P.s0, P.s2, w.off1, w.ch2, w.moff, w.rec1, w.rec2));
            if (check_mode()) check_holes(g, w.rec2, nrec, "scatter_l2");
        }
        break;
    }
    if (fast_out) *fast_out = fast;
    if (apply) pass_apply(g, ps, fast);
    return ps;
}

// (B) one workgroup per window: LDS bitmap of its winners
static void pass_mark_local(Graph *g, PassState &ps, bool want_new) {
    Workspace &w = g->ws;
    const PassGeo &q = ps.q;
    hipStream_t st = g->stream;
    if (ps.coarse) {
        // LDS: a bit per k-mer (winners) or a 4-bit loser count
        const size_t lds = ((size_t)1 << ps.js) / (ps.losers ? 2 : 8);
        TIMED("mark", hipLaunchKernelGGL(k_mark_wf, dim3(ps.FJ), dim3(PT_THREADS), lds, st, ps.wout, w.moff, w.cmbase,
                                         w.cnk, ps.fpc, ps.js, w.ctr, want_new ? w.newbits : nullptr,
                                         ps.losers ? (uint32_t)g->prm.n : 0u, ps.nkmers));
        return;
    }
    TIMED("mark", hipLaunchKernelGGL(k_mark, dim3(q.FJ), dim3(PT_THREADS), ((size_t)1 << q.js) / 8, st, ps.wout,
                                     w.moff, w.mcnt, q.nchw, q.FJ, q.js, w.ctr, want_new ? w.newbits : nullptr));
}

// (C) bigcount candidates (fullf complete), outputs, counters
template <class Src>
static void pass_stage_c(Graph *g, const Src &src, PassState &ps, const PassOut *out) {
    Workspace &w = g->ws;
    const Params &P = g->prm;
    hipStream_t st = g->stream;
    const uint64_t nkmers = ps.nkmers;
    const bool bigc = ps.bigc;
    const bool want_new = out && (out->h_new || out->h_newbits);
    const uint64_t flag_bytes = (nkmers + 15) & ~15ull;
    uint64_t *d_out_hash = nullptr;
    if (out && out->h_hash) d_out_hash = w.rec2;  // level-2 records are dead after crossing
    const uint64_t nchunk = flag_bytes / 16;
    const unsigned fgrid = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>((nchunk + FIN_THREADS - 1) / FIN_THREADS, 4096));
    if (bigc || d_out_hash)
        TIMED("finalize", hipLaunchKernelGGL(k_finalize<Src>, dim3(fgrid), dim3(FIN_THREADS), 0, st, P, src, nkmers,
                                             w.fullf, w.ctr, bigc ? w.bck : nullptr, w.bcv, w.cap_bcmap - 1,
                                             d_out_hash));
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(w.h_ctr, w.ctr, CTR_N * 8, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> hbits;
    if (want_new && out->h_newbits) {
        KH_HIP(hipMemcpyAsync(out->h_newbits, w.newbits, (nkmers + 31) / 32 * 4, hipMemcpyDeviceToHost, st));
    } else if (want_new) {
        hbits.resize((nkmers + 31) / 32);
        KH_HIP(hipMemcpyAsync(hbits.data(), w.newbits, hbits.size() * 4, hipMemcpyDeviceToHost, st));
    }
    if (d_out_hash) KH_HIP(hipMemcpyAsync(out->h_hash, d_out_hash, nkmers * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    engine_collect_events(g);
    if (want_new && !out->h_newbits)
        for (uint64_t j = 0; j < nkmers; j++) out->h_new[j] = (uint8_t)((hbits[j >> 5] >> (j & 31)) & 1);
    // bigcount map overflow (a probe run too long): grow it and redo the
    // finalize of this pass (fullf and the source are intact; the map is per pass)
    while (bigc && (w.h_ctr[CTR_ERR] & 2)) {
        bcmap_alloc(w, w.cap_bcmap * 4);
        bcmap_clear(w, st);
        KH_HIP(hipMemsetAsync(w.ctr + CTR_NBC, 0, 16, st));    // CTR_NBC, CTR_ERR
        KH_HIP(hipMemsetAsync(w.ctr + CTR_BCFF, 0, 8, st));
        TIMED("finalize", hipLaunchKernelGGL(k_finalize<Src>, dim3(fgrid), dim3(FIN_THREADS), 0, st, P, src, nkmers,
                                             w.fullf, w.ctr, w.bck, w.bcv, w.cap_bcmap - 1, (uint64_t *)nullptr));
        KH_HIP(hipMemcpyAsync(w.h_ctr, w.ctr, CTR_N * 8, hipMemcpyDeviceToHost, st));
        KH_HIP(hipStreamSynchronize(st));
        engine_collect_events(g);
    }
    if (w.h_ctr[CTR_ERR]) fail(KH_EDEVICE, "device pipeline error flag set");
    g->n_occupied += w.h_ctr[CTR_OCC];
    g->n_unique += w.h_ctr[CTR_UNIQUE];
    if (bigc) bcmap_merge(g, w.h_ctr[CTR_NBC], w.h_ctr[CTR_BCFF]);
}

// passes of at most SMALL_PASS k-mers run k_small_pass (sequential semantics,
// no partition); KH_SMALL_PASS overrides the threshold (0 disables)
static uint64_t small_pass_max() { return (uint64_t)std::max(0, test_env_int("KH_SMALL_PASS", 2048)); }

template <class Src>
static void run_pass_small(Graph *g, const Src &src, uint64_t nkmers, const PassOut *out) {
    Workspace &w = g->ws;
    hipStream_t st = g->stream;
    ensure((void **)&w.sm_flags, &w.cap_sm, nkmers, 1);
    ensure((void **)&w.sm_hash, &w.cap_smh, nkmers, 8);
    TIMED("small_pass", hipLaunchKernelGGL(k_small_pass<Src>, dim3(1), dim3(64), 0, st, g->prm, src, nkmers, g->d_tab,
                                           w.sm_flags, w.sm_hash));
    KH_HIP(hipGetLastError());
    std::vector<uint8_t> fl(nkmers);
    std::vector<uint64_t> hs(nkmers);
    KH_HIP(hipMemcpyAsync(fl.data(), w.sm_flags, nkmers, hipMemcpyDeviceToHost, st));
    KH_HIP(hipMemcpyAsync(hs.data(), w.sm_hash, nkmers * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    engine_collect_events(g);
    for (uint64_t j = 0; j < nkmers; j++) {
        g->n_unique += fl[j] & 1;
        g->n_occupied += (fl[j] >> 1) & 1;
        if (fl[j] & 4) {   // ByteStorage::add bigcount update (storage.hh:606-616)
            auto it = g->bigcounts.find(hs[j]);
            g->bigcounts[hs[j]] = it == g->bigcounts.end() ? 256 : (uint16_t)std::min<uint32_t>(it->second + 1u, 65535u);
            g->bc_dirty = true;
        }
        if (out && out->h_new) out->h_new[j] = fl[j] & 1;
        if (out && out->h_newbits) {
            if (!(j & 31)) out->h_newbits[j >> 5] = 0;
            out->h_newbits[j >> 5] |= (uint32_t)(fl[j] & 1) << (j & 31);
        }
        if (out && out->h_hash) out->h_hash[j] = hs[j];
    }
}

template <class Src>
static void run_pass(Graph *g, const Src &src, uint64_t nkmers, const PassOut *out) {
    if (nkmers == 0) return;
    if (nkmers <= small_pass_max() && g->world == 1) {
        run_pass_small(g, src, nkmers, out);
        return;
    }
    PassState ps = pass_stage_a(g, src, nkmers);
    pass_mark_local(g, ps, out && (out->h_new || out->h_newbits));
    pass_stage_c(g, src, ps, out);
}

// ---------------------------------------------------------------------------
// batching of read sets
// fixed-length reads of kpr k-mers; nreads bounds the read index of the
// buffer the source walks (div_f64 needs it below 2^31)
static void set_fixed(SrcCommon &s, uint64_t kpr, uint64_t nreads) {
    s.kpr = kpr;
    s.kpr_m = kpr ? barrett_m(kpr) : 0;
    s.kpr_ip = kpr && nreads < (1ull << 31) && nreads * kpr < (1ull << 52) ? 1.0 / (double)kpr : 0.0;
}

template <class Src>
static void consume_reads(Graph *g, Src base, const uint64_t *d_koff, uint64_t nreads, uint64_t nkmers,
                          uint64_t kpr, const PassOut *out) {
    if (nkmers == 0 || nreads == 0) return;
    const uint64_t B = g->batch_kmers;
    set_fixed(base, kpr, nreads);
    base.koff = d_koff;
    base.nreads = nreads;
    base.kbase = 0;
    base.rbase = 0;
    if (out || nkmers <= std::min<uint64_t>(B + (B >> 4), MAX_PASS_KMERS)) {   // one pass (koff[0] == 0 by contract)
        run_pass(g, base, nkmers, out);
        return;
    }
    if (kpr) {   // fixed-length reads: equal batches of whole reads, no offsets needed
        const uint64_t rpb0 = std::max<uint64_t>(1, std::min(B, MAX_PASS_KMERS) / kpr);
        const uint64_t npass = (nreads + rpb0 - 1) / rpb0;
        const uint64_t rpb = (nreads + npass - 1) / npass;
        for (uint64_t r0 = 0; r0 < nreads; r0 += rpb) {
            Src s = base;
            s.kbase = r0 * kpr;
            run_pass(g, s, std::min(rpb, nreads - r0) * kpr, out);
        }
        return;
    }
    const uint64_t B0 = std::min(B, MAX_PASS_KMERS);
    const uint64_t nchunks = (nkmers + B0 - 1) / B0;
    const uint64_t Bb = (nkmers + nchunks - 1) / nchunks;   // equal passes
    std::vector<uint64_t> rr(nchunks + 1), kk(nchunks + 1);
    uint64_t *d = nullptr;
    KH_HIP(hipMalloc((void **)&d, (nchunks + 1) * 16));
    hipLaunchKernelGGL(k_chunk_bounds, dim3((unsigned)std::min<uint64_t>((nchunks + 256) / 256, 4096)), dim3(256), 0,
                       g->stream, d_koff, nreads, Bb, nchunks, d, d + nchunks + 1);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(rr.data(), d, (nchunks + 1) * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(kk.data(), d + nchunks + 1, (nchunks + 1) * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    KH_HIP(hipFree(d));
    uint64_t done = 0;
    for (uint64_t i = 0; i < nchunks; i++) {
        const uint64_t r0 = rr[i], r1 = rr[i + 1];
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

static SrcTwoBit src_twobit(Graph *g, const uint64_t *d_words) {
    SrcTwoBit s{};
    s.words = d_words;
    s.k = g->k;
    return s;
}
// a Murmur source over nbytes of reads (k-mer offsets d_koff, or fixed kpr
// k-mers per read when d_koff is null); builds the reads' reverse-complement
// stream in the workspace first
static SrcBytes src_bytes(Graph *g, const uint8_t *d_bytes, const uint64_t *d_koff, uint64_t nreads, uint64_t kpr,
                          uint64_t nbytes) {
    SrcBytes s{};
    s.bytes = d_bytes;
    s.k = g->k;
    Workspace &w = g->ws;
    ensure((void **)&w.d_rbytes, &w.cap_rbytes, nbytes + 64, 1);
    s.rbytes = w.d_rbytes;
    if (nreads && g->k <= MURMUR_WORDS_MAX) {
        const unsigned grid = (unsigned)std::min<uint64_t>((nreads + 3) / 4, 16384);
        hipLaunchKernelGGL(k_revcomp_reads, dim3(grid), dim3(256), 0, g->stream, d_bytes, d_koff, kpr, g->k, nreads,
                           w.d_rbytes);
        KH_HIP(hipGetLastError());
    }
    return s;
}
static SrcBytes src_bytes_host(Graph *g, const HostBatch &b) {
    return src_bytes(g, g->ws.d_bytes, g->ws.d_koff, b.nreads(), 0, b.bytes.size());
}

void engine_consume_twobit(Graph *g, const uint64_t *d_words, const uint64_t *d_koff, uint64_t nreads,
                           uint64_t nkmers, const PassOut *out) {
    consume_reads(g, src_twobit(g, d_words), d_koff, nreads, nkmers, 0, out);
}

void engine_consume_twobit_fixed(Graph *g, const uint64_t *d_words, uint64_t nreads, uint64_t read_len,
                                 const PassOut *out) {
    if (read_len < (uint64_t)g->k) fail(KH_EVALUE, "reads shorter than k");
    const uint64_t kpr = read_len - g->k + 1;
    consume_reads(g, src_twobit(g, d_words), nullptr, nreads, nreads * kpr, kpr, out);
}

void engine_consume_bytes(Graph *g, const uint8_t *d_bytes, const uint64_t *d_koff, uint64_t nreads,
                          uint64_t nkmers, const PassOut *out) {
    uint64_t kend = 0;
    KH_HIP(hipMemcpy(&kend, d_koff + nreads, 8, hipMemcpyDeviceToHost));
    consume_reads(g, src_bytes(g, d_bytes, d_koff, nreads, 0, kend + nreads * (uint64_t)(g->k - 1)), d_koff, nreads,
                  nkmers, 0, out);
}

// Passes run in stream order, so per-k-mer outputs of consecutive passes are
// exact when each pass writes its own slice of them.
void engine_consume_hashes(Graph *g, const uint64_t *d_hashes, uint64_t n, const PassOut *out) {
    if (out && out->h_newbits) fail(KH_EVALUE, "hash batches report new flags per k-mer (h_new), not as a bitmap");
    const uint64_t B = std::min<uint64_t>(g->batch_kmers, MAX_PASS_KMERS);
    for (uint64_t a = 0; a < n; a += B) {
        SrcHashes s{};
        s.h = d_hashes + a;
        s.k = g->k;
        PassOut o;
        if (out) {
            o.h_new = out->h_new ? out->h_new + a : nullptr;
            o.h_hash = out->h_hash ? out->h_hash + a : nullptr;
        }
        run_pass(g, s, std::min(B, n - a), out ? &o : nullptr);
    }
}

// ---------------------------------------------------------------------------
// host-fed batches
static void upload_batch(Graph *g, const HostBatch &b) {
    Workspace &w = g->ws;
    const uint64_t nr = b.nreads();
    ensure((void **)&w.d_koff, &w.cap_koff, nr + 1, 8);
    KH_HIP(hipMemcpyAsync(w.d_koff, b.koff.data(), (nr + 1) * 8, hipMemcpyHostToDevice, g->stream));
    if (b.hash == MURMUR) {
        ensure((void **)&w.d_bytes, &w.cap_bytes, b.bytes.size() + 64, 1);
        KH_HIP(hipMemcpyAsync(w.d_bytes, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice, g->stream));
    } else {
        const uint64_t nw = (b.nbases + 31) / 32 + 1;
        ensure((void **)&w.d_words, &w.cap_words, nw, 8);
        KH_HIP(hipMemcpyAsync(w.d_words, b.words.data(), nw * 8, hipMemcpyHostToDevice, g->stream));
    }
}

static uint64_t batch_kpr(const HostBatch &b) {
    const uint64_t nr = b.nreads();
    if (!nr) return 0;
    const uint64_t kpr = b.koff[1] - b.koff[0];
    return b.koff[nr] == nr * kpr ? (b.uniform ? kpr : 0) : 0;
}

void engine_consume_host(Graph *g, const HostBatch &b, const PassOut *out) {
    if (b.nkmers() == 0) return;
    upload_batch(g, b);
    const uint64_t kpr = batch_kpr(b);
    if (b.hash == MURMUR)
        consume_reads(g, src_bytes_host(g, b), g->ws.d_koff, b.nreads(), b.nkmers(), kpr, out);
    else
        consume_reads(g, src_twobit(g, g->ws.d_words), g->ws.d_koff, b.nreads(), b.nkmers(), kpr, out);
}

void engine_hash_batch(Graph *g, const HostBatch &b, uint64_t *h_out) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nk) return;
    upload_batch(g, b);
    DevBuf dbuf(nk * 8);
    uint64_t *d = dbuf.as<uint64_t>();
    const uint64_t tiles = (nk + Q_TILE - 1) / Q_TILE;
    const size_t lds = 16 + (Q_TILE + 2) * 8;
    if (b.hash == MURMUR) {
        SrcBytes s = src_bytes_host(g, b);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_hashes<SrcBytes>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, s, nk, d);
    } else {
        SrcTwoBit s = src_twobit(g, g->ws.d_words);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_hashes<SrcTwoBit>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, s, nk,
                           d);
    }
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(h_out, d, nk * 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

uint64_t engine_consume_filtered(Graph *g, const HostBatch &b, const BandMask &f) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nk) return 0;
    KmerFilter F{};
    F.band = f.num_bands != 0;
    F.band_lo = f.band_lo;
    F.band_hi = f.band_hi;
    if (f.mask) {
        engine_sync_bigcounts(f.mask);
        F.mask = 1;
        F.MP = f.mask->prm;
        F.mtab = f.mask->d_tab;
        F.mbc_keys = f.mask->d_bc_keys;
        F.mbc_vals = f.mask->d_bc_vals;
        F.mbc_n = f.mask->d_bc_n;
        F.threshold = f.threshold;
        F.consume_masked = f.consume_masked;
    }
    upload_batch(g, b);
    DevBuf b_h(nk * 8), b_sel(nk * 8), b_keep(nk), b_n(8), b_tmp;
    uint64_t *d_h = b_h.as<uint64_t>(), *d_sel = b_sel.as<uint64_t>(), *d_n = b_n.as<uint64_t>();
    uint8_t *d_keep = b_keep.as<uint8_t>();
    const uint64_t tiles = (nk + Q_TILE - 1) / Q_TILE;
    const size_t lds = 16 + (Q_TILE + 2) * 8;
    if (b.hash == MURMUR) {
        SrcBytes s = src_bytes_host(g, b);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_filter<SrcBytes>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, s, nk, F,
                           d_h, d_keep);
    } else {
        SrcTwoBit s = src_twobit(g, g->ws.d_words);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_filter<SrcTwoBit>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, s, nk,
                           F, d_h, d_keep);
    }
    KH_HIP(hipGetLastError());
    size_t bytes = 0;
    KH_HIP(rocprim::select(nullptr, bytes, d_h, d_keep, d_sel, d_n, (size_t)nk, g->stream));
    b_tmp.alloc(bytes);
    KH_HIP(rocprim::select(b_tmp.p, bytes, d_h, d_keep, d_sel, d_n, (size_t)nk, g->stream));
    uint64_t kept = 0;
    KH_HIP(hipMemcpyAsync(&kept, d_n, 8, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
    if (kept) engine_consume_hashes(g, d_sel, kept, nullptr);
    KH_HIP(hipStreamSynchronize(g->stream));
    return kept;
}

void engine_get_counts(Graph *g, const uint64_t *h_hashes, uint64_t n, uint16_t *out) {
    if (!n) return;
    engine_sync_bigcounts(g);
    Workspace &w = g->ws;
    ensure((void **)&w.q_hashes, &w.cap_q, n, 8);
    uint64_t cap16 = w.cap_q16;
    ensure((void **)&w.q_counts, &cap16, n, 2);
    w.cap_q16 = cap16;
    KH_HIP(hipMemcpyAsync(w.q_hashes, h_hashes, n * 8, hipMemcpyHostToDevice, g->stream));
    const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 65536);
    hipLaunchKernelGGL(k_get_counts, dim3(grid), dim3(256), 0, g->stream, g->prm, g->d_tab, w.q_hashes, n, w.q_counts,
                       g->d_bc_keys, g->d_bc_vals, g->d_bc_n);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(out, w.q_counts, n * 2, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

// per-k-mer counts of an uploaded host batch into d_counts (device)
static void batch_counts(Graph *g, const HostBatch &b, uint16_t *d_counts) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    const uint64_t tiles = (nk + Q_TILE - 1) / Q_TILE;
    const size_t lds = 16 + (Q_TILE + 2) * 8;
    if (!tiles) return;
    if (b.hash == MURMUR) {
        SrcBytes s = src_bytes_host(g, b);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_counts<SrcBytes>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, g->prm, s,
                           nk, g->d_tab, d_counts, g->d_bc_keys, g->d_bc_vals, g->d_bc_n);
    } else {
        SrcTwoBit s = src_twobit(g, g->ws.d_words);
        s.koff = g->ws.d_koff;
        s.nreads = nr;
        hipLaunchKernelGGL(k_kmer_counts<SrcTwoBit>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, g->prm,
                           s, nk, g->d_tab, d_counts, g->d_bc_keys, g->d_bc_vals, g->d_bc_n);
    }
    KH_HIP(hipGetLastError());
}

// Hashtable::get_kmer_counts (src/oxli/hashtable.cc:403-413) over a batch
void engine_kmer_counts(Graph *g, const HostBatch &b, uint16_t *h_out) {
    const uint64_t nk = b.nkmers();
    if (!nk) return;
    engine_sync_bigcounts(g);
    upload_batch(g, b);
    DevBuf b_counts(nk * 2 + 64);
    batch_counts(g, b, b_counts.as<uint16_t>());
    KH_HIP(hipMemcpyAsync(h_out, b_counts.p, nk * 2, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

// Hashtable::median_at_least (src/oxli/hashtable.cc:333-364) per read of a batch
void engine_median_at_least(Graph *g, const HostBatch &b, uint32_t cutoff, uint8_t *h_out) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nr) return;
    engine_sync_bigcounts(g);
    upload_batch(g, b);
    DevBuf b_counts(nk * 2 + 64), b_out(nr + 64);
    batch_counts(g, b, b_counts.as<uint16_t>());
    const unsigned grid = (unsigned)std::min<uint64_t>((nr + 255) / 256, 65536);
    hipLaunchKernelGGL(k_at_least, dim3(grid), dim3(256), 0, g->stream, g->ws.d_koff, nr, b_counts.as<uint16_t>(),
                       cutoff, b_out.as<uint8_t>());
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(h_out, b_out.p, nr, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

void engine_median(Graph *g, const HostBatch &b, uint16_t *med, float *avg, float *sd) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nr) return;
    engine_sync_bigcounts(g);
    upload_batch(g, b);
    DevBuf b_counts(nk * 2 + 64), b_med(nr * 2 + 64), b_avg(nr * 4 + 64), b_sd(nr * 4 + 64);
    uint16_t *d_counts = b_counts.as<uint16_t>(), *d_med = b_med.as<uint16_t>();
    float *d_avg = b_avg.as<float>(), *d_sd = b_sd.as<float>();
    batch_counts(g, b, d_counts);
    const unsigned grid = (unsigned)std::min<uint64_t>((nr + 255) / 256, 65536);
    hipLaunchKernelGGL(k_median, dim3(grid), dim3(256), 0, g->stream, g->ws.d_koff, nr, d_counts, d_med, d_avg, d_sd);
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(med, d_med, nr * 2, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(avg, d_avg, nr * 4, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipMemcpyAsync(sd, d_sd, nr * 4, hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

// Caller-owned ASCII reads are hashed from aligned 8-byte word windows that
// read up to 64 bytes past the last read (load_window): when the allocation
// holding them does not extend that far, they are copied into a padded
// workspace buffer first (include/khmer_hip.h, kh_consume_bytes_fixed_device).
static const uint8_t *padded_bytes(Graph *g, const uint8_t *d, uint64_t n) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d) == hipSuccess && base &&
        (uint64_t)((const uint8_t *)d - (const uint8_t *)base) + n + 64 <= (uint64_t)size)
        return d;
    (void)hipGetLastError();
    Workspace &w = g->ws;
    ensure((void **)&w.d_bytes, &w.cap_bytes, n + 64, 1);
    KH_HIP(hipMemcpyAsync(w.d_bytes, d, n, hipMemcpyDeviceToDevice, g->stream));
    KH_HIP(hipMemsetAsync(w.d_bytes + n, 0, 64, g->stream));
    return w.d_bytes;
}

// get_median_count over device-resident fixed-length reads (packed 2-bit words
// for 2-bit graphs, ASCII bytes for Murmur ones); outputs stay on the device
void engine_median_fixed_device(Graph *g, const void *d_reads, uint64_t nreads, uint64_t read_len, uint16_t *d_med,
                                float *d_avg, float *d_sd) {
    if (read_len < (uint64_t)g->k) fail(KH_EVALUE, "reads shorter than k");
    const uint64_t kpr = read_len - g->k + 1;
    if (kpr > 256) fail(KH_EVALUE, "device median path takes at most 256 k-mers per read");
    if (!nreads) return;
    engine_sync_bigcounts(g);
    const unsigned grid = (unsigned)std::min<uint64_t>((nreads + 3) / 4, 8192);
    if (g->hash == MURMUR) {
        // pieces of at most 2^24 reads: each builds its own reverse-complement
        // stream, so the workspace stays bounded for any number of reads
        const uint64_t cr = 1ull << 24;
        for (uint64_t r0 = 0; r0 < nreads; r0 += cr) {
            const uint64_t n = std::min(cr, nreads - r0);
            const uint8_t *rd = padded_bytes(g, (const uint8_t *)d_reads + r0 * read_len, n * read_len);
            SrcBytes s = src_bytes(g, rd, nullptr, n, kpr, n * read_len);
            set_fixed(s, kpr, n);
            const unsigned gr = (unsigned)std::min<uint64_t>((n + 3) / 4, 8192);
            TIMED("median", hipLaunchKernelGGL(k_median_fixed<SrcBytes>, dim3(gr), dim3(256), 0, g->stream, g->prm,
                                               s, n, (uint32_t)kpr, g->d_tab, g->d_bc_keys, g->d_bc_vals, g->d_bc_n,
                                               d_med + r0, d_avg + r0, d_sd + r0));
        }
    } else {
        SrcTwoBit s = src_twobit(g, (const uint64_t *)d_reads);
        set_fixed(s, kpr, nreads);
        TIMED("median", hipLaunchKernelGGL(k_median_fixed<SrcTwoBit>, dim3(grid), dim3(256), 0, g->stream, g->prm, s,
                                           nreads, (uint32_t)kpr, g->d_tab, g->d_bc_keys, g->d_bc_vals, g->d_bc_n,
                                           d_med, d_avg, d_sd));
    }
    KH_HIP(hipGetLastError());
    KH_HIP(hipStreamSynchronize(g->stream));
    engine_collect_events(g);
}

void engine_consume_bytes_fixed(Graph *g, const uint8_t *d_bytes, uint64_t nreads, uint64_t read_len) {
    if (read_len < (uint64_t)g->k) fail(KH_EVALUE, "reads shorter than k");
    const uint64_t kpr = read_len - g->k + 1;
    // pieces of at most one device pass: the reverse-complement stream
    // (src_bytes) is built per piece, so its workspace stays bounded for any
    // number of reads; passes run in stream order, so the result is the
    // whole stream's
    uint64_t cr = std::max<uint64_t>(1, std::min<uint64_t>(g->batch_kmers, MAX_PASS_KMERS) / kpr);
    const uint64_t np = (nreads + cr - 1) / std::max<uint64_t>(cr, 1);
    if (np) cr = (nreads + np - 1) / np;   // equal pieces
    for (uint64_t r0 = 0; r0 < nreads; r0 += cr) {
        const uint64_t n = std::min(cr, nreads - r0);
        const uint8_t *d = padded_bytes(g, d_bytes + r0 * read_len, n * read_len);
        consume_reads(g, src_bytes(g, d, nullptr, n, kpr, n * read_len), nullptr, n, n * kpr, kpr, nullptr);
    }
}

void engine_unpack_ascii(int device, const uint64_t *d_words, uint64_t nbases, uint8_t *d_bytes) {
    KH_HIP(hipSetDevice(device));
    const uint64_t nw = (nbases + 31) / 32;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nw + 255) / 256, 65536));
    hipLaunchKernelGGL(k_unpack_ascii, dim3(grid), dim3(256), 0, nullptr, d_words, nbases, d_bytes);
    KH_HIP(hipGetLastError());
    KH_HIP(hipDeviceSynchronize());
}

void engine_download_table(Graph *g, int i, uint8_t *dst) {
    KH_HIP(hipMemcpyAsync(dst, g->d_tab + g->prm.tbyte[i], g->nbytes[(size_t)i], hipMemcpyDeviceToHost, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

void engine_upload_table(Graph *g, int i, const uint8_t *src) {
    KH_HIP(hipMemcpyAsync(g->d_tab + g->prm.tbyte[i], src, g->nbytes[(size_t)i], hipMemcpyHostToDevice, g->stream));
    KH_HIP(hipStreamSynchronize(g->stream));
}

void engine_synth_packed(int device, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L, int k,
                         uint64_t *d_words, uint64_t *d_koff) {
    KH_HIP(hipSetDevice(device));
    const uint64_t nwords = (nreads * (uint64_t)L + 31) / 32 + 1;
    const unsigned grid = (unsigned)std::min<uint64_t>((nwords + 255) / 256, 1u << 16);
    if (genome)
        hipLaunchKernelGGL(k_synth_genomic, dim3(grid), dim3(256), 0, 0, seed, genome, r0, nreads, L, k, d_words,
                           nwords, d_koff);
    else
        hipLaunchKernelGGL(k_synth_packed, dim3(grid), dim3(256), 0, 0, seed, r0, nreads, L, k, d_words, nwords,
                           d_koff);
    KH_HIP(hipGetLastError());
    KH_HIP(hipDeviceSynchronize());
}

// ---------------------------------------------------------------------------
// graph creation: table arena + partition geometry

void graph_prepare_params(Graph *g) {
    Params &P = g->prm;
    memset(&P, 0, sizeof P);
    P.kind = g->kind;
    P.hash = g->hash;
    P.k = g->k;
    P.n = g->n;
    P.use_bigcount = g->use_bigcount ? 1 : 0;
#ifdef KH_ABLATE
    // timing-only switches that skip work (wrong results): development builds only
    const char *ab = getenv("KH_ABLATE");
    P.ablate = ab ? atoi(ab) : 0;
#endif
    // regions of 2^14 bins (Byte/Nibble: 1024-thread apply, ~154 KiB of LDS;
    // KH_S0=13 selects the 2^13-bin, 512-thread variant)
    static const int s0_env = env_seg("KH_S0", 14);
    P.s0 = g->kind == BIT ? 14 : (s0_env == 13 ? 13 : 14);
    // regions per level-1 bucket: about sqrt(total regions), so both levels
    // fan out to a few hundred destinations (few same-address LDS atomics in
    // the tile ranks), at most 1024 (C2 on one device: 477 x 1024; a shard of
    // an 8-way group: 240 x 256 instead of 60 x 1024)
    uint64_t maxreg = 1, nreg = 0;
    for (int i = 0; i < g->n; i++) {
        const uint64_t r = (g->lsz[i] + (1ull << P.s0) - 1) >> P.s0;
        maxreg = std::max<uint64_t>(maxreg, r);
        nreg += r;
    }
    const int half = (ceil_log2(std::max<uint64_t>(nreg, 1)) + 1) / 2;
    P.s2 = std::min({10, ceil_log2(maxreg), std::max(half + 1, 1)});
    static const int s2_env = env_seg("KH_S2", 0);   // development: force the level-2 fan-out
    if (s2_env > 0) P.s2 = std::min({10, s2_env, std::max(ceil_log2(maxreg), 1)});
    if (g->force_s2 >= 0) P.s2 = g->force_s2;
    const uint64_t span = 1ull << (P.s0 + P.s2);
    uint64_t base = 0, byteoff = 0;
    for (int i = 0; i < g->n; i++) {
        P.p[i] = g->sizes[i];
        P.m[i] = barrett_m(g->sizes[i]);
        P.ip[i] = 1.0 / (double)g->sizes[i];
        P.lo[i] = g->lo[i];
        P.lsz[i] = g->lsz[i];
        P.tbase[i] = base;
        base += (g->lsz[i] + span - 1) / span * span;
        P.tbyte[i] = byteoff;
        P.tbytes[i] = g->nbytes[i];
        byteoff += (g->nbytes[i] + 255) / 256 * 256;
    }
    // local_bin's double-multiply remainder: every table below 2^30 bins and
    // every hash below 2^31 table sizes (2-bit k-mers are below 4^k; Murmur
    // hashes span 64 bits)
    const double hmax = g->hash == TWOBIT && g->k < 32 ? std::ldexp(1.0, 2 * g->k) : std::ldexp(1.0, 64);
    P.fm32 = 1;
    for (int i = 0; i < g->n; i++)
        if (g->sizes[i] >= (1ull << 30) || hmax >= std::ldexp((double)g->sizes[i], 31)) P.fm32 = 0;
    uint64_t F1 = base / span;
    if (F1 > 4096) fail(KH_EVALUE, "tables too large for one device (more than 4096 level-1 buckets)");
    if (F1 == 0) F1 = 1;
    P.F1 = (uint32_t)F1;
}

// allow the large dynamic LDS footprints (gfx950: 160 KiB per workgroup)
static void set_lds_limits() {
    static bool done = false;
    if (done) return;
    done = true;
    const int lim = 160 * 1024;
    (void)hipFuncSetAttribute((const void *)k_apply_count<BYTE, 512>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<NIBBLE, 512>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<BYTE, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<NIBBLE, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<BYTE, 512, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<NIBBLE, 512, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<BYTE, 1024, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_sparse<BYTE, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_sparse<BYTE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_sparse<NIBBLE, false>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_sparse<NIBBLE, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_count<NIBBLE, 1024, true>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_bit<APPLY_THREADS>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_apply_bit<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
#define KH_LDS_MAX(...) (void)hipFuncSetAttribute((const void *)__VA_ARGS__, hipFuncAttributeMaxDynamicSharedMemorySize, lim)
    for (int kpt : {1, 2, 4, 8})
        for (bool seg : {false, true}) {
            KH_LDS_MAX(l1_kernel<SrcTwoBit>(seg, kpt));
            KH_LDS_MAX(l1_kernel<SrcBytes>(seg, kpt));
            KH_LDS_MAX(l1_kernel<SrcHashes>(seg, kpt));
        }
    KH_LDS_MAX((k_scatter_l2<PT_THREADS, L2_SEG, L2_RPT>));
    KH_LDS_MAX((k_scatter_l2f<PT_THREADS, L2_RPT>));
    for (int kpt : {1, 2, 4, 8}) {
        KH_LDS_MAX(l1f_kernel<SrcTwoBit>(kpt, 8));
        KH_LDS_MAX(l1f_kernel<SrcTwoBit>(kpt, 8, true));
        KH_LDS_MAX(l1f_kernel<SrcBytes>(kpt, 8));
        KH_LDS_MAX(l1f_kernel<SrcHashes>(kpt, 8));
    }
    KH_LDS_MAX((k_scatter_l1<SrcHashes, 2, L1_MAX_RPT, L1_MAX_RPT, true>));
    for (int kpt : {1, 2, 4, 8}) {
        KH_LDS_MAX(own_l1f_kernel<SrcTwoBit>(kpt, false));
        KH_LDS_MAX(own_l1f_kernel<SrcTwoBit>(kpt, true));
        KH_LDS_MAX(own_l1f_kernel<SrcBytes>(kpt, false));
        KH_LDS_MAX(own_l1f_kernel<SrcHashes>(kpt, false));
    }
    KH_LDS_MAX((k_own_filter<SrcTwoBit, 1>));
    KH_LDS_MAX((k_own_filter<SrcTwoBit, 2>));
    KH_LDS_MAX((k_own_filter<SrcTwoBit, 4>));
    KH_LDS_MAX((k_own_filter<SrcTwoBit, 8>));
    KH_LDS_MAX((k_own_filter<SrcTwoBit, 16>));
    KH_LDS_MAX((k_own_filter<SrcBytes, 1>));
    KH_LDS_MAX((k_own_filter<SrcBytes, 2>));
    KH_LDS_MAX((k_own_filter<SrcBytes, 4>));
    KH_LDS_MAX((k_own_filter<SrcBytes, 8>));
    KH_LDS_MAX((k_own_filter<SrcBytes, 16>));
    KH_LDS_MAX((k_own_filter<SrcHashes, 1>));
    KH_LDS_MAX((k_own_filter<SrcHashes, 2>));
    KH_LDS_MAX((k_own_filter<SrcHashes, 4>));
    KH_LDS_MAX((k_own_filter<SrcHashes, 8>));
    KH_LDS_MAX((k_own_filter<SrcHashes, 16>));
    KH_LDS_MAX((k_scatter_w<PT_THREADS, 2>));
    KH_LDS_MAX((k_scatter_l1p<2>));
    KH_LDS_MAX(k_scatter_n1);
    KH_LDS_MAX((k_scatter_n2<PT_THREADS, 2>));
    KH_LDS_MAX((k_scatter_n2<PT_THREADS, 3>));
    KH_LDS_MAX((k_scatter_n2<PT_THREADS, 4>));
    KH_LDS_MAX((k_apply_delta<BYTE, 1024>));
    KH_LDS_MAX((k_apply_delta<NIBBLE, 1024>));
    KH_LDS_MAX((k_apply_delta<BIT, 1024>));
    KH_LDS_MAX((k_apply_delta<BYTE, 512>));
    KH_LDS_MAX((k_apply_delta<NIBBLE, 512>));
    KH_LDS_MAX((k_apply_delta<BIT, 512>));
#undef KH_LDS_MAX
    (void)hipFuncSetAttribute((const void *)k_mark, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipFuncSetAttribute((const void *)k_mark_wf, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    (void)hipGetLastError();
}

// A graph holding bins [lo_i, hi_i) of every table: the contiguous 8-bin
// aligned slice of shard `rank` of `world` (shard_lo), or explicit bounds
// (blo/bhi, exchange-mode groups).  tables = false builds the geometry and
// workspace only (an exchange-mode rank's unsharded level-1 view).
static Graph *graph_build(int kind, int hash, int k, const uint64_t *sizes, int n, int device, int world, int rank,
                          const uint64_t *blo, const uint64_t *bhi, int force_s2, bool tables);
Graph *graph_create_shard(int kind, int hash, int k, const uint64_t *sizes, int n, int device, int world, int rank) {
    return graph_build(kind, hash, k, sizes, n, device, world, rank, nullptr, nullptr, -1, true);
}
static Graph *graph_build(int kind, int hash, int k, const uint64_t *sizes, int n, int device, int world, int rank,
                          const uint64_t *blo, const uint64_t *bhi, int force_s2, bool tables) {
    if (n < 1 || n > MAXT) fail(KH_EVALUE, "number of tables must be in [1, 32]");
    if (kind != BYTE && kind != BIT && kind != NIBBLE) fail(KH_EVALUE, "unknown storage kind");
    if (hash == TWOBIT && (k < 1 || k > 32)) fail(KH_EVALUE, "k-mer size must be <= 32 for 2-bit hashing");
    if (hash == MURMUR && (k < 1 || k > 127)) fail(KH_EVALUE, "k-mer size must be in [1, 127]");
    if (world < 1 || rank < 0 || rank >= world) fail(KH_EVALUE, "invalid shard rank / world size");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail(KH_EDEVICE, "no HIP device available");
    if (device < 0 || device >= ndev) fail(KH_EDEVICE, "invalid HIP device");
    std::unique_ptr<Graph> g(new Graph());
    g->kind = kind;
    g->hash = hash;
    g->k = k;
    g->n = n;
    g->device = device;
    g->world = world;
    g->rank = rank;
    for (int i = 0; i < n; i++) {
        if (sizes[i] == 0) fail(KH_EVALUE, "table size must be > 0");
        g->sizes.push_back(sizes[i]);
        // contiguous slices, 8-bin aligned so Bit/Nibble slices start on a byte
        const uint64_t lo = blo ? blo[i] : shard_lo(sizes[i], world, rank);
        const uint64_t hi = bhi ? bhi[i] : shard_lo(sizes[i], world, rank + 1);
        g->lo.push_back(lo);
        g->lsz.push_back(hi - lo);
        // storage.hh:127-140 (bit), 297-310 (nibble), 502-511 (byte); a slice
        // carries the same trailing byte so the last shard matches the layout
        const uint64_t m = hi - lo;
        g->nbytes.push_back(kind == BIT ? m / 8 + 1 : kind == NIBBLE ? m / 2 + 1 : m);
    }
    g->force_s2 = force_s2;
    KH_HIP(hipSetDevice(device));
    set_lds_limits();
    graph_prepare_params(g.get());
    if (!tables) {
        KH_HIP(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
        return g.release();
    }
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
    dev_fill(g->d_tab, 0, arena, g->stream);
    KH_HIP(hipStreamSynchronize(g->stream));
    return g.release();
}

Graph *graph_create(int kind, int hash, int k, const uint64_t *sizes, int n, int device) {
    return graph_create_shard(kind, hash, k, sizes, n, device, 1, 0);
}

Graph::~Graph() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    Workspace &w = ws;
    void *ptrs[] = {d_tab, d_bc_keys, d_bc_vals, w.rec1, w.rec2, w.fullf, w.newbits, w.bc, w.bcn, w.bck, w.bcv,
                    w.off1, w.ch2, w.off2, w.mcnt, w.moff, w.scan_tmp, w.wcnt, w.xseg, w.reg_base, w.reg_cur, w.bkt_base, w.bkt_cur, w.ctr, w.d_words, w.d_koff, w.d_bytes,
                    w.q_hashes, w.q_counts, w.frec, w.fcount, w.d_rbytes, w.sm_flags, w.sm_hash, w.cw_cur, w.cmbase,
                    w.cnk, w.wch, w.np_cur, w.np_blkj, w.np_fcur, w.sp_cnt, w.sp_off};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (w.h_ctr) (void)hipHostFree(w.h_ctr);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
}

}  // namespace kh

extern "C" int kh_debug_read(uint64_t *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kh::g_dbg), 64 * 8) != hipSuccess) return 5;
    static const uint64_t z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(kh::g_dbg), z, 64 * 8) != hipSuccess) return 5;
    return 0;
}

// ===========================================================================
// Sharded groups ("read broadcast + owner-computes", exact):
// rank r of a G-rank group holds bins [lo_r, lo_r+1) of every table (8-bin
// aligned contiguous slices).  Input reads are consumed in rank order as ONE
// global stream: source s's packed reads are broadcast (RCCL over xGMI) and
// every rank hashes every k-mer but keeps only the (k-mer, table) records of
// bins it owns, so each table byte is updated exactly as on one device.  The
// order-dependent counters stay exact: winners (first inserters of zero bins)
// are routed to the rank owning their k-mer window, which ORs all shards'
// winners in an LDS bitmap; bigcount "full" tallies (rare) are all-gathered
// and summed on every rank, so the bigcount map is replicated.
// Loopback mode runs all G shards in one process on one device (device
// copies instead of RCCL), which is how the protocol is tested on one GPU.
#include <rccl/rccl.h>

namespace kh {

#define KH_NCCL(x)                                                                                    \
    do {                                                                                              \
        ncclResult_t r_ = (x);                                                                        \
        if (r_ != ncclSuccess) fail(KH_EDEVICE, std::string("RCCL: ") + ncclGetErrorString(r_));     \
    } while (0)

struct ShardGroup {
    int world = 1, rank0 = 0, nlocal = 1;
    std::vector<Graph *> shards;
    // exchange mode (Option A): each rank hashes only its own reads into the
    // unsharded level-1 buckets (views[l]: geometry + workspace, no tables)
    // and sends every bucket to its owner; rank r owns buckets [B[r], B[r+1])
    // = bins [blo, bhi) of each table ([world][n])
    bool a2a = false;
    // delta mode (KH_GROUP_DELTA, group_consume_delta): the same ownership and
    // views as exchange mode, but the views hold full-size tables: each rank
    // applies its own chunk into them, and only per-bin table bytes travel
    bool delta = false;
    std::vector<Graph *> views;
    std::vector<uint32_t> B;
    std::vector<uint64_t> blo, bhi;
    ncclComm_t comm = nullptr;
    ncclComm_t comm_b = nullptr;     // source-read broadcasts (own stream, overlapped with compute)
    bool hosted = false;             // one shard per process, collectives through host callbacks
    kh_transport tp{};
    struct Local {
        uint64_t *src = nullptr;
        uint64_t cap_src = 0;        // broadcast reads of another rank (RCCL)
        uint32_t *recv = nullptr;
        uint64_t cap_recv = 0;       // winners routed to this rank
        uint64_t *ws = nullptr;
        uint64_t cap_ws = 0;         // own window starts
        uint64_t *ws_all = nullptr;
        uint64_t cap_ws_all = 0;     // every shard's window starts
        uint64_t *roff = nullptr;
        uint64_t cap_roff = 0;
        uint64_t *flist = nullptr;
        uint64_t cap_flist = 0;      // own full-tally list
        uint64_t *fall = nullptr;
        uint64_t cap_fall = 0;       // gathered full-tally lists
        // source reads in flight: two slots filled on the transfer stream
        // (RCCL broadcast on comm_b; a device copy in loopback) while the
        // compute stream consumes the other one
        uint64_t *seg = nullptr;
        uint64_t cap_seg = 0;        // exchange mode: level-2 segment starts and ends
        uint64_t *slot[2] = {nullptr, nullptr};
        uint64_t cap_slot[2] = {0, 0};
        uint8_t *q8 = nullptr;
        uint64_t cap_q8 = 0;         // sharded query: per-k-mer minima (owner lookups / own bins)
        uint8_t *o8 = nullptr;
        uint64_t cap_o8 = 0;         // sharded query: the reduced minima of this rank's k-mers
        uint8_t *dbuf = nullptr;
        uint64_t cap_dbuf = 0;       // delta mode: every rank's delta (then prefix) of the owned slices
        uint64_t *d_sz = nullptr;
        uint64_t cap_dsz = 0;        // sparse delta pieces: payload sizes sent / received
        uint8_t *stage = nullptr;
        uint64_t cap_stage = 0;      // sparse delta pieces' staging when the dead record buffer is too small
        // hosted delta mode: the alltoallv's host staging, kept across passes
        // (about one table each way; only the slices' bytes are meaningful)
        std::vector<uint8_t> hsend, hrecv;
        hipStream_t st_x = nullptr;
        hipEvent_t ev_ready[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
        bool freed[2] = {false, false};
    };
    std::vector<Local> loc;
    uint64_t wire_dense = 0, wire_sent = 0;   // delta mode: bytes of the pieces between ranks, dense / as sent
    uint64_t *d_red = nullptr;
    std::vector<uint64_t> h_ws;      // [G][FJ+1]
    ~ShardGroup() {
        for (size_t l = 0; l < loc.size(); l++) {
            (void)hipSetDevice(shards[l]->device);
            auto &lc = loc[l];
            if (lc.st_x) (void)hipStreamSynchronize(lc.st_x);
            for (void *p : {(void *)lc.src, (void *)lc.recv, (void *)lc.ws, (void *)lc.ws_all, (void *)lc.roff,
                            (void *)lc.flist, (void *)lc.fall, (void *)lc.slot[0], (void *)lc.slot[1], (void *)lc.seg,
                            (void *)lc.q8, (void *)lc.o8, (void *)lc.dbuf, (void *)lc.d_sz, (void *)lc.stage})
                if (p) (void)hipFree(p);
            for (int b = 0; b < 2; b++) {
                if (lc.ev_ready[b]) (void)hipEventDestroy(lc.ev_ready[b]);
                if (lc.ev_free[b]) (void)hipEventDestroy(lc.ev_free[b]);
            }
            if (lc.st_x) (void)hipStreamDestroy(lc.st_x);
        }
        if (d_red) (void)hipFree(d_red);
        if (comm_b) (void)ncclCommDestroy(comm_b);
        if (comm) (void)ncclCommDestroy(comm);
        for (Graph *g : shards) delete g;
        for (Graph *g : views) delete g;
    }
};

constexpr uint64_t FULL_LIST_CAP = 1ull << 24;

// ---- collectives of a one-shard-per-process group: RCCL, or the host
// transport (staged through host memory, synchronous with the stream) ----
static bool per_rank(const ShardGroup *G) { return G->comm != nullptr || G->hosted; }

static void host_rc(int rc, const char *what) {
    if (rc) fail(KH_EDEVICE, std::string("host transport: ") + what + " failed");
}

static void coll_allgather_u64(ShardGroup *G, hipStream_t st, const uint64_t *d_send, uint64_t *d_recv, uint64_t n) {
    if (G->comm) {
        KH_NCCL(ncclAllGather(d_send, d_recv, n, ncclUint64, G->comm, st));
        return;
    }
    std::vector<uint64_t> snd(n), rcv(n * (uint64_t)G->world);
    KH_HIP(hipMemcpyAsync(snd.data(), d_send, n * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    host_rc(G->tp.allgather(G->tp.ctx, snd.data(), rcv.data(), n * 8), "allgather");
    KH_HIP(hipMemcpyAsync(d_recv, rcv.data(), rcv.size() * 8, hipMemcpyHostToDevice, st));
    KH_HIP(hipStreamSynchronize(st));
}

enum { RED_SUM, RED_MAX, RED_MIN };
static void coll_allreduce_u64(ShardGroup *G, hipStream_t st, const uint64_t *d_send, uint64_t *d_recv, uint64_t n,
                               int op) {
    if (G->comm) {
        const ncclRedOp_t o = op == RED_SUM ? ncclSum : op == RED_MAX ? ncclMax : ncclMin;
        KH_NCCL(ncclAllReduce(d_send, d_recv, n, ncclUint64, o, G->comm, st));
        return;
    }
    std::vector<uint64_t> snd(n), rcv(n * (uint64_t)G->world), red(n);
    KH_HIP(hipMemcpyAsync(snd.data(), d_send, n * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    host_rc(G->tp.allgather(G->tp.ctx, snd.data(), rcv.data(), n * 8), "allreduce");
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v = rcv[i];
        for (int r = 1; r < G->world; r++) {
            const uint64_t x = rcv[(uint64_t)r * n + i];
            v = op == RED_SUM ? v + x : op == RED_MAX ? std::max(v, x) : std::min(v, x);
        }
        red[i] = v;
    }
    KH_HIP(hipMemcpyAsync(d_recv, red.data(), n * 8, hipMemcpyHostToDevice, st));
    KH_HIP(hipStreamSynchronize(st));
}

void group_unique_id(unsigned char *out, size_t n) {
    ncclUniqueId id;
    if (n < sizeof id) fail(KH_EVALUE, "unique id buffer too small");
    KH_NCCL(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
}

// Exchange-mode ownership: the unsharded geometry's level-1 buckets (2^(s0+s2)
// bins each, tables back to back at V.tbase) in `world` contiguous ranges;
// rank r owns buckets [B[r], B[r+1]), i.e. bins [blo, bhi) of every table.
// Its shard's own geometry (same s2) then numbers those buckets 0, 1, ... in
// the same order with the same in-bucket offsets, so level-1 records travel
// unchanged.
static void a2a_plan(const Params &V, const uint64_t *sizes, int n, int world, std::vector<uint32_t> &B,
                     std::vector<uint64_t> &blo, std::vector<uint64_t> &bhi) {
    const uint64_t span = 1ull << (V.s0 + V.s2);
    B.assign(world + 1, 0);
    for (int r = 0; r <= world; r++) B[r] = (uint32_t)((uint64_t)V.F1 * (uint64_t)r / (uint64_t)world);
    blo.assign((size_t)world * n, 0);
    bhi.assign((size_t)world * n, 0);
    for (int r = 0; r < world; r++)
        for (int i = 0; i < n; i++) {
            auto bin_of = [&](uint64_t bkt) -> uint64_t {
                const uint64_t x = bkt * span;
                return x <= V.tbase[i] ? 0 : std::min<uint64_t>(sizes[i], x - V.tbase[i]);
            };
            blo[(size_t)r * n + i] = bin_of(B[r]);
            bhi[(size_t)r * n + i] = bin_of(B[r + 1]);
        }
}

static void group_make_shards(ShardGroup *G, int kind, int hash, int k, const uint64_t *sizes, int n,
                              const int *devices, int mode) {
    const int world = G->world;
    const bool exchange = mode != 0;   // KH_GROUP_EXCHANGE or KH_GROUP_DELTA
    G->delta = mode == 2;
    if (G->delta) {
        // Delta mode keeps three table arenas a rank: the full-size view (its
        // delta, then its prefix), the owner's delta buffer (about one table)
        // and the rank's shard (1 / world of a table) -- it does not shard
        // memory.  Fail before allocating when a device cannot hold its ranks'
        // arenas (the record buffers of a pass come on top).
        uint64_t tb = 0;
        for (int i = 0; i < n; i++)
            tb += kind == BIT ? sizes[i] / 8 + 1 : kind == NIBBLE ? sizes[i] / 2 + 1 : sizes[i];
        const double per_rank = (double)tb * (2.0 + 1.0 / world);
        for (int l = 0; l < G->nlocal; l++) {
            int same = 0;
            for (int m = 0; m < G->nlocal; m++) same += devices[m] == devices[l];
            size_t freeb = 0, total = 0;
            KH_HIP(hipSetDevice(devices[l]));
            if (hipMemGetInfo(&freeb, &total) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            if (per_rank * same > 0.95 * (double)freeb) {
                char msg[256];
                snprintf(msg, sizeof msg,
                         "delta mode needs %.1f GB of table arenas per rank (%d on device %d, %.1f GB free); "
                         "exchange mode shards the tables (--group-mode exchange)",
                         per_rank / 1e9, same, devices[l], (double)freeb / 1e9);
                fail(KH_EVALUE, msg);
            }
        }
    }
    if (exchange) {
        // exchange-mode views hold only a geometry and a workspace; delta-mode
        // views also a full-size table arena (the rank's delta, then its prefix)
        for (int l = 0; l < G->nlocal; l++)
            G->views.push_back(graph_build(kind, hash, k, sizes, n, devices[l], 1, 0, nullptr, nullptr, -1, G->delta));
        const Params &V = G->views[0]->prm;
        if (V.F1 < (uint32_t)world) fail(KH_EVALUE, "exchange mode needs at least one level-1 bucket per rank");
        // level 1 of the unsharded view runs in launch windows of <= 1024
        // buckets (l1f_windows): any table of at most 1024 buckets (1.7e10 bins)
        if (l1f_windows(V, l1f_tables_per_launch()).empty())
            fail(KH_EVALUE, "exchange mode: a table has more than 1024 level-1 buckets");
        a2a_plan(V, sizes, n, world, G->B, G->blo, G->bhi);
        G->a2a = true;
    }
    for (int l = 0; l < G->nlocal; l++) {
        const int r = G->rank0 + l;
        G->shards.push_back(exchange ? graph_build(kind, hash, k, sizes, n, devices[l], world, r, &G->blo[(size_t)r * n],
                                                   &G->bhi[(size_t)r * n], G->views[0]->prm.s2, true)
                                     : graph_create_shard(kind, hash, k, sizes, n, devices[l], world, r));
        G->shards.back()->grouped = true;
    }
}

ShardGroup *group_create(int kind, int hash, int k, const uint64_t *sizes, int n, int world, int rank, int nlocal,
                         const int *devices, const unsigned char *uid, int mode) {
    if (world < 1 || world > 64) fail(KH_EVALUE, "group size must be in [1, 64]");
    if (nlocal != 1 && nlocal != world) fail(KH_EVALUE, "a process holds one shard (RCCL) or all shards (loopback)");
    if (nlocal == 1 && (rank < 0 || rank >= world)) fail(KH_EVALUE, "invalid rank");
    std::unique_ptr<ShardGroup> G(new ShardGroup());
    G->world = world;
    G->nlocal = nlocal;
    G->rank0 = nlocal == world ? 0 : rank;
    group_make_shards(G.get(), kind, hash, k, sizes, n, devices, mode);
    G->loc.resize(nlocal);
    // RCCL for one shard per process; a 1-rank group given a unique id runs
    // every RCCL call site too (communicator creation, split, collectives)
    if (nlocal == 1 && (world > 1 || uid)) {
        if (!uid) fail(KH_EVALUE, "an RCCL group needs the unique id of rank 0");
        ncclUniqueId id;
        memcpy(&id, uid, sizeof id);
        KH_HIP(hipSetDevice(devices[0]));
        KH_NCCL(ncclCommInitRank(&G->comm, world, id, rank));
        KH_NCCL(ncclCommSplit(G->comm, 0, rank, &G->comm_b, nullptr));
        KH_HIP(hipMalloc((void **)&G->d_red, 256 * 8));   // [0,64) gathers, [128,..) scalars
    }
    return G.release();
}

ShardGroup *group_create_hosted(int kind, int hash, int k, const uint64_t *sizes, int n, int world, int rank,
                                int device, const kh_transport *t, int mode) {
    if (world < 1 || world > 64) fail(KH_EVALUE, "group size must be in [1, 64]");
    if (rank < 0 || rank >= world) fail(KH_EVALUE, "invalid rank");
    if (!t->allgather || !t->broadcast || !t->alltoallv) fail(KH_EVALUE, "incomplete host transport");
    std::unique_ptr<ShardGroup> G(new ShardGroup());
    G->world = world;
    G->nlocal = 1;
    G->rank0 = rank;
    G->hosted = true;
    G->tp = *t;
    group_make_shards(G.get(), kind, hash, k, sizes, n, &device, mode);
    G->loc.resize(1);
    KH_HIP(hipSetDevice(device));
    KH_HIP(hipMalloc((void **)&G->d_red, 256 * 8));
    return G.release();
}

void group_comm_info(ShardGroup *G, int *nranks, int *device) {
    *nranks = 0;
    *device = -1;
    if (!G->comm) return;
    KH_NCCL(ncclCommCount(G->comm, nranks));
    KH_NCCL(ncclCommCuDevice(G->comm, device));
}

void group_destroy(ShardGroup *G) { delete G; }

static uint32_t group_wlo(uint32_t FJ, int W, int r) { return (uint32_t)((uint64_t)FJ * (uint64_t)r / (uint64_t)W); }

// winners of every shard -> window owners -> LDS-bitmap union (n_unique partials)
static void group_route_winners(ShardGroup *G, std::vector<PassState> &ps) {
    const int W = G->world, NL = G->nlocal;
    const uint32_t FJ = ps[0].q.FJ;
    const int js = ps[0].q.js;
    for (int l = 0; l < NL; l++) {
        Graph *g = G->shards[l];
        auto &lc = G->loc[l];
        KH_HIP(hipSetDevice(g->device));
        ensure((void **)&lc.ws, &lc.cap_ws, FJ + 1, 8);
        ensure((void **)&lc.ws_all, &lc.cap_ws_all, (uint64_t)W * (FJ + 1), 8);
        ensure((void **)&lc.roff, &lc.cap_roff, W, 8);
        if (ps[l].coarse)
            TIMED("route", hipLaunchKernelGGL(k_window_starts_cw, dim3((FJ + 256) / 256), dim3(256), 0, g->stream,
                                              g->ws.moff, g->ws.cmbase, g->ws.cnk, ps[l].fpc, FJ, lc.ws));
        else
            TIMED("route", hipLaunchKernelGGL(k_window_starts, dim3((FJ + 256) / 256), dim3(256), 0, g->stream,
                                              g->ws.moff, g->ws.mcnt, ps[l].q.nchw, FJ, lc.ws));
    }
    G->h_ws.assign((size_t)W * (FJ + 1), 0);
    if (per_rank(G)) {
        Graph *g = G->shards[0];
        auto &lc = G->loc[0];
        coll_allgather_u64(G, g->stream, lc.ws, lc.ws_all, FJ + 1);
        KH_HIP(hipMemcpyAsync(G->h_ws.data(), lc.ws_all, G->h_ws.size() * 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
    } else {
        for (int s = 0; s < NL; s++) {
            KH_HIP(hipSetDevice(G->shards[s]->device));
            KH_HIP(hipMemcpyAsync(G->h_ws.data() + (size_t)s * (FJ + 1), G->loc[s].ws, (FJ + 1) * 8,
                                  hipMemcpyDeviceToHost, G->shards[s]->stream));
        }
        for (int s = 0; s < NL; s++) KH_HIP(hipStreamSynchronize(G->shards[s]->stream));
        for (int l = 0; l < NL; l++)
            KH_HIP(hipMemcpy(G->loc[l].ws_all, G->h_ws.data(), G->h_ws.size() * 8, hipMemcpyHostToDevice));
    }
    auto wsv = [&](int s, uint32_t w) { return G->h_ws[(size_t)s * (FJ + 1) + w]; };
    for (int l = 0; l < NL; l++) {
        const int r = G->rank0 + l;
        Graph *g = G->shards[l];
        auto &lc = G->loc[l];
        KH_HIP(hipSetDevice(g->device));
        const uint32_t wl = group_wlo(FJ, W, r), wh = group_wlo(FJ, W, r + 1);
        std::vector<uint64_t> roff(W);
        uint64_t tot = 0;
        for (int s = 0; s < W; s++) {
            roff[s] = tot;
            tot += wsv(s, wh) - wsv(s, wl);
        }
        ensure((void **)&lc.recv, &lc.cap_recv, tot + 1, 4);
        KH_HIP(hipMemcpyAsync(lc.roff, roff.data(), W * 8, hipMemcpyHostToDevice, g->stream));
        if (G->comm) {
            // own part first (device copy), then the grouped point-to-point exchange
            const uint64_t own = wsv(r, wh) - wsv(r, wl);
            if (own)
                KH_HIP(hipMemcpyAsync(lc.recv + roff[r], ps[0].wout + wsv(r, wl), own * 4, hipMemcpyDeviceToDevice,
                                      g->stream));
            KH_NCCL(ncclGroupStart());
            for (int d = 0; d < W; d++) {
                if (d == r) continue;
                const uint64_t c = wsv(r, group_wlo(FJ, W, d + 1)) - wsv(r, group_wlo(FJ, W, d));
                if (c)
                    KH_NCCL(ncclSend(ps[0].wout + wsv(r, group_wlo(FJ, W, d)), c, ncclUint32, d, G->comm,
                                     g->stream));
                const uint64_t cin = wsv(d, wh) - wsv(d, wl);
                if (cin) KH_NCCL(ncclRecv(lc.recv + roff[d], cin, ncclUint32, d, G->comm, g->stream));
            }
            KH_NCCL(ncclGroupEnd());
        } else if (G->hosted) {
            // the rank's winners are partitioned by window, so the blocks for
            // ranks 0..W-1 lie back to back: one alltoallv
            std::vector<uint64_t> sb(W), rb(W);
            for (int d = 0; d < W; d++) {
                sb[d] = 4 * (wsv(r, group_wlo(FJ, W, d + 1)) - wsv(r, group_wlo(FJ, W, d)));
                rb[d] = 4 * (wsv(d, wh) - wsv(d, wl));
            }
            const uint64_t nsend = wsv(r, FJ) - wsv(r, 0);
            std::vector<uint32_t> hs(nsend + 1), hr(tot + 1);
            KH_HIP(hipMemcpyAsync(hs.data(), ps[0].wout + wsv(r, 0), nsend * 4, hipMemcpyDeviceToHost, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
            host_rc(G->tp.alltoallv(G->tp.ctx, hs.data(), sb.data(), hr.data(), rb.data()), "alltoallv");
            KH_HIP(hipMemcpyAsync(lc.recv, hr.data(), tot * 4, hipMemcpyHostToDevice, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
        } else {
            for (int s = 0; s < W; s++) {
                const uint64_t c = wsv(s, wh) - wsv(s, wl);
                if (c)
                    KH_HIP(hipMemcpyAsync(lc.recv + roff[s], ps[s].wout + wsv(s, wl), c * 4, hipMemcpyDeviceToDevice,
                                          g->stream));
            }
        }
        if (wh > wl)
            TIMED("mark", hipLaunchKernelGGL(k_mark_multi, dim3(wh - wl), dim3(PT_THREADS), ((size_t)1 << js) / 8,
                                             g->stream, lc.recv, lc.ws_all, lc.roff, W, FJ, wl, js, g->ws.ctr));
    }
}

// bigcount: per-k-mer full tallies of all shards summed on every rank.  Sparse
// (each rank's nonzero tallies compacted and all-gathered) while the lists
// are small; dense (the whole per-k-mer byte array summed: an RCCL uint8
// all-reduce) when a list would outgrow FULL_LIST_CAP or the dense array --
// a saturated stream makes most k-mers full in some table
static void group_merge_full_dense(ShardGroup *G, uint64_t nkb) {
    const int W = G->world, NL = G->nlocal;
    if (G->comm) {
        Graph *g = G->shards[0];
        KH_HIP(hipSetDevice(g->device));
        KH_NCCL(ncclAllReduce(g->ws.fullf, g->ws.fullf, nkb, ncclUint8, ncclSum, G->comm, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        return;
    }
    if (G->hosted) {
        // in slices of at most 256 MB: a rank holds W slices at a time, not W
        // whole per-k-mer arrays (up to 3.3 GB each)
        Graph *g = G->shards[0];
        KH_HIP(hipSetDevice(g->device));
        const uint64_t piece = std::min<uint64_t>(nkb, 256ull << 20);
        std::vector<uint8_t> mine(piece), all((size_t)W * piece);
        for (uint64_t a = 0; a < nkb; a += piece) {
            const uint64_t n = std::min(piece, nkb - a);
            KH_HIP(hipMemcpyAsync(mine.data(), g->ws.fullf + a, n, hipMemcpyDeviceToHost, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
            host_rc(G->tp.allgather(G->tp.ctx, mine.data(), all.data(), n), "allgather");
            for (uint64_t i = 0; i < n; i++) {
                uint32_t v = 0;
                for (int r = 0; r < W; r++) v += all[(size_t)r * n + i];
                mine[i] = (uint8_t)v;
            }
            KH_HIP(hipMemcpyAsync(g->ws.fullf + a, mine.data(), n, hipMemcpyHostToDevice, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
        }
        return;
    }
    // loopback: sum every shard's array into shard 0's, then copy it back out
    Graph *g0 = G->shards[0];
    KH_HIP(hipSetDevice(g0->device));
    for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nkb / 16 / 256 + 1, 4096));
    uint8_t *tmp = nullptr;
    KH_HIP(hipMalloc((void **)&tmp, nkb + 64));
    for (int l = 1; l < NL; l++) {
        KH_HIP(hipMemcpyAsync(tmp, G->shards[l]->ws.fullf, nkb, hipMemcpyDefault, g0->stream));
        hipLaunchKernelGGL(k_add_bytes, dim3(grid), dim3(256), 0, g0->stream, g0->ws.fullf, tmp, nkb);
    }
    KH_HIP(hipStreamSynchronize(g0->stream));
    KH_HIP(hipFree(tmp));
    for (int l = 1; l < NL; l++)
        KH_HIP(hipMemcpy(G->shards[l]->ws.fullf, g0->ws.fullf, nkb, hipMemcpyDefault));
    KH_HIP(hipGetLastError());
}

static void group_merge_full(ShardGroup *G, std::vector<PassState> &ps) {
    const int W = G->world, NL = G->nlocal;
    const uint64_t nk = ps[0].nkmers, nkb = (nk + 15) & ~15ull;
    std::vector<uint64_t> cnt(W, 0);
    for (int l = 0; l < NL; l++) {
        Graph *g = G->shards[l];
        auto &lc = G->loc[l];
        KH_HIP(hipSetDevice(g->device));
        ensure((void **)&lc.flist, &lc.cap_flist, 1024, 8);
        const uint64_t cap = std::min<uint64_t>(FULL_LIST_CAP, lc.cap_flist);
        KH_HIP(hipMemsetAsync(g->ws.ctr + CTR_NFULL, 0, 8, g->stream));
        hipLaunchKernelGGL(k_full_compact, dim3(2048), dim3(256), 0, g->stream, g->ws.fullf, nk, lc.flist, cap,
                           g->ws.ctr);
        uint64_t h[CTR_N];
        KH_HIP(hipMemcpyAsync(h, g->ws.ctr, CTR_N * 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        cnt[G->rank0 + l] = h[CTR_NFULL];
    }
    if (per_rank(G)) {
        Graph *g = G->shards[0];
        KH_HIP(hipSetDevice(g->device));
        KH_HIP(hipMemcpyAsync(G->d_red + 128, &cnt[G->rank0], 8, hipMemcpyHostToDevice, g->stream));
        coll_allgather_u64(G, g->stream, G->d_red + 128, G->d_red, 1);
        KH_HIP(hipMemcpyAsync(cnt.data(), G->d_red, W * 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
    }
    const uint64_t mx = *std::max_element(cnt.begin(), cnt.end());
    if (!mx) return;
    if (mx > FULL_LIST_CAP || mx * 8 > nkb) {   // every rank decides alike (same counts)
        group_merge_full_dense(G, nkb);
        return;
    }
    // sparse: every list complete (re-compacted into a larger list if its first
    // buffer was short), padded to the longest, gathered and scattered back
    for (int l = 0; l < NL; l++) {
        Graph *g = G->shards[l];
        auto &lc = G->loc[l];
        const uint64_t c = cnt[G->rank0 + l];
        KH_HIP(hipSetDevice(g->device));
        if (c > lc.cap_flist || mx > lc.cap_flist) {
            if (lc.flist) KH_HIP(hipFree(lc.flist));
            lc.flist = nullptr;
            lc.cap_flist = 0;
            ensure((void **)&lc.flist, &lc.cap_flist, mx, 8);
            KH_HIP(hipMemsetAsync(g->ws.ctr + CTR_NFULL, 0, 8, g->stream));
            hipLaunchKernelGGL(k_full_compact, dim3(2048), dim3(256), 0, g->stream, g->ws.fullf, nk, lc.flist,
                               lc.cap_flist, g->ws.ctr);
        }
        if (mx > c) KH_HIP(hipMemsetAsync(lc.flist + c, 0xFF, (mx - c) * 8, g->stream));
    }
    if (per_rank(G)) {
        Graph *g = G->shards[0];
        auto &lc = G->loc[0];
        ensure((void **)&lc.fall, &lc.cap_fall, (uint64_t)W * mx, 8);
        coll_allgather_u64(G, g->stream, lc.flist, lc.fall, mx);
        dev_fill(g->ws.fullf, 0, nkb, g->stream);
        hipLaunchKernelGGL(k_full_scatter, dim3(2048), dim3(256), 0, g->stream, lc.fall, (uint64_t)W * mx,
                           g->ws.fullf);
    } else {
        for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
        for (int l = 0; l < NL; l++) {
            Graph *g = G->shards[l];
            KH_HIP(hipSetDevice(g->device));
            dev_fill(g->ws.fullf, 0, nkb, g->stream);
            for (int s = 0; s < W; s++)
                if (cnt[s])
                    hipLaunchKernelGGL(k_full_scatter, dim3(2048), dim3(256), 0, g->stream, G->loc[s].flist, cnt[s],
                                       g->ws.fullf);
        }
    }
    KH_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Exchange mode (Option A, SURVEY.md §8(e) "north star"): every rank hashes
// only its own reads.  A pass takes the next chunk of every rank's reads; the
// pass's stream is the rank chunks in rank order (k-mer index j = rank *
// stride + index in the chunk), so the exact counters follow that order.
//   1. level 1 of the own chunk into the unsharded level-1 buckets (view)
//   2. every rank's bucket bases and fill levels (allgather)
//   3. bucket range [B[d], B[d+1]) to its owner d (grouped ncclSend/ncclRecv;
//      host transport: alltoallv; loopback: device copies)
//   4. the owner's level 2 over its (source, bucket) segments, apply, winners
//   5. winners routed by window, bigcount tallies merged (as Option B)
//   6. finalize of the own chunk's k-mers; bigcount events replicated

// level 1 of one chunk in the unsharded geometry; a bucket overflow grows the
// capacity margin and redoes it (the chunk is still in place)
template <class Src>
static void a2a_level1(Graph *V, const Src &src, uint64_t nkmers, uint32_t jbase) {
    const Params &P = V->prm;
    Workspace &w = V->ws;
    hipStream_t st = V->stream;
    if constexpr (std::is_same<Src, SrcBytes>::value) {
        // Murmur over several level-1 windows: hash once (as pass_stage_a)
        if (l1f_windows(P, l1f_tables_per_launch()).size() > 1) {
            ensure((void **)&w.frec, &w.cap_frec, nkmers, 8);
            const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nkmers + 255) / 256, 4096));
            TIMED_G(V, "hash", hipLaunchKernelGGL(k_hash_kmers<Src>, dim3(grid), dim3(256), 0, st, src, nkmers,
                                                  w.frec));
            KH_HIP(hipGetLastError());
            SrcHashes hs{};
            static_cast<SrcCommon &>(hs) = static_cast<const SrcCommon &>(src);
            hs.koff = nullptr;
            hs.kpr = 0;
            hs.kbase = 0;
            hs.h = w.frec;
            a2a_level1(V, hs, nkmers, jbase);
            return;
        }
    }
    const PassGeo q = pass_geo(P, nkmers);
    ws_prepare(V, q);
    const uint64_t F1 = P.F1;
    w.l1_exact = !std::is_same<Src, SrcHashes>::value && !l1f_direct(P);
    if (w.l1_exact) {
        // more buckets than one fast launch holds at two workgroups per CU
        // (C3 / C4 / C5 tables): the exact two-pass level 1
        // (as pass_stage_a) -- bucket b's records are [off1[b], off1[b + 1])
        KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
        TIMED_G(V, "hist_l1", hipLaunchKernelGGL(k_hist_l1<Src>, dim3(q.nch1), dim3(L1_THREADS),
                                                 lds_hist_l1(P, false), st, P, src, nkmers, q.ck1, q.nch1, w.mcnt));
        TIMED_G(V, "scan", scan_counts(V, w.mcnt, w.moff, F1 * q.nch1));
        TIMED_G(V, "plan_l2", hipLaunchKernelGGL(k_plan_l2, dim3(1), dim3(1024), F1 * 8 + 1025 * 8, st, (uint32_t)F1,
                                                 q.nch1, w.moff, w.mcnt, w.off1, w.ch2));
        uint64_t nrec = 0;
        KH_HIP(hipMemcpyAsync(&nrec, w.off1 + F1, 8, hipMemcpyDeviceToHost, st));
        KH_HIP(hipStreamSynchronize(st));
        ensure_recs(V, nrec, false);
        for (int t0 = 0; t0 < P.n; t0 += L1_MAX_RPT) {
            const int nt = std::min(L1_MAX_RPT, P.n - t0);
            const int kpt = std::max(1, L1_MAX_RPT / nt);
            TIMED_G(V, "scatter_l1", hipLaunchKernelGGL(l1_kernel<Src>(l1_seg(P) != 0, kpt), dim3(q.nch1),
                                                        dim3(L1_THREADS), lds_scatter_l1(P, false, L1_THREADS * kpt),
                                                        st, P, src, nkmers, q.ck1, q.nch1, t0, nt, w.moff, w.rec1,
                                                        jbase, 0u));
        }
        KH_HIP(hipGetLastError());
        return;
    }
    for (;;) {
        const uint64_t cap1 = bkt_plan(V, nkmers);
        ensure_recs(V, cap1, false);
        KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
        hipLaunchKernelGGL(k_reg_reset, dim3((unsigned)((F1 + 255) / 256)), dim3(256), 0, st, w.bkt_base,
                           (unsigned long long *)w.bkt_cur, (uint64_t)F1);
        launch_l1f(V, src, nkmers, false, jbase);
        uint64_t err = 0;
        KH_HIP(hipMemcpyAsync(&err, w.ctr + CTR_ERR, 8, hipMemcpyDeviceToHost, st));
        KH_HIP(hipStreamSynchronize(st));
        if (!(err & 8)) break;
        if (V->cap_sigma < 72.0) {
            V->cap_sigma *= 3.0;
            continue;
        }
        fail(KH_EDEVICE, "exchange mode: a level-1 bucket overflowed at the largest capacity margin (skewed input)");
    }
    KH_HIP(hipGetLastError());
}

// every source's bucket bases and fill levels: meta[s][0..F1] = bases,
// meta[s][F1+1 .. 2F1+1] = ends (the last entry repeats the final base)
static void a2a_meta(ShardGroup *G, std::vector<uint64_t> &meta) {
    const int W = G->world, NL = G->nlocal;
    const uint64_t F1 = G->views[0]->prm.F1, M = 2 * (F1 + 1);
    meta.assign((size_t)W * M, 0);
    for (int l = 0; l < NL; l++) {
        Graph *V = G->views[l];
        KH_HIP(hipSetDevice(V->device));
        uint64_t *h = meta.data() + (size_t)(G->rank0 + l) * M;
        if (V->ws.l1_exact) {   // exact level 1: contiguous buckets, ends = the next bucket's start
            KH_HIP(hipMemcpyAsync(h, V->ws.off1, (F1 + 1) * 8, hipMemcpyDeviceToHost, V->stream));
            KH_HIP(hipMemcpyAsync(h + F1 + 1, V->ws.off1 + 1, F1 * 8, hipMemcpyDeviceToHost, V->stream));
        } else {
            KH_HIP(hipMemcpyAsync(h, V->ws.bkt_base, (F1 + 1) * 8, hipMemcpyDeviceToHost, V->stream));
            KH_HIP(hipMemcpyAsync(h + F1 + 1, V->ws.bkt_cur, F1 * 8, hipMemcpyDeviceToHost, V->stream));
        }
        KH_HIP(hipStreamSynchronize(V->stream));
        h[2 * F1 + 1] = h[F1];
    }
    if (per_rank(G)) {
        Graph *V = G->views[0];
        auto &lc = G->loc[0];
        ensure((void **)&lc.seg, &lc.cap_seg, (uint64_t)W * M, 8);
        uint64_t *d_mine = lc.seg + (size_t)G->rank0 * M;
        KH_HIP(hipMemcpyAsync(d_mine, meta.data() + (size_t)G->rank0 * M, M * 8, hipMemcpyHostToDevice, V->stream));
        std::vector<uint64_t> tmp(M);
        // allgather into a separate device block, then back to the host
        uint64_t *d_all = nullptr;
        KH_HIP(hipMalloc((void **)&d_all, (size_t)W * M * 8));
        coll_allgather_u64(G, V->stream, d_mine, d_all, M);
        KH_HIP(hipMemcpyAsync(meta.data(), d_all, (size_t)W * M * 8, hipMemcpyDeviceToHost, V->stream));
        KH_HIP(hipStreamSynchronize(V->stream));
        KH_HIP(hipFree(d_all));
    }
}

// the records of rank `s`'s buckets [B[r], B[r+1]) land at rbase[s] of
// owner r's level-1 buffer
static void a2a_exchange(ShardGroup *G, const std::vector<uint64_t> &meta, std::vector<std::vector<uint64_t>> &rbase) {
    const int W = G->world, NL = G->nlocal;
    const uint64_t F1 = G->views[0]->prm.F1, M = 2 * (F1 + 1);
    auto base = [&](int s, uint32_t b) { return meta[(size_t)s * M + b]; };
    rbase.assign(NL, std::vector<uint64_t>(W + 1, 0));
    for (int l = 0; l < NL; l++) {
        const int r = G->rank0 + l;
        uint64_t acc = 0;
        for (int s = 0; s < W; s++) {
            rbase[l][s] = acc;
            acc += base(s, G->B[r + 1]) - base(s, G->B[r]);
        }
        rbase[l][W] = acc;
    }
    if (G->comm) {
        Graph *g = G->shards[0];
        Graph *V = G->views[0];
        const int r = G->rank0;
        KH_HIP(hipSetDevice(g->device));
        KH_HIP(hipStreamSynchronize(V->stream));
        const uint64_t own = base(r, G->B[r + 1]) - base(r, G->B[r]);
        if (own)
            KH_HIP(hipMemcpyAsync(g->ws.rec1 + rbase[0][r], V->ws.rec1 + base(r, G->B[r]), own * 8,
                                  hipMemcpyDeviceToDevice, g->stream));
        KH_NCCL(ncclGroupStart());
        for (int d = 0; d < W; d++) {
            if (d == r) continue;
            const uint64_t c = base(r, G->B[d + 1]) - base(r, G->B[d]);
            if (c) KH_NCCL(ncclSend(V->ws.rec1 + base(r, G->B[d]), c, ncclUint64, d, G->comm, g->stream));
            const uint64_t cin = base(d, G->B[r + 1]) - base(d, G->B[r]);
            if (cin) KH_NCCL(ncclRecv(g->ws.rec1 + rbase[0][d], cin, ncclUint64, d, G->comm, g->stream));
        }
        KH_NCCL(ncclGroupEnd());
    } else if (G->hosted) {
        Graph *g = G->shards[0];
        Graph *V = G->views[0];
        const int r = G->rank0;
        KH_HIP(hipSetDevice(g->device));
        std::vector<uint64_t> sb(W), rb(W);
        for (int d = 0; d < W; d++) {
            sb[d] = 8 * (base(r, G->B[d + 1]) - base(r, G->B[d]));
            rb[d] = 8 * (rbase[0][d + 1] - rbase[0][d]);
        }
        const uint64_t n0 = base(r, G->B[0]), nsend = base(r, G->B[W]) - n0;
        std::vector<uint64_t> hs(nsend + 1), hr(rbase[0][W] + 1);
        KH_HIP(hipMemcpyAsync(hs.data(), V->ws.rec1 + n0, nsend * 8, hipMemcpyDeviceToHost, V->stream));
        KH_HIP(hipStreamSynchronize(V->stream));
        host_rc(G->tp.alltoallv(G->tp.ctx, hs.data(), sb.data(), hr.data(), rb.data()), "alltoallv");
        KH_HIP(hipMemcpyAsync(g->ws.rec1, hr.data(), rbase[0][W] * 8, hipMemcpyHostToDevice, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
    } else {
        for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->views[l]->stream));
        for (int l = 0; l < NL; l++) {
            const int r = G->rank0 + l;
            Graph *g = G->shards[l];
            KH_HIP(hipSetDevice(g->device));
            for (int s = 0; s < W; s++) {
                const uint64_t c = rbase[l][s + 1] - rbase[l][s];
                if (c)
                    KH_HIP(hipMemcpyAsync(g->ws.rec1 + rbase[l][s], G->views[s]->ws.rec1 + base(s, G->B[r]), c * 8,
                                          hipMemcpyDeviceToDevice, g->stream));
            }
        }
    }
}

// the owner's received records as W * NB segments (lc.seg: starts, then
// ends): segment s * NB + b = source s's bucket B[r] + b inside its block of
// rec1.  Returns the number of segments.
static uint64_t a2a_segments(ShardGroup *G, int l, const std::vector<uint64_t> &meta, const std::vector<uint64_t> &rb) {
    const int W = G->world, r = G->rank0 + l;
    Graph *g = G->shards[l];
    const uint64_t F1v = G->views[0]->prm.F1, M = 2 * (F1v + 1);
    const uint32_t NB = G->B[r + 1] - G->B[r];
    const uint64_t nseg = (uint64_t)W * NB;
    std::vector<uint64_t> seg(2 * (nseg + 1));
    for (int s = 0; s < W; s++)
        for (uint32_t b = 0; b < NB; b++) {
            const uint64_t bb = meta[(size_t)s * M + G->B[r] + b], b0 = meta[(size_t)s * M + G->B[r]];
            const uint64_t e = meta[(size_t)s * M + F1v + 1 + G->B[r] + b];
            seg[s * NB + b] = rb[s] + (bb - b0);
            seg[nseg + 1 + s * NB + b] = rb[s] + (e - b0);
        }
    seg[nseg] = rb[W];
    seg[2 * nseg + 1] = rb[W];
    auto &lc = G->loc[l];
    ensure((void **)&lc.seg, &lc.cap_seg, 2 * (nseg + 1), 8);
    KH_HIP(hipMemcpyAsync(lc.seg, seg.data(), seg.size() * 8, hipMemcpyHostToDevice, g->stream));
    return nseg;
}

// the owner's level 2 over its (source, bucket) segments, apply and winners
static PassState a2a_owner_pass(ShardGroup *G, int l, const std::vector<uint64_t> &meta,
                                const std::vector<uint64_t> &rb, uint64_t nk) {
    const int W = G->world, r = G->rank0 + l;
    Graph *g = G->shards[l];
    const Params &P = g->prm;
    Workspace &w = g->ws;
    hipStream_t st = g->stream;
    KH_HIP(hipSetDevice(g->device));
    const uint32_t NB = G->B[r + 1] - G->B[r];
    if (NB != P.F1) fail(KH_EDEVICE, "exchange mode: owner geometry does not match its bucket range");
    PassState ps;
    ps.q = pass_geo(P, nk);
    ps.nkmers = nk;
    ps.bigc = P.kind == BYTE && P.use_bigcount;
    ws_prepare(g, ps.q);
    KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
    if (ps.bigc) {
        dev_fill(w.fullf, 0, (nk + 15) & ~15ull, st);
        bcmap_clear(w, st);
    }
    const uint64_t nseg = a2a_segments(G, l, meta, rb);
    auto &lc = G->loc[l];
    const uint64_t F2 = 1ull << P.s2, nreg = (uint64_t)P.F1 * F2;
    // W segments per bucket: split each into parts / W so a region has as many
    // writing workgroups (partial blocks) as reg_plan's slack allows
    const uint32_t parts = std::max<uint32_t>(1, l2f_parts(P.F1) / (uint32_t)W);
    for (;;) {
        const uint64_t cap2 = reg_plan(g, nk);
        if (cap2 > w.cap_recs) {
            // a larger margin after an overflow: grow both buffers, keeping
            // the received level-1 records
            const uint64_t keep = rb[W];
            uint64_t *tmp = nullptr;
            KH_HIP(hipMalloc((void **)&tmp, keep * 8 + 64));
            KH_HIP(hipMemcpyAsync(tmp, w.rec1, keep * 8, hipMemcpyDeviceToDevice, st));
            KH_HIP(hipStreamSynchronize(st));
            ensure_recs(g, cap2);
            KH_HIP(hipMemcpyAsync(w.rec1, tmp, keep * 8, hipMemcpyDeviceToDevice, st));
            KH_HIP(hipStreamSynchronize(st));
            KH_HIP(hipFree(tmp));
        }
        hipLaunchKernelGGL(k_reg_reset, dim3((unsigned)std::min<uint64_t>((nreg + 255) / 256, 4096)), dim3(256), 0, st,
                           w.reg_base, (unsigned long long *)w.reg_cur, nreg);
        TIMED("scatter_l2", hipLaunchKernelGGL((k_scatter_l2f<PT_THREADS, L2_RPT>), dim3((unsigned)(nseg * parts)),
                                               dim3(PT_THREADS), lds_scatter_l2f(P), st, (uint32_t)NB, P.s0, P.s2,
                                               parts, lc.seg, lc.seg + nseg + 1, w.reg_base,
                                               (unsigned long long *)w.reg_cur, w.rec1, w.rec2, w.ctr, l2f_blk_sh()));
        uint64_t err = 0;
        KH_HIP(hipMemcpyAsync(&err, w.ctr + CTR_ERR, 8, hipMemcpyDeviceToHost, st));
        KH_HIP(hipStreamSynchronize(st));
        if (!(err & 4)) break;
        KH_HIP(hipMemsetAsync(w.ctr + CTR_ERR, 0, 8, st));
        if (g->cap_sigma < 72.0 && recs_fit(g, nk, g->cap_sigma * 3.0)) {
            g->cap_sigma *= 3.0;
            continue;
        }
        fail(KH_EDEVICE, "exchange mode: a level-2 region overflowed at the largest capacity margin (skewed input)");
    }
    pass_apply(g, ps, true);
    return ps;
}

// finalize of the own chunk (its k-mers are [r * stride, r * stride + nkc) of
// the pass), counters, and the bigcount events of every rank merged into
// every rank's map (ByteStorage::add's saturating sum is order-free).
// on_views (delta mode): the chunk was applied on the rank's view, whose
// per-k-mer full tallies and counters are complete for its own k-mers (index
// 0 .. nkc); the counters still go to the shard.
template <class Src>
static void a2a_stage_c(ShardGroup *G, std::vector<PassState> &ps, const std::vector<Src> &srcs, uint64_t stride,
                        uint64_t nkc, bool on_views = false) {
    const int W = G->world, NL = G->nlocal;
    std::vector<std::vector<uint64_t>> keys(W);
    std::vector<std::vector<uint32_t>> cnts(W);
    std::vector<uint64_t> nff(W, 0);
    const bool bigc = ps[0].bigc;
    for (int l = 0; l < NL; l++) {
        const int r = G->rank0 + l;
        Graph *g = on_views ? G->views[l] : G->shards[l];
        Graph *home = G->shards[l];
        const uint64_t foff = on_views ? 0 : (uint64_t)r * stride;
        Workspace &w = g->ws;
        const Params &P = g->prm;
        hipStream_t st = g->stream;
        KH_HIP(hipSetDevice(g->device));
        const uint64_t nchunk = (nkc + 15) / 16;
        const unsigned fgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nchunk + FIN_THREADS - 1) / FIN_THREADS, 4096));
        for (;;) {
            if (bigc)
                TIMED("finalize", hipLaunchKernelGGL(k_finalize<Src>, dim3(fgrid), dim3(FIN_THREADS), 0, st, P,
                                                     srcs[l], nkc, w.fullf + foff, w.ctr, w.bck, w.bcv,
                                                     w.cap_bcmap - 1, (uint64_t *)nullptr));
            KH_HIP(hipGetLastError());
            KH_HIP(hipMemcpyAsync(w.h_ctr, w.ctr, CTR_N * 8, hipMemcpyDeviceToHost, st));
            KH_HIP(hipStreamSynchronize(st));
            if (!(bigc && (w.h_ctr[CTR_ERR] & 2))) break;
            bcmap_alloc(w, w.cap_bcmap * 4);
            bcmap_clear(w, st);
            KH_HIP(hipMemsetAsync(w.ctr + CTR_NBC, 0, 16, st));    // CTR_NBC, CTR_ERR
            KH_HIP(hipMemsetAsync(w.ctr + CTR_BCFF, 0, 8, st));
        }
        engine_collect_events(g);
        if (on_views) move_kstats(home, g);
        if (w.h_ctr[CTR_ERR]) fail(KH_EDEVICE, "device pipeline error flag set");
        home->n_occupied += w.h_ctr[CTR_OCC];
        home->n_unique += w.h_ctr[CTR_UNIQUE];
        if (!bigc) continue;
        const uint64_t nkeys = w.h_ctr[CTR_NBC];
        nff[r] = w.h_ctr[CTR_BCFF];
        keys[r].resize(nkeys);
        cnts[r].resize(nkeys);
        if (nkeys) {
            KH_HIP(hipMemsetAsync(w.ctr + CTR_BCOUT, 0, 8, st));
            const unsigned grid = (unsigned)std::min<uint64_t>((w.cap_bcmap + 255) / 256, 8192);
            hipLaunchKernelGGL(k_bc_compact, dim3(grid), dim3(256), 0, st, w.bck, w.bcv, w.cap_bcmap, w.ctr, w.bc,
                               w.bcn);
            KH_HIP(hipMemcpyAsync(keys[r].data(), w.bc, nkeys * 8, hipMemcpyDeviceToHost, st));
            KH_HIP(hipMemcpyAsync(cnts[r].data(), w.bcn, nkeys * 4, hipMemcpyDeviceToHost, st));
            KH_HIP(hipStreamSynchronize(st));
        }
    }
    if (!bigc) return;
    if (per_rank(G)) {
        // sizes, then (key, count) pairs padded to the largest list
        Graph *g = G->shards[0];
        const int r = G->rank0;
        KH_HIP(hipSetDevice(g->device));
        uint64_t mine[2] = {keys[r].size(), nff[r]};
        KH_HIP(hipMemcpyAsync(G->d_red + 160, mine, 16, hipMemcpyHostToDevice, g->stream));
        coll_allgather_u64(G, g->stream, G->d_red + 160, G->d_red, 2);
        std::vector<uint64_t> sz(2 * W);
        KH_HIP(hipMemcpyAsync(sz.data(), G->d_red, 2 * W * 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        uint64_t mx = 0;
        for (int s = 0; s < W; s++) {
            mx = std::max<uint64_t>(mx, sz[2 * s]);
            nff[s] = sz[2 * s + 1];
        }
        if (mx) {
            std::vector<uint64_t> send(2 * mx, 0), all((size_t)W * 2 * mx);
            for (uint64_t i = 0; i < keys[r].size(); i++) {
                send[2 * i] = keys[r][i];
                send[2 * i + 1] = cnts[r][i];
            }
            uint64_t *d = nullptr;
            KH_HIP(hipMalloc((void **)&d, (size_t)(W + 1) * 2 * mx * 8));
            KH_HIP(hipMemcpyAsync(d, send.data(), 2 * mx * 8, hipMemcpyHostToDevice, g->stream));
            coll_allgather_u64(G, g->stream, d, d + 2 * mx, 2 * mx);
            KH_HIP(hipMemcpyAsync(all.data(), d + 2 * mx, all.size() * 8, hipMemcpyDeviceToHost, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
            KH_HIP(hipFree(d));
            for (int s = 0; s < W; s++) {
                if (s == r) continue;
                keys[s].resize(sz[2 * s]);
                cnts[s].resize(sz[2 * s]);
                for (uint64_t i = 0; i < sz[2 * s]; i++) {
                    keys[s][i] = all[(size_t)s * 2 * mx + 2 * i];
                    cnts[s][i] = (uint32_t)all[(size_t)s * 2 * mx + 2 * i + 1];
                }
            }
        }
    }
    for (int l = 0; l < NL; l++) {
        Graph *g = G->shards[l];
        auto bump = [&](uint64_t h, uint64_t f) {
            auto it = g->bigcounts.find(h);
            const uint64_t b = it == g->bigcounts.end() ? 255 : it->second;
            g->bigcounts[h] = (uint16_t)std::min<uint64_t>(b + f, 65535);
        };
        bool any = false;
        for (int s = 0; s < W; s++) {
            if (nff[s]) bump(BC_EMPTY, nff[s]), any = true;
            for (size_t i = 0; i < keys[s].size(); i++) bump(keys[s][i], cnts[s][i]), any = true;
        }
        if (any) g->bc_dirty = true;
    }
}

// A group consume call's input: every rank's own fixed-length reads, packed
// 2-bit words (2-bit hashed graphs) or ASCII bytes (the Murmur-hashed
// Counttable family), the same count and length on every rank.
struct GroupReads {
    bool bytes = false;
    const void *const *d = nullptr;   // one device buffer per local shard
    uint64_t nreads = 0, read_len = 0, kpr = 0;
    // broadcast units (u64 words or bytes) of one rank's reads
    uint64_t units() const { return bytes ? nreads * read_len : (nreads * read_len + 31) / 32 + 1; }
    size_t esize() const { return bytes ? 1 : 8; }
    ncclDataType_t nccl_type() const { return bytes ? ncclUint8 : ncclUint64; }
};

// the source of reads [r0, r0 + nr) of buffer `buf` (a rank's reads) for graph g
template <class Src>
static Src group_src(Graph *g, const GroupReads &R, const void *buf, uint64_t r0, uint64_t nr);
template <>
SrcTwoBit group_src<SrcTwoBit>(Graph *g, const GroupReads &R, const void *buf, uint64_t r0, uint64_t nr) {
    SrcTwoBit s = src_twobit(g, (const uint64_t *)buf);
    set_fixed(s, R.kpr, R.nreads);
    s.koff = nullptr;
    s.nreads = nr;
    s.kbase = r0 * R.kpr;
    s.rbase = 0;
    return s;
}
template <>
SrcBytes group_src<SrcBytes>(Graph *g, const GroupReads &R, const void *buf, uint64_t r0, uint64_t nr) {
    // the windows read up to 64 bytes past the pass's last read (padded_bytes);
    // the pass's reverse-complement stream goes to g's workspace
    const uint8_t *b = padded_bytes(g, (const uint8_t *)buf + r0 * R.read_len, nr * R.read_len);
    SrcBytes s = src_bytes(g, b, nullptr, nr, R.kpr, nr * R.read_len);
    set_fixed(s, R.kpr, R.nreads);
    s.koff = nullptr;
    s.nreads = nr;
    s.kbase = 0;
    s.rbase = 0;
    return s;
}

// Pass-level failure agreement (collective).  In a one-shard-per-process
// group a rank that fails on its own (a capacity overflow at the largest
// margin, an allocation failure) would leave its peers blocked in the pass's
// next collective; instead every rank reaches this point, the error flags are
// all-reduced, and all ranks fail together.  Loopback: rethrow directly.
static void group_agree(ShardGroup *G, std::exception_ptr err) {
    if (per_rank(G) && G->world > 1) {
        Graph *g = G->shards[0];
        KH_HIP(hipSetDevice(g->device));
        const uint64_t mine = err ? 1 : 0;
        uint64_t any = 0;
        KH_HIP(hipMemcpyAsync(G->d_red + 170, &mine, 8, hipMemcpyHostToDevice, g->stream));
        coll_allreduce_u64(G, g->stream, G->d_red + 170, G->d_red + 171, 1, RED_MAX);
        KH_HIP(hipMemcpyAsync(&any, G->d_red + 171, 8, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
        if (any && !err) fail(KH_EDEVICE, "sharded consume: another rank failed in this pass");
    }
    if (err) std::rethrow_exception(err);
}
#define GROUP_TRY(...)                                                                             \
    do {                                                                                           \
        std::exception_ptr e_;                                                                     \
        try { __VA_ARGS__; } catch (...) { e_ = std::current_exception(); }                        \
        group_agree(G, e_);                                                                        \
    } while (0)

// Exchange-mode passes: a pass takes the next rpb reads of every rank; its
// k-mer index space W * stride (stride a multiple of 16: fullf chunks) stays
// below 2^32 (khmer_amd.parallel.exchange_passes restates this plan)
static void a2a_pass_plan(ShardGroup *G, Graph *g0, const GroupReads &R, uint64_t *rpb, uint64_t *stride) {
    const uint64_t cap = std::min<uint64_t>(g0->batch_kmers, MAX_PASS_KMERS) / (uint64_t)G->world;
    const uint64_t rpb0 = std::max<uint64_t>(1, (cap > 16 ? cap - 16 : 1) / R.kpr);
    const uint64_t npass = std::max<uint64_t>(1, (R.nreads + rpb0 - 1) / rpb0);
    *rpb = std::max<uint64_t>(1, (R.nreads + npass - 1) / npass);
    *stride = (*rpb * R.kpr + 15) & ~15ull;
}

template <class Src>
static void group_consume_a2a(ShardGroup *G, const GroupReads &R) {
    const int W = G->world, NL = G->nlocal;
    Graph *g0 = G->shards[0];
    const uint64_t kpr = R.kpr, nreads = R.nreads;
    uint64_t rpb, stride;
    a2a_pass_plan(G, g0, R, &rpb, &stride);
    const uint64_t nk = (uint64_t)W * stride;
    for (uint64_t r0 = 0; r0 < nreads; r0 += rpb) {
        const uint64_t nr = std::min(rpb, nreads - r0), nkc = nr * kpr;
        std::vector<Src> srcs(NL);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            Graph *V = G->views[l];
            KH_HIP(hipSetDevice(V->device));
            V->use_bigcount = false;   // the owners finalize; the view only runs level 1
            V->profile = G->shards[l]->profile;
            srcs[l] = group_src<Src>(V, R, R.d[l], r0, nr);
            a2a_level1(V, srcs[l], nkc, (uint32_t)((uint64_t)(G->rank0 + l) * stride));
            move_kstats(G->shards[l], V);
        });
        std::vector<uint64_t> meta;
        a2a_meta(G, meta);
        // owner buffers: the received records (level 1) and the level-2 regions
        const uint64_t F1v = G->views[0]->prm.F1, M = 2 * (F1v + 1);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            const int r = G->rank0 + l;
            Graph *g = G->shards[l];
            KH_HIP(hipSetDevice(g->device));
            uint64_t need = 0;
            for (int s = 0; s < W; s++) need += meta[(size_t)s * M + G->B[r + 1]] - meta[(size_t)s * M + G->B[r]];
            ensure_recs(g, std::max(need, reg_plan(g, nk)));
        });
        std::vector<std::vector<uint64_t>> rb;
        a2a_exchange(G, meta, rb);
        std::vector<PassState> ps(NL);
        GROUP_TRY(for (int l = 0; l < NL; l++) ps[l] = a2a_owner_pass(G, l, meta, rb[l], nk));
        group_route_winners(G, ps);
        if (ps[0].bigc) group_merge_full(G, ps);
        a2a_stage_c(G, ps, srcs, stride, nkc);
    }
    for (int l = 0; l < NL; l++) {
        KH_HIP(hipSetDevice(G->shards[l]->device));
        KH_HIP(hipStreamSynchronize(G->views[l]->stream));
        KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
    }
}

// ---------------------------------------------------------------------------
// Delta mode (KH_GROUP_DELTA, khmer_hip.h): per pass, every rank
//   1. partitions its own chunk on its full-geometry view (single-GPU level 1
//      and level 2, k-mer indices local to the chunk) and writes the chunk's
//      delta tables D_r (k_apply_delta) into the view's arena;
//   2. sends owner o the bytes of o's slice (all-to-all of table bytes);
//   3. as owner, turns the W deltas of its slice into the prefixes
//      P_r = T + D_0 + ... + D_{r-1} and its new slice T + D_0 + ... +
//      D_{W-1} (k_delta_prefix, saturating in the storage's layout);
//   4. receives its own prefix P_r of every slice back into the view's arena;
//   5. applies its chunk over P_r with the single-GPU apply: a bin's value
//      there is exactly what the stream (the rank chunks in rank order) shows
//      when the rank's chunk begins, so the apply's is_new winners, table-0
//      first touches and full inserts are the reference's for the rank's own
//      k-mers (storage.hh:571-624, 320-359, 172-199) -- n_unique,
//      n_occupied and bigcount events need no routing;
//   6. finalize + counters + bigcount events merged (a2a_stage_c on views).
// The view's arena then holds P_r plus its own inserts and is overwritten by
// the next pass's delta.

// bytes [*b0, *b0 + *nb) of table i's reference layout held by rank o: the
// bytes of its bucket-aligned bin slice (bin slices start on byte
// boundaries).  Only bytes that hold bins travel: a Bit / Nibble table's
// trailing byte past its last bin (p/8 + 1, p/2 + 1 bytes of storage)
// stays 0 on every rank.
static void delta_slice(const ShardGroup *G, int o, int i, uint64_t *b0, uint64_t *nb) {
    const Graph *V = G->views[0];
    const int n = V->n;
    const uint64_t lo = G->blo[(size_t)o * n + i], hi = G->bhi[(size_t)o * n + i];
    const uint64_t bpb = V->kind == BIT ? 8 : V->kind == NIBBLE ? 2 : 1;   // bins per byte
    *b0 = lo / bpb;
    *nb = lo < hi ? (hi + bpb - 1) / bpb - *b0 : 0;
}
// owner o's delta buffer: W blocks of `stride` bytes (one per source rank),
// table i's slice at offset soff[i] of a block (256-B aligned: the prefix
// kernel's 16-B accesses)
static uint64_t delta_layout(const ShardGroup *G, int o, std::vector<uint64_t> &soff) {
    const int n = G->views[0]->n;
    soff.assign(n, 0);
    uint64_t acc = 0;
    for (int i = 0; i < n; i++) {
        uint64_t b0, nb;
        delta_slice(G, o, i, &b0, &nb);
        soff[i] = acc;
        acc += (nb + 255) / 256 * 256;
    }
    return std::max<uint64_t>(acc, 256);
}

// step 1b: the chunk's delta tables into the view's arena
static void delta_apply(Graph *V, PassState &ps, bool l2f) {
    const Params &P = V->prm;
    Workspace &w = V->ws;
    ApplyArgs A{};
    A.rlo = l2f ? w.reg_base : w.off2;
    A.rhi = l2f ? w.reg_cur : w.off2 + 1;
    A.rec = w.rec2;
    A.tab = V->d_tab;
    A.rprefix[0] = 0;
    for (int i = 0; i < P.n; i++) A.rprefix[i + 1] = A.rprefix[i] + ((P.lsz[i] + (1ull << P.s0) - 1) >> P.s0);
    const uint64_t total = A.rprefix[P.n];
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(total, 4 * device_cus(V)));
    const int th = 1 << (P.s0 - 4);
    const size_t lds = ((size_t)1 << P.s0) * 4;
    hipStream_t st = V->stream;
    Graph *g = V;
    if (th == 1024) {
        if (P.kind == BYTE) TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<BYTE, 1024>), dim3(grid), dim3(1024), lds, st, P, A));
        else if (P.kind == NIBBLE) TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<NIBBLE, 1024>), dim3(grid), dim3(1024), lds, st, P, A));
        else TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<BIT, 1024>), dim3(grid), dim3(1024), lds, st, P, A));
    } else {
        if (P.kind == BYTE) TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<BYTE, 512>), dim3(grid), dim3(512), lds, st, P, A));
        else if (P.kind == NIBBLE) TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<NIBBLE, 512>), dim3(grid), dim3(512), lds, st, P, A));
        else TIMED("apply_delta", hipLaunchKernelGGL((k_apply_delta<BIT, 512>), dim3(grid), dim3(512), lds, st, P, A));
    }
    KH_HIP(hipGetLastError());
    (void)ps;
}

// steps 2 and 4: forward = every rank's delta slices to their owners'
// buffers; backward = every owner's prefix slices back into the ranks' views
// Sparse pieces of the delta exchange (kh_apply.cuh k_sp_*): a table slice
// travels as a bitmap of its nonzero bytes plus those bytes -- C4's deltas
// are ~93 % zeros, so a rank-pass sends ~1/5 of the table bytes.
// KH_DELTA_SPARSE=0 sends them dense (read in every build: the tests compare).
static bool delta_sparse_on() { return test_env_int("KH_DELTA_SPARSE", 1) != 0; }
static uint64_t sp_bm_bytes(uint64_t nb) { return ((nb + 15) / 16 * 2 + 15) & ~15ull; }
static uint64_t sp_worst(uint64_t nb) { return sp_bm_bytes(nb) + ((nb + 15) & ~15ull); }
static bool sp_aligned(const void *p) { return ((uintptr_t)p & 15) == 0; }
// [src, src + nb) -> out (bitmap, then the payload at out + sp_bm_bytes(nb));
// the payload's byte count into *d_size (device), on g's stream
static void sp_pack(Graph *g, const uint8_t *src, uint64_t nb, uint8_t *out, uint64_t *d_size) {
    Workspace &w = g->ws;
    const uint64_t nch = (nb + SP_CHUNK - 1) / SP_CHUNK;
    ensure((void **)&w.sp_cnt, &w.cap_spcnt, nch + 1, 4);
    ensure((void **)&w.sp_off, &w.cap_spoff, nch + 1, 8);
    KTimer kt_(g, "delta_pack");
    hipLaunchKernelGGL(k_sp_count, dim3((unsigned)nch), dim3(SP_THREADS), 0, g->stream, src, nullptr, nb, w.sp_cnt);
    scan_counts(g, w.sp_cnt, w.sp_off, nch + 1);
    hipLaunchKernelGGL(k_sp_pack, dim3((unsigned)nch), dim3(SP_THREADS), 0, g->stream, src, nb, w.sp_off,
                       (uint16_t *)out, out + sp_bm_bytes(nb));
    KH_HIP(hipMemcpyAsync(d_size, w.sp_off + nch, 8, hipMemcpyDeviceToDevice, g->stream));
    KH_HIP(hipGetLastError());
}
static void sp_unpack(Graph *g, const uint8_t *in, uint64_t nb, uint8_t *dst) {
    Workspace &w = g->ws;
    const uint64_t nch = (nb + SP_CHUNK - 1) / SP_CHUNK;
    ensure((void **)&w.sp_cnt, &w.cap_spcnt, nch + 1, 4);
    ensure((void **)&w.sp_off, &w.cap_spoff, nch + 1, 8);
    KTimer kt_(g, "delta_unpack");
    hipLaunchKernelGGL(k_sp_count, dim3((unsigned)nch), dim3(SP_THREADS), 0, g->stream, nullptr,
                       (const uint16_t *)in, nb, w.sp_cnt);
    scan_counts(g, w.sp_cnt, w.sp_off, nch + 1);
    hipLaunchKernelGGL(k_sp_unpack, dim3((unsigned)nch), dim3(SP_THREADS), 0, g->stream, (const uint16_t *)in,
                       in + sp_bm_bytes(nb), w.sp_off, nb, dst);
    KH_HIP(hipGetLastError());
}

static void delta_exchange(ShardGroup *G, bool forward) {
    const int W = G->world, NL = G->nlocal, n = G->views[0]->n;
    std::vector<std::vector<uint64_t>> soff(W);
    std::vector<uint64_t> stride(W);
    for (int o = 0; o < W; o++) stride[o] = delta_layout(G, o, soff[o]);
    auto slice = [&](int o, int i, uint64_t *b0, uint64_t *nb) { delta_slice(G, o, i, b0, nb); };
    if (G->comm) {
        Graph *V = G->views[0];
        auto &lc = G->loc[0];
        const int r = G->rank0;
        KH_HIP(hipSetDevice(V->device));
        hipStream_t st = V->stream;
        // own slice: a device copy
        for (int i = 0; i < n; i++) {
            uint64_t b0, nb;
            slice(r, i, &b0, &nb);
            if (!nb) continue;
            uint8_t *vt = V->d_tab + V->prm.tbyte[i] + b0;
            uint8_t *bt = lc.dbuf + (uint64_t)r * stride[r] + soff[r][i];
            KH_HIP(hipMemcpyAsync(forward ? bt : vt, forward ? vt : bt, nb, hipMemcpyDeviceToDevice, st));
        }
        // the pieces to and from every other rank: (table i of peer d) ->
        // send src / receive dst and byte count, in (d, i) order
        struct Piece { const uint8_t *src; uint8_t *dst; uint64_t nb; int d, i; };
        std::vector<Piece> sends, recvs;
        uint64_t need = 0;
        bool aligned = true;
        for (int d = 0; d < W; d++) {
            if (d == r) continue;
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                if (forward) {
                    slice(d, i, &b0, &nb);
                    if (nb) sends.push_back({V->d_tab + V->prm.tbyte[i] + b0, nullptr, nb, d, i});
                    slice(r, i, &b0, &nb);
                    if (nb) recvs.push_back({nullptr, lc.dbuf + (uint64_t)d * stride[r] + soff[r][i], nb, d, i});
                } else {
                    slice(r, i, &b0, &nb);
                    if (nb) sends.push_back({lc.dbuf + (uint64_t)d * stride[r] + soff[r][i], nullptr, nb, d, i});
                    slice(d, i, &b0, &nb);
                    if (nb) recvs.push_back({nullptr, V->d_tab + V->prm.tbyte[i] + b0, nb, d, i});
                }
            }
        }
        for (const Piece &p : sends) { need += sp_worst(p.nb); aligned = aligned && sp_aligned(p.src); }
        for (const Piece &p : recvs) { need += sp_worst(p.nb); aligned = aligned && sp_aligned(p.dst); }
        // KH_DELTA_PROBE=1 at world 1 (tools/rank_model.py): no piece leaves
        // the rank, so pack the own slices instead and count them, for the
        // sparse wire estimate of a larger group
        // (the deltas only: the prefixes of a larger group are denser than a
        // world-1 rank's, which is the table before the pass)
        if (forward && sends.empty() && W == 1 && test_env_int("KH_DELTA_PROBE", 0)) {
            ensure((void **)&lc.d_sz, &lc.cap_dsz, 2, 8);
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                slice(r, i, &b0, &nb);
                const uint8_t *src = V->d_tab + V->prm.tbyte[i] + b0;
                if (!nb || !sp_aligned(src)) continue;
                ensure((void **)&lc.stage, &lc.cap_stage, sp_worst(nb), 1);
                sp_pack(V, src, nb, lc.stage, lc.d_sz);
                uint64_t sz = 0;
                KH_HIP(hipMemcpyAsync(&sz, lc.d_sz, 8, hipMemcpyDeviceToHost, st));
                KH_HIP(hipStreamSynchronize(st));
                G->wire_dense += nb;
                G->wire_sent += std::min(sp_bm_bytes(nb) + sz, nb);
            }
        }
        // staging: the view's level-1 record buffer (dead between level 2 and
        // the apply that follows the exchange)
        if (!sends.empty() && delta_sparse_on() && aligned) {
            uint8_t *stage = (uint8_t *)V->ws.rec1;
            if (need > V->ws.cap_recs * 8) {
                ensure((void **)&lc.stage, &lc.cap_stage, need, 1);
                stage = lc.stage;
            }
            ensure((void **)&lc.d_sz, &lc.cap_dsz, 2 * (uint64_t)W * n, 8);
            uint64_t *d_ssz = lc.d_sz, *d_rsz = lc.d_sz + (uint64_t)W * n;
            KH_HIP(hipMemsetAsync(lc.d_sz, 0, 2 * (uint64_t)W * n * 8, st));
            std::vector<uint64_t> sb(sends.size()), rb(recvs.size());
            uint64_t at = 0;
            for (size_t k = 0; k < sends.size(); k++) {
                sb[k] = at;
                at += sp_worst(sends[k].nb);
                sp_pack(V, sends[k].src, sends[k].nb, stage + sb[k], d_ssz + (uint64_t)sends[k].d * n + sends[k].i);
            }
            for (size_t k = 0; k < recvs.size(); k++) {
                rb[k] = at;
                at += sp_worst(recvs[k].nb);
            }
            // payload sizes first (n per peer), then the pieces
            KH_NCCL(ncclGroupStart());
            for (int d = 0; d < W; d++) {
                if (d == r) continue;
                KH_NCCL(ncclSend(d_ssz + (uint64_t)d * n, n, ncclUint64, d, G->comm, st));
                KH_NCCL(ncclRecv(d_rsz + (uint64_t)d * n, n, ncclUint64, d, G->comm, st));
            }
            KH_NCCL(ncclGroupEnd());
            std::vector<uint64_t> hsz(2 * (uint64_t)W * n);
            KH_HIP(hipMemcpyAsync(hsz.data(), lc.d_sz, hsz.size() * 8, hipMemcpyDeviceToHost, st));
            KH_HIP(hipStreamSynchronize(st));
            KH_NCCL(ncclGroupStart());
            // a piece whose sparse form is not smaller travels dense (both
            // sides decide from the same payload size)
            std::vector<char> rsparse(recvs.size(), 0);
            for (size_t k = 0; k < sends.size(); k++) {
                const uint64_t bytes = sp_bm_bytes(sends[k].nb) + hsz[(uint64_t)sends[k].d * n + sends[k].i];
                G->wire_dense += sends[k].nb;
                G->wire_sent += std::min(bytes, sends[k].nb);
                if (bytes < sends[k].nb)
                    KH_NCCL(ncclSend(stage + sb[k], bytes, ncclUint8, sends[k].d, G->comm, st));
                else
                    KH_NCCL(ncclSend(sends[k].src, sends[k].nb, ncclUint8, sends[k].d, G->comm, st));
            }
            for (size_t k = 0; k < recvs.size(); k++) {
                const uint64_t sz = hsz[(uint64_t)W * n + (uint64_t)recvs[k].d * n + recvs[k].i];
                if (sz > recvs[k].nb) fail(KH_EDEVICE, "sparse delta piece larger than its slice");
                const uint64_t bytes = sp_bm_bytes(recvs[k].nb) + sz;
                rsparse[k] = bytes < recvs[k].nb;
                if (rsparse[k])
                    KH_NCCL(ncclRecv(stage + rb[k], bytes, ncclUint8, recvs[k].d, G->comm, st));
                else
                    KH_NCCL(ncclRecv(recvs[k].dst, recvs[k].nb, ncclUint8, recvs[k].d, G->comm, st));
            }
            KH_NCCL(ncclGroupEnd());
            for (size_t k = 0; k < recvs.size(); k++)
                if (rsparse[k]) sp_unpack(V, stage + rb[k], recvs[k].nb, recvs[k].dst);
            return;
        }
        for (const Piece &p : sends) {
            G->wire_dense += p.nb;
            G->wire_sent += p.nb;
        }
        KH_NCCL(ncclGroupStart());
        for (int d = 0; d < W; d++) {
            if (d == r) continue;
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                if (forward) {
                    slice(d, i, &b0, &nb);   // my delta of d's slice -> d
                    if (nb) KH_NCCL(ncclSend(V->d_tab + V->prm.tbyte[i] + b0, nb, ncclUint8, d, G->comm, st));
                    slice(r, i, &b0, &nb);   // d's delta of my slice
                    if (nb) KH_NCCL(ncclRecv(lc.dbuf + (uint64_t)d * stride[r] + soff[r][i], nb, ncclUint8, d, G->comm, st));
                } else {
                    slice(r, i, &b0, &nb);   // d's prefix of my slice -> d
                    if (nb) KH_NCCL(ncclSend(lc.dbuf + (uint64_t)d * stride[r] + soff[r][i], nb, ncclUint8, d, G->comm, st));
                    slice(d, i, &b0, &nb);   // my prefix of d's slice
                    if (nb) KH_NCCL(ncclRecv(V->d_tab + V->prm.tbyte[i] + b0, nb, ncclUint8, d, G->comm, st));
                }
            }
        }
        KH_NCCL(ncclGroupEnd());
        return;
    }
    if (G->hosted) {
        // one alltoallv; every (source, owner) block is the owner's padded
        // layout, so a received block drops into the delta buffer as it is
        Graph *V = G->views[0];
        auto &lc = G->loc[0];
        const int r = G->rank0;
        KH_HIP(hipSetDevice(V->device));
        hipStream_t st = V->stream;
        std::vector<uint64_t> sb(W), rb(W), at(W + 1, 0);
        for (int d = 0; d < W; d++) {
            sb[d] = forward ? stride[d] : stride[r];
            rb[d] = forward ? stride[r] : stride[d];
            at[d + 1] = at[d] + sb[d];
        }
        std::vector<uint8_t> &hs = lc.hsend, &hr = lc.hrecv;
        if (hs.size() < at[W] + 1) hs.resize(at[W] + 1);
        KH_HIP(hipStreamSynchronize(st));
        for (int d = 0; d < W; d++)
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                if (forward) {
                    slice(d, i, &b0, &nb);
                    if (nb) KH_HIP(hipMemcpy(hs.data() + at[d] + soff[d][i], V->d_tab + V->prm.tbyte[i] + b0, nb,
                                             hipMemcpyDeviceToHost));
                } else {
                    slice(r, i, &b0, &nb);
                    if (nb) KH_HIP(hipMemcpy(hs.data() + at[d] + soff[r][i], lc.dbuf + (uint64_t)d * stride[r] + soff[r][i],
                                             nb, hipMemcpyDeviceToHost));
                }
            }
        uint64_t rtot = 0;
        for (int d = 0; d < W; d++) rtot += rb[d];
        if (hr.size() < rtot + 1) hr.resize(rtot + 1);
        host_rc(G->tp.alltoallv(G->tp.ctx, hs.data(), sb.data(), hr.data(), rb.data()), "alltoallv");
        uint64_t q = 0;
        for (int s = 0; s < W; s++) {
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                if (forward) {
                    slice(r, i, &b0, &nb);
                    if (nb) KH_HIP(hipMemcpy(lc.dbuf + (uint64_t)s * stride[r] + soff[r][i], hr.data() + q + soff[r][i], nb,
                                             hipMemcpyHostToDevice));
                } else {
                    slice(s, i, &b0, &nb);
                    if (nb) KH_HIP(hipMemcpy(V->d_tab + V->prm.tbyte[i] + b0, hr.data() + q + soff[s][i], nb,
                                             hipMemcpyHostToDevice));
                }
            }
            q += rb[s];
        }
        return;
    }
    // loopback: device copies between the local views and owners; pieces
    // between two ranks of one device go through the sparse codec, as they
    // would on the wire (packed into the owner's dead level-1 buffer and
    // unpacked from it, one piece at a time on the owner's stream)
    for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->views[l]->stream));
    for (int o = 0; o < W; o++) {
        auto &lc = G->loc[o];
        Graph *Vo = G->views[o];
        KH_HIP(hipSetDevice(Vo->device));
        for (int s = 0; s < W; s++) {
            Graph *Vs = G->views[s];
            for (int i = 0; i < n; i++) {
                uint64_t b0, nb;
                slice(o, i, &b0, &nb);
                if (!nb) continue;
                uint8_t *vt = Vs->d_tab + Vs->prm.tbyte[i] + b0;
                uint8_t *bt = lc.dbuf + (uint64_t)s * stride[o] + soff[o][i];
                const uint8_t *src = forward ? vt : bt;
                uint8_t *dst = forward ? bt : vt;
                if (s != o && delta_sparse_on() && Vs->device == Vo->device && sp_aligned(src) && sp_aligned(dst)) {
                    uint8_t *stage = (uint8_t *)Vo->ws.rec1;
                    if (sp_worst(nb) > Vo->ws.cap_recs * 8) {
                        ensure((void **)&lc.stage, &lc.cap_stage, sp_worst(nb), 1);
                        stage = lc.stage;
                    }
                    ensure((void **)&lc.d_sz, &lc.cap_dsz, 2, 8);
                    sp_pack(Vo, src, nb, stage, lc.d_sz);
                    uint64_t sz = 0;
                    KH_HIP(hipMemcpyAsync(&sz, lc.d_sz, 8, hipMemcpyDeviceToHost, Vo->stream));
                    KH_HIP(hipStreamSynchronize(Vo->stream));
                    G->wire_dense += nb;
                    G->wire_sent += std::min(sp_bm_bytes(nb) + sz, nb);
                    if (sp_bm_bytes(nb) + sz < nb) {   // else dense, as on the wire
                        sp_unpack(Vo, stage, nb, dst);
                        continue;
                    }
                    KH_HIP(hipMemcpyAsync(dst, src, nb, hipMemcpyDefault, Vo->stream));
                    continue;
                }
                if (s != o) {
                    G->wire_dense += nb;
                    G->wire_sent += nb;
                }
                KH_HIP(hipMemcpyAsync(dst, src, nb, hipMemcpyDefault, Vo->stream));
            }
        }
    }
    for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->views[l]->stream));
}

// step 3: the owner's prefixes and its new slice
static void delta_prefix(ShardGroup *G, int l) {
    const int W = G->world, r = G->rank0 + l;
    Graph *g = G->shards[l];
    Graph *V = G->views[l];
    auto &lc = G->loc[l];
    std::vector<uint64_t> soff;
    const uint64_t stride = delta_layout(G, r, soff);
    KH_HIP(hipSetDevice(g->device));
    for (int i = 0; i < g->n; i++) {
        uint64_t b0, nb;
        delta_slice(G, r, i, &b0, &nb);
        if (!nb) continue;
        uint8_t *T = g->d_tab + g->prm.tbyte[i];
        uint8_t *buf = lc.dbuf + soff[i];
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nb + 16 * 256 - 1) / (16 * 256), 8192));
        Graph *gt = V;   // timed on the view's stream (the pass's stream)
        {
            KTimer kt_(gt, "delta_prefix");
            if (g->kind == BYTE)
                hipLaunchKernelGGL(k_delta_prefix<BYTE>, dim3(grid), dim3(256), 0, V->stream, T, buf, nb, stride, W);
            else if (g->kind == NIBBLE)
                hipLaunchKernelGGL(k_delta_prefix<NIBBLE>, dim3(grid), dim3(256), 0, V->stream, T, buf, nb, stride, W);
            else
                hipLaunchKernelGGL(k_delta_prefix<BIT>, dim3(grid), dim3(256), 0, V->stream, T, buf, nb, stride, W);
        }
        KH_HIP(hipGetLastError());
    }
}

// Delta-mode passes: up to the graph's batch (<= MAX_PASS_KMERS) of every
// rank's own reads per pass (a2a_pass_plan at world 1;
// khmer_amd.parallel.delta_passes restates it)
template <class Src>
static void group_consume_delta(ShardGroup *G, const GroupReads &R) {
    const int W = G->world, NL = G->nlocal;
    Graph *g0 = G->shards[0];
    const uint64_t kpr = R.kpr, nreads = R.nreads;
    const uint64_t cap = std::min<uint64_t>(g0->batch_kmers, MAX_PASS_KMERS);
    const uint64_t rpb0 = std::max<uint64_t>(1, (cap > 16 ? cap - 16 : 1) / kpr);
    const uint64_t npass = std::max<uint64_t>(1, (nreads + rpb0 - 1) / rpb0);
    const uint64_t rpb = std::max<uint64_t>(1, (nreads + npass - 1) / npass);
    GROUP_TRY(for (int l = 0; l < NL; l++) {
        const int r = G->rank0 + l;
        std::vector<uint64_t> soff;
        const uint64_t stride = delta_layout(G, r, soff);
        KH_HIP(hipSetDevice(G->shards[l]->device));
        ensure((void **)&G->loc[l].dbuf, &G->loc[l].cap_dbuf, (uint64_t)W * stride, 1);
    });
    for (uint64_t r0 = 0; r0 < nreads; r0 += rpb) {
        const uint64_t nr = std::min(rpb, nreads - r0), nkc = nr * kpr;
        std::vector<Src> srcs(NL);
        std::vector<PassState> ps(NL);
        std::vector<char> fast(NL, 0);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            Graph *V = G->views[l];
            Graph *sh = G->shards[l];
            KH_HIP(hipSetDevice(V->device));
            V->use_bigcount = sh->use_bigcount;
            V->prm.use_bigcount = sh->prm.use_bigcount;
            V->profile = sh->profile;
            srcs[l] = group_src<Src>(V, R, R.d[l], r0, nr);
            bool f = false;
            // complement mode's winner-share estimate: the table's occupancy,
            // scaled up from the home shard's slice of table 0 (the view's own
            // counters stay 0: a2a_stage_c counts into the home shard)
            const Params &SP = sh->prm;
            V->occ_hint = SP.lsz[0] ? (int64_t)((double)sh->n_occupied * (double)SP.p[0] / (double)SP.lsz[0]) : -1;
            ps[l] = pass_stage_a(V, srcs[l], nkc, false, &f);
            fast[l] = f;
            delta_apply(V, ps[l], f);
        });
        delta_exchange(G, true);
        GROUP_TRY(for (int l = 0; l < NL; l++) delta_prefix(G, l));
        delta_exchange(G, false);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            Graph *V = G->views[l];
            KH_HIP(hipSetDevice(V->device));
            pass_apply(V, ps[l], fast[l] != 0);
            pass_mark_local(V, ps[l], false);
        });
        a2a_stage_c(G, ps, srcs, 0, nkc, true);
    }
    for (int l = 0; l < NL; l++) {
        KH_HIP(hipSetDevice(G->shards[l]->device));
        KH_HIP(hipStreamSynchronize(G->views[l]->stream));
        KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
    }
}

// the broadcast-mode consume (Option B) of every rank's reads, source by source
template <class Src>
static void group_consume_bcast(ShardGroup *G, const GroupReads &R) {
    const int W = G->world, NL = G->nlocal;
    Graph *g0 = G->shards[0];
    const uint64_t kpr = R.kpr, nreads = R.nreads;
    const uint64_t nunits = R.units();
    const size_t esz = R.esize();
    const uint64_t slot_words = (nunits * esz + 64 + 7) / 8;   // + the windows' 64-byte read-ahead
    const uint64_t rpb0 = std::max<uint64_t>(1, std::min<uint64_t>(g0->batch_kmers, MAX_PASS_KMERS) / kpr);
    const uint64_t npass = std::max<uint64_t>(1, (nreads + rpb0 - 1) / rpb0);
    const uint64_t rpb = std::max<uint64_t>(1, (nreads + npass - 1) / npass);   // equal passes
    // Source s's reads travel into slot s & 1 on the transfer stream while the
    // compute stream consumes source s - 1 from the other slot: events order
    // slot reuse (ev_free, recorded after a source's last pass) and use
    // (ev_ready).  RCCL: a broadcast on comm_b, the root in place on its own
    // buffer.  Loopback: a device copy (the same schedule without RCCL).
    for (int l = 0; l < NL; l++) {
        auto &lc = G->loc[l];
        KH_HIP(hipSetDevice(G->shards[l]->device));
        if (!lc.st_x) {
            KH_HIP(hipStreamCreateWithFlags(&lc.st_x, hipStreamNonBlocking));
            for (int b = 0; b < 2; b++) {
                KH_HIP(hipEventCreateWithFlags(&lc.ev_ready[b], hipEventDisableTiming));
                KH_HIP(hipEventCreateWithFlags(&lc.ev_free[b], hipEventDisableTiming));
            }
        }
        for (int b = 0; b < 2; b++) lc.freed[b] = false;   // each slot's last reader is done (synchronised)
    }
    const bool rccl = G->comm != nullptr;
    auto own = [&](int s, int l) { return per_rank(G) && G->rank0 + l == s; };
    auto transfer = [&](int s) {
        for (int l = 0; l < NL; l++) {
            auto &lc = G->loc[l];
            const int b = s & 1;
            KH_HIP(hipSetDevice(G->shards[l]->device));
            if (lc.freed[b]) KH_HIP(hipStreamWaitEvent(lc.st_x, lc.ev_free[b], 0));
            if (!own(s, l)) {
                if (lc.cap_slot[b] < slot_words) KH_HIP(hipStreamSynchronize(lc.st_x));   // about to be reallocated
                ensure((void **)&lc.slot[b], &lc.cap_slot[b], slot_words, 8);
                KH_HIP(hipMemsetAsync((uint8_t *)lc.slot[b] + nunits * esz, 0, 64, lc.st_x));
            }
            if (G->hosted) {
                // synchronous: the root's reads through host memory into the slot
                std::vector<uint8_t> hb(nunits * esz);
                if (own(s, l)) {
                    KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
                    KH_HIP(hipMemcpy(hb.data(), R.d[0], hb.size(), hipMemcpyDeviceToHost));
                }
                host_rc(G->tp.broadcast(G->tp.ctx, hb.data(), hb.size(), s), "broadcast");
                if (!own(s, l)) {
                    KH_HIP(hipMemcpyAsync(lc.slot[b], hb.data(), hb.size(), hipMemcpyHostToDevice, lc.st_x));
                    KH_HIP(hipStreamSynchronize(lc.st_x));
                }
            } else if (own(s, l)) {
                void *w = const_cast<void *>(R.d[0]);
                KH_NCCL(ncclBroadcast(w, w, nunits, R.nccl_type(), s, G->comm_b, lc.st_x));
            } else if (rccl) {
                KH_NCCL(ncclBroadcast(lc.slot[b], lc.slot[b], nunits, R.nccl_type(), s, G->comm_b, lc.st_x));
            } else {
                KH_HIP(hipMemcpyAsync(lc.slot[b], R.d[s], nunits * esz, hipMemcpyDeviceToDevice, lc.st_x));
            }
            KH_HIP(hipEventRecord(lc.ev_ready[b], lc.st_x));
        }
    };
    transfer(0);
    for (int s = 0; s < W; s++) {
        if (s + 1 < W) transfer(s + 1);
        std::vector<const void *> buf(NL);
        for (int l = 0; l < NL; l++) {
            auto &lc = G->loc[l];
            KH_HIP(hipSetDevice(G->shards[l]->device));
            KH_HIP(hipStreamWaitEvent(G->shards[l]->stream, lc.ev_ready[s & 1], 0));
            buf[l] = own(s, l) ? R.d[0] : (const void *)lc.slot[s & 1];
        }
        for (uint64_t r0 = 0; r0 < nreads; r0 += rpb) {
            const uint64_t nr = std::min(rpb, nreads - r0);
            std::vector<PassState> ps(NL);
            std::vector<Src> srcs(NL);
            GROUP_TRY(for (int l = 0; l < NL; l++) {
                Graph *g = G->shards[l];
                KH_HIP(hipSetDevice(g->device));
                srcs[l] = group_src<Src>(g, R, buf[l], r0, nr);
                ps[l] = pass_stage_a(g, srcs[l], nr * kpr);
            });
            if (r0 == 0 && s + 1 < W) {
                // No comm_b broadcast is ever in flight together with an
                // operation on G->comm: broadcast s+1 starts after source
                // s-1's last pass (ev_free) and must finish before source s's
                // first collective.  Same order on every rank, so the two
                // communicators' kernels never wait on each other.  It still
                // overlaps the first pass's hashing and level-1 work.
                for (int l = 0; l < NL; l++) {
                    KH_HIP(hipSetDevice(G->shards[l]->device));
                    KH_HIP(hipStreamWaitEvent(G->shards[l]->stream, G->loc[l].ev_ready[(s + 1) & 1], 0));
                }
            }
            group_route_winners(G, ps);
            if (ps[0].bigc) group_merge_full(G, ps);
            GROUP_TRY(for (int l = 0; l < NL; l++) {
                KH_HIP(hipSetDevice(G->shards[l]->device));
                pass_stage_c(G->shards[l], srcs[l], ps[l], nullptr);
            });
        }
        for (int l = 0; l < NL; l++) {
            auto &lc = G->loc[l];
            KH_HIP(hipSetDevice(G->shards[l]->device));
            KH_HIP(hipEventRecord(lc.ev_free[s & 1], G->shards[l]->stream));
            lc.freed[s & 1] = true;
        }
    }
    for (int l = 0; l < NL; l++) {
        KH_HIP(hipSetDevice(G->shards[l]->device));
        KH_HIP(hipStreamSynchronize(G->loc[l].st_x));
        KH_HIP(hipStreamSynchronize(G->shards[l]->stream));   // the slots are free for the next call
    }
}

// every rank must pass the same shape (the collective schedule depends on it)
static void group_check_shape(ShardGroup *G, uint64_t nreads, uint64_t read_len) {
    if (!per_rank(G)) return;
    Graph *g0 = G->shards[0];
    uint64_t h[2] = {nreads, read_len};
    KH_HIP(hipSetDevice(g0->device));
    KH_HIP(hipMemcpyAsync(G->d_red + 140, h, 16, hipMemcpyHostToDevice, g0->stream));
    coll_allreduce_u64(G, g0->stream, G->d_red + 140, G->d_red + 142, 2, RED_MAX);
    coll_allreduce_u64(G, g0->stream, G->d_red + 140, G->d_red + 144, 2, RED_MIN);
    uint64_t mm[4];
    KH_HIP(hipMemcpyAsync(mm, G->d_red + 142, 32, hipMemcpyDeviceToHost, g0->stream));
    KH_HIP(hipStreamSynchronize(g0->stream));
    if (mm[0] != mm[2] || mm[1] != mm[3]) fail(KH_EVALUE, "ranks passed different read counts or lengths");
}

static GroupReads group_reads(ShardGroup *G, bool bytes, const void *const *d, uint64_t nreads, uint64_t read_len) {
    Graph *g0 = G->shards[0];
    if (bytes && g0->hash != MURMUR) fail(KH_EVALUE, "ASCII reads are for Murmur-hashed (Counttable) groups");
    if (!bytes && g0->hash != TWOBIT) fail(KH_EVALUE, "packed 2-bit reads are for 2-bit hashed groups");
    if (read_len < (uint64_t)g0->k) fail(KH_EVALUE, "reads shorter than k");
    group_check_shape(G, nreads, read_len);
    GroupReads R;
    R.bytes = bytes;
    R.d = d;
    R.nreads = nreads;
    R.read_len = read_len;
    R.kpr = read_len - g0->k + 1;
    return R;
}

// collective: every rank passes its own fixed-length packed reads (same
// count and length on every rank); consumed as the stream rank 0, 1, ...
// (exchange mode: pass-interleaved, see group_consume_a2a)
void group_consume_fixed(ShardGroup *G, const uint64_t *const *d_words, uint64_t nreads, uint64_t read_len) {
    const GroupReads R = group_reads(G, false, (const void *const *)d_words, nreads, read_len);
    if (!nreads) return;
    if (G->delta) group_consume_delta<SrcTwoBit>(G, R);
    else if (G->a2a) group_consume_a2a<SrcTwoBit>(G, R);
    else group_consume_bcast<SrcTwoBit>(G, R);
}

// the same for ASCII reads of a Murmur-hashed (Counttable family) group
void group_consume_bytes_fixed(ShardGroup *G, const uint8_t *const *d_bytes, uint64_t nreads, uint64_t read_len) {
    const GroupReads R = group_reads(G, true, (const void *const *)d_bytes, nreads, read_len);
    if (!nreads) return;
    if (G->delta) group_consume_delta<SrcBytes>(G, R);
    else if (G->a2a) group_consume_a2a<SrcBytes>(G, R);
    else group_consume_bcast<SrcBytes>(G, R);
}

// ---------------------------------------------------------------------------
// Sharded get_median_count (Hashtable::get_median_count,
// src/oxli/hashtable.cc:299-328) of every rank's own fixed-length reads.  A
// k-mer's N bins live on different ranks, so its count -- the minimum over
// the tables, then the bigcount value when a Byte minimum is 255
// (storage.hh:627-649) -- is assembled from the owners:
//   exchange mode: the k-mers are partitioned into the unsharded level-1
//     buckets exactly as in a consume pass (a2a_level1) and every bucket
//     range goes to its owner (a2a_exchange); the owner reads each routed
//     record's table value and keeps the per-k-mer minimum in a u8 array over
//     the pass's k-mer index space (k_lookup_min); a MIN reduce-scatter over
//     ranks leaves every rank the minima of its own k-mers.
//   broadcast mode: every source's reads are broadcast, every rank takes the
//     minimum over the tables whose bin it owns (k_own_min), and a MIN reduce
//     to the source rank completes them.
// The read's home rank then computes median / average / stddev from the
// minima (k_median_fixed with cnt8; bigcount map replicated on every rank).
struct QueryOut {
    uint16_t *const *med;
    float *const *avg;
    float *const *sd;
};

template <class Src>
static void group_median_reads(Graph *g, const GroupReads &R, const void *buf, uint64_t r0, uint64_t nr,
                               const uint8_t *cnt8, uint16_t *med, float *avg, float *sd) {
    const Src src = group_src<Src>(g, R, buf, r0, nr);
    const unsigned grid = (unsigned)std::min<uint64_t>((nr + 3) / 4, 8192);
    TIMED("median", hipLaunchKernelGGL(k_median_fixed<Src>, dim3(grid), dim3(256), 0, g->stream, g->prm, src, nr,
                                       (uint32_t)R.kpr, g->d_tab, g->d_bc_keys, g->d_bc_vals, g->d_bc_n, med + r0,
                                       avg + r0, sd + r0, cnt8));
    KH_HIP(hipGetLastError());
}

template <class Src>
static void group_median_a2a(ShardGroup *G, const GroupReads &R, const QueryOut &Q) {
    const int W = G->world, NL = G->nlocal;
    Graph *g0 = G->shards[0];
    uint64_t rpb, stride;
    a2a_pass_plan(G, g0, R, &rpb, &stride);
    const uint64_t nk = (uint64_t)W * stride;
    constexpr uint32_t PARTS = 4;   // workgroups per (source, bucket) segment
    for (uint64_t r0 = 0; r0 < R.nreads; r0 += rpb) {
        const uint64_t nr = std::min(rpb, R.nreads - r0), nkc = nr * R.kpr;
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            Graph *V = G->views[l];
            KH_HIP(hipSetDevice(V->device));
            V->use_bigcount = false;
            a2a_level1(V, group_src<Src>(V, R, R.d[l], r0, nr), nkc, (uint32_t)((uint64_t)(G->rank0 + l) * stride));
        });
        std::vector<uint64_t> meta;
        a2a_meta(G, meta);
        const uint64_t F1v = G->views[0]->prm.F1, M = 2 * (F1v + 1);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            const int r = G->rank0 + l;
            Graph *g = G->shards[l];
            auto &lc = G->loc[l];
            KH_HIP(hipSetDevice(g->device));
            uint64_t need = 0;
            for (int s = 0; s < W; s++) need += meta[(size_t)s * M + G->B[r + 1]] - meta[(size_t)s * M + G->B[r]];
            ensure_recs(g, need);
            ensure((void **)&lc.q8, &lc.cap_q8, nk + 64, 1);
            ensure((void **)&lc.o8, &lc.cap_o8, std::max<uint64_t>(stride, nk) + 64, 1);
        });
        std::vector<std::vector<uint64_t>> rb;
        a2a_exchange(G, meta, rb);
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            const int r = G->rank0 + l;
            Graph *g = G->shards[l];
            auto &lc = G->loc[l];
            KH_HIP(hipSetDevice(g->device));
            const uint64_t nseg = a2a_segments(G, l, meta, rb[l]);
            dev_fill(lc.q8, 0xFF, (nk + 3) & ~3ull, g->stream);
            if (nseg)
                TIMED("lookup", hipLaunchKernelGGL(k_lookup_min, dim3((unsigned)(nseg * PARTS)), dim3(256), 0,
                                                   g->stream, g->prm, g->d_tab, g->ws.rec1, lc.seg,
                                                   lc.seg + nseg + 1, G->B[r + 1] - G->B[r], PARTS,
                                                   (uint32_t *)lc.q8));
            KH_HIP(hipGetLastError());
        });
        // MIN reduce-scatter: rank r's minima = min over ranks of chunk r
        if (G->comm) {
            Graph *g = G->shards[0];
            auto &lc = G->loc[0];
            KH_NCCL(ncclReduceScatter(lc.q8, lc.o8, stride, ncclUint8, ncclMin, G->comm, g->stream));
        } else if (G->hosted) {
            Graph *g = G->shards[0];
            auto &lc = G->loc[0];
            std::vector<uint8_t> hs(nk), hr(nk);
            std::vector<uint64_t> sb(W, stride), rbb(W, stride);
            KH_HIP(hipMemcpyAsync(hs.data(), lc.q8, nk, hipMemcpyDeviceToHost, g->stream));
            KH_HIP(hipStreamSynchronize(g->stream));
            host_rc(G->tp.alltoallv(G->tp.ctx, hs.data(), sb.data(), hr.data(), rbb.data()), "alltoallv");
            KH_HIP(hipMemcpyAsync(lc.q8, hr.data(), nk, hipMemcpyHostToDevice, g->stream));
            KH_HIP(hipMemsetAsync(lc.o8, 0xFF, stride, g->stream));
            hipLaunchKernelGGL(k_min_bytes, dim3((unsigned)std::min<uint64_t>((stride + 255) / 256, 8192)), dim3(256),
                               0, g->stream, lc.o8, lc.q8, stride, W, stride);
        } else {
            for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
            for (int l = 0; l < NL; l++) {
                Graph *g = G->shards[l];
                auto &lc = G->loc[l];
                KH_HIP(hipMemsetAsync(lc.o8, 0xFF, stride, g->stream));
                for (int s = 0; s < W; s++)
                    hipLaunchKernelGGL(k_min_bytes, dim3((unsigned)std::min<uint64_t>((stride + 255) / 256, 8192)),
                                       dim3(256), 0, g->stream, lc.o8, G->loc[s].q8 + (uint64_t)l * stride, 0, 1,
                                       stride);
            }
            for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
        }
        KH_HIP(hipGetLastError());
        GROUP_TRY(for (int l = 0; l < NL; l++) {
            Graph *g = G->shards[l];
            KH_HIP(hipSetDevice(g->device));
            group_median_reads<Src>(g, R, R.d[l], r0, nr, G->loc[l].o8, Q.med[l], Q.avg[l], Q.sd[l]);
            (void)nkc;
        });
    }
}

template <class Src>
static void group_median_bcast(ShardGroup *G, const GroupReads &R, const QueryOut &Q) {
    const int W = G->world, NL = G->nlocal;
    Graph *g0 = G->shards[0];
    const uint64_t nunits = R.units();
    const size_t esz = R.esize();
    const uint64_t slot_words = (nunits * esz + 64 + 7) / 8;
    const uint64_t rpb0 = std::max<uint64_t>(1, std::min<uint64_t>(g0->batch_kmers, MAX_PASS_KMERS) / R.kpr);
    const uint64_t npass = std::max<uint64_t>(1, (R.nreads + rpb0 - 1) / rpb0);
    const uint64_t rpb = std::max<uint64_t>(1, (R.nreads + npass - 1) / npass);
    auto own = [&](int s, int l) { return per_rank(G) && G->rank0 + l == s; };
    for (int s = 0; s < W; s++) {
        // source s's reads on every local shard (loopback: read in place)
        std::vector<const void *> buf(NL);
        for (int l = 0; l < NL; l++) {
            Graph *g = G->shards[l];
            auto &lc = G->loc[l];
            KH_HIP(hipSetDevice(g->device));
            if (!per_rank(G)) {
                buf[l] = R.d[s];
                continue;
            }
            if (!own(s, l)) {
                ensure((void **)&lc.slot[0], &lc.cap_slot[0], slot_words, 8);
                KH_HIP(hipMemsetAsync((uint8_t *)lc.slot[0] + nunits * esz, 0, 64, g->stream));
            }
            void *dst = own(s, l) ? const_cast<void *>(R.d[0]) : (void *)lc.slot[0];
            if (G->comm) {
                KH_NCCL(ncclBroadcast(dst, dst, nunits, R.nccl_type(), s, G->comm_b, g->stream));
            } else {
                std::vector<uint8_t> hb(nunits * esz);
                KH_HIP(hipStreamSynchronize(g->stream));
                if (own(s, l)) KH_HIP(hipMemcpy(hb.data(), R.d[0], hb.size(), hipMemcpyDeviceToHost));
                host_rc(G->tp.broadcast(G->tp.ctx, hb.data(), hb.size(), s), "broadcast");
                if (!own(s, l)) KH_HIP(hipMemcpy(dst, hb.data(), hb.size(), hipMemcpyHostToDevice));
            }
            buf[l] = dst;
        }
        for (uint64_t r0 = 0; r0 < R.nreads; r0 += rpb) {
            const uint64_t nr = std::min(rpb, R.nreads - r0), nk = nr * R.kpr;
            GROUP_TRY(for (int l = 0; l < NL; l++) {
                Graph *g = G->shards[l];
                auto &lc = G->loc[l];
                KH_HIP(hipSetDevice(g->device));
                ensure((void **)&lc.q8, &lc.cap_q8, nk + 64, 1);
                const Src src = group_src<Src>(g, R, buf[l], r0, nr);
                const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nk + 255) / 256, 16384));
                TIMED("own_min", hipLaunchKernelGGL(k_own_min<Src>, dim3(grid), dim3(256), 0, g->stream, g->prm, src,
                                                    nk, g->d_tab, lc.q8));
                KH_HIP(hipGetLastError());
            });
            // MIN reduce to the source rank
            int root_l = -1;
            if (G->comm) {
                Graph *g = G->shards[0];
                auto &lc = G->loc[0];
                KH_NCCL(ncclReduce(lc.q8, lc.q8, nk, ncclUint8, ncclMin, s, G->comm, g->stream));
                if (own(s, 0)) root_l = 0;
            } else if (G->hosted) {
                // MIN reduce to the source only (an alltoallv whose only
                // destination is s), in slices of at most 256 MB: the source
                // holds W slices at a time, every other rank one (ADVICE r4:
                // an all-gather of whole passes held W x 3.3 GB per rank)
                Graph *g = G->shards[0];
                auto &lc = G->loc[0];
                const bool root = own(s, 0);
                const uint64_t piece = std::min<uint64_t>(nk, 256ull << 20);
                std::vector<uint8_t> mine(piece), all(root ? (size_t)W * piece : 1);
                std::vector<uint64_t> sb(W, 0), rb(W, 0);
                for (uint64_t a = 0; a < nk; a += piece) {
                    const uint64_t n = std::min(piece, nk - a);
                    KH_HIP(hipMemcpyAsync(mine.data(), lc.q8 + a, n, hipMemcpyDeviceToHost, g->stream));
                    KH_HIP(hipStreamSynchronize(g->stream));
                    sb[s] = n;
                    for (int t = 0; t < W; t++) rb[t] = root ? n : 0;
                    host_rc(G->tp.alltoallv(G->tp.ctx, mine.data(), sb.data(), all.data(), rb.data()), "alltoallv");
                    if (!root) continue;
                    for (uint64_t q = 0; q < n; q++) {
                        uint8_t c = 0xFF;
                        for (int t = 0; t < W; t++) c = std::min(c, all[(size_t)t * n + q]);
                        mine[q] = c;
                    }
                    KH_HIP(hipMemcpyAsync(lc.q8 + a, mine.data(), n, hipMemcpyHostToDevice, g->stream));
                    KH_HIP(hipStreamSynchronize(g->stream));
                }
                if (root) root_l = 0;
            } else {
                for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
                Graph *g = G->shards[s];
                for (int t = 0; t < W; t++)
                    if (t != s)
                        hipLaunchKernelGGL(k_min_bytes, dim3((unsigned)std::min<uint64_t>((nk + 255) / 256, 8192)),
                                           dim3(256), 0, g->stream, G->loc[s].q8, G->loc[t].q8, 0, 1, nk);
                root_l = s;
            }
            KH_HIP(hipGetLastError());
            if (root_l >= 0) {
                Graph *g = G->shards[root_l];
                KH_HIP(hipSetDevice(g->device));
                group_median_reads<Src>(g, R, buf[root_l], r0, nr, G->loc[root_l].q8, Q.med[root_l], Q.avg[root_l],
                                        Q.sd[root_l]);
            }
            // the next pass reuses every shard's q8
            for (int l = 0; l < NL; l++) KH_HIP(hipStreamSynchronize(G->shards[l]->stream));
        }
    }
}

// collective: d_reads[l] = local shard l's own fixed-length reads (packed
// 2-bit words, or ASCII bytes for Murmur groups); its outputs go to
// d_med[l] / d_avg[l] / d_sd[l] (device, one entry per read)
void group_median_fixed(ShardGroup *G, const void *const *d_reads, uint64_t nreads, uint64_t read_len,
                        uint16_t *const *d_med, float *const *d_avg, float *const *d_sd) {
    Graph *g0 = G->shards[0];
    const bool bytes = g0->hash == MURMUR;
    const GroupReads R = group_reads(G, bytes, d_reads, nreads, read_len);
    if (R.kpr > 256) fail(KH_EVALUE, "device median path takes at most 256 k-mers per read");
    if (!nreads) return;
    for (Graph *g : G->shards) {
        KH_HIP(hipSetDevice(g->device));
        engine_sync_bigcounts(g);
    }
    const QueryOut Q{d_med, d_avg, d_sd};
    if (G->a2a) {
        if (bytes) group_median_a2a<SrcBytes>(G, R, Q);
        else group_median_a2a<SrcTwoBit>(G, R, Q);
    } else {
        if (bytes) group_median_bcast<SrcBytes>(G, R, Q);
        else group_median_bcast<SrcTwoBit>(G, R, Q);
    }
    for (Graph *g : G->shards) {
        KH_HIP(hipSetDevice(g->device));
        KH_HIP(hipStreamSynchronize(g->stream));
        engine_collect_events(g);
    }
    for (Graph *V : G->views) KH_HIP(hipStreamSynchronize(V->stream));
}

void group_wire_stats(const ShardGroup *G, uint64_t *dense_bytes, uint64_t *sent_bytes) {
    if (dense_bytes) *dense_bytes = G->wire_dense;
    if (sent_bytes) *sent_bytes = G->wire_sent;
}

// n_unique / n_occupied of the whole group (collective in RCCL mode)
void group_counters(ShardGroup *G, uint64_t *n_unique, uint64_t *n_occupied) {
    uint64_t h[2] = {0, 0};
    for (Graph *g : G->shards) {
        h[0] += g->n_unique;
        h[1] += g->n_occupied;
    }
    if (per_rank(G)) {
        Graph *g = G->shards[0];
        KH_HIP(hipSetDevice(g->device));
        KH_HIP(hipMemcpyAsync(G->d_red + 150, h, 16, hipMemcpyHostToDevice, g->stream));
        coll_allreduce_u64(G, g->stream, G->d_red + 150, G->d_red + 152, 2, RED_SUM);
        KH_HIP(hipMemcpyAsync(h, G->d_red + 152, 16, hipMemcpyDeviceToHost, g->stream));
        KH_HIP(hipStreamSynchronize(g->stream));
    }
    *n_unique = h[0];
    *n_occupied = h[1];
}

void group_rank_slice(ShardGroup *G, int rank, int table, uint64_t *lo, uint64_t *size) {
    const Graph *g = G->shards[0];
    if (rank < 0 || rank >= G->world) fail(KH_EVALUE, "invalid rank");
    if (table < 0 || table >= g->n) fail(KH_EVALUE, "no such table");
    if (G->a2a) {
        *lo = G->blo[(size_t)rank * g->n + table];
        *size = G->bhi[(size_t)rank * g->n + table] - *lo;
    } else {
        *lo = shard_lo(g->sizes[(size_t)table], G->world, rank);
        *size = shard_lo(g->sizes[(size_t)table], G->world, rank + 1) - *lo;
    }
}
int group_exchange(ShardGroup *G) { return G->delta ? 2 : G->a2a ? 1 : 0; }
int group_world(ShardGroup *G) { return G->world; }
int group_nlocal(ShardGroup *G) { return G->nlocal; }
int group_rank(ShardGroup *G, int l) { return G->rank0 + l; }
Graph *group_shard(ShardGroup *G, int l) {
    if (l < 0 || l >= G->nlocal) fail(KH_EVALUE, "no such local shard");
    return G->shards[l];
}

}  // namespace kh
