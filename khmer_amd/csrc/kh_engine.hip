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
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kh_apply.cuh"
#include "kh_internal.h"
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

static void ws_prepare(Graph *g, uint64_t nkmers) {
    Workspace &w = g->ws;
    const uint64_t recs = nkmers * (uint64_t)g->n;
    if (nkmers > w.cap_kmers) {
        uint64_t cap = std::max<uint64_t>(nkmers, w.cap_kmers + w.cap_kmers / 2);
        cap = (cap + 15) & ~15ull;
        if (w.newf) KH_HIP(hipFree(w.newf));
        if (w.fullf) KH_HIP(hipFree(w.fullf));
        w.newf = w.fullf = nullptr;
        KH_HIP(hipMalloc((void **)&w.newf, cap + 64));
        KH_HIP(hipMalloc((void **)&w.fullf, cap + 64));
        w.cap_kmers = cap;
    }
    if (recs > w.cap_recs) {
        uint64_t cap = std::max<uint64_t>(recs, w.cap_recs + w.cap_recs / 2);
        for (uint64_t **pp : {&w.rec1, &w.rec2}) {
            if (*pp) KH_HIP(hipFree(*pp));
            *pp = nullptr;
            KH_HIP(hipMalloc((void **)pp, cap * 8 + 64));
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

// LDS footprints
static size_t lds_window(bool window, int tile_kmers) { return 16 + (window ? (size_t)(tile_kmers + 2) * 8 : 0); }
static size_t lds_count_l1(const Params &P, bool window, int tile_kmers) {
    return (size_t)((P.F1 + 3) & ~3u) * 4 + lds_window(window, tile_kmers);
}
static size_t lds_scatter_l1(const Params &P, bool window, int tile_kmers) {
    const size_t F1a = (P.F1 + 3) & ~3u;
    return F1a * 8 + (size_t)L1_TILE_RECS * 8 + F1a * 4 * 2 + (size_t)L1_TILE_RECS * 2 + lds_window(window, tile_kmers);
}
static size_t lds_scatter_l2(const Params &P) {
    const size_t F2 = (size_t)1 << P.s2;
    return F2 * 8 + (size_t)L2_TILE_RECS * 8 + F2 * 4 * 2 + (size_t)L2_TILE_RECS * 2;
}
static size_t lds_apply(const Params &P) {
    const size_t R = (size_t)1 << P.s0;
    return P.kind == BIT ? R * 4 + 16 + R / 8 : R * 4 * 2 + (R / 512) * 4 + R;
}

// ---------------------------------------------------------------------------
// one device pass over a batch of <= 2^32 - 16 k-mers
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
    const bool bigc = P.kind == BYTE && P.use_bigcount;
    const bool window = [&] {
        if constexpr (!Src::kReads) return false;
        else return src.kpr == 0;
    }();
    const uint64_t flag_bytes = (nkmers + 15) & ~15ull;

    KH_HIP(hipMemsetAsync(w.cnt1, 0, F1 * 4, st));
    KH_HIP(hipMemsetAsync(w.cnt2, 0, F1 * F2 * 4, st));
    KH_HIP(hipMemsetAsync(w.ctr, 0, CTR_N * 8, st));
    KH_HIP(hipMemsetAsync(w.newf, 0, flag_bytes, st));
    if (bigc) KH_HIP(hipMemsetAsync(w.fullf, 0, flag_bytes, st));

    const int ctile = 4096;
    const uint64_t nct = (nkmers + ctile - 1) / ctile;
    TIMED("count_l1", hipLaunchKernelGGL(k_count_l1<Src>, dim3((unsigned)nct), dim3(L1_THREADS),
                                         lds_count_l1(P, window, ctile), st, P, src, nkmers, ctile, w.cnt1));
    TIMED("scan_l1", hipLaunchKernelGGL(k_scan_l1, dim3(1), dim3(1024), F1 * 8 + 1025 * 8, st, (uint32_t)F1,
                                        w.cnt1, w.off1, w.cur1, w.tile1));
    for (int t0 = 0; t0 < P.n; t0 += L1_MAX_RPT) {
        const int nt = std::min(L1_MAX_RPT, P.n - t0);
        const int kpt = std::max(1, L1_MAX_RPT / nt);
        const int tile_kmers = L1_THREADS * kpt;
        const uint64_t ntiles = (nkmers + tile_kmers - 1) / tile_kmers;
        TIMED("scatter_l1", hipLaunchKernelGGL(k_scatter_l1<Src>, dim3((unsigned)ntiles), dim3(L1_THREADS),
                                               lds_scatter_l1(P, window, tile_kmers), st, P, src, nkmers, kpt, t0,
                                               nt, w.cur1, w.rec1));
    }
    const uint64_t ntiles2 = (recs + L2_TILE_RECS - 1) / L2_TILE_RECS + F1;
    TIMED("count_l2", hipLaunchKernelGGL(k_count_l2, dim3((unsigned)ntiles2), dim3(L2_THREADS), F2 * 4, st,
                                         (uint32_t)F1, P.s0, P.s2, w.off1, w.tile1, w.rec1, w.cnt2));
    TIMED("scan_l2", hipLaunchKernelGGL(k_scan_l2, dim3((unsigned)F1), dim3(1024), F2 * 8 + 1025 * 8, st, P.s2,
                                        (uint32_t)F1, w.off1, w.cnt2, w.off2, w.cur2));
    TIMED("scatter_l2", hipLaunchKernelGGL(k_scatter_l2, dim3((unsigned)ntiles2), dim3(L2_THREADS),
                                           lds_scatter_l2(P), st, (uint32_t)F1, P.s0, P.s2, w.off1, w.tile1, w.cur2,
                                           w.rec1, w.rec2));

    ApplyArgs A;
    A.off2 = w.off2;
    A.rec = w.rec2;
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
    const unsigned agrid = (unsigned)std::min<uint64_t>(real_regions, 256 * 2 * 4);
    if (P.kind == BIT)
        TIMED("apply_bit", hipLaunchKernelGGL(k_apply_bit, dim3(agrid), dim3(APPLY_THREADS), lds_apply(P), st, P, A));
    else if (P.kind == NIBBLE)
        TIMED("apply_nibble", hipLaunchKernelGGL(k_apply_count<NIBBLE>, dim3(agrid), dim3(APPLY_THREADS),
                                                 lds_apply(P), st, P, A));
    else
        TIMED("apply_byte", hipLaunchKernelGGL(k_apply_count<BYTE>, dim3(agrid), dim3(APPLY_THREADS), lds_apply(P),
                                               st, P, A));
    if (bigc)
        TIMED("crossing", hipLaunchKernelGGL(k_crossing, dim3(1024), dim3(256), 0, st, P, w.off2, w.rec2, w.cross,
                                             w.ctr, w.cap_cross, w.fullf));

    uint64_t *d_out_hash = nullptr;
    if (out && out->h_hash) d_out_hash = w.rec1;  // level-1 records are dead after scatter_l2
    const uint64_t nchunk = flag_bytes / 16;
    const unsigned fgrid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((nchunk + FIN_THREADS - 1) / FIN_THREADS,
                                                                              4096));
    TIMED("finalize", hipLaunchKernelGGL(k_finalize<Src>, dim3(fgrid), dim3(FIN_THREADS), 0, st, P, src, nkmers,
                                         w.newf, w.fullf, w.ctr, w.bc, w.cap_bc, d_out_hash));
    KH_HIP(hipGetLastError());
    KH_HIP(hipMemcpyAsync(w.h_ctr, w.ctr, CTR_N * 8, hipMemcpyDeviceToHost, st));
    if (out && out->h_new) KH_HIP(hipMemcpyAsync(out->h_new, w.newf, nkmers, hipMemcpyDeviceToHost, st));
    if (d_out_hash) KH_HIP(hipMemcpyAsync(out->h_hash, d_out_hash, nkmers * 8, hipMemcpyDeviceToHost, st));
    KH_HIP(hipStreamSynchronize(st));
    engine_collect_events(g);
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
            const uint64_t base = it == g->bigcounts.end() ? 255 : it->second;
            g->bigcounts[hs[a]] = (uint16_t)std::min<uint64_t>(base + (b - a), 65535);
            a = b;
        }
        g->bc_dirty = true;
    }
}

// ---------------------------------------------------------------------------
// batching of read sets
static void set_fixed(SrcCommon &s, uint64_t kpr) {
    s.kpr = kpr;
    s.kpr_m = kpr ? barrett_m(kpr) : 0;
}

template <class Src>
static void consume_reads(Graph *g, Src base, const uint64_t *d_koff, uint64_t nreads, uint64_t nkmers,
                          uint64_t kpr, const PassOut *out) {
    if (nkmers == 0 || nreads == 0) return;
    const uint64_t B = g->batch_kmers;
    set_fixed(base, kpr);
    base.koff = d_koff;
    base.nreads = nreads;
    base.kbase = 0;
    base.rbase = 0;
    if (out || nkmers <= B + (B >> 4)) {   // one pass (koff[0] == 0 by contract)
        run_pass(g, base, nkmers, out);
        return;
    }
    if (kpr) {   // fixed-length reads: batches of whole reads, no offsets needed
        const uint64_t rpb = std::max<uint64_t>(1, B / kpr);
        for (uint64_t r0 = 0; r0 < nreads; r0 += rpb) {
            Src s = base;
            s.kbase = r0 * kpr;
            run_pass(g, s, std::min(rpb, nreads - r0) * kpr, out);
        }
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
static SrcBytes src_bytes(Graph *g, const uint8_t *d_bytes) {
    SrcBytes s{};
    s.bytes = d_bytes;
    s.k = g->k;
    return s;
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
    consume_reads(g, src_bytes(g, d_bytes), d_koff, nreads, nkmers, 0, out);
}

void engine_consume_hashes(Graph *g, const uint64_t *d_hashes, uint64_t n, const PassOut *out) {
    const uint64_t B = g->batch_kmers;
    if (n > B && out) fail(KH_EVALUE, "per-k-mer outputs need a single device batch");
    for (uint64_t a = 0; a < n; a += B) {
        SrcHashes s{};
        s.h = d_hashes + a;
        s.k = g->k;
        run_pass(g, s, std::min(B, n - a), out);
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
        ensure((void **)&w.d_bytes, &w.cap_bytes, b.bytes.size() + 8, 1);
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
        consume_reads(g, src_bytes(g, g->ws.d_bytes), g->ws.d_koff, b.nreads(), b.nkmers(), kpr, out);
    else
        consume_reads(g, src_twobit(g, g->ws.d_words), g->ws.d_koff, b.nreads(), b.nkmers(), kpr, out);
}

void engine_hash_batch(Graph *g, const HostBatch &b, uint64_t *h_out) {
    const uint64_t nk = b.nkmers(), nr = b.nreads();
    if (!nk) return;
    upload_batch(g, b);
    uint64_t *d = nullptr;
    KH_HIP(hipMalloc((void **)&d, nk * 8));
    const uint64_t tiles = (nk + Q_TILE - 1) / Q_TILE;
    const size_t lds = 16 + (Q_TILE + 2) * 8;
    if (b.hash == MURMUR) {
        SrcBytes s = src_bytes(g, g->ws.d_bytes);
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
    KH_HIP(hipFree(d));
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
    const uint64_t tiles = (nk + Q_TILE - 1) / Q_TILE;
    const size_t lds = 16 + (Q_TILE + 2) * 8;
    if (tiles) {
        if (b.hash == MURMUR) {
            SrcBytes s = src_bytes(g, g->ws.d_bytes);
            s.koff = g->ws.d_koff;
            s.nreads = nr;
            hipLaunchKernelGGL(k_kmer_counts<SrcBytes>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream, g->prm,
                               s, nk, g->d_tab, d_counts, g->d_bc_keys, g->d_bc_vals, g->d_bc_n);
        } else {
            SrcTwoBit s = src_twobit(g, g->ws.d_words);
            s.koff = g->ws.d_koff;
            s.nreads = nr;
            hipLaunchKernelGGL(k_kmer_counts<SrcTwoBit>, dim3((unsigned)tiles), dim3(Q_THREADS), lds, g->stream,
                               g->prm, s, nk, g->d_tab, d_counts, g->d_bc_keys, g->d_bc_vals, g->d_bc_n);
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
    // KH_ABLATE: timing-only switches that skip work (wrong results); bench
    // ablation studies only
    const char *ab = getenv("KH_ABLATE");
    P.ablate = ab ? atoi(ab) : 0;
    P.s0 = g->kind == BIT ? 14 : 13;
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
    if (F1 > 4096) fail(KH_EVALUE, "tables too large for one device (more than 4096 level-1 buckets)");
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
    void *ptrs[] = {d_tab, d_bc_keys, d_bc_vals, w.rec1, w.rec2, w.newf, w.fullf, w.bc, w.cnt1, w.off1,
                    w.cur1, w.tile1, w.cnt2, w.off2, w.cur2, w.cross, w.ctr, w.d_words, w.d_koff, w.d_bytes,
                    w.q_hashes, w.q_counts};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (w.h_ctr) (void)hipHostFree(w.h_ctr);
    for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
}

}  // namespace kh
