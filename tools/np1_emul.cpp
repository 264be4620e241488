// Development: a CPU emulation of k_scatter_n1 (khmer_amd/csrc/kh_nearprime.cuh)
// with every LDS and global index bounds-checked.  Workgroups run round-robin
// one barrier phase at a time (so the chunk-queue atomics interleave as on the
// device); inside a phase the 512 threads run one after another.
//   g++ -O2 -std=c++17 -I khmer_amd/csrc tools/np1_emul.cpp -o /tmp/np1_emul
//   /tmp/np1_emul <k> <table size x> <reads> [jlim]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "kh_device.h"

using namespace kh;
static const int THREADS = 512, KPT = 8, TILE = THREADS * KPT, NP_TW = 192, S0 = 14;
static const int SLOT_B = 55, SLOT_K = 42;
static const uint32_t EMPTY = 0x1FFF, DEAD = 0xFFFFFFFFu;
static const uint64_t PAY = (1ull << SLOT_K) - 1;

template <class T>
struct Arr {   // bounds-checked array
    std::vector<T> v;
    const char *name;
    Arr(size_t n, const char *nm, T init = T()) : v(n, init), name(nm) {}
    T &operator[](uint64_t i) {
        if (i >= v.size()) {
            fprintf(stderr, "OOB %s[%llu] (size %zu)\n", name, (unsigned long long)i, v.size());
            throw std::runtime_error("oob");
        }
        return v[i];
    }
};

static bool is_prime(uint64_t n) {
    if (n < 2) return false;
    for (uint64_t d = 2; d * d <= n; d++)
        if (n % d == 0) return false;
    return true;
}
static int ceil_log2(uint64_t x) { int s = 0; while ((1ull << s) < x) s++; return s; }

struct Geo {
    uint64_t pm; double ipm; uint32_t rp, magic, nb, rloc; int ob, pb; uint32_t jlim; int n; uint64_t cap;
};

int main(int argc, char **argv) {
    const int k = atoi(argv[1]);
    const double x = atof(argv[2]);
    const uint64_t nreads = strtoull(argv[3], 0, 10);
    const int L = 150, n = 4;
    std::vector<uint64_t> p;
    for (uint64_t v = (uint64_t)x; p.size() < (size_t)n; v--)
        if (is_prime(v)) p.push_back(v);
    Geo N{};
    N.n = n;
    N.pm = p[0];
    uint64_t dmax = p[0] - p[n - 1];
    const uint64_t qmax = ((1ull << (2 * k)) - 1) / N.pm;
    const uint64_t maxoff = qmax * dmax;
    N.rloc = 1024 / n;
    const uint64_t E = (maxoff + (1 << S0) - 1) >> S0;
    N.rp = N.rloc - (uint32_t)E - 1;
    const uint64_t Rm = (N.pm + (1 << S0) - 1) >> S0;
    N.nb = (uint32_t)((Rm + N.rp - 1) / N.rp);
    N.ob = ceil_log2((uint64_t)N.rp * (1 << S0) + 1);
    N.pb = N.ob + ceil_log2(qmax + 1);
    N.jlim = 64 - N.pb >= 32 ? 0xFFFFFFFFu : (uint32_t)((1ull << (64 - N.pb)) - 1);
    if (argc > 4) N.jlim = (uint32_t)atoll(argv[4]);
    N.magic = (uint32_t)(((1ull << 32) + N.rp - 1) / N.rp);
    N.ipm = 1.0 / (double)N.pm;
    const uint64_t kpr = L - k + 1, nkmers = nreads * kpr;
    const uint64_t tiles = (nkmers + TILE - 1) / TILE;
    const uint32_t nwg = (uint32_t)std::min<uint64_t>(tiles / 4 + 1, 768);
    const int blk_sh = 8;
    const uint32_t BLK = 1u << blk_sh;
    const double mean = (double)nkmers * (double)((uint64_t)N.rp << S0) / (double)N.pm;
    uint64_t cap = (uint64_t)(mean + 8 * sqrt(mean)) + (uint64_t)(nwg + 1) * BLK;
    cap = (cap + BLK - 1) / BLK * BLK;
    N.cap = cap;
    const uint32_t cht = 8;
    printf("k %d pm %llu nb %u rp %u pb %d jlim %u nkmers %llu nwg %u cap %llu\n", k, (unsigned long long)N.pm, N.nb,
           N.rp, N.pb, N.jlim, (unsigned long long)nkmers, nwg, (unsigned long long)cap);
    // the packed reads: random words (any bits hash to some canonical k-mer)
    const uint64_t nwords = nreads * L / 32 + 2;
    std::vector<uint64_t> words(nwords);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    for (auto &w : words) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; w = st; }
    Arr<uint64_t> rec(cap * N.nb, "rec", ~0ull);
    Arr<uint32_t> blkj(cap / BLK * N.nb + 1, "blkj");
    Arr<unsigned long long> bkt_cur(N.nb + 1, "bkt_cur");
    for (uint32_t d = 0; d < N.nb; d++) bkt_cur[d] = d * cap;
    unsigned long long l1q = 0;
    uint64_t err = 0;
    const uint32_t F1 = N.nb, F1a = (F1 + 3) & ~3u, NSLOT = TILE + 2 * F1a;
    const uint64_t CK = (uint64_t)cht * TILE;
    const uint32_t nchunks = (uint32_t)((nkmers + CK - 1) / CK);
    auto read_of = [&](uint64_t ja) { return ja / kpr; };
    auto tile_w0 = [&](uint64_t j0) -> uint64_t { return ((j0 + read_of(j0) * (uint64_t)(k - 1)) * 2) >> 6; };
    auto tile_nw = [&](uint64_t j0, uint64_t j1) -> uint32_t { return (uint32_t)(tile_w0(j1 - 1) + 2 - tile_w0(j0)); };
    const uint32_t S = N.rp << S0;

    struct WG {
        uint32_t id;
        Arr<uint64_t> s_tw, tail, slot;
        Arr<uint32_t> dlx, dly, qqx, qqy, bcur, cnt, hist2, lstart, bjb, obase, s_misc;
        std::vector<uint64_t> rr;   // [THREADS][KPT]
        std::vector<uint64_t> rsv;
        std::vector<uint64_t> tw_next;
        unsigned long long qn = 0;
        uint32_t cb;
        uint64_t hj0, hj1, hce, n0, n1;
        bool htop = true;
        uint32_t ti = 0;
        int phase = 0;   // 0 prologue-a, 1 prologue-b, 2 P1, 3 P2, 4 P3, 5 epilogue, 6 done
        WG(uint32_t F1a, uint32_t NSLOT)
            : s_tw(2 * NP_TW, "s_tw"), tail(F1a, "tail"), slot(NSLOT, "slot"), dlx(F1a, "dlx"), dly(F1a, "dly"),
              qqx(F1a, "qqx"), qqy(F1a, "qqy"), bcur(F1a, "bcur"), cnt(F1a, "cnt"), hist2(2 * F1a, "hist2"),
              lstart(F1a, "lstart"), bjb(F1a, "bjb"), obase(F1a, "obase"), s_misc(4, "s_misc"),
              rr(THREADS * KPT), rsv(THREADS), tw_next(THREADS) {}
    };
    std::vector<WG *> wgs;
    for (uint32_t w = 0; w < nwg; w++) {
        WG *g = new WG(F1a, NSLOT);
        g->id = w;
        g->cb = w + nwg;
        g->hj0 = std::min<uint64_t>(nkmers, (uint64_t)w * CK);
        g->hce = std::min<uint64_t>(nkmers, g->hj0 + CK);
        wgs.push_back(g);
    }
    auto next_tile = [&](WG *g, uint64_t j1, uint64_t *n0, uint64_t *n1) {
        *n0 = j1;
        *n1 = j1;
        if (j1 < g->hce) *n1 = std::min<uint64_t>(g->hce, j1 + TILE);
        else if (g->cb < nchunks) {
            *n0 = (uint64_t)g->cb * CK;
            *n1 = std::min<uint64_t>(nkmers, *n0 + (uint64_t)TILE);
        }
    };
    auto hash_rank = [&](WG *g, uint64_t j0, uint64_t j1, uint32_t hoff, uint32_t buf) {
        const uint64_t tw_w0 = tile_w0(j0);
        for (uint32_t t = 0; t < THREADS; t++)
            for (int a = 0; a < KPT; a++) {
                const uint64_t j = j0 + (uint64_t)a * THREADS + t;
                uint64_t &r_ = g->rr[t * KPT + a];
                r_ = ~0ull;
                if (j < j1) {
                    const uint64_t bpos = (j + read_of(j) * (uint64_t)(k - 1)) * 2;
                    const uint32_t wi = (uint32_t)((bpos >> 6) - tw_w0);
                    const uint64_t w0 = g->s_tw[buf * NP_TW + wi], w1 = g->s_tw[buf * NP_TW + wi + 1];
                    const uint32_t sh = (uint32_t)(bpos & 63);
                    const uint64_t xx = sh ? ((w0 << sh) | (w1 >> (64 - sh))) : w0;
                    const uint64_t h = canonical2(xx >> (64 - 2 * k), k);
                    const uint64_t q = h / N.pm, r = h % N.pm;
                    const uint32_t b = (uint32_t)(((r >> S0) * (uint64_t)N.magic) >> 32);
                    if (b >= F1) { fprintf(stderr, "bucket %u\n", b); throw std::runtime_error("b"); }
                    const uint64_t pay = (q << N.ob) | (r - (uint64_t)b * S);
                    const uint32_t rank = g->hist2[hoff + b]++;
                    r_ = ((uint64_t)b << SLOT_B) | ((uint64_t)rank << SLOT_K) | pay;
                }
            }
    };
    uint64_t steps = 0;
    try {
        for (bool any = true; any;) {
            any = false;
            for (WG *g : wgs) {
                if (g->phase == 6) continue;
                any = true;
                steps++;
                const uint32_t F1l = F1;
                switch (g->phase) {
                case 0: {
                    for (uint32_t b = 0; b < F1l; b++) { g->bcur[b] = 0; g->cnt[b] = 0; g->hist2[b] = 0; g->hist2[F1a + b] = 0; g->bjb[b] = 0; }
                    g->hj1 = std::min<uint64_t>(g->hce, g->hj0 + TILE);
                    if (g->hce > g->hj0) {
                        const uint32_t nw = tile_nw(g->hj0, g->hj1);
                        for (uint32_t t = 0; t < THREADS && t < nw; t++) g->s_tw[t] = words.at(tile_w0(g->hj0) + t);
                        g->qn = l1q++;
                    }
                    g->phase = 1;
                    break;
                }
                case 1: {
                    next_tile(g, g->hj1, &g->n0, &g->n1);
                    if (g->hce > g->hj0) {
                        if (g->n1 > g->n0) {
                            const uint32_t nw = tile_nw(g->n0, g->n1);
                            for (uint32_t t = 0; t < THREADS && t < nw; t++) g->tw_next[t] = words.at(tile_w0(g->n0) + t);
                        }
                        hash_rank(g, g->hj0, g->hj1, 0, 0);
                    }
                    g->phase = g->hce > g->hj0 ? 2 : 5;
                    break;
                }
                case 2: {   // P1
                    const uint32_t hoff = (g->ti & 1) * F1a;
                    for (uint32_t d = 0; d < THREADS; d++) {
                        g->rsv[d] = 0;
                        if (d < F1l && g->bcur[d] != DEAD) {
                            const uint32_t h = g->hist2[hoff + d], L0 = g->cnt[d];
                            const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (((L0 + BLK - 1) & ~(BLK - 1)) >> blk_sh);
                            if (need) { g->rsv[d] = bkt_cur[d]; bkt_cur[d] += (unsigned long long)need * BLK; }
                        }
                    }
                    uint32_t base = 0;
                    for (uint32_t b = 0; b < 256; b++) {
                        const uint32_t h = b < F1l ? g->hist2[hoff + b] : 0u;
                        const uint32_t par = b < F1l ? (g->cnt[b] & 1u) : 0u;
                        const uint32_t rs = h ? (h + par + 1u) & ~1u : 0u;
                        if (b < F1l) g->lstart[b] = base + par;
                        base += rs;
                    }
                    g->s_misc[1] = base;
                    g->phase = 3;
                    break;
                }
                case 3: {   // P2
                    const uint32_t hoff = (g->ti & 1) * F1a;
                    const uint64_t j0 = g->hj0;
                    const bool last = g->n1 == g->n0;
                    const bool top = g->htop;
                    const uint32_t tb = (uint32_t)j0;
                    const uint32_t nhi = last ? tb : (uint32_t)(g->n1 - 1);
                    for (uint32_t t = 0; t < THREADS; t++)
                        for (int a = 0; a < KPT; a++) {
                            const uint64_t r_ = g->rr[t * KPT + a];
                            if (r_ == ~0ull) continue;
                            const uint32_t b = (uint32_t)(r_ >> SLOT_B);
                            const uint32_t pos = g->lstart[b] + (uint32_t)((r_ >> SLOT_K) & EMPTY);
                            g->slot[pos] = ((uint64_t)b << SLOT_B) | ((uint64_t)(a * THREADS + t) << SLOT_K) | (r_ & PAY);
                        }
                    if (!last) for (uint32_t t = 0; t < NP_TW; t++) g->s_tw[((g->ti + 1) & 1) * NP_TW + t] = g->tw_next[t];
                    if (top) g->s_misc[0] = (uint32_t)std::min<unsigned long long>(g->qn + 2ull * nwg, nchunks);
                    for (uint32_t d = 0; d < F1l; d++) {
                        const uint32_t h = g->hist2[hoff + d], L0 = g->cnt[d];
                        const uint32_t split = (L0 + BLK - 1) & ~(BLK - 1);
                        const uint32_t need = ((L0 + h + BLK - 1) >> blk_sh) - (split >> blk_sh);
                        const uint32_t bc = g->bcur[d];
                        const uint32_t e = L0 + h;
                        const uint32_t jb_old = g->bjb[d];
                        const uint32_t jb_new = need ? tb : jb_old;
                        const bool stale = !last && (e & (BLK - 1)) != 0 && nhi - jb_new > N.jlim;
                        if (!(h || last || stale)) continue;
                        uint32_t nb = 0;
                        if (bc == DEAD) nb = DEAD;
                        else if (need) {
                            nb = (uint32_t)(g->rsv[d] - (uint64_t)d * cap);
                            if ((uint64_t)nb + (uint64_t)need * BLK > cap) { err |= 8; nb = DEAD; }
                        }
                        const uint32_t fe = (last || stale) ? e : (e & ~1u);
                        if ((L0 & 1) && fe > L0 - 1 && bc != DEAD) rec[(uint64_t)d * cap + bc + ((L0 - 1) & (BLK - 1))] = g->tail[d];
                        const uint32_t q0 = g->lstart[d];
                        if (h) {
                            if (L0 & 1) g->slot[q0 - 1] = ((uint64_t)d << SLOT_B) | ((uint64_t)EMPTY << SLOT_K);
                            if ((q0 + h) & 1) g->slot[q0 + h] = ((uint64_t)d << SLOT_B) | ((uint64_t)EMPTY << SLOT_K);
                        }
                        const bool dead = bc == DEAD || nb == DEAD;
                        g->dlx[d] = bc + (L0 & (BLK - 1)) - q0;
                        g->dly[d] = nb + L0 - split - q0;
                        g->qqx[d] = q0 + (split - L0);
                        g->qqy[d] = dead ? 0 : q0 + (fe > L0 ? fe - L0 : 0);
                        g->obase[d] = jb_old;
                        if (h) {
                            if (nb == DEAD) g->bcur[d] = DEAD;
                            else if (need) g->bcur[d] = nb + (need - 1) * BLK;
                            g->cnt[d] = e;
                            g->hist2[hoff + d] = 0;
                            g->bjb[d] = jb_new;
                            if (need && nb != DEAD)
                                for (uint32_t z = 0; z < need; z++) blkj[(((uint64_t)d * cap + nb) >> blk_sh) + z] = tb;
                        }
                        if (stale && !dead) {
                            const uint64_t pb0 = (uint64_t)d * cap + g->bcur[d];
                            for (uint32_t s = e & (BLK - 1); s < BLK; s++) rec[pb0 + s] = ~0ull;
                            g->cnt[d] = (e + BLK - 1) & ~(BLK - 1);
                        }
                    }
                    g->phase = 4;
                    break;
                }
                case 4: {   // P3
                    const uint64_t j0 = g->hj0;
                    const bool last = g->n1 == g->n0;
                    const uint32_t tb = (uint32_t)j0;
                    const uint32_t nslot = g->s_misc[1];
                    for (uint32_t m = 0; 2 * m < nslot; m++) {
                        const uint64_t sx = g->slot[2 * m], sy = g->slot[2 * m + 1];
                        const uint32_t dd = (uint32_t)(sx >> SLOT_B);
                        const uint32_t k0 = (uint32_t)(sx >> SLOT_K) & EMPTY, k1 = (uint32_t)(sy >> SLOT_K) & EMPTY;
                        if ((uint32_t)(sy >> SLOT_B) != dd) { fprintf(stderr, "pair straddles buckets\n"); throw std::runtime_error("pair"); }
                        const uint32_t q = 2 * m;
                        const bool nw = q >= g->qqx[dd];
                        const uint32_t base = nw ? tb : g->obase[dd];
                        const bool r0 = k0 != EMPTY, r1 = k1 != EMPTY;
                        const uint64_t v0 = ((uint64_t)(tb + k0 - base) << N.pb) | (sx & PAY);
                        const uint64_t v1 = ((uint64_t)(tb + k1 - base) << N.pb) | (sy & PAY);
                        if (r0 && (uint64_t)(tb + k0 - base) > N.jlim) { fprintf(stderr, "jrel overflow\n"); throw std::runtime_error("jrel"); }
                        const uint64_t o = (uint64_t)dd * cap + (uint32_t)((nw ? g->dly[dd] : g->dlx[dd]) + q);
                        if (q < g->qqy[dd]) {
                            if (r0 && r1) { rec[o] = v0; rec[o + 1] = v1; }
                            else if (r0) rec[o] = v0;
                            else if (r1) rec[o + 1] = v1;
                        } else if (r0) {
                            g->tail[dd] = v0;
                        }
                    }
                    if (last) { g->phase = 5; break; }
                    if (g->hj1 >= g->hce) {
                        g->hce = std::min<uint64_t>(nkmers, (uint64_t)g->cb * CK + CK);
                        g->cb = g->s_misc[0];
                        g->htop = true;
                    } else {
                        g->htop = false;
                    }
                    g->hj0 = g->n0;
                    g->hj1 = g->n1;
                    next_tile(g, g->hj1, &g->n0, &g->n1);
                    if (g->htop) g->qn = l1q++;
                    if (g->n1 > g->n0) {
                        const uint32_t nw = tile_nw(g->n0, g->n1);
                        if (nw > NP_TW) { fprintf(stderr, "tile words %u\n", nw); throw std::runtime_error("nw"); }
                        for (uint32_t t = 0; t < THREADS && t < nw; t++) g->tw_next[t] = words.at(tile_w0(g->n0) + t);
                    }
                    hash_rank(g, g->hj0, g->hj1, ((g->ti + 1) & 1) * F1a, (g->ti + 1) & 1);
                    g->ti++;
                    g->phase = 2;
                    break;
                }
                case 5: {   // epilogue
                    for (uint32_t y = 0; y < F1l * BLK; y++) {
                        const uint32_t dd = y >> blk_sh, sl = y & (BLK - 1);
                        const uint32_t c = g->cnt[dd] & (BLK - 1);
                        if (c == 0 || sl < c || g->bcur[dd] == DEAD) continue;
                        rec[(uint64_t)dd * cap + g->bcur[dd] + sl] = ~0ull;
                    }
                    g->phase = 6;
                    break;
                }
                }
            }
        }
    } catch (std::exception &e) {
        printf("FAILED after %llu phase steps: %s\n", (unsigned long long)steps, e.what());
        return 1;
    }
    // every reserved slot of every bucket is a record or a sentinel; count records
    uint64_t recs = 0;
    for (uint32_t d = 0; d < N.nb; d++)
        for (uint64_t i = (uint64_t)d * cap; i < bkt_cur[d]; i++) recs += rec[i] != ~0ull;
    printf("level 1 ok: err %llu, records %llu of %llu k-mers, queue %llu\n", (unsigned long long)err,
           (unsigned long long)recs, (unsigned long long)nkmers, l1q);
    if (recs != nkmers) return 2;

    // ---- level 2 (k_scatter_n2<1024, 4, 4>), workgroups one after another
    const int span_bits = 24;
    std::vector<uint64_t> tbase(n), rt(n), rbase(n), dd_(n);
    uint64_t base = 0;
    for (int i = 0; i < n; i++) {
        tbase[i] = base;
        base += (p[i] + (1ull << span_bits) - 1) >> span_bits << span_bits;
        rt[i] = (p[i] + (1 << S0) - 1) >> S0;
        rbase[i] = tbase[i] >> S0;
        dd_[i] = N.pm - p[i];
    }
    const uint64_t nreg = base >> S0;
    const int parts = 16, blk2 = 6;
    const uint32_t BLK2 = 1u << blk2;
    std::vector<uint64_t> reg_base(nreg + 1, 0);
    {
        uint64_t acc = 0;
        const uint64_t slack = (2 * 16 + 1) * BLK2 + 16;
        int i = 0;
        for (uint64_t g = 0; g < nreg; g++) {
            reg_base[g] = acc;
            const uint64_t lo = g << S0;
            while (i + 1 < n && lo >= tbase[i + 1]) i++;
            if (lo >= tbase[i] + p[i]) continue;
            const uint64_t nbn = std::min<uint64_t>(1 << S0, tbase[i] + p[i] - lo);
            const double m = (double)nkmers * (double)nbn / (double)p[i];
            uint64_t c = (uint64_t)(m + 8 * sqrt(m)) + slack;
            acc += (c + 15) & ~15ull;
        }
        reg_base[nreg] = acc;
    }
    Arr<uint64_t> rec2(reg_base[nreg], "rec2", ~0ull);
    std::vector<unsigned long long> reg_cur(reg_base.begin(), reg_base.end() - 1);
    const uint32_t F2 = 4 * N.rloc;
    const int IN = 2, T2 = 1024, TILE2 = T2 * IN;
    uint64_t err2 = 0;
    try {
        for (uint32_t wg = 0; wg < N.nb * parts; wg++) {
            const uint32_t b = wg / parts, pp = wg % parts;
            const uint64_t b0 = (uint64_t)b * cap, b1 = std::min<uint64_t>(bkt_cur[b], b0 + cap);
            const uint64_t len = ((b1 - b0 + parts - 1) / parts + 1) & ~1ull;
            const uint64_t r0 = std::min(b1, b0 + (uint64_t)pp * len), r1 = std::min(b1, r0 + len);
            Arr<uint64_t> bcur(F2, "n2.bcur", 0), nbase(F2, "n2.nbase", 0), tail(F2 * 16, "n2.tail", 0);
            Arr<uint32_t> cnt(F2, "n2.cnt", 0), hist(F2, "n2.hist", 0);
            const uint64_t bin0 = (uint64_t)b * ((uint64_t)N.rp << S0);
            const uint32_t rb = b * N.rp;
            const uint32_t ntiles = (uint32_t)((r1 - r0 + TILE2 - 1) / TILE2);
            for (uint32_t ti = 0; ti < ntiles; ti++) {
                const uint64_t t0 = r0 + (uint64_t)ti * TILE2;
                const bool last = ti + 1 == ntiles;
                const uint64_t n1 = std::min(r1, t0 + TILE2);
                std::vector<uint64_t> X;   // (x) in thread order
                std::vector<uint32_t> R;
                for (uint64_t idx = t0; idx < n1; idx++) {
                    const uint64_t v = rec[idx];
                    if (v == ~0ull) continue;
                    const uint32_t jb = blkj[idx >> blk_sh];
                    const uint64_t jv = (uint64_t)(jb + (uint32_t)(v >> N.pb)) << 32;
                    const uint64_t pay = v & ((1ull << N.pb) - 1);
                    const uint64_t qv = pay >> N.ob, r = bin0 + (pay & ((1ull << N.ob) - 1));
                    for (int i = 0; i < n; i++) {
                        uint64_t bin = r + qv * dd_[i];
                        if (bin >= p[i]) bin -= p[i];
                        const uint32_t rho = (uint32_t)(bin >> S0);
                        int32_t loc = (int32_t)(rho - rb);
                        if (loc < 0) loc += (int32_t)rt[i];
                        if ((uint32_t)loc >= N.rloc) { err2 |= 16; continue; }
                        const uint32_t dst = (uint32_t)i * N.rloc + (uint32_t)loc;
                        const uint64_t x = jv | ((uint64_t)dst << 16) | (bin & ((1 << S0) - 1));
                        X.push_back(x);
                        R.push_back(hist[dst]++);
                    }
                }
                // reservations + flush list
                std::vector<uint32_t> flist;
                for (uint32_t d = 0; d < F2; d++) {
                    const uint32_t h = hist[d], c0 = cnt[d];
                    const bool dead = bcur[d] == ~0ull;
                    uint64_t nb = 0;
                    if (h) {
                        const uint32_t need = ((c0 + h + BLK2 - 1) >> blk2) - ((c0 + BLK2 - 1) >> blk2);
                        if (dead) nb = ~0ull;
                        else if (need) {
                            const uint32_t il = d / N.rloc;
                            uint32_t rho = rb + (d - il * N.rloc);
                            if (rho >= rt[il]) rho -= rt[il];
                            const uint64_t g = rbase[il] + rho;
                            if (g >= nreg) throw std::runtime_error("greg");
                            nb = reg_cur.at(g);
                            reg_cur.at(g) += (uint64_t)need * BLK2;
                            if (nb + (uint64_t)need * BLK2 > reg_base.at(g + 1)) { err2 |= 4; nb = ~0ull; }
                        }
                    }
                    nbase[d] = nb;
                    const uint32_t a = c0 & ~15u, e = c0 + h;
                    if (!dead && c0 != a && (last ? e : (e & ~15u)) > a) flist.push_back(d);
                }
                for (uint32_t d : flist) {
                    const uint32_t c0 = cnt[d], a = c0 & ~15u;
                    for (uint32_t sl = 0; sl < 16; sl++)
                        if (a + sl < c0) rec2[bcur[d] + ((a + sl) & (BLK2 - 1))] = tail[d * 16 + sl];
                }
                for (size_t q = 0; q < X.size(); q++) {
                    const uint32_t d = ((uint32_t)X[q]) >> 16;
                    const uint32_t L = cnt[d] + R[q], e = cnt[d] + hist[d];
                    const uint64_t val = X[q] & 0xFFFFFFFF0000FFFFull;
                    if (L < (last ? e : (e & ~15u))) {
                        const uint32_t split = (cnt[d] + BLK2 - 1) & ~(BLK2 - 1);
                        uint64_t pos;
                        if (L < split) pos = bcur[d] == ~0ull ? ~0ull : bcur[d] + (L & (BLK2 - 1));
                        else pos = nbase[d] == ~0ull ? ~0ull : nbase[d] + (L - split);
                        if (pos != ~0ull) rec2[pos] = val;
                    } else {
                        tail[d * 16 + (L & 15)] = val;
                    }
                }
                for (uint32_t d = 0; d < F2; d++) {
                    const uint32_t h = hist[d];
                    if (!h) continue;
                    const uint32_t c0 = cnt[d];
                    const uint32_t need = ((c0 + h + BLK2 - 1) >> blk2) - ((c0 + BLK2 - 1) >> blk2);
                    if (nbase[d] == ~0ull) bcur[d] = ~0ull;
                    else if (need) bcur[d] = nbase[d] + (uint64_t)(need - 1) * BLK2;
                    cnt[d] = c0 + h;
                    hist[d] = 0;
                }
            }
            for (uint32_t y = 0; y < F2 * BLK2; y++) {
                const uint32_t d = y >> blk2, sl = y & (BLK2 - 1);
                const uint32_t c = cnt[d] & (BLK2 - 1);
                if (c == 0 || sl < c || bcur[d] == ~0ull) continue;
                rec2[bcur[d] + sl] = ~0ull;
            }
        }
    } catch (std::exception &e) {
        printf("LEVEL 2 FAILED: %s\n", e.what());
        return 1;
    }
    uint64_t recs2 = 0;
    for (uint64_t g = 0; g < nreg; g++)
        for (uint64_t i = reg_base[g]; i < reg_cur[g]; i++) recs2 += rec2[i] != ~0ull;
    printf("level 2: err %llu, records %llu of %llu\n", (unsigned long long)err2, (unsigned long long)recs2,
           (unsigned long long)nkmers * n);
    return recs2 == nkmers * n ? 0 : 3;
}
