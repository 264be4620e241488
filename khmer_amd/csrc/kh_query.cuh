// kh_query.cuh -- read-only device kernels: get_count, k-mer hashes/counts,
// get_median_count, batch boundaries, synthetic reads.  Included by kh_engine.hip.
#pragma once
#include "kh_src.cuh"

namespace kh {

constexpr int Q_THREADS = 256;
constexpr int Q_TILE = 2048;

// ---------------------------------------------------------------------------
// queries: Storage::get_count (storage.hh:206-219, 362-379, 627-649)
// The table gathers of a query are non-temporal loads: one byte used of
// every line fetched, so keeping the lines in L2 only evicts useful ones.
// Same FETCH_SIZE, C5 query 520 -> 474.5 ms/step (same box, median digests
// matched).  -DKH_QUERY_TEMPORAL restores plain loads (A/B).
#ifdef KH_QUERY_TEMPORAL
#define KH_TLOAD(p) (*(p))
#else
#define KH_TLOAD(p) __builtin_nontemporal_load(p)
#endif
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
            const uint8_t byte = KH_TLOAD(&tab[P.tbyte[i] + (bin >> 1)]);
            const uint32_t c = (bin & 1) ? (byte & 0x0F) : (byte >> 4);
            mn = c < mn ? c : mn;
        }
        return mn;
    }
    uint32_t mn = 255;
    for (int i = 0; i < P.n; i++) {
        const uint32_t c = KH_TLOAD(&tab[P.tbyte[i] + mod_barrett(h, P.p[i], P.m[i])]);
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
__global__ void __launch_bounds__(Q_THREADS) k_kmer_hashes(Src src, uint64_t nkmers, uint64_t *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * Q_TILE;
    const uint64_t j1 = min(nkmers, j0 + Q_TILE);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    block_sync();
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) out[j] = kmer_hash(src, s_koff, tr, j);
}

// Band / mask filter of the consume_seqfile_banding / _with_mask variants
// (src/oxli/hashtable.cc:152-274): keep k-mer j iff its hash lies in
// [band_lo, band_hi) (when banding) and the mask table's count c satisfies
// c >= threshold (consume_masked) or c <= threshold (otherwise).  Writes the
// hash and a keep flag per k-mer; order is preserved by the compaction after.
struct KmerFilter {
    int band;                 // banding on
    uint64_t band_lo, band_hi;
    int mask;                 // mask on
    Params MP;                // mask table geometry
    const uint8_t *mtab;
    const uint64_t *mbc_keys;
    const uint16_t *mbc_vals;
    uint64_t mbc_n;
    uint32_t threshold;
    int consume_masked;
};

template <class Src>
__global__ void __launch_bounds__(Q_THREADS) k_kmer_filter(Src src, uint64_t nkmers, KmerFilter F, uint64_t *out,
                                                         uint8_t *keep) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * Q_TILE;
    const uint64_t j1 = min(nkmers, j0 + Q_TILE);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    block_sync();
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        const uint64_t h = kmer_hash(src, s_koff, tr, j);
        bool k = !F.band || (h >= F.band_lo && h < F.band_hi);
        if (k && F.mask) {
            const uint32_t c = get_count_dev(F.MP, F.mtab, h, F.mbc_keys, F.mbc_vals, F.mbc_n);
            k = F.consume_masked ? c >= F.threshold : c <= F.threshold;
        }
        out[j] = h;
        keep[j] = k ? 1 : 0;
    }
}

// counts of every k-mer of a batch (for get_median_count)
template <class Src>
__global__ void __launch_bounds__(Q_THREADS) k_kmer_counts(Params P, Src src, uint64_t nkmers, const uint8_t *tab,
                                                            uint16_t *out, const uint64_t *bc_keys,
                                                            const uint16_t *bc_vals, uint64_t bc_n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *s_meta = (uint64_t *)smem;
    uint64_t *s_koff = s_meta + 2;
    const uint64_t j0 = (uint64_t)blockIdx.x * Q_TILE;
    const uint64_t j1 = min(nkmers, j0 + Q_TILE);
    TileReads tr = load_tile_reads(src, j0, j1, s_koff, s_meta);
    block_sync();
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

// Hashtable::median_at_least (src/oxli/hashtable.cc:333-364), one thread per
// read over its k-mer counts: the reference's two loops return true exactly
// when at least min_req = unsigned(0.5 + float(n) / 2) of the n k-mers have a
// count >= cutoff (the early exits only stop the scan), so the count decides.
__global__ void k_at_least(const uint64_t *koff, uint64_t nreads, const uint16_t *counts, uint32_t cutoff,
                           uint8_t *out) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < nreads;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = koff[r], n = koff[r + 1] - a;
        const uint64_t min_req = (uint64_t)(0.5 + (double)((float)n / 2.0f));
        uint64_t num = 0;
        for (uint64_t t = 0; t < n; t++) num += (uint32_t)counts[a + t] >= cutoff ? 1 : 0;
        out[r] = num >= min_req ? 1 : 0;
    }
}

// Hashtable::get_median_count over fixed-length device reads, one wave per read
// (kpr = k-mers per read <= 256, four per lane): the k-mer counts stay in
// registers.  average: the partial sums are integers below 2^24 (kpr <= 256,
// counts <= 65535), so the reference's sequential float32 sum equals the
// exact integer sum; the squared deviations are summed in stream order by a
// uniform loop (the same rounding sequence as the reference); median =
// sorted[kpr / 2] by a radix select over the counts with wave ballots.
//
// cnt8 != null (a sharded group's query, kh_engine.hip group_median_fixed):
// the k-mer counts are the per-k-mer minima over the tables gathered from the
// shards that own the bins (u8: tables are at most 8-bit), and a Byte count
// of 255 becomes the bigcount value from the replicated map, as
// ByteStorage::get_count does (storage.hh:627-649).
__device__ __forceinline__ uint32_t bigcount_or(uint64_t h, uint32_t c, const uint64_t *bc_keys,
                                                const uint16_t *bc_vals, uint64_t bc_n) {
    uint64_t lo = 0, hi = bc_n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (bc_keys[mid] < h) lo = mid + 1; else hi = mid;
    }
    return lo < bc_n && bc_keys[lo] == h ? bc_vals[lo] : c;
}
template <class Src>
__global__ void __launch_bounds__(256) k_median_fixed(Params P, Src src, uint64_t nreads, uint32_t kpr,
                                                      const uint8_t *tab, const uint64_t *bc_keys,
                                                      const uint16_t *bc_vals, uint64_t bc_n, uint16_t *med,
                                                      float *avg, float *sd, const uint8_t *cnt8 = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = wave; r < nreads; r += nwaves) {
        uint32_t c[4];
        bool ok[4];
        uint32_t sum = 0, mx = 0;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t t = lane + 64u * s;
            ok[s] = t < kpr;
            if (!ok[s]) {
                c[s] = 0;
            } else if (cnt8) {
                c[s] = cnt8[r * kpr + t];
                if (c[s] == 255 && P.kind == BYTE && P.use_bigcount && bc_n)
                    c[s] = bigcount_or(kmer_hash_global(src, r * kpr + t), c[s], bc_keys, bc_vals, bc_n);
            } else {
                c[s] = get_count_dev(P, tab, kmer_hash_global(src, r * kpr + t), bc_keys, bc_vals, bc_n);
            }
            sum += c[s];
            mx = c[s] > mx ? c[s] : mx;
        }
        sum = (uint32_t)wave_sum(sum);
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t y = __shfl_xor(mx, d, 64);
            mx = y > mx ? y : mx;
        }
        const float n = (float)kpr;
        const float average = div_rn_exact((float)sum, n);
        float d2[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const float d = __fsub_rn((float)c[s], average);
            d2[s] = __fmul_rn(d, d);
        }
        float var = 0.f;
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const uint32_t lim = kpr > 64u * s ? min(64u, kpr - 64u * s) : 0u;
            const int v = __float_as_int(d2[s]);
            for (uint32_t l = 0; l < lim; l++) var = __fadd_rn(var, __int_as_float(__builtin_amdgcn_readlane(v, l)));
        }
        var = sqrt_rn_exact(div_rn_exact(var, n));
        // radix select of element kpr / 2
        uint32_t m = kpr / 2, prefix = 0;
        const int nbits = 32 - __clz(mx | 1);
        for (int b = nbits - 1; b >= 0; b--) {
            uint32_t cnt0 = 0;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const bool cand = ok[s] && ((c[s] >> b) >> 1) == ((prefix >> b) >> 1) && !((c[s] >> b) & 1);
                cnt0 += __popcll(__ballot(cand));
            }
            if (m >= cnt0) {
                m -= cnt0;
                prefix |= 1u << b;
            }
        }
        if (lane == 0) {
            med[r] = (uint16_t)prefix;
            avg[r] = average;
            sd[r] = var;
        }
    }
}

// ---------------------------------------------------------------------------
// Sharded get_median_count (kh_engine.hip group_median_fixed): the minimum
// over the tables of every k-mer, gathered from the shards owning its bins.

// table value of local bin `bin` of table i (Storage::get_count's per-table
// read, storage.hh:206-219, 362-379, 627-649; a shard's slice starts on a
// multiple of 8 bins, so the nibble parity and bit position are the global ones)
__device__ __forceinline__ uint32_t table_value(const Params &P, const uint8_t *tab, int i, uint64_t bin) {
    if (P.kind == BIT) return (tab[P.tbyte[i] + (bin >> 3)] >> (bin & 7)) & 1;
    if (P.kind == NIBBLE) {
        const uint8_t byte = tab[P.tbyte[i] + (bin >> 1)];
        return (bin & 1) ? (byte & 0x0F) : (byte >> 4);
    }
    return tab[P.tbyte[i] + bin];
}

// res[j] = min(res[j], c) on a byte array through CAS on its 32-bit word
__device__ __forceinline__ void atomic_min_u8(uint32_t *res32, uint64_t j, uint32_t c) {
    uint32_t *p = res32 + (j >> 2);
    const int sh = (int)(j & 3) * 8;
    uint32_t cur = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (((cur >> sh) & 0xFFu) > c) {
        const uint32_t nw = (cur & ~(0xFFu << sh)) | (c << sh);
        const uint32_t prev = atomicCAS(p, cur, nw);
        if (prev == cur) break;
        cur = prev;
    }
}

// Exchange mode: the owner looks up the level-1 records routed to it.
// Segment x = s * NB + b holds source s's records of the owner's bucket b:
// (j << 32) | offset inside the bucket's 2^(s0+s2) bins (sentinel ~0 in
// partially filled blocks).  `parts` workgroups per segment.
__global__ void k_lookup_min(Params P, const uint8_t *tab, const uint64_t *rec, const uint64_t *seg_lo,
                             const uint64_t *seg_hi, uint32_t NB, uint32_t parts, uint32_t *res32) {
    const uint64_t x = blockIdx.x / parts, part = blockIdx.x % parts;
    const uint64_t lo = seg_lo[x], hi = seg_hi[x];
    const uint32_t b = (uint32_t)(x % NB);
    const int shift = P.s0 + P.s2;
    // the bucket's table (tables start on bucket boundaries)
    int ti = 0;
    const uint64_t g0 = (uint64_t)b << shift;
    while (ti + 1 < P.n && g0 >= P.tbase[ti + 1]) ti++;
    const uint64_t base = g0 - P.tbase[ti];
    const uint64_t n = hi > lo ? hi - lo : 0, per = (n + parts - 1) / parts;
    const uint64_t a0 = lo + part * per, a1 = min(hi, a0 + per);
    for (uint64_t a = a0 + threadIdx.x; a < a1; a += blockDim.x) {
        const uint64_t v = rec[a];
        if (v == ~0ull) continue;
        const uint64_t bin = base + (v & ((1ull << shift) - 1));
        atomic_min_u8(res32, v >> 32, table_value(P, tab, ti, bin));
    }
}

// Broadcast mode: every rank hashes every k-mer of a source's reads and
// takes the minimum over the tables whose bin it owns (0xFF: none)
template <class Src>
__global__ void __launch_bounds__(256) k_own_min(Params P, Src src, uint64_t nkmers, const uint8_t *tab,
                                                 uint8_t *out) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < nkmers;
         j += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = kmer_hash_global(src, j);
        uint32_t c = 0xFF;
        for (int i = 0; i < P.n; i++) {
            const uint64_t bin = mod_barrett(h, P.p[i], P.m[i]) - P.lo[i];
            if (bin < P.lsz[i]) {
                const uint32_t v = table_value(P, tab, i, bin);
                c = v < c ? v : c;
            }
        }
        out[j] = (uint8_t)c;
    }
}

// dst[q] = min over the `nsrc` arrays src + t * stride (bytes), q < n
__global__ void k_min_bytes(uint8_t *dst, const uint8_t *src, uint64_t stride, int nsrc, uint64_t n) {
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t c = dst[q];
        for (int t = 0; t < nsrc; t++) {
            const uint32_t v = src[(uint64_t)t * stride + q];
            c = v < c ? v : c;
        }
        dst[q] = (uint8_t)c;
    }
}

// every read of a byte batch reverse-complemented in place (the complement of
// _revcomp, src/oxli/kmer_hash.cc:52-55, IUPAC and all): read r occupies bytes
// [koff[r] + r*(k-1), +len) (fixed length: [r*L, +L)); one wave per read
__global__ void k_revcomp_reads(const uint8_t *bytes, const uint64_t *koff, uint64_t kpr, int k, uint64_t nreads,
                                uint8_t *rbytes) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = wave; r < nreads; r += nwaves) {
        uint64_t start, len;
        if (koff) {
            start = koff[r] + r * (uint64_t)(k - 1);
            len = koff[r + 1] - koff[r] + (uint64_t)(k - 1);
        } else {
            len = kpr + (uint64_t)(k - 1);
            start = r * len;
        }
        for (uint64_t t = lane; t < len; t += 64) rbytes[start + t] = (uint8_t)iupac_comp(bytes[start + len - 1 - t]);
    }
}

// 2-bit packed bases -> ASCII (code 0..3 = A, T, C, G; kh_device.h order)
__global__ void k_unpack_ascii(const uint64_t *words, uint64_t nbases, uint8_t *out) {
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w * 32 < nbases;
         w += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = words[w];
        uint8_t b[32];
#pragma unroll
        for (int i = 0; i < 32; i++) b[i] = "ATCG"[(x >> (62 - 2 * i)) & 3];
        if (w * 32 + 32 <= nbases) {
            uint4 *o = (uint4 *)(out + w * 32);
            o[0] = *(const uint4 *)&b[0];
            o[1] = *(const uint4 *)&b[16];
        } else {
            for (uint64_t i = 0; w * 32 + i < nbases; i++) out[w * 32 + i] = b[i];
        }
    }
}

// ---------------------------------------------------------------------------
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

// genomic stream (khmer_amd/synth.py genomic_codes): read r samples L bases at
// a uniform start (either strand) of a random genome of G bases (seed+1) and
// substitutes 1% of them (seed+3).  One output word per thread; the genome word
// and the read's (start, strand) are cached across the word's 32 bases.
__global__ void k_synth_genomic(uint64_t seed, uint64_t G, uint64_t r0, uint64_t nreads, int L, int k,
                                uint64_t *words, uint64_t nwords, uint64_t *koff) {
    const uint64_t nbases = nreads * (uint64_t)L;
    for (uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t out = 0;
        uint64_t cur_r = ~0ull, start = 0, gw_key = ~0ull, gsrc = 0;
        bool rc = false;
        for (int b = 0; b < 32; b++) {
            const uint64_t p = w * 32 + b;
            uint64_t code = 0;
            if (p < nbases) {
                const uint64_t r = p / (uint64_t)L, i = p % (uint64_t)L;
                if (r != cur_r) {
                    cur_r = r;
                    start = synth_word(seed + 2, r0 + r, 0) % (G - (uint64_t)L + 1);
                    rc = synth_word(seed + 2, r0 + r, 1) & 1;
                }
                const uint64_t gi = rc ? start + (uint64_t)L - 1 - i : start + i;
                const uint64_t gw = gi >> 5;
                if (gw != gw_key) { gsrc = synth_word(seed + 1, gw >> 20, gw & 0xFFFFF); gw_key = gw; }
                code = (gsrc >> (62 - 2 * (gi & 31))) & 3;
                if (rc) code ^= 1;
                const uint64_t u = synth_word(seed + 3, r0 + r, i);
                if (u % 100 == 0) code = (code + 1 + (u >> 32) % 3) & 3;
            }
            out = (out << 2) | code;
        }
        words[w] = out;
    }
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r <= nreads;
         r += (uint64_t)gridDim.x * blockDim.x)
        koff[r] = r * (uint64_t)(L - k + 1);
}

}  // namespace kh
