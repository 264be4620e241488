// kh_device.h -- arithmetic shared by the HIP kernels and the host side of
// libkhmer_hip.so.  Everything here is integer/byte work (no MFMA).
//
// 2-bit code (include/oxli/kmer_hash.hh:62-96): A=0 T=1 C=2 G=3, anything
// else 3; complement = code ^ 1 for every code (A<->T, C<->G, else 3->2), so a
// packed read carries the reference's hashing semantics exactly, cleaned or not.
//
// Packed read stream: 32 bases per u64 word, first base in the two most
// significant bits (base p lives at word p>>5, shift 62-2*(p&31)); the buffer
// carries one zero padding word so a window never reads past the end.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KH_HD __host__ __device__ __forceinline__
#else
#define KH_HD static inline
#endif

namespace kh {

// storage kinds == reference file type codes (include/oxli/oxli.hh:91-97)
enum StorageKind : int { BYTE = 1, BIT = 2, NIBBLE = 7 };
enum HashKind : int { TWOBIT = 0, MURMUR = 1 };

KH_HD uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// Exact h % p for any 64-bit h and p >= 1 (replaces the reference's
// `khash % _tablesizes[i]`, include/oxli/storage.hh:577).  m = floor(2^64/p)
// (UINT64_MAX for p == 1); Barrett's estimate is at most one short, so one
// conditional subtraction makes it exact.
KH_HD uint64_t barrett_m(uint64_t p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return p <= 1 ? ~0ull : (~0ull / p) + ((~0ull % p) == p - 1 ? 1 : 0);
#else
    return p <= 1 ? ~0ull : (uint64_t)(((unsigned __int128)1 << 64) / p);
#endif
}
KH_HD uint64_t mod_barrett(uint64_t h, uint64_t p, uint64_t m) {
    uint64_t q = umulhi64(h, m);
    uint64_t r = h - q * p;
    return r >= p ? r - p : r;
}

// The same remainder from one double multiply, for p < 2^30 and h / p < 2^31
// (Params::fm32; fewer VALU instructions than the 64-bit Barrett product):
// with ip = fl(1/p), x = fl(fl(h) * ip) is within 2^-20 of h / p, so q =
// trunc(x) is floor(h / p) or one off, the remainder estimate h - q * p lies
// in [-p, 2p) -- exact in 32-bit two's complement -- and one correction each
// way makes it h % p.
KH_HD uint32_t mod_f64_32(uint64_t h, uint32_t p, double ip) {
    const uint32_t q = (uint32_t)((double)h * ip);
    int32_t r = (int32_t)((uint32_t)h - q * p);
    r += r < 0 ? (int32_t)p : 0;
    r -= r >= (int32_t)p ? (int32_t)p : 0;
    return (uint32_t)r;
}
// floor(x / d) for x < 2^53 and a quotient below 2^31 (SrcCommon::kpr_ip),
// the same bound: the double estimate is exact or one off either way
KH_HD uint64_t div_f64(uint64_t x, uint64_t d, double id) {
    const uint32_t q = (uint32_t)((double)x * id);
    const int64_t r = (int64_t)(x - (uint64_t)q * d);
    return r < 0 ? q - 1 : (r >= (int64_t)d ? q + 1 : q);
}

KH_HD uint64_t kmer_mask(int k) { return k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1); }

KH_HD uint64_t bitrev64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__) || defined(__clang__)
    return __builtin_bitreverse64(x);
#else
    x = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = ((x >> 8) & 0x00FF00FF00FF00FFull) | ((x & 0x00FF00FF00FF00FFull) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFull) | ((x & 0x0000FFFF0000FFFFull) << 16);
    return (x >> 32) | (x << 32);
#endif
}

// reverse complement of a forward 2-bit k-mer (low 2k bits), i.e. the
// reference's rolling `_kmer_r` (src/oxli/kmer_hash.cc:330-336).
KH_HD uint64_t revcomp2(uint64_t f, int k) {
    uint64_t c = f ^ 0x5555555555555555ull;  // complement every base (x^1)
    uint64_t y = bitrev64(c);                // reverse base order (bits swapped)
    y = ((y >> 1) & 0x5555555555555555ull) | ((y & 0x5555555555555555ull) << 1);
    return y >> (64 - 2 * k);
}

// forward 2-bit window of k bases starting at base position pos
KH_HD uint64_t window2(const uint64_t *words, uint64_t pos, int k) {
    uint64_t b = pos * 2;
    uint64_t w0 = words[b >> 6];
    uint64_t w1 = words[(b >> 6) + 1];
    unsigned sh = (unsigned)(b & 63);
    uint64_t x = sh ? ((w0 << sh) | (w1 >> (64 - sh))) : w0;
    return x >> (64 - 2 * k);
}

KH_HD uint64_t canonical2(uint64_t f, int k) {
    uint64_t r = revcomp2(f, k);
    return f < r ? f : r;
}

// ---- MurmurHash3_x64_128, first output word (the *table family hash,
// src/oxli/kmer_hash.cc:177-198 over third-party/smhasher/MurmurHash3.cc:67-144)
KH_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
KH_HD uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// Murmur over `len` bytes produced by a byte-source functor get(i)
template <class Get>
KH_HD uint64_t murmur3_x64_128_h1(Get get, int len) {
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    uint64_t h1 = 0, h2 = 0;
    const int nblocks = len / 16;
    for (int i = 0; i < nblocks; i++) {
        uint64_t k1 = 0, k2 = 0;
        for (int b = 7; b >= 0; b--) k1 = (k1 << 8) | (uint8_t)get(16 * i + b);
        for (int b = 7; b >= 0; b--) k2 = (k2 << 8) | (uint8_t)get(16 * i + 8 + b);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const int tail = nblocks * 16;
    const int rem = len & 15;
    uint64_t k1 = 0, k2 = 0;
    if (rem > 8) {
        for (int b = rem - 1; b >= 8; b--) k2 = (k2 << 8) | (uint8_t)get(tail + b);
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    if (rem > 0) {
        int top = rem > 8 ? 7 : rem - 1;
        for (int b = top; b >= 0; b--) k1 = (k1 << 8) | (uint8_t)get(tail + b);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

// complement table of _revcomp (src/oxli/kmer_hash.cc:52-55), upper and lower
// case to upper-case IUPAC complements, anything else to ' '.
KH_HD char iupac_comp(uint8_t c) {
    switch (c | 0x20) {
    case 'a': return 'T';
    case 'b': return 'V';
    case 'c': return 'G';
    case 'd': return 'H';
    case 'f': return 'F';
    case 'g': return 'C';
    case 'h': return 'D';
    case 'k': return 'M';
    case 'm': return 'K';
    case 'n': return 'N';
    case 'r': return 'Y';
    case 's': return 'S';
    case 't': return 'A';
    case 'u': return 'A';
    case 'v': return 'B';
    case 'w': return 'W';
    case 'y': return 'R';
    case 'z': return c == 'z' ? 0 : ' ';
    default: return ' ';
    }
}

// canonical Murmur k-mer hash over raw ASCII (kmer_hash.cc:177-198)
KH_HD uint64_t murmur_canonical(const uint8_t *s, int k) {
    uint64_t h = murmur3_x64_128_h1([&](int i) { return s[i]; }, k);
    bool self = true;
    for (int i = 0; i < k; i++)
        if ((uint8_t)iupac_comp(s[k - 1 - i]) != s[i]) { self = false; break; }
    if (self) return h;
    uint64_t r = murmur3_x64_128_h1([&](int i) { return (uint8_t)iupac_comp(s[k - 1 - i]); }, k);
    return h ^ r;
}

// ---- device fast path: Murmur over byte-aligned little-endian words ----
// k-mers of up to MURMUR_WORDS_MAX bytes are hashed from eight aligned 8-byte
// loads per window (a funnel shift aligns them), the reverse complement from a
// second window into the reads' precomputed reverse-complement stream
// (k_revcomp_reads), so no byte loads and no complement table per k-mer.
constexpr int MURMUR_WORDS_MAX = 56;

KH_HD uint64_t murmur_tail_mask(int nbytes) { return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1); }

// MurmurHash3_x64_128 h1 of `len` (<= 56) bytes held little-endian in v[0..6]
KH_HD uint64_t murmur3_h1_words(const uint64_t *v, int len) {
    const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
    uint64_t h1 = 0, h2 = 0;
    const int nblocks = len / 16;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (i < nblocks) {
            uint64_t k1 = v[2 * i], k2 = v[2 * i + 1];
            k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
            h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
            k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
            h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
        }
    }
    const int rem = len & 15;
    uint64_t t1 = 0, t2 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (i == nblocks) { t1 = v[2 * i]; t2 = i < 3 ? v[2 * i + 1] : 0; }
    if (rem > 8) {
        uint64_t k2 = t2 & murmur_tail_mask(rem - 8);
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    }
    if (rem > 0) {
        uint64_t k1 = t1 & murmur_tail_mask(rem);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

// the 7 little-endian words of the bytes at p (8 aligned loads; reads at most
// 7 bytes past p + 56)
KH_HD void load_window(const uint8_t *p, uint64_t *v) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint64_t *w = (const uint64_t *)(uintptr_t)(a & ~7ull);
    const unsigned sh = (unsigned)(a & 7) * 8;
    uint64_t x[8];
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = w[i];
#pragma unroll
    for (int i = 0; i < 7; i++) v[i] = sh ? ((x[i] >> sh) | (x[i + 1] << (64 - sh))) : x[i];
}

// canonical Murmur hash of the k-mer at p whose reverse complement is at q
// (same value as murmur_canonical(p, k) for k <= MURMUR_WORDS_MAX)
KH_HD uint64_t murmur_canonical_windows(const uint8_t *p, const uint8_t *q, int k) {
    uint64_t v[7], u[7];
    load_window(p, v);
    load_window(q, u);
    const uint64_t h = murmur3_h1_words(v, k);
    bool self = true;
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const int nb = k - 8 * i;
        if (nb > 0) self = self && ((v[i] ^ u[i]) & murmur_tail_mask(nb)) == 0;
    }
    if (self) return h;
    return h ^ murmur3_h1_words(u, k);
}

}  // namespace kh
