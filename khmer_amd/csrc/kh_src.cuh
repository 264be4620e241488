// kh_src.cuh -- k-mer sources of a device batch (included by kh_engine.hip).
//
// A batch is a sub-range of a read set.  Batch-local k-mer j is absolute k-mer
// kbase + j; the base of read r in the packed stream is koff[r] + r*(k-1)
// (reads are packed back to back, every read holds >= 1 k-mer).
//   * fixed-length reads (kpr = k-mers per read != 0): the read of absolute
//     k-mer ja is ja / kpr (Barrett), no offset array is touched;
//   * variable-length reads: an LDS window of the batch's k-mer offsets per
//     tile and a binary search in LDS.
#pragma once
#include "kh_internal.h"

namespace kh {

// Workgroup barrier with an explicit wait for this wave's LDS operations.
// hipcc (ROCm 7.2, gfx950) was observed to emit a loop-header s_barrier with
// no lgkmcnt wait on the back edge, so LDS stores at the end of one iteration
// could land after other waves' LDS atomics of the next (lost counts).
__device__ __forceinline__ void block_sync() {
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0), vmcnt/expcnt untouched
    __syncthreads();
}

__device__ __forceinline__ uint64_t div_barrett(uint64_t x, uint64_t d, uint64_t m) {
    uint64_t q = umulhi64(x, m);
    return (x - q * d >= d) ? q + 1 : q;
}

struct SrcCommon {
    const uint64_t *koff;   // offsets of this batch's reads (absolute values); unused when kpr != 0
    uint64_t nreads;        // reads in this batch (variable-length mode)
    uint64_t kbase;         // absolute index of batch k-mer 0
    uint64_t rbase;         // absolute index of koff[0]'s read
    uint64_t kpr, kpr_m;    // fixed k-mers per read and its Barrett constant (0 = variable)
    double kpr_ip = 0;      // 1 / kpr when every read index is below 2^31 (div_f64), else 0
    int k;
    // read of absolute k-mer index ja (fixed-length reads)
    __device__ __forceinline__ uint64_t read_of(uint64_t ja) const {
        return kpr_ip != 0.0 ? div_f64(ja, kpr, kpr_ip) : div_barrett(ja, kpr, kpr_m);
    }
};

// Every source also splits a hash into fetch() (issue the global loads) and
// finish() (compute from the loaded registers), so a kernel can fetch the next
// tile's k-mers a whole tile ahead of using them.
struct SrcTwoBit : SrcCommon {
    const uint64_t *words;
    static constexpr bool kReads = true;
    __device__ __forceinline__ uint64_t at(uint64_t ja, uint64_t r) const {
        return canonical2(window2(words, ja + r * (uint64_t)(k - 1), k), k);
    }
    struct Pend {
        uint64_t w0, w1;
        uint32_t sh;
    };
    __device__ __forceinline__ Pend fetch(uint64_t ja, uint64_t r) const {
        const uint64_t b = (ja + r * (uint64_t)(k - 1)) * 2;
        return Pend{words[b >> 6], words[(b >> 6) + 1], (uint32_t)(b & 63)};
    }
    __device__ __forceinline__ uint64_t finish(const Pend &p) const {
        const uint64_t x = p.sh ? ((p.w0 << p.sh) | (p.w1 >> (64 - p.sh))) : p.w0;
        return canonical2(x >> (64 - 2 * k), k);
    }
};

// ASCII reads for the Murmur (Counttable family) hash.  rbytes holds every
// read reverse-complemented in place (k_revcomp_reads): the reverse complement
// of the k-mer at read position i is the window at position len - k - i
struct SrcBytes : SrcCommon {
    const uint8_t *bytes;
    const uint8_t *rbytes;
    static constexpr bool kReads = true;
    __device__ __forceinline__ uint64_t at(uint64_t ja, uint64_t r) const {
        const uint64_t pos = ja + r * (uint64_t)(k - 1);
        if (k > MURMUR_WORDS_MAX) return murmur_canonical(bytes + pos, k);
        uint64_t rpos;
        if (kpr) {
            rpos = r * (kpr + (uint64_t)(k - 1)) + (kpr - 1) - (ja - r * kpr);
        } else {
            const uint64_t k0 = koff[r - rbase], nk = koff[r - rbase + 1] - k0;
            rpos = k0 + r * (uint64_t)(k - 1) + (nk - 1) - (ja - k0);
        }
        return murmur_canonical_windows(bytes + pos, rbytes + rpos, k);
    }
    using Pend = uint64_t;   // Murmur reads k bytes: hashed at fetch time
    __device__ __forceinline__ Pend fetch(uint64_t ja, uint64_t r) const { return at(ja, r); }
    __device__ __forceinline__ uint64_t finish(Pend p) const { return p; }
};

struct SrcHashes : SrcCommon {
    const uint64_t *h;
    static constexpr bool kReads = false;
    __device__ __forceinline__ uint64_t at(uint64_t ja, uint64_t) const { return h[ja - kbase]; }
    using Pend = uint64_t;
    __device__ __forceinline__ Pend fetch(uint64_t ja, uint64_t) const { return h[ja - kbase]; }
    __device__ __forceinline__ uint64_t finish(Pend p) const { return p; }
};

// LDS window of read offsets covering k-mer tile [j0, j1) (variable mode)
struct TileReads {
    uint64_t rlo;
    uint32_t n;
};

template <class Src>
__device__ __forceinline__ bool needs_window(const Src &src) {
    if constexpr (!Src::kReads) return false;
    else return src.kpr == 0;
}

// All threads of the block must call this (it synchronises when a window is
// needed; the caller must __syncthreads() itself otherwise).
template <class Src>
__device__ __forceinline__ TileReads load_tile_reads(const Src &src, uint64_t j0, uint64_t j1,
                                                     uint64_t *s_koff, uint64_t *s_meta) {
    TileReads tr{0, 0};
    if (!needs_window(src)) return tr;
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
    block_sync();
    tr.rlo = s_meta[0];
    tr.n = (uint32_t)s_meta[1];
    for (uint32_t t = threadIdx.x; t <= tr.n; t += blockDim.x) s_koff[t] = src.koff[tr.rlo + t];
    block_sync();
    return tr;
}

// hash of batch k-mer j inside a tile
template <class Src>
__device__ __forceinline__ uint64_t kmer_hash(const Src &src, const uint64_t *s_koff, const TileReads &tr,
                                              uint64_t j) {
    const uint64_t ja = j + src.kbase;
    if constexpr (!Src::kReads) {
        return src.at(ja, 0);
    } else {
        uint64_t r;
        if (src.kpr) {
            r = src.read_of(ja);
        } else {
            uint32_t lo = 0, hi = tr.n;
            while (hi - lo > 1) {
                uint32_t mid = (lo + hi) >> 1;
                if (s_koff[mid] <= ja) lo = mid; else hi = mid;
            }
            r = src.rbase + tr.rlo + lo;
        }
        return src.at(ja, r);
    }
}

// fetch half of kmer_hash for sources without a read window (fixed-length
// reads or explicit hashes)
template <class Src>
__device__ __forceinline__ typename Src::Pend kmer_fetch(const Src &src, uint64_t j) {
    const uint64_t ja = j + src.kbase;
    if constexpr (!Src::kReads) return src.fetch(ja, 0);
    else return src.fetch(ja, src.read_of(ja));
}

// hash of batch k-mer j without a tile window (rare paths: bigcount, outputs)
template <class Src>
__device__ __forceinline__ uint64_t kmer_hash_global(const Src &src, uint64_t j) {
    const uint64_t ja = j + src.kbase;
    if constexpr (!Src::kReads) {
        return src.at(ja, 0);
    } else {
        uint64_t r;
        if (src.kpr) {
            r = src.read_of(ja);
        } else {
            uint64_t lo = 0, hi = src.nreads;
            while (hi - lo > 1) {
                uint64_t mid = (lo + hi) >> 1;
                if (src.koff[mid] <= ja) lo = mid; else hi = mid;
            }
            r = src.rbase + lo;
        }
        return src.at(ja, r);
    }
}

// bin of hash h in table i (h mod p_i, storage.hh:577) as a bin of the local
// bin space (table bases P.tbase); false when another shard owns it
__device__ __forceinline__ bool local_bin(const Params &P, int i, uint64_t h, uint64_t *G) {
    const uint64_t b = (P.fm32 ? (uint64_t)mod_f64_32(h, (uint32_t)P.p[i], P.ip[i]) : mod_barrett(h, P.p[i], P.m[i])) - P.lo[i];
    *G = P.tbase[i] + b;
    return b < P.lsz[i];
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

}  // namespace kh
