// kh_host.cpp -- host-side helpers of libkhmer_hip.so: scalar hashing
// utilities (the khmer._khmer module functions), primes, read packing.
#include <immintrin.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "kh_internal.h"

namespace kh {

// twobit_repr (include/oxli/kmer_hash.hh:69-73): A=0 T=1 C=2 else 3
static inline uint64_t repr(unsigned char c) { return c == 'A' ? 0 : c == 'T' ? 1 : c == 'C' ? 2 : 3; }

// _hash (src/oxli/kmer_hash.cc:65-95)
uint64_t hash_twobit(const char *kmer, int k, uint64_t *f, uint64_t *r) {
    if (k > 32) fail(1, "Supplied kmer string doesn't match the underlying k-size.");
    if ((int)strnlen(kmer, (size_t)k) < k) fail(1, "k-mer is too short to hash.");
    uint64_t h = 0;
    for (int i = 0; i < k; i++) h = (h << 2) | repr((unsigned char)kmer[i]);
    uint64_t rc = revcomp2(h, k);
    if (f) *f = h;
    if (r) *r = rc;
    return h < rc ? h : rc;
}

// _revhash (src/oxli/kmer_hash.cc:134-150)
std::string revhash(uint64_t h, int k) {
    std::string s((size_t)k, 'A');
    static const char sym[4] = {'A', 'T', 'C', 'G'};
    for (int i = k - 1; i >= 0; i--) { s[(size_t)i] = sym[h & 3]; h >>= 2; }
    return s;
}

// _revcomp (src/oxli/kmer_hash.cc:152-166)
std::string revcomp(const char *s, size_t len) {
    std::string out(len, ' ');
    for (size_t i = 0; i < len; i++) out[len - 1 - i] = iupac_comp((uint8_t)s[i]);
    return out;
}

// _hash_murmur / _hash_murmur_forward (src/oxli/kmer_hash.cc:177-207)
uint64_t hash_murmur(const char *kmer, int k) { return murmur_canonical((const uint8_t *)kmer, k); }
uint64_t hash_murmur_fwd(const char *kmer, int k) {
    const uint8_t *s = (const uint8_t *)kmer;
    return murmur3_x64_128_h1([&](int i) { return s[i]; }, k);
}

// is_prime / get_n_primes_near_x (include/oxli/hashtable.hh:79-123)
bool is_prime(uint64_t n) {
    if (n < 2) return false;
    if (n == 2) return true;
    if (n % 2 == 0) return false;
    for (unsigned long long i = 3; i < sqrt((double)n) + 1; i += 2)
        if (n % i == 0) return false;
    return true;
}

std::vector<uint64_t> primes_near(uint32_t n, uint64_t x) {
    std::vector<uint64_t> out;
    if (x == 1) { out.push_back(1); return out; }
    uint64_t i = x - 1;
    if (i % 2 == 0) i--;
    while (out.size() != n) {
        if (is_prime(i)) out.push_back(i);
        if (i == 1) break;
        i -= 2;
    }
    return out;
}

// k-mer hash iteration over one string (KmerIterator, src/oxli/kmer_hash.cc:278-343;
// MurmurKmerHashIterator, include/oxli/hashtable.hh:436-491); length = strlen.
void kmer_hashes_host(int hash_kind, int k, const char *seq, size_t len, std::vector<uint64_t> &out) {
    size_t slen = strnlen(seq, len);
    if (slen < (size_t)k || k < 1) return;
    if (hash_kind == MURMUR) {
        for (size_t i = 0; i + (size_t)k <= slen; i++) out.push_back(hash_murmur(seq + i, k));
        return;
    }
    if (k > 32) fail(1, "Supplied kmer string doesn't match the underlying k-size.");
    uint64_t mask = kmer_mask(k), f = 0;
    for (size_t i = 0; i < slen; i++) {
        f = ((f << 2) | repr((unsigned char)seq[i])) & mask;
        if (i + 1 >= (size_t)k) out.push_back(canonical2(f, k));
    }
}

// ---- byte maps -------------------------------------------------------------
struct Maps {
    uint8_t clean2[256], raw2[256], cleanc[256];
    Maps() {
        for (int c = 0; c < 256; c++) {
            raw2[c] = (uint8_t)repr((unsigned char)c);
            // _to_valid_dna (src/oxli/read_parsers.cc:53-69): ACGT/acgt kept
            // (upper-cased), everything else becomes 'A'
            char cc;
            switch (c) {
            case 'A': case 'C': case 'G': case 'T': cc = (char)c; break;
            case 'a': case 'c': case 'g': case 't': cc = (char)(c - 32); break;
            default: cc = 'A';
            }
            cleanc[c] = (uint8_t)cc;
            clean2[c] = (uint8_t)repr((unsigned char)cc);
        }
    }
};
static const Maps g_maps;

// 8 cleaned bases -> 16 bits, first base in the top bits (BMI2 pext; x86-64
// hosts with BMI2, checked once at run time).  A byte b is a valid base iff
// (b | 0x20) is 'a', 'c', 'g' or 't' (exactly upper- and lower-case ACGT);
// its code is ((b >> 1) & 3) with the two bits swapped (A 0, C 2, G 3, T 1),
// anything else cleans to 'A' (0): _to_valid_dna + twobit_repr
// (src/oxli/read_parsers.cc:53-69, include/oxli/kmer_hash.hh:62-70).
__attribute__((target("bmi2"))) static inline uint32_t pack8_clean(uint64_t x) {
    const uint64_t L = 0x0101010101010101ull, H7 = 0x7F7F7F7F7F7F7F7Full;
    const uint64_t v = x | (0x20 * L);
    auto eq = [&](uint64_t c) {   // 0x80 in the bytes of v equal to c
        const uint64_t t = v ^ (c * L);
        return ~(((t & H7) + H7) | t | H7);
    };
    const uint64_t valid = eq('a') | eq('c') | eq('g') | eq('t');
    const uint64_t y = (x >> 1) & (3 * L);
    uint64_t z = ((y & L) << 1) | ((y >> 1) & L);
    z &= (valid >> 7) * 0xFF;
    return (uint32_t)_pext_u64(__builtin_bswap64(z), 3 * L);
}
__attribute__((target("bmi2"))) static size_t pack_body_bmi2(const char *s, size_t len, uint64_t *dst) {
    size_t i = 0, w = 0;
    for (; i + 32 <= len; i += 32, w++) {
        uint64_t q[4];
        memcpy(q, s + i, 32);
        dst[w] = ((uint64_t)pack8_clean(q[0]) << 48) | ((uint64_t)pack8_clean(q[1]) << 32) |
                 ((uint64_t)pack8_clean(q[2]) << 16) | (uint64_t)pack8_clean(q[3]);
    }
    return i;
}
static bool have_bmi2() {
    static const bool v = [] {
        const char *e = getenv("KH_PACK_SCALAR");   // development A/B
        return !(e && atoi(e)) && __builtin_cpu_supports("bmi2");
    }();
    return v;
}

void HostBatch::append(const char *s, size_t len, int k, bool clean) {
    uint64_t nk = len - (uint64_t)k + 1;
    if (hash == MURMUR) {
        const uint8_t *mp = clean ? g_maps.cleanc : nullptr;
        size_t off = bytes.size();
        bytes.resize(off + len);
        if (mp) for (size_t i = 0; i < len; i++) bytes[off + i] = mp[(uint8_t)s[i]];
        else memcpy(bytes.data() + off, s, len);
    } else {
        const uint8_t *mp = clean ? g_maps.clean2 : g_maps.raw2;
        uint64_t need_words = (nbases + len + 31) / 32 + 1;  // +1 padding word
        if (words.size() < need_words) words.resize(std::max<size_t>(need_words, words.size() * 3 / 2 + 1), 0);
        uint64_t p = nbases;
        size_t i = 0;
        // head: fill the partial word
        while (i < len && (p & 31)) {
            words[p >> 5] |= (uint64_t)mp[(uint8_t)s[i]] << (62 - 2 * (p & 31));
            i++; p++;
        }
        // body: 32 bases per word
        if (clean && have_bmi2() && i + 32 <= len) {
            const size_t done = pack_body_bmi2(s + i, len - i, words.data() + (p >> 5));
            i += done;
            p += done;
        }
        while (i + 32 <= len) {
            uint64_t w = 0;
            for (int b = 0; b < 32; b++) w = (w << 2) | mp[(uint8_t)s[i + b]];
            words[p >> 5] = w;
            i += 32; p += 32;
        }
        while (i < len) {
            words[p >> 5] |= (uint64_t)mp[(uint8_t)s[i]] << (62 - 2 * (p & 31));
            i++; p++;
        }
    }
    if (!read_kmers.empty() && read_kmers.back() != nk) uniform = false;
    nbases += len;
    koff.push_back(koff.back() + nk);
    read_kmers.push_back((uint32_t)nk);
}

void HostBatch::merge(const HostBatch &o) {
    if (hash == MURMUR) {
        bytes.insert(bytes.end(), o.bytes.begin(), o.bytes.end());
    } else if (o.nbases) {
        // o's bases start at base nbases: its words shifted right by the
        // offset inside the partial word (bits past nbases are zero)
        const uint64_t p = nbases, nw = (o.nbases + 31) / 32;
        const uint64_t need = (p + o.nbases + 31) / 32 + 1;
        if (words.size() < need) words.resize(need, 0);
        uint64_t *d = words.data() + (p >> 5);
        const unsigned sh = 2 * (unsigned)(p & 31);
        if (sh == 0) {
            memcpy(d, o.words.data(), nw * 8);
        } else {
            for (uint64_t i = 0; i < nw; i++) {
                d[i] |= o.words[i] >> sh;
                d[i + 1] = o.words[i] << (64 - sh);
            }
        }
    }
    const uint64_t base = koff.back();
    for (size_t i = 1; i < o.koff.size(); i++) koff.push_back(base + o.koff[i]);
    if (!read_kmers.empty() && !o.read_kmers.empty() && read_kmers.back() != o.read_kmers.front()) uniform = false;
    uniform = uniform && o.uniform;
    read_kmers.insert(read_kmers.end(), o.read_kmers.begin(), o.read_kmers.end());
    nbases += o.nbases;
}

}  // namespace kh
