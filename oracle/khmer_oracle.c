/*
 * khmer_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Plain-C restatement of the reference oxli hot path.  Every function cites the
 * reference file:line it restates.  Parity is pinned by the reference's own
 * known-answer tests (tests/test_oracle_kats.py); the reference itself could not
 * be executed here.  Never linked into the product library.
 */
#define _GNU_SOURCE
#include "khmer_oracle.h"

#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <string.h>
#include <zlib.h>

#define MAX_KCOUNT 255      /* include/oxli/oxli.hh:81 */
#define MAX_BIGCOUNT 65535  /* include/oxli/oxli.hh:82 */
#define TAG_DENSITY 40      /* include/oxli/oxli.hh:83 */

static __thread char g_err[512];
static void set_err(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}
const char *or_last_error(void) { return g_err; }

/* ------------------------------------------------------------------------ */
/* 2-bit encoding: include/oxli/kmer_hash.hh:62-96 (no KHMER_EXTRA_SANITY_CHECKS,
 * canonical: built without NO_UNIQUE_RC).                          */
static inline uint64_t twobit_repr(unsigned char c) {
    return c == 'A' ? 0 : c == 'T' ? 1 : c == 'C' ? 2 : 3;
}
static inline uint64_t twobit_comp(unsigned char c) {
    return c == 'A' ? 1 : c == 'T' ? 0 : c == 'C' ? 3 : 2;
}
static inline char revtwobit_repr(unsigned n) {
    return n == 0 ? 'A' : n == 1 ? 'T' : n == 2 ? 'C' : 'G';
}

/* _hash: src/oxli/kmer_hash.cc:65-95 */
int or_hash2bit(const char *kmer, int k, uint64_t *fwd, uint64_t *rc, uint64_t *out) {
    if (k > 32) { set_err("Supplied kmer string doesn't match the underlying k-size."); return -1; }
    if ((int)strnlen(kmer, (size_t)k) < k) { set_err("k-mer is too short to hash."); return -1; }
    uint64_t h = twobit_repr((unsigned char)kmer[0]);
    uint64_t r = twobit_comp((unsigned char)kmer[k - 1]);
    for (int i = 1, j = k - 2; i < k; i++, j--) {
        h = (h << 2) | twobit_repr((unsigned char)kmer[i]);
        r = (r << 2) | twobit_comp((unsigned char)kmer[j]);
    }
    if (fwd) *fwd = h;
    if (rc) *rc = r;
    if (out) *out = h < r ? h : r;
    return 0;
}

/* _revhash: src/oxli/kmer_hash.cc:134-150 */
void or_revhash(uint64_t h, int k, char *out) {
    for (int i = k - 1; i >= 0; i--) {
        out[i] = revtwobit_repr((unsigned)(h & 3));
        h >>= 2;
    }
    out[k] = 0;
}

/* complement table of _revcomp: src/oxli/kmer_hash.cc:52-55 (IUPAC aware,
 * upper- and lower-case map to upper-case complements, others to ' ') */
static char comp_tbl[256];
static void init_comp_tbl(void) {
    static int done = 0;
    if (done) return;
    for (int i = 0; i < 256; i++) comp_tbl[i] = ' ';
    const char *from = "ABCDFGHKMNRSTUVWY";
    const char *to   = "TVGHFCDMKNYSAABWR";
    for (int i = 0; from[i]; i++) {
        comp_tbl[(unsigned char)from[i]] = to[i];
        comp_tbl[(unsigned char)(from[i] + 32)] = to[i];
    }
    comp_tbl['z'] = 0; /* reference reads the table's NUL terminator there */
    done = 1;
}

/* _revcomp: src/oxli/kmer_hash.cc:152-166 */
void or_revcomp(const char *in, size_t len, char *out) {
    init_comp_tbl();
    for (size_t i = 0; i < len; i++) out[len - 1 - i] = comp_tbl[(unsigned char)in[i]];
    out[len] = 0;
}

/* MurmurHash3_x64_128 (public-domain algorithm by A. Appleby; vendored by the
 * reference as third-party/smhasher/MurmurHash3.cc:67-144).  Restated from the
 * published algorithm; little-endian block reads. */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
void or_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t out[2]) {
    const uint8_t *data = (const uint8_t *)key;
    const int nblocks = len / 16;
    uint64_t h1 = seed, h2 = seed;
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    for (int i = 0; i < nblocks; i++) {
        uint64_t k1, k2;
        memcpy(&k1, data + 16 * i, 8);
        memcpy(&k2, data + 16 * i + 8, 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t *tail = data + nblocks * 16;
    uint64_t k1 = 0, k2 = 0;
    switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)tail[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)tail[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)tail[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)tail[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)tail[9] << 8;   /* fallthrough */
    case 9:  k2 ^= (uint64_t)tail[8];
             k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; /* fallthrough */
    case 8:  k1 ^= (uint64_t)tail[7] << 56; /* fallthrough */
    case 7:  k1 ^= (uint64_t)tail[6] << 48; /* fallthrough */
    case 6:  k1 ^= (uint64_t)tail[5] << 40; /* fallthrough */
    case 5:  k1 ^= (uint64_t)tail[4] << 32; /* fallthrough */
    case 4:  k1 ^= (uint64_t)tail[3] << 24; /* fallthrough */
    case 3:  k1 ^= (uint64_t)tail[2] << 16; /* fallthrough */
    case 2:  k1 ^= (uint64_t)tail[1] << 8;  /* fallthrough */
    case 1:  k1 ^= (uint64_t)tail[0];
             k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    out[0] = h1; out[1] = h2;
}

/* _hash_murmur: src/oxli/kmer_hash.cc:177-198 */
uint64_t or_hash_murmur(const char *kmer, int k) {
    uint64_t out[2];
    char rev[256];
    or_murmur3_x64_128(kmer, k, 0, out);
    uint64_t h = out[0];
    or_revcomp(kmer, (size_t)k, rev);
    if (memcmp(rev, kmer, (size_t)k) == 0) return h;  /* self-complement */
    or_murmur3_x64_128(rev, k, 0, out);
    return h ^ out[0];
}

/* _hash_murmur_forward: src/oxli/kmer_hash.cc:200-207 */
uint64_t or_hash_murmur_forward(const char *kmer, int k) {
    uint64_t out[2];
    or_murmur3_x64_128(kmer, k, 0, out);
    return out[0];
}

/* ------------------------------------------------------------------------ */
/* primes: include/oxli/hashtable.hh:79-123 */
int or_is_prime(uint64_t n) {
    if (n < 2) return 0;
    if (n == 2) return 1;
    if (n % 2 == 0) return 0;
    for (unsigned long long i = 3; i < sqrt((double)n) + 1; i += 2)
        if (n % i == 0) return 0;
    return 1;
}

int or_get_n_primes_near_x(uint32_t n, uint64_t x, uint64_t *out) {
    int found = 0;
    if (x == 1) { out[0] = 1; return 1; }
    uint64_t i = x - 1;
    if (i % 2 == 0) i--;
    while ((uint32_t)found != n) {
        if (or_is_prime(i)) out[found++] = i;
        if (i == 1) break;
        i -= 2;
    }
    return found;
}

/* ------------------------------------------------------------------------ */
/* small open-addressing maps for bigcounts (u64->u16) and tags (u64 set) */
typedef struct { uint64_t *keys; uint16_t *vals; uint8_t *used; uint64_t cap, n; } u64map;

static void map_grow(u64map *m);
static uint64_t mix(uint64_t x) { return fmix64(x + 0x9e3779b97f4a7c15ULL); }
static int64_t map_find(const u64map *m, uint64_t key) {
    if (!m->cap) return -1;
    uint64_t i = mix(key) & (m->cap - 1);
    while (m->used[i]) {
        if (m->keys[i] == key) return (int64_t)i;
        i = (i + 1) & (m->cap - 1);
    }
    return -1;
}
static uint64_t map_slot(u64map *m, uint64_t key, int *created) {
    if ((m->n + 1) * 2 > m->cap) map_grow(m);
    uint64_t i = mix(key) & (m->cap - 1);
    while (m->used[i]) {
        if (m->keys[i] == key) { *created = 0; return i; }
        i = (i + 1) & (m->cap - 1);
    }
    m->used[i] = 1; m->keys[i] = key; m->vals[i] = 0; m->n++;
    *created = 1;
    return i;
}
static void map_grow(u64map *m) {
    u64map nm;
    nm.cap = m->cap ? m->cap * 2 : 64;
    nm.n = 0;
    nm.keys = calloc(nm.cap, 8); nm.vals = calloc(nm.cap, 2); nm.used = calloc(nm.cap, 1);
    for (uint64_t i = 0; i < m->cap; i++)
        if (m->used[i]) {
            int c;
            uint64_t s = map_slot(&nm, m->keys[i], &c);
            nm.vals[s] = m->vals[i];
        }
    free(m->keys); free(m->vals); free(m->used);
    *m = nm;
}
static void map_free(u64map *m) { free(m->keys); free(m->vals); free(m->used); memset(m, 0, sizeof *m); }
static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* ------------------------------------------------------------------------ */
struct or_table {
    int kind, hash, k, n;
    uint64_t sizes[64];
    uint64_t nbytes[64];
    uint8_t *tab[64];
    uint64_t occupied, unique;
    int use_bigcount;
    u64map bigcounts;
    u64map tags;
};

or_table *or_table_new(int kind, int hash, int k, const uint64_t *sizes, int n) {
    if (n < 1 || n > 64) { set_err("bad number of tables"); return NULL; }
    or_table *t = calloc(1, sizeof *t);
    t->kind = kind; t->hash = hash; t->k = k; t->n = n;
    for (int i = 0; i < n; i++) {
        t->sizes[i] = sizes[i];
        /* allocation sizes: storage.hh:127-140 (bit), :297-310 (nibble), :502-511 (byte) */
        t->nbytes[i] = kind == OR_BIT ? sizes[i] / 8 + 1 : kind == OR_NIBBLE ? sizes[i] / 2 + 1 : sizes[i];
        /* allocate + memset like the reference (storage.hh:502-511): pages are
         * touched at construction, not inside a timed consume */
        /* 2 MB aligned and backed by transparent huge pages where the kernel
         * allows it: a GB table's random adds miss the TLB on 4 KB pages */
        void *mem = NULL;
        const size_t want = t->nbytes[i] ? t->nbytes[i] : 1;
        if (posix_memalign(&mem, (size_t)2 << 20, want) != 0) mem = NULL;
        t->tab[i] = mem;
        if (!t->tab[i]) { set_err("out of memory"); or_table_free(t); return NULL; }
        if (want >= ((size_t)2 << 20)) madvise(mem, want, MADV_HUGEPAGE);
        memset(t->tab[i], 0, t->nbytes[i] ? t->nbytes[i] : 1);
        for (uint64_t b = 0; b < t->nbytes[i]; b += 4096) ((volatile uint8_t *)t->tab[i])[b] = 0;
    }
    return t;
}

void or_table_free(or_table *t) {
    if (!t) return;
    for (int i = 0; i < t->n; i++) free(t->tab[i]);
    map_free(&t->bigcounts); map_free(&t->tags);
    free(t);
}

void or_set_bigcount(or_table *t, int on) { t->use_bigcount = on; }
uint64_t or_n_unique(const or_table *t) { return t->unique; }
uint64_t or_n_occupied(const or_table *t) { return t->occupied; }
uint64_t or_table_nbytes(const or_table *t, int i) { return t->nbytes[i]; }
const uint8_t *or_table_data(const or_table *t, int i) { return t->tab[i]; }
uint64_t or_bigcount_size(const or_table *t) { return t->bigcounts.n; }
void or_bigcount_export(const or_table *t, uint64_t *keys, uint16_t *vals) {
    uint64_t j = 0;
    for (uint64_t i = 0; i < t->bigcounts.cap; i++)
        if (t->bigcounts.used[i]) keys[j++] = t->bigcounts.keys[i];
    qsort(keys, j, 8, cmp_u64);
    for (uint64_t i = 0; i < j; i++) vals[i] = t->bigcounts.vals[map_find(&t->bigcounts, keys[i])];
}

/* bins of hash h: bin_i = h % p_i (storage.hh:177, 321, 576) */
static inline void bins_of(const or_table *t, uint64_t h, uint64_t *bins) {
    for (int i = 0; i < t->n; i++) bins[i] = h % t->sizes[i];
}

/* BitStorage::test_and_set_bits: include/oxli/storage.hh:172-199 */
static int bit_add_b(or_table *t, const uint64_t *bins) {
    int is_new = 0;
    for (int i = 0; i < t->n; i++) {
        uint64_t bin = bins[i];
        uint8_t bit = (uint8_t)(1u << (bin % 8));
        uint8_t orig = t->tab[i][bin / 8];
        t->tab[i][bin / 8] = orig | bit;
        if (!(orig & bit)) {
            if (i == 0) t->occupied++;
            is_new = 1;
        }
    }
    if (is_new) t->unique++;
    return is_new;
}

/* NibbleStorage::add: include/oxli/storage.hh:320-359 (even bin -> high nibble) */
static int nibble_add_b(or_table *t, const uint64_t *bins) {
    int is_new = 0;
    for (int i = 0; i < t->n; i++) {
        uint64_t bin = bins[i];
        uint64_t idx = bin / 2;
        uint8_t mask = (bin % 2) ? 0x0F : 0xF0;
        int shift = (bin % 2) ? 0 : 4;
        uint8_t cur = (uint8_t)((t->tab[i][idx] & mask) >> shift);
        if (!is_new && cur == 0) {
            is_new = 1;
            if (i == 0) t->occupied++;
        }
        if (cur == 15) continue;
        uint8_t nc = (uint8_t)((cur + 1) << shift);
        t->tab[i][idx] = (uint8_t)((t->tab[i][idx] & ~mask) | (nc & mask));
    }
    if (is_new) t->unique++;
    return is_new;
}

/* ByteStorage::add: include/oxli/storage.hh:571-624 */
static int byte_add_b(or_table *t, uint64_t h, const uint64_t *bins) {
    int is_new = 0;
    int n_full = 0;
    for (int i = 0; i < t->n; i++) {
        uint64_t bin = bins[i];
        uint8_t cur = t->tab[i][bin];
        if (!is_new && cur == 0) {
            is_new = 1;
            if (i == 0) t->occupied++;
        }
        if (cur < MAX_KCOUNT) t->tab[i][bin] = (uint8_t)(cur + 1);
        else n_full++;
    }
    if (n_full == t->n && t->use_bigcount) {
        int created;
        uint64_t s = map_slot(&t->bigcounts, h, &created);
        if (t->bigcounts.vals[s] == 0) t->bigcounts.vals[s] = MAX_KCOUNT + 1;
        else if (t->bigcounts.vals[s] < MAX_BIGCOUNT) t->bigcounts.vals[s]++;
    }
    if (is_new) t->unique++;
    return is_new;
}

static int add_b(or_table *t, uint64_t h, const uint64_t *bins) {
    switch (t->kind) {
    case OR_BIT: return bit_add_b(t, bins);
    case OR_NIBBLE: return nibble_add_b(t, bins);
    default: return byte_add_b(t, h, bins);
    }
}
static int bit_add(or_table *t, uint64_t h) {
    uint64_t b[64];
    bins_of(t, h, b);
    return bit_add_b(t, b);
}

int or_add(or_table *t, uint64_t h) {
    uint64_t b[64];
    bins_of(t, h, b);
    return add_b(t, h, b);
}

/* get_count: storage.hh:206-219 (bit), :362-379 (nibble), :627-649 (byte) */
int or_get(const or_table *t, uint64_t h) {
    if (t->kind == OR_BIT) {
        for (int i = 0; i < t->n; i++) {
            uint64_t bin = h % t->sizes[i];
            if (!(t->tab[i][bin / 8] & (1u << (bin % 8)))) return 0;
        }
        return 1;
    }
    if (t->kind == OR_NIBBLE) {
        int mn = 15;
        for (int i = 0; i < t->n; i++) {
            uint64_t bin = h % t->sizes[i];
            int c = (bin % 2) ? (t->tab[i][bin / 2] & 0x0F) : (t->tab[i][bin / 2] >> 4);
            if (c < mn) mn = c;
        }
        return mn;
    }
    int mn = MAX_KCOUNT;
    for (int i = 0; i < t->n; i++) {
        int c = t->tab[i][h % t->sizes[i]];
        if (c < mn) mn = c;
    }
    if (mn == MAX_KCOUNT && t->use_bigcount) {
        int64_t s = map_find(&t->bigcounts, h);
        if (s >= 0) mn = t->bigcounts.vals[s];
    }
    return mn;
}

/* test_and_set_bits: bit storage returns is_new (storage.hh:172-199); byte and
 * nibble return !get_count-before then add (storage.hh:254-258, 564-569) */
int or_test_and_set(or_table *t, uint64_t h) {
    if (t->kind == OR_BIT) return bit_add(t, h);
    int x = or_get(t, h);
    or_add(t, h);
    return !x;
}

/* ------------------------------------------------------------------------ */
/* k-mer iteration.  2-bit: KmerIterator src/oxli/kmer_hash.cc:278-343 (rolling,
 * length = strlen); Murmur: MurmurKmerHashIterator include/oxli/hashtable.hh:436-491. */
typedef void (*kmer_cb)(void *ctx, uint64_t h);

static uint64_t iterate_kmers(const or_table *t, const char *s, size_t len, kmer_cb cb, void *ctx) {
    size_t slen = strnlen(s, len);
    int k = t->k;
    if (slen < (size_t)k) return 0;
    uint64_t n = 0;
    if (t->hash == OR_HASH_MURMUR) {
        for (size_t i = 0; i + (size_t)k <= slen; i++) {
            cb(ctx, or_hash_murmur(s + i, k));
            n++;
        }
        return n;
    }
    uint64_t mask = (k == 32) ? ~0ULL : ((1ULL << (2 * k)) - 1);
    int nbits_sub_1 = 2 * k - 2;
    uint64_t f = 0, r = 0, h;
    or_hash2bit(s, k, &f, &r, &h);
    cb(ctx, h);
    n++;
    for (size_t idx = (size_t)k; idx < slen; idx++) {
        unsigned char c = (unsigned char)s[idx];
        f = ((f << 2) | twobit_repr(c)) & mask;
        r = (r >> 2) | (twobit_comp(c) << nbits_sub_1);
        cb(ctx, f < r ? f : r);
        n++;
    }
    return n;
}

static void cb_add(void *ctx, uint64_t h) { or_add((or_table *)ctx, h); }

/* Hashtable::consume_string: src/oxli/hashtable.cc:280-294 */
uint32_t or_consume_string(or_table *t, const char *s, size_t len) {
    return (uint32_t)iterate_kmers(t, s, len, cb_add, t);
}

typedef struct { uint64_t *out; uint64_t n; } hash_sink;
static void cb_store(void *ctx, uint64_t h) { hash_sink *hs = ctx; hs->out[hs->n++] = h; }

/* Hashtable::get_kmer_hashes: src/oxli/hashtable.cc:378-388 */
uint64_t or_kmer_hashes(const or_table *t, const char *s, size_t len, uint64_t *out) {
    hash_sink hs = { out, 0 };
    return iterate_kmers(t, s, len, cb_store, &hs);
}

/* Read cleaning: _to_valid_dna src/oxli/read_parsers.cc:53-69 */
static inline char clean_base(unsigned char c) {
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': return (char)c;
    case 'a': case 'c': case 'g': case 't': return (char)(c - 32);
    default: return 'A';
    }
}

/* Hashgraph::consume_sequence_and_tag: src/oxli/hashgraph.cc:200-271 */
typedef struct { or_table *t; uint64_t n_consumed; unsigned since; uint64_t last; } tag_ctx;
static void cb_tag(void *ctx, uint64_t h) {
    tag_ctx *c = ctx;
    int is_new = or_test_and_set(c->t, h);
    if (is_new) c->n_consumed++;
    if (is_new) {
        c->since++;
    } else if (map_find(&c->t->tags, h) >= 0) {
        c->since = 1;
    } else {
        c->since++;
    }
    if (c->since >= TAG_DENSITY) {
        int created;
        map_slot(&c->t->tags, h, &created);
        c->since = 1;
    }
    c->last = h;
}
static uint64_t consume_and_tag(or_table *t, const char *s, size_t len) {
    tag_ctx c = { t, 0, TAG_DENSITY / 2 + 1, 0 };
    iterate_kmers(t, s, len, cb_tag, &c);
    /* the reference inserts the (possibly uninitialised, read shorter than k)
     * last k-mer; we only do so when at least one k-mer was seen */
    if (c.since >= TAG_DENSITY / 2 - 1 && strnlen(s, len) >= (size_t)t->k) {
        int created;
        map_slot(&t->tags, c.last, &created);
    }
    return c.n_consumed;
}
uint64_t or_n_tags(const or_table *t) { return t->tags.n; }
void or_tags_export(const or_table *t, uint64_t *out) {
    uint64_t j = 0;
    for (uint64_t i = 0; i < t->tags.cap; i++)
        if (t->tags.used[i]) out[j++] = t->tags.keys[i];
    qsort(out, j, 8, cmp_u64);
}

/* ------------------------------------------------------------------------ */
/* FASTA/FASTQ reader.  Record semantics of FastxReader::get_next_read
 * (src/oxli/read_parsers.cc:329-372) over the vendored seqan record reader
 * (third-party/seqan/core/include/seqan/seq_io/read_fasta_fastq.h:300-650):
 *  - format fixed by the file's first character ('>' FASTA, '@' FASTQ);
 *  - name = rest of the header line (readLine: \n, \r\n or \r);
 *  - sequence = non-space chars of the following lines, up to a line that
 *    starts with '>' (FASTA) / '+' (FASTQ); the first sequence line is never a
 *    stop line (afterEol starts false);
 *  - FASTQ: '+' line must be empty or equal the name, then exactly len(seq)
 *    non-space quality chars (EOF before that is tolerated), rest of line skipped;
 *  - empty sequence -> "Sequence is empty"; quality length mismatch once
 *    qualities were seen -> "Sequence and quality lengths differ";
 *    malformed record -> StreamReadError (OSError in Python).
 * Input may be gzip-compressed (zlib reads plain files transparently). */
struct or_parser {
    gzFile gz;
    unsigned char buf[1 << 16]; int pos, len;
    int fastq;
    char *name; size_t name_len, name_cap;
    char *seq; size_t seq_len, seq_cap;
    char *qual; size_t qual_len, qual_cap;
    char *tmp; size_t tmp_len, tmp_cap;
    uint64_t num_reads;
    int have_qualities;
};

static int cr_peek(or_parser *p) {
    if (p->pos < p->len) return p->buf[p->pos];
    p->len = gzread(p->gz, p->buf, sizeof p->buf);
    p->pos = 0;
    if (p->len <= 0) { p->len = 0; return -1; }
    return p->buf[0];
}
static void cr_next(or_parser *p) { p->pos++; }
static int cr_at_end(or_parser *p) { return cr_peek(p) < 0; }

static void buf_append(char **b, size_t *len, size_t *cap, const char *s, size_t n) {
    if (*len + n + 1 > *cap) {
        size_t nc = (*cap ? *cap : 256);
        while (nc < *len + n + 1) nc *= 2;
        *b = realloc(*b, nc);
        *cap = nc;
    }
    memcpy(*b + *len, s, n);
    *len += n;
    (*b)[*len] = 0;
}
static void buf_push(char **b, size_t *len, size_t *cap, char c) { buf_append(b, len, cap, &c, 1); }

/* seqan readLine: tokenize.h:1519-1560 */
static void cr_read_line(or_parser *p, char **b, size_t *len, size_t *cap) {
    buf_append(b, len, cap, "", 0);
    int c;
    while ((c = cr_peek(p)) >= 0) {
        if (c == '\n') { cr_next(p); return; }
        if (c == '\r') {
            cr_next(p);
            if (cr_peek(p) == '\n') cr_next(p);
            return;
        }
        buf_push(b, len, cap, (char)c);
        cr_next(p);
    }
}
/* seqan skipLine: tokenize.h:1626-1637 */
static void cr_skip_line(or_parser *p) {
    int c;
    while ((c = cr_peek(p)) >= 0 && c != '\n') cr_next(p);
    if (c == '\n') cr_next(p);
}

or_parser *or_parser_open(const char *path) {
    gzFile gz = gzopen(path, "rb");
    if (!gz) {
        set_err("File %s contains badly formatted sequence or does not exist.", path);
        return NULL;
    }
    or_parser *p = calloc(1, sizeof *p);
    p->gz = gz;
    int c = cr_peek(p);
    if (c < 0) {
        set_err("File %s does not contain any sequences!", path);
        or_parser_close(p);
        return NULL;
    }
    if (c != '>' && c != '@') {
        set_err("File %s contains badly formatted sequence or does not exist.", path);
        or_parser_close(p);
        return NULL;
    }
    p->fastq = (c == '@');
    return p;
}

/* seqan readRecord (FASTA / FASTQ with qualities) -> 0 ok, -1 invalid format */
static int read_record(or_parser *p) {
    p->name_len = p->seq_len = p->qual_len = 0;
    buf_append(&p->name, &p->name_len, &p->name_cap, "", 0);
    buf_append(&p->seq, &p->seq_len, &p->seq_cap, "", 0);
    buf_append(&p->qual, &p->qual_len, &p->qual_cap, "", 0);
    char marker = p->fastq ? '@' : '>';
    char stop = p->fastq ? '+' : '>';
    if (cr_peek(p) != marker) return -1;
    cr_next(p);
    if (cr_at_end(p)) return 0;
    cr_read_line(p, &p->name, &p->name_len, &p->name_cap);
    if (cr_at_end(p)) return 0;
    int after_eol = 0, c;
    while ((c = cr_peek(p)) >= 0) {
        if (c == '\r' || c == '\n') { after_eol = 1; cr_next(p); continue; }
        if (after_eol && c == stop) break;
        if (!isspace(c)) buf_push(&p->seq, &p->seq_len, &p->seq_cap, (char)c);
        after_eol = 0;
        cr_next(p);
    }
    if (!p->fastq) return 0;
    if (cr_at_end(p)) return 0;
    if (cr_peek(p) != '+') return -1;
    cr_next(p);
    if (cr_at_end(p)) return 0;
    p->tmp_len = 0;
    cr_read_line(p, &p->tmp, &p->tmp_len, &p->tmp_cap);
    if (p->tmp_len && strcmp(p->tmp, p->name) != 0) return -1;
    if (cr_at_end(p)) return 0;
    while (p->qual_len < p->seq_len && (c = cr_peek(p)) >= 0) {
        if (!isspace(c)) buf_push(&p->qual, &p->qual_len, &p->qual_cap, (char)c);
        cr_next(p);
    }
    if (p->qual_len == p->seq_len) cr_skip_line(p);
    return 0;
}

int or_parser_next(or_parser *p, const char **name, const char **seq, const char **qual,
                   size_t *seqlen, size_t *quallen) {
    if (cr_at_end(p)) return 0;
    if (read_record(p) != 0) { set_err("Generic StreamReadError error"); return -3; }
    if (p->num_reads == 0 && p->qual_len != 0) p->have_qualities = 1;
    if (p->seq_len == 0) { set_err("Sequence is empty"); return -1; }
    if (p->have_qualities && p->seq_len != p->qual_len) {
        set_err("Sequence and quality lengths differ");
        return -1;
    }
    p->num_reads++;
    *name = p->name; *seq = p->seq; *qual = p->qual;
    *seqlen = p->seq_len; *quallen = p->qual_len;
    return 1;
}

uint64_t or_parser_num_reads(const or_parser *p) { return p->num_reads; }
void or_parser_close(or_parser *p) {
    if (!p) return;
    if (p->gz) gzclose(p->gz);
    free(p->tmp); free(p->name); free(p->seq); free(p->qual);
    free(p);
}

/* Hashtable::consume_seqfile src/oxli/hashtable.cc:125-150 and
 * Hashgraph::consume_seqfile_and_tag src/oxli/hashgraph.cc:290-320 */
int or_consume_fastx(or_table *t, const char *path, int mode, uint32_t *reads, uint64_t *kmers) {
    or_parser *p = or_parser_open(path);
    *reads = 0; *kmers = 0;
    if (!p) return -1;
    const char *name, *seq, *qual;
    size_t sl, ql;
    char *clean = NULL;
    size_t clean_cap = 0;
    int rc;
    while ((rc = or_parser_next(p, &name, &seq, &qual, &sl, &ql)) == 1) {
        if (sl + 1 > clean_cap) { clean_cap = (sl + 1) * 2; clean = realloc(clean, clean_cap); }
        for (size_t i = 0; i < sl; i++) clean[i] = clean_base((unsigned char)seq[i]);
        clean[sl] = 0;
        if (mode == 1) *kmers += consume_and_tag(t, clean, sl);
        else *kmers += or_consume_string(t, clean, sl);
        (*reads)++;
    }
    free(clean);
    or_parser_close(p);
    return rc == -3 ? -3 : (rc < 0 ? -2 : 0);
}

/* Hashtable::consume_seqfile_with_mask / _banding / _banding_with_mask:
 * src/oxli/hashtable.cc:152-274; band interval: compute_band_interval
 * src/oxli/kmer_hash.cc:262-276 (u64 wraparound kept).  num_bands == 0: no
 * banding; mask == NULL: no mask.  Returns -4 for band > num_bands. */
typedef struct {
    or_table *t;
    const or_table *mask;
    int band;
    uint64_t lo, hi;
    uint32_t threshold;
    int consume_masked;
    uint64_t n;
} filt_ctx;
static void cb_filtered(void *ctx, uint64_t h) {
    filt_ctx *f = ctx;
    if (f->band && !(h >= f->lo && h < f->hi)) return;
    if (f->mask) {
        uint32_t c = (uint32_t)or_get(f->mask, h);
        if (!(f->consume_masked ? c >= f->threshold : c <= f->threshold)) return;
    }
    or_add(f->t, h);
    f->n++;
}
int or_consume_fastx_filtered(or_table *t, const char *path, uint32_t num_bands, uint32_t band,
                              const or_table *mask, uint32_t threshold, int consume_masked,
                              uint32_t *reads, uint64_t *kmers) {
    *reads = 0; *kmers = 0;
    filt_ctx f = { t, mask, num_bands != 0, 0, 0, threshold, consume_masked, 0 };
    if (num_bands) {
        if (band > num_bands) {
            set_err("'band' must be in the interval [0, 'num_bands'), %u not in [0, %u)", band, num_bands);
            return -4;
        }
        uint64_t bs = UINT64_MAX / num_bands;
        f.lo = bs * band;
        f.hi = bs * (uint64_t)(band + 1);
    }
    or_parser *p = or_parser_open(path);
    if (!p) return -1;
    const char *name, *seq, *qual;
    size_t sl, ql;
    char *clean = NULL;
    size_t cap = 0;
    int rc;
    while ((rc = or_parser_next(p, &name, &seq, &qual, &sl, &ql)) == 1) {
        if (sl + 1 > cap) { cap = (sl + 1) * 2; clean = realloc(clean, cap); }
        for (size_t i = 0; i < sl; i++) clean[i] = clean_base((unsigned char)seq[i]);
        clean[sl] = 0;
        iterate_kmers(t, clean, sl, cb_filtered, &f);
        (*reads)++;
    }
    *kmers = f.n;
    free(clean);
    or_parser_close(p);
    return rc == -3 ? -3 : (rc < 0 ? -2 : 0);
}

uint64_t or_consume_batch(or_table *t, const char *seqs, const uint64_t *offs, uint64_t nreads) {
    uint64_t total = 0;
    char *clean = NULL;
    size_t cap = 0;
    for (uint64_t r = 0; r < nreads; r++) {
        size_t len = (size_t)(offs[r + 1] - offs[r]);
        if (len + 1 > cap) { cap = (len + 1) * 2; clean = realloc(clean, cap); }
        for (size_t i = 0; i < len; i++) clean[i] = clean_base((unsigned char)seqs[offs[r] + i]);
        clean[len] = 0;
        total += or_consume_string(t, clean, len);
    }
    free(clean);
    return total;
}


/* Hashtable::abundance_distribution: src/oxli/hashtable.cc:451-493.
 * dist must hold 65536 entries. */
typedef struct { or_table *t, *tracking; uint64_t *dist; } abund_ctx;
static void cb_abund(void *ctx, uint64_t h) {
    abund_ctx *a = ctx;
    if (!or_get(a->tracking, h)) {
        or_add(a->tracking, h);
        a->dist[or_get(a->t, h)]++;
    }
}
int or_abundance_distribution(or_table *t, or_table *tracking, const char *path, uint64_t *dist) {
    memset(dist, 0, 65536 * sizeof(uint64_t));
    or_parser *p = or_parser_open(path);
    if (!p) return -1;
    const char *name, *seq, *qual;
    size_t sl, ql;
    char *clean = NULL;
    size_t cap = 0;
    int rc;
    abund_ctx a = { t, tracking, dist };
    while ((rc = or_parser_next(p, &name, &seq, &qual, &sl, &ql)) == 1) {
        if (sl + 1 > cap) { cap = (sl + 1) * 2; clean = realloc(clean, cap); }
        for (size_t i = 0; i < sl; i++) clean[i] = clean_base((unsigned char)seq[i]);
        clean[sl] = 0;
        iterate_kmers(t, clean, sl, cb_abund, &a);
    }
    free(clean);
    or_parser_close(p);
    return rc == -3 ? -3 : (rc < 0 ? -2 : 0);
}

/* ------------------------------------------------------------------------ */
/* Hashtable::get_median_count: src/oxli/hashtable.cc:299-328.  float32, the
 * reference's sequential summation order, no contraction (compiled with
 * -ffp-contract=off). */
typedef struct { const or_table *t; uint16_t *counts; uint64_t n; } cnt_sink;
static void cb_count(void *ctx, uint64_t h) {
    cnt_sink *c = ctx;
    c->counts[c->n++] = (uint16_t)or_get(c->t, h);
}
static int cmp_u16(const void *a, const void *b) {
    return (int)*(const uint16_t *)a - (int)*(const uint16_t *)b;
}
int or_median(const or_table *t, const char *s, size_t len, uint16_t *med, float *avg, float *sd) {
    uint16_t *counts = malloc((len + 1) * sizeof(uint16_t));
    cnt_sink c = { t, counts, 0 };
    iterate_kmers(t, s, len, cb_count, &c);
    if (!c.n) { free(counts); set_err("no k-mer counts for this string; too short?"); return -1; }
    float average = 0;
    for (uint64_t i = 0; i < c.n; i++) average += counts[i];
    average /= (float)c.n;
    float stddev = 0;
    for (uint64_t i = 0; i < c.n; i++) {
        float d = (float)counts[i] - average;
        stddev += d * d;
    }
    stddev /= (float)c.n;
    stddev = sqrtf(stddev);
    qsort(counts, c.n, sizeof(uint16_t), cmp_u16);
    *med = counts[c.n / 2];
    *avg = average;
    *sd = stddev;
    free(counts);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* file writers: src/oxli/storage.cc:99-136 (bit), 582-638 (byte), 772-803
 * (nibble); layout doc/dev/binary-file-formats.rst.  Bigcount pairs are written
 * in ascending key order (the reference writes unordered_map order). */
int or_save(const or_table *t, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f) { set_err("%s", strerror(errno)); return -1; }
    unsigned char version = 4;
    unsigned char type = (unsigned char)t->kind;
    uint32_t k = (uint32_t)t->k;
    unsigned char n = (unsigned char)t->n;
    uint64_t occ = t->occupied;
    fwrite("OXLI", 1, 4, f);
    fwrite(&version, 1, 1, f);
    fwrite(&type, 1, 1, f);
    if (t->kind == OR_BYTE) {
        unsigned char bc = t->use_bigcount ? 1 : 0;
        fwrite(&bc, 1, 1, f);
    }
    fwrite(&k, 4, 1, f);
    fwrite(&n, 1, 1, f);
    fwrite(&occ, 8, 1, f);
    for (int i = 0; i < t->n; i++) {
        uint64_t sz = t->sizes[i];
        fwrite(&sz, 8, 1, f);
        fwrite(t->tab[i], 1, t->nbytes[i], f);
    }
    if (t->kind == OR_BYTE) {
        uint64_t nb = t->bigcounts.n;
        fwrite(&nb, 8, 1, f);
        if (nb) {
            uint64_t *keys = malloc(nb * 8);
            uint16_t *vals = malloc(nb * 2);
            or_bigcount_export(t, keys, vals);
            for (uint64_t i = 0; i < nb; i++) { fwrite(&keys[i], 8, 1, f); fwrite(&vals[i], 2, 1, f); }
            free(keys); free(vals);
        }
    }
    fclose(f);
    return 0;
}

/* Hashgraph::save_tagset: src/oxli/hashgraph.cc:55-88 (std::set -> ascending) */
int or_save_tagset(const or_table *t, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f) { set_err("%s", strerror(errno)); return -1; }
    unsigned char version = 4, type = 3;
    uint32_t k = (uint32_t)t->k;
    uint64_t n = t->tags.n;
    uint32_t density = TAG_DENSITY;
    fwrite("OXLI", 1, 4, f);
    fwrite(&version, 1, 1, f);
    fwrite(&type, 1, 1, f);
    fwrite(&k, 4, 1, f);
    fwrite(&n, 8, 1, f);
    fwrite(&density, 4, 1, f);
    uint64_t *tags = malloc((n ? n : 1) * 8);
    or_tags_export(t, tags);
    fwrite(tags, 8, n, f);
    free(tags);
    fclose(f);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline with threads: the reference's -T>1 mode (storage.hh:571-624):
 * per-bin atomic increments; read-then-increment races are tolerated exactly as
 * the reference tolerates them.  Used only by bench.py's cpu_baseline leg. */
typedef struct {
    or_table *t; const char *seqs; const uint64_t *offs; uint64_t r0, r1; uint64_t kmers;
} mt_job;

static void mt_add(or_table *t, uint64_t h) {
    for (int i = 0; i < t->n; i++) {
        uint64_t bin = h % t->sizes[i];
        if (t->kind == OR_BIT) {
            uint8_t bit = (uint8_t)(1u << (bin % 8));
            uint8_t orig = __sync_fetch_and_or(&t->tab[i][bin / 8], bit);
            if (!(orig & bit) && i == 0) __sync_add_and_fetch(&t->occupied, 1);
        } else {
            uint8_t cur = t->tab[i][bin];
            if (cur == 0 && i == 0) __sync_add_and_fetch(&t->occupied, 1);
            if (cur < MAX_KCOUNT) __sync_add_and_fetch(&t->tab[i][bin], 1);
        }
    }
}

static void *mt_worker(void *arg) {
    mt_job *j = arg;
    or_table *t = j->t;
    int k = t->k;
    uint64_t mask = (k == 32) ? ~0ULL : ((1ULL << (2 * k)) - 1);
    int nbits_sub_1 = 2 * k - 2;
    for (uint64_t r = j->r0; r < j->r1; r++) {
        const char *s = j->seqs + j->offs[r];
        uint64_t len = j->offs[r + 1] - j->offs[r];
        if (len < (uint64_t)k) continue;
        uint64_t f = 0, rc = 0;
        for (uint64_t i = 0; i < len; i++) {
            unsigned char c = (unsigned char)clean_base((unsigned char)s[i]);
            f = ((f << 2) | twobit_repr(c)) & mask;
            rc = (rc >> 2) | (twobit_comp(c) << nbits_sub_1);
            if (i + 1 >= (uint64_t)k) {
                mt_add(t, f < rc ? f : rc);
                j->kmers++;
            }
        }
    }
    return NULL;
}

uint64_t or_consume_batch_mt(or_table *t, const char *seqs, const uint64_t *offs,
                             uint64_t nreads, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (t->kind == OR_NIBBLE || t->hash != OR_HASH_TWOBIT) return or_consume_batch(t, seqs, offs, nreads);
    pthread_t th[256];
    mt_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int i = 0; i < nthreads; i++) {
        jobs[i].t = t; jobs[i].seqs = seqs; jobs[i].offs = offs;
        jobs[i].r0 = nreads * (uint64_t)i / (uint64_t)nthreads;
        jobs[i].r1 = nreads * (uint64_t)(i + 1) / (uint64_t)nthreads;
        jobs[i].kmers = 0;
        pthread_create(&th[i], NULL, mt_worker, &jobs[i]);
    }
    uint64_t total = 0;
    for (int i = 0; i < nthreads; i++) { pthread_join(th[i], NULL); total += jobs[i].kmers; }
    return total;
}

/* ------------------------------------------------------------------------ */
/* Synthetic input streams.  These are NOT reference
 * functions: they regenerate, on the host, the exact read streams the
 * benchmark generates in HBM (khmer_amd/synth.py defines them; the device
 * twins are kh_query.cuh k_synth_packed / k_synth_genomic), so that the oracle
 * can consume the benchmark's own workload for full-size golden fixtures.
 * Codes: A=0 T=1 C=2 G=3 (twobit_repr, include/oxli/kmer_hash.hh:62-73). */
static inline uint64_t synth_word(uint64_t seed, uint64_t r, uint64_t t) {
    uint64_t z = seed + ((r << 20) + t) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static const char synth_ascii[4] = { 'A', 'T', 'C', 'G' };

void or_synth_read(uint64_t seed, uint64_t r, int L, char *out) {
    for (int i = 0; i < L; i++)
        out[i] = synth_ascii[(synth_word(seed, r, (uint64_t)i >> 5) >> (62 - 2 * (i & 31))) & 3];
    out[L] = 0;
}

/* genomic stream: reads of L bases sampled uniformly (either strand) from a
 * random genome of G bases (seed+1), with a 1% substitution rate (seed+3). */
static inline unsigned genome_base(uint64_t seed, uint64_t g) {
    const uint64_t w = g >> 5;
    return (unsigned)((synth_word(seed + 1, w >> 20, w & 0xFFFFF) >> (62 - 2 * (g & 31))) & 3);
}

void or_synth_genomic_read(uint64_t seed, uint64_t G, uint64_t r, int L, char *out) {
    const uint64_t start = synth_word(seed + 2, r, 0) % (G - (uint64_t)L + 1);
    const int rc = (int)(synth_word(seed + 2, r, 1) & 1);
    for (int i = 0; i < L; i++) {
        unsigned c = rc ? (genome_base(seed, start + (uint64_t)(L - 1 - i)) ^ 1u)
                        : genome_base(seed, start + (uint64_t)i);
        const uint64_t u = synth_word(seed + 3, r, (uint64_t)i);
        if (u % 100 == 0) c = (unsigned)((c + 1 + (u >> 32) % 3) & 3);
        out[i] = synth_ascii[c];
    }
    out[L] = 0;
}

/* consume reads r0..r0+nreads-1 of a synthetic stream in stream order
 * (genome == 0: iid uniform stream; otherwise the genomic stream).  The
 * k-mers of a group of reads are hashed and binned first, then added one by
 * one in stream order (the same add as or_consume_string) while the table
 * bytes of the k-mer PF_AHEAD places later are prefetched: GB tables make
 * every add a cache miss, and the golden fixtures run 5e10 adds. */
struct sink_h { uint64_t *h; uint64_t n; };
static void cb_sink(void *ctx, uint64_t h) { struct sink_h *s = ctx; s->h[s->n++] = h; }
#define PF_GROUP 64
#define PF_AHEAD 24
uint64_t or_consume_synth(or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L) {
    char *buf = malloc((size_t)L + 1);
    const int n = t->n;
    const uint64_t cap = (uint64_t)PF_GROUP * (uint64_t)(L + 1);
    uint64_t *hs = malloc(cap * 8), *bins = malloc(cap * (uint64_t)n * 8);
    const int shift = t->kind == OR_BIT ? 3 : t->kind == OR_NIBBLE ? 1 : 0;
    uint64_t total = 0;
    for (uint64_t g = r0; g < r0 + nreads; g += PF_GROUP) {
        const uint64_t ge = g + PF_GROUP < r0 + nreads ? g + PF_GROUP : r0 + nreads;
        struct sink_h sk = {hs, 0};
        for (uint64_t r = g; r < ge; r++) {
            if (genome) or_synth_genomic_read(seed, genome, r, L, buf);
            else or_synth_read(seed, r, L, buf);
            iterate_kmers(t, buf, (size_t)L, cb_sink, &sk);
        }
        for (uint64_t j = 0; j < sk.n; j++) bins_of(t, hs[j], bins + j * (uint64_t)n);
        for (uint64_t j = 0; j < sk.n; j++) {
            if (j + PF_AHEAD < sk.n) {
                const uint64_t *b = bins + (j + PF_AHEAD) * (uint64_t)n;
                for (int i = 0; i < n; i++) __builtin_prefetch(t->tab[i] + (b[i] >> shift), 1, 0);
            }
            add_b(t, hs[j], bins + j * (uint64_t)n);
        }
        total += sk.n;
    }
    free(hs);
    free(bins);
    free(buf);
    return total;
}

/* The same stream-order consume spread over threads, for the full-size golden
 * fixtures (5e10 adds into 16-32 GB tables: one cache/TLB miss per (k-mer,
 * table) makes the single-threaded loop ~2 M k-mers/s).  Nothing about the
 * result changes:
 *  - the reads of a super-group are synthesised and hashed by worker threads
 *    (pure functions of the read index) into contiguous per-worker slices, so
 *    the concatenation is the stream order;
 *  - table i is updated by its own thread, k-mer by k-mer in stream order, so
 *    every bin sees exactly the sequence of values it sees in add_b; the
 *    thread records per k-mer whether its bin was zero (is_new, occupied) and
 *    whether it was full (ByteStorage's n_full);
 *  - the calling thread then combines the flags in stream order: unique and
 *    occupied as add_b counts them, and the bigcount increments (saturating
 *    increments of one key per k-mer: storage.hh:606-616).
 * The previous super-group's table updates overlap the next one's hashing. */
#define SG_READS 16384
struct synth_job {
    const or_table *t; uint64_t seed, genome, r0, r1; int L;
    uint64_t *hs; uint64_t n;
};
static void *synth_hash_worker(void *arg) {
    struct synth_job *j = arg;
    char *buf = malloc((size_t)j->L + 1);
    struct sink_h sk = {j->hs, 0};
    for (uint64_t r = j->r0; r < j->r1; r++) {
        if (j->genome) or_synth_genomic_read(j->seed, j->genome, r, j->L, buf);
        else or_synth_read(j->seed, r, j->L, buf);
        iterate_kmers(j->t, buf, (size_t)j->L, cb_sink, &sk);
    }
    j->n = sk.n;
    free(buf);
    return NULL;
}
struct table_job {
    or_table *t; int i; const uint64_t *hs; uint64_t nh; uint8_t *flags;   /* bit 0: was zero, bit 1: full */
};
static void *table_add_worker(void *arg) {
    struct table_job *j = arg;
    or_table *t = j->t;
    const uint64_t p = t->sizes[j->i];
    uint8_t *tab = t->tab[j->i];
    const uint64_t *hs = j->hs;
    for (uint64_t x = 0; x < j->nh; x++) {
        if (x + PF_AHEAD < j->nh) {
            const uint64_t b = hs[x + PF_AHEAD] % p;
            __builtin_prefetch(tab + (t->kind == OR_BIT ? b / 8 : t->kind == OR_NIBBLE ? b / 2 : b), 1, 0);
        }
        const uint64_t bin = hs[x] % p;
        uint8_t f = 0;
        if (t->kind == OR_BIT) {                         /* storage.hh:172-199 */
            const uint8_t bit = (uint8_t)(1u << (bin % 8));
            const uint8_t orig = tab[bin / 8];
            tab[bin / 8] = orig | bit;
            f = !(orig & bit);
        } else if (t->kind == OR_NIBBLE) {               /* storage.hh:320-359 */
            const uint64_t idx = bin / 2;
            const uint8_t mask = (bin % 2) ? 0x0F : 0xF0;
            const int shift = (bin % 2) ? 0 : 4;
            const uint8_t cur = (uint8_t)((tab[idx] & mask) >> shift);
            f = cur == 0;
            if (cur != 15) tab[idx] = (uint8_t)((tab[idx] & ~mask) | ((uint8_t)((cur + 1) << shift) & mask));
        } else {                                         /* storage.hh:571-624 */
            const uint8_t cur = tab[bin];
            f = cur == 0;
            if (cur < MAX_KCOUNT) tab[bin] = (uint8_t)(cur + 1);
            else f |= 2;
        }
        j->flags[x] = f;
    }
    return NULL;
}
uint64_t or_consume_synth_mt(or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L,
                             int nthreads) {
    if (nthreads < 2) return or_consume_synth(t, seed, genome, r0, nreads, L);
    if (nthreads > 64) nthreads = 64;
    const int n = t->n;
    const uint64_t per = (uint64_t)(L + 1) * SG_READS;
    uint64_t *hbuf[2] = {malloc(per * 8), malloc(per * 8)};
    uint64_t *hcat = malloc(per * 8);
    uint8_t *flags = malloc(per * (uint64_t)n);
    struct synth_job jobs[2][64];
    struct table_job tj[64];
    pthread_t th[64], tt[64];
    uint64_t total = 0, nprev = 0;
    const uint64_t end = r0 + nreads;
    int cur = 0;
    for (uint64_t g = r0;; g += SG_READS) {
        const uint64_t ge = g < end ? (g + SG_READS < end ? g + SG_READS : end) : g;
        int nt = 0;
        if (g < end) {
            uint64_t off = 0;
            for (int i = 0; i < nthreads; i++) {
                struct synth_job *j = &jobs[cur][i];
                j->t = t; j->seed = seed; j->genome = genome; j->L = L;
                j->r0 = g + (ge - g) * (uint64_t)i / (uint64_t)nthreads;
                j->r1 = g + (ge - g) * (uint64_t)(i + 1) / (uint64_t)nthreads;
                j->hs = hbuf[cur] + off;
                off += (j->r1 - j->r0) * (uint64_t)(L + 1);
                pthread_create(&th[i], NULL, synth_hash_worker, j);
                nt++;
            }
        }
        if (nprev) {   /* the previous super-group (hashes in hcat, stream order) */
            for (int i = 0; i < n; i++) {
                tj[i] = (struct table_job){t, i, hcat, nprev, flags + (uint64_t)i * per};
                pthread_create(&tt[i], NULL, table_add_worker, &tj[i]);
            }
            for (int i = 0; i < n; i++) pthread_join(tt[i], NULL);
            for (uint64_t x = 0; x < nprev; x++) {
                int is_new = 0, nfull = 0;
                for (int i = 0; i < n; i++) {
                    const uint8_t f = flags[(uint64_t)i * per + x];
                    if ((f & 1) && !is_new) {
                        is_new = 1;
                        if (i == 0) t->occupied++;
                    }
                    nfull += (f >> 1) & 1;
                }
                if (t->kind == OR_BYTE && nfull == n && t->use_bigcount) {
                    int created;
                    const uint64_t s = map_slot(&t->bigcounts, hcat[x], &created);
                    if (t->bigcounts.vals[s] == 0) t->bigcounts.vals[s] = MAX_KCOUNT + 1;
                    else if (t->bigcounts.vals[s] < MAX_BIGCOUNT) t->bigcounts.vals[s]++;
                }
                if (is_new) t->unique++;
            }
            total += nprev;
            nprev = 0;
        }
        for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
        if (g >= end) break;
        for (int i = 0; i < nthreads; i++) {   /* gather the slices in stream order */
            memcpy(hcat + nprev, jobs[cur][i].hs, jobs[cur][i].n * 8);
            nprev += jobs[cur][i].n;
        }
        cur ^= 1;
    }
    free(hbuf[0]);
    free(hbuf[1]);
    free(hcat);
    free(flags);
    return total;
}

/* get_median_count (or_median, src/oxli/hashtable.cc:299-328) of reads
 * r0..r0+nreads-1 of a synthetic stream, one output triple per read (the
 * golden fixtures' query digests) */
int or_median_synth(const or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L,
                    uint16_t *med, float *avg, float *sd) {
    char *buf = malloc((size_t)L + 1);
    int rc = 0;
    for (uint64_t r = 0; r < nreads && rc == 0; r++) {
        if (genome) or_synth_genomic_read(seed, genome, r0 + r, L, buf);
        else or_synth_read(seed, r0 + r, L, buf);
        rc = or_median(t, buf, (size_t)L, &med[r], &avg[r], &sd[r]);
    }
    free(buf);
    return rc;
}
