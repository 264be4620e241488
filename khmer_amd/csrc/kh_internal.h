// kh_internal.h -- internal structures of libkhmer_hip.so (not part of the ABI).
#pragma once
#include <stdint.h>

#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <hip/hip_runtime.h>

#include "kh_device.h"
#include "../../include/khmer_hip.h"

namespace kh {

// ---- errors: mapped to status codes at the C-ABI edge (kh_capi.cpp) ----
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] inline void fail(int code, const std::string &msg) { throw Error(code, msg); }

#define KH_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) {                                                             \
            if (e_ == hipErrorOutOfMemory)                                                  \
                ::kh::fail(4, std::string("device out of memory: ") + #expr);               \
            ::kh::fail(5, std::string("HIP error ") + hipGetErrorString(e_) + " at " + #expr); \
        }                                                                                   \
    } while (0)

// device scratch owned by a scope: freed on every path, including throws
struct DevBuf {
    void *p = nullptr;
    DevBuf() = default;
    explicit DevBuf(size_t bytes) { alloc(bytes); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { if (p) (void)hipFree(p); }
    void alloc(size_t bytes) {
        if (p) { (void)hipFree(p); p = nullptr; }
        KH_HIP(hipMalloc(&p, bytes ? bytes : 1));
    }
    template <class T> T *as() const { return (T *)p; }
};

constexpr int MAXT = 32;  // tables per graph on device (NibbleStorage's own cap, storage.hh:290)
// k-mers of one device pass: at most 3200 winner windows of 2^20 k-mers (the
// LDS of k_scatter_w's per-window tails, ~115 KB, and k_mark's 2^20-bit
// bitmap); batch k-mer indices stay 32-bit (3200 * 2^20 < 2^32 - 1 = NO_J).
// The C2 step (6.5e9 k-mers) runs as two passes of 3.25e9.
constexpr uint64_t MAX_PASS_KMERS = 3200ull << 20;

// ---- partition geometry -----------------------------------------------------
// Every table bin gets a global id G = tbase[i] + bin.  Regions are 2^s0 bins
// (one LDS-resident workgroup each); level-1 buckets are 2^(s0+s2) bins; each
// table starts on a bucket boundary.
struct Geometry {
    int s0 = 14;          // log2 region bins
    int s2 = 10;          // log2 regions per level-1 bucket
    uint32_t F1 = 1;      // level-1 buckets
    uint64_t tbase[MAXT];
    uint32_t bucket_table[8192];
};

// Development knobs: the environment variables that switch kernel paths or
// schedules for A/B timing (INTEGRATION.md "Development knobs") are read only
// by a development build (make DEV=1, i.e. -DKH_DEV); the product library
// ignores them and always takes its defaults.  Variables the test suite sets
// (feed chunk sizes, the owned-filter thresholds, KH_SMALL_PASS, the BGZF and
// packer switches) are read with getenv in every build.
static inline const char *dev_getenv(const char *name) {
#ifdef KH_DEV
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// kernel parameter block (passed by value)
// Timing-only ablations (bench.py --ablate, tools/lb_ablate.sh): switches that
// skip work and give wrong tables.  They exist only in a development build
// compiled with -DKH_ABLATE (make EXTRA_HIPFLAGS=-DKH_ABLATE); in the product
// library KH_ABL is constant false and the KH_ABLATE variable is ignored.
#ifdef KH_ABLATE
#define KH_ABL(P, bit) ((P).ablate & (bit))
#else
#define KH_ABL(P, bit) 0
#endif

struct Params {
    int kind, hash, k, n;
    int s0, s2;
    uint32_t F1;
    int use_bigcount;
    int ablate;               // timing-only ablation bits (KH_ABLATE env, -DKH_ABLATE builds only)
    uint64_t p[MAXT];         // table sizes (bins) -- the primes the hash is reduced by
    uint64_t lo[MAXT];        // first bin of table i held here (0 unless sharded)
    uint64_t lsz[MAXT];       // bins of table i held here (p[i] unless sharded)
    uint64_t m[MAXT];         // Barrett constants
    double ip[MAXT];          // 1 / p[i] (mod_f64_32) when fm32
    int fm32;                 // every p[i] < 2^30 and every hash / p[i] < 2^31: local_bin uses mod_f64_32
    uint64_t tbase[MAXT];     // global bin base of table i
    uint64_t tbyte[MAXT];     // byte offset of table i in the table arena
    uint64_t tbytes[MAXT];    // storage bytes of table i
};

// device workspace of one pipeline pass (grown on demand)
struct Workspace {
    uint64_t cap_kmers = 0, cap_recs = 0;
    uint64_t *rec1 = nullptr, *rec2 = nullptr;   // (k-mer index << 32) | bin offset
    uint64_t *frec = nullptr;                    // a shard's owned records (k_own_filter)
    uint64_t cap_frec = 0;
    unsigned long long *fcount = nullptr;        // k_own_filter output counter
    uint8_t *fullf = nullptr;                    // per k-mer bigcount "full" tallies
    uint32_t *newbits = nullptr;                 // per k-mer new flags (bitmap)
    // bigcount events of a pass, aggregated on the device: open-addressing map
    // hash -> number of "full" inserts (cleared per pass), compacted into
    // (bc, bcn) for the host merge into Graph::bigcounts
    uint64_t *bck = nullptr;                     // map keys (BC_EMPTY = free)
    uint32_t *bcv = nullptr;                     // map counts
    uint64_t *bc = nullptr;                      // compacted keys
    uint32_t *bcn = nullptr;                     // compacted counts
    uint64_t cap_bcmap = 0;                      // map slots (power of two); bc/bcn hold as many
    // partition bookkeeping
    uint64_t *off1 = nullptr;        // [F1+1] level-1 bucket offsets
    uint32_t *ch2 = nullptr;         // [F1+1] level-2 chunk prefix per bucket
    uint64_t *off2 = nullptr;        // [F1*2^s2 + 1] region offsets
    uint32_t *mcnt = nullptr;        // (destination, chunk) count matrix
    uint64_t *moff = nullptr;        // its exclusive scan
    void *scan_tmp = nullptr;        // rocPRIM scan temporary storage
    uint32_t *wcnt = nullptr;        // [regions] winners per region
    // coarse-window winner path (unsharded passes; kh_apply.cuh k_*_wf)
    unsigned long long *cw_cur = nullptr;   // [64] append cursors
    uint64_t *cmbase = nullptr;              // [65] count-matrix base per coarse window
    uint32_t *cnk = nullptr;                 // [64] chunks per coarse window
    void *wch = nullptr;                     // WChunk descriptors
    uint64_t cap_wch = 0;
    uint64_t cap_m = 0, cap_moff = 0, cap_scan = 0, cap_newbits = 0, cap_wcnt = 0;
    uint4 *xseg = nullptr;           // crossing-bin segments, one per region with crossings
    // fixed-capacity level 2 (k_scatter_l2f): region g holds [reg_base[g], reg_cur[g])
    uint64_t *reg_base = nullptr;    // [regions + 1] capacity prefix for passes of reg_nkmers k-mers
    uint64_t *reg_cur = nullptr;     // [regions] append cursors
    uint64_t cap_reg = 0, reg_nkmers = 0, reg_total = 0, reg_max = 0;   // reg_max: largest region capacity
    uint64_t reg_np = 0;             // planned for the near-prime level 2: its rp, rloc, parts (0: not)
    // near-prime level 1 (kh_nearprime.cuh): bucket d holds [d cap, np_cur[d]);
    // np_blkj[block] = the k-mer index base of a level-1 block
    unsigned long long *np_cur = nullptr;
    uint32_t *np_blkj = nullptr;
    uint64_t cap_npcur = 0, cap_blkj = 0;
    // three-level near-prime: fine bucket b holds [b cap_f, np_fcur[b]) of
    // the fine records (kh_nearprime.cuh k_scatter_n1b)
    unsigned long long *np_fcur = nullptr;
    uint64_t cap_npfcur = 0;
    // sparse delta pieces (kh_engine.hip sp_pack / sp_unpack): chunk counts, offsets
    uint32_t *sp_cnt = nullptr;
    uint64_t *sp_off = nullptr;
    uint64_t cap_spcnt = 0, cap_spoff = 0;
    double reg_sigma = 0, bkt_sigma = 0;          // capacity margins the plans were made with
    // fixed-capacity level 1 (k_scatter_l1f): bucket b holds [bkt_base[b], bkt_cur[b])
    uint64_t *bkt_base = nullptr, *bkt_cur = nullptr;
    uint64_t bkt_nkmers = 0, bkt_total = 0;
    bool l1_exact = false;           // exchange-mode view: level 1 took the exact path (buckets = off1)
    uint64_t *ctr = nullptr;         // counters, see CTR_*
    uint64_t *h_ctr = nullptr;       // pinned host mirror
    uint64_t cap_regions = 0, cap_xseg = 0;
    // staging for host-fed batches
    uint64_t *d_words = nullptr, *d_koff = nullptr;
    uint8_t *d_bytes = nullptr;
    uint8_t *d_rbytes = nullptr;     // reverse complement of every read of d_bytes (Murmur sources)
    uint64_t cap_words = 0, cap_koff = 0, cap_bytes = 0, cap_rbytes = 0;
    // small passes (k_small_pass): per-k-mer flags and hashes
    uint8_t *sm_flags = nullptr;
    uint64_t *sm_hash = nullptr;
    uint64_t cap_sm = 0, cap_smh = 0;
    // query staging
    uint64_t *q_hashes = nullptr;
    uint16_t *q_counts = nullptr;
    uint64_t cap_q = 0, cap_q16 = 0;
};
enum { CTR_OCC = 0, CTR_UNIQUE, CTR_NCROSS, CTR_NBC, CTR_ERR, CTR_NFULL, CTR_BCFF, CTR_BCOUT, CTR_L1Q, CTR_APQ, CTR_N };
constexpr uint64_t BC_EMPTY = ~0ull;   // free map slot; events of hash ~0 count in CTR_BCFF

// Hashgraph::all_tags (include/oxli/hashgraph.hh:113, a std::set<HashIntoType>):
// an open-addressing set of u64 k-mer hashes (linear probing, load <= 1/2);
// ordered output (save_tagset, get_tags) sorts on demand
class TagSet {
    static constexpr uint64_t EMPTY = ~0ull;
    std::vector<uint64_t> slot_;
    uint64_t n_ = 0;
    bool has_empty_ = false;   // the key ~0 itself
    static uint64_t mix(uint64_t x) {
        x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
        return x;
    }
    void rehash(uint64_t cap) {
        std::vector<uint64_t> old;
        old.swap(slot_);
        slot_.assign(cap, EMPTY);
        for (uint64_t x : old)
            if (x != EMPTY) place(x);
    }
    void grow() { rehash(slot_.empty() ? 1024 : slot_.size() * 2); }
    void place(uint64_t x) {
        const uint64_t m = slot_.size() - 1;
        for (uint64_t i = mix(x) & m;; i = (i + 1) & m)
            if (slot_[i] == EMPTY) { slot_[i] = x; return; }
    }
  public:
    uint64_t size() const { return n_ + (has_empty_ ? 1 : 0); }
    bool count(uint64_t x) const {
        if (x == EMPTY) return has_empty_;
        if (slot_.empty()) return false;
        const uint64_t m = slot_.size() - 1;
        for (uint64_t i = mix(x) & m;; i = (i + 1) & m) {
            if (slot_[i] == x) return true;
            if (slot_[i] == EMPTY) return false;
        }
    }
    void insert(uint64_t x) {
        if (x == EMPTY) { has_empty_ = true; return; }
        if (2 * (n_ + 1) > slot_.size()) grow();
        const uint64_t m = slot_.size() - 1;
        for (uint64_t i = mix(x) & m;; i = (i + 1) & m) {
            if (slot_[i] == x) return;
            if (slot_[i] == EMPTY) { slot_[i] = x; n_++; return; }
        }
    }
    void clear() { slot_.clear(); n_ = 0; has_empty_ = false; }
    // capacity for n keys at load <= 1/2 (one rehash instead of a doubling chain)
    void reserve(uint64_t n) {
        uint64_t c = 1024;
        while (c < 2 * n) c *= 2;
        if (c > slot_.size()) rehash(c);
    }
    // n inserts with their slots prefetched first: the table is far larger
    // than the caches, so one-at-a-time inserts wait on a miss each
    void insert_batch(const uint64_t *x, uint64_t n) {
        reserve(n_ + n);
        const uint64_t m = slot_.size() - 1;
        for (uint64_t a = 0; a < n; a++) __builtin_prefetch(&slot_[mix(x[a]) & m], 1);
        for (uint64_t a = 0; a < n; a++) insert(x[a]);
    }
    std::vector<uint64_t> sorted() const;   // ascending (std::set order)
};

struct Graph {
    int kind = BYTE, hash = TWOBIT, k = 0, n = 0, device = 0;
    std::vector<uint64_t> sizes, nbytes;
    // shard of a multi-GPU group: this graph holds bins [lo, lo + lsz) of every
    // table (lo = 0, lsz = sizes when not sharded); nbytes are the slice's bytes
    int world = 1, rank = 0;
    bool grouped = false;             // a shard of a ShardGroup (its winners are routed by window)
    int l1_chunk = -1, apply_dyn = -1;   // work distribution (kh_graph_set_schedule; -1: default)
    int force_s2 = -1;                // level-2 fan-out fixed by the group (exchange mode: the
                                      // unsharded geometry's, so level-1 buckets line up)
    std::vector<uint64_t> lo, lsz;
    Geometry geo;
    Params prm;
    uint8_t *d_tab = nullptr;         // table arena
    uint64_t arena_bytes = 0;
    hipStream_t stream = nullptr;
    uint64_t n_unique = 0, n_occupied = 0;
    int64_t occ_hint = -1;            // delta-mode views: the table occupancy complement_mode estimates from (-1: n_occupied)
    bool use_bigcount = false;
    std::unordered_map<uint64_t, uint16_t> bigcounts;   // storage.hh:498 KmerCountMap
    // device mirror of bigcounts for queries (sorted keys / values)
    uint64_t *d_bc_keys = nullptr;
    uint16_t *d_bc_vals = nullptr;
    uint64_t d_bc_n = 0, d_bc_cap = 0;
    bool bc_dirty = true;
    TagSet tags;                                        // hashgraph.hh:113 all_tags
    uint64_t batch_kmers = 1ull << 27;
    int l2_cool = 0;                  // passes left on the exact level 2 after a capacity overflow
    // capacity margin of the fixed-capacity partition, in Poisson sigmas of
    // each bucket's / region's expected record count; grown (x3, sticky) when
    // a pass overflows -- skewed input (repeated k-mers) spreads region
    // counts far wider than Poisson
    double cap_sigma = 8.0;
    Workspace ws;
    // optional per-kernel HIP-event timing (kh_graph_set_profiling)
    bool profile = false;
    struct KStat { double ms = 0; uint64_t n = 0; };
    std::vector<std::pair<std::string, KStat>> kstats;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> ev_pending;
    size_t ev_next = 0;
    std::recursive_mutex mu;
    ~Graph();
};

// ---- host helpers (kh_host.cpp) ----
uint64_t hash_twobit(const char *kmer, int k, uint64_t *f, uint64_t *r);
uint64_t hash_murmur(const char *kmer, int k);
uint64_t hash_murmur_fwd(const char *kmer, int k);
std::string revhash(uint64_t h, int k);
std::string revcomp(const char *s, size_t len);
bool is_prime(uint64_t n);
std::vector<uint64_t> primes_near(uint32_t n, uint64_t x);
void kmer_hashes_host(int hash_kind, int k, const char *seq, size_t len, std::vector<uint64_t> &out);

// host-side batch of reads ready for the device
struct HostBatch {
    int hash = TWOBIT;
    std::vector<uint64_t> words;     // 2-bit packed (TWOBIT)
    std::vector<uint8_t> bytes;      // ASCII (MURMUR)
    std::vector<uint64_t> koff{0};   // k-mer prefix offsets per packed read
    std::vector<uint32_t> read_kmers;  // per packed read
    uint64_t nbases = 0;
    bool uniform = true;             // every packed read has the same length
    uint64_t nkmers() const { return koff.back(); }
    uint64_t nreads() const { return koff.size() - 1; }
    void clear() {
        words.clear(); bytes.clear(); koff.assign(1, 0); read_kmers.clear(); nbases = 0; uniform = true;
    }
    // append a read (reads shorter than k are skipped by the caller)
    void append(const char *s, size_t len, int k, bool clean);
    // append batch o's reads after this batch's (same hash kind)
    void merge(const HostBatch &o);
};

// raw reads for the pipelined host feed: concatenated sequences >= k bases
struct RawBatch {
    std::vector<char> seq;
    std::vector<uint32_t> len;
    uint64_t nkmers = 0, nreads_parsed = 0;
};

// ---- parser (kh_parser.cpp) ----
struct Parser;
struct ReadView {
    const char *name; size_t name_len;
    const char *seq; size_t seq_len;
    const char *qual; size_t qual_len;
};

// ---- engine (kh_engine.hip) ----
Graph *graph_create(int kind, int hash, int k, const uint64_t *sizes, int n, int device);
Graph *graph_create_shard(int kind, int hash, int k, const uint64_t *sizes, int n, int device, int world, int rank);
// first bin of shard r of a p-bin table split over `world` shards (8-aligned)
inline uint64_t shard_lo(uint64_t p, int world, int r) {
    if (r >= world) return p;
    const uint64_t x = (uint64_t)(((unsigned __int128)p * (unsigned)r) / (unsigned)world);
    return x & ~7ull;
}
void graph_zero_counters(Graph *g);
// fill `bytes` bytes of device memory at p with v on stream st (64-bit
// indices, 16-byte stores; large ranges never go through hipMemsetAsync)
void dev_fill(void *p, int v, uint64_t bytes, hipStream_t st);
void graph_prepare_params(Graph *g);
// run one device pipeline pass over a device-resident batch.
// Optional outputs: per-k-mer is-new flags and hashes (device pointers filled
// into ws; copied to host by the caller).
struct PassOut {
    uint8_t *h_new = nullptr;     // host [nkmers]
    uint32_t *h_newbits = nullptr;   // host [(nkmers + 31) / 32]: the same flags as a bitmap (bit j & 31 of word j >> 5)
    uint64_t *h_hash = nullptr;   // host [nkmers]
};
void engine_consume_twobit(Graph *g, const uint64_t *d_words, const uint64_t *d_koff,
                           uint64_t nreads, uint64_t nkmers, const PassOut *out);
void engine_consume_twobit_fixed(Graph *g, const uint64_t *d_words, uint64_t nreads, uint64_t read_len,
                                 const PassOut *out);
void engine_consume_bytes(Graph *g, const uint8_t *d_bytes, const uint64_t *d_koff,
                          uint64_t nreads, uint64_t nkmers, const PassOut *out);
void engine_consume_hashes(Graph *g, const uint64_t *d_hashes, uint64_t n, const PassOut *out);
void engine_consume_host(Graph *g, const HostBatch &b, const PassOut *out);
void engine_get_counts(Graph *g, const uint64_t *h_hashes, uint64_t n, uint16_t *out);
// consume_seqfile_banding / _with_mask (hashtable.cc:152-274): only k-mers in
// the band and passing the mask are counted; returns how many were
struct BandMask {
    uint32_t num_bands = 0;          // 0: no banding
    uint64_t band_lo = 0, band_hi = 0;
    Graph *mask = nullptr;           // nullptr: no mask
    uint32_t threshold = 0;
    int consume_masked = 0;
};
uint64_t engine_consume_filtered(Graph *g, const HostBatch &b, const BandMask &f);
void engine_median(Graph *g, const HostBatch &b, uint16_t *med, float *avg, float *sd);
void engine_kmer_counts(Graph *g, const HostBatch &b, uint16_t *h_out);
void engine_median_at_least(Graph *g, const HostBatch &b, uint32_t cutoff, uint8_t *h_out);
void engine_hash_batch(Graph *g, const HostBatch &b, uint64_t *h_out);
void engine_median_fixed_device(Graph *g, const void *d_reads, uint64_t nreads, uint64_t read_len, uint16_t *d_med,
                                float *d_avg, float *d_sd);
void engine_consume_bytes_fixed(Graph *g, const uint8_t *d_bytes, uint64_t nreads, uint64_t read_len);
void engine_unpack_ascii(int device, const uint64_t *d_words, uint64_t nbases, uint8_t *d_bytes);
void engine_sync_bigcounts(Graph *g);
void engine_download_table(Graph *g, int i, uint8_t *dst);
void engine_upload_table(Graph *g, int i, const uint8_t *src);
void engine_collect_events(Graph *g);

// ---- sharded groups (kh_engine.hip) ----
struct ShardGroup;
void group_unique_id(unsigned char *out, size_t n);
ShardGroup *group_create(int kind, int hash, int k, const uint64_t *sizes, int n, int world, int rank, int nlocal,
                         const int *devices, const unsigned char *uid, int mode);   // mode: KH_GROUP_*
ShardGroup *group_create_hosted(int kind, int hash, int k, const uint64_t *sizes, int n, int world, int rank,
                                int device, const kh_transport *t, int mode);
void group_rank_slice(ShardGroup *G, int rank, int table, uint64_t *lo, uint64_t *size);
int group_exchange(ShardGroup *G);   // the group's KH_GROUP_* mode
void group_comm_info(ShardGroup *G, int *nranks, int *device);
void group_destroy(ShardGroup *G);
void group_consume_fixed(ShardGroup *G, const uint64_t *const *d_words, uint64_t nreads, uint64_t read_len);
void group_consume_bytes_fixed(ShardGroup *G, const uint8_t *const *d_bytes, uint64_t nreads, uint64_t read_len);
void group_median_fixed(ShardGroup *G, const void *const *d_reads, uint64_t nreads, uint64_t read_len,
                        uint16_t *const *d_med, float *const *d_avg, float *const *d_sd);
void group_counters(ShardGroup *G, uint64_t *n_unique, uint64_t *n_occupied);
void group_wire_stats(const ShardGroup *G, uint64_t *dense_bytes, uint64_t *sent_bytes);
int group_world(ShardGroup *G);
int group_nlocal(ShardGroup *G);
int group_rank(ShardGroup *G, int l);
Graph *group_shard(ShardGroup *G, int l);

}  // namespace kh
