// kh_capi.cpp -- the extern "C" boundary of libkhmer_hip.so (include/khmer_hip.h).
// Every entry point converts exceptions into status codes + a thread-local
// message (the reference maps C++ exceptions to Python ones,
// khmer/_oxli/oxli_exception_convert.cc:9-31).
#include <errno.h>
#include <limits.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <fstream>
#include <memory>
#include <mutex>
#include <new>
#include <condition_variable>
#include <deque>
#include <exception>
#include <string>
#include <functional>
#include <thread>

#include "../../include/khmer_hip.h"
#include "kh_internal.h"

namespace kh {
struct Parser;
Parser *parser_open(const char *path);
void parser_close(Parser *p);
int parser_next_read(Parser *p, ReadView *rv);
uint64_t parser_num_reads(Parser *p);
bool parser_is_complete(Parser *p);
void parser_fill_batch(Parser *p, HostBatch &b, int k, uint64_t max_kmers, uint64_t max_bases, bool *done,
                       uint64_t *taken);
void parser_fill_raw(Parser *p, RawBatch &b, int k, uint64_t max_kmers, uint64_t max_bases, bool *done,
                     uint64_t *taken);
struct PlainFile;
PlainFile *parser_plain_open(Parser *pr);
void parser_plain_close(PlainFile *f);
void parser_plain_commit(Parser *pr);
size_t plain_size(const PlainFile *f);
bool plain_chunkable(const PlainFile *f, size_t CH);
void plain_parse_chunk(const PlainFile *f, size_t c, size_t CH, int k, uint64_t max_kmers, std::vector<RawBatch> &out,
                       uint64_t *nreads, size_t *start, size_t *end, bool *redo);
void plain_parse_rest(const PlainFile *f, size_t from, size_t CH, int k, uint64_t max_kmers,
                      const std::function<void(RawBatch &)> &sink, uint64_t *nreads);
uint64_t plain_parse_range(const PlainFile *f, size_t start, size_t stop, int k, uint64_t max_kmers,
                           std::vector<RawBatch> &out, uint64_t *nreads);
void parser_mark_drained(Parser *pr, uint64_t nreads);
void engine_synth_packed(int device, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L, int k,
                         uint64_t *d_words, uint64_t *d_koff);
}  // namespace kh

using namespace kh;

struct kh_graph { Graph *g; bool owned = true; };
struct kh_group { ShardGroup *G; };
struct kh_parser { Parser *p; };

static thread_local std::string tl_err;

template <class F>
static int guard(F &&f) {
    try {
        f();
        return KH_OK;
    } catch (const Error &e) {
        tl_err = e.what();
        return e.code;
    } catch (const std::bad_alloc &) {
        tl_err = "out of memory";
        return KH_ENOMEM;
    } catch (const std::exception &e) {
        tl_err = e.what();
        return KH_ERUNTIME;
    }
}

#define CHECK_PTR(p) do { if (!(p)) fail(KH_EVALUE, "null handle"); } while (0)

extern "C" {

const char *kh_last_error(void) { return tl_err.c_str(); }
int kh_abi_version(void) { return KH_ABI_VERSION; }

int kh_device_count(int *n) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return KH_OK;
}

// ---------------- hashing ---------------------------------------------------
int kh_hash_twobit(const char *kmer, int k, uint64_t *fwd, uint64_t *rc, uint64_t *canon) {
    return guard([&] {
        uint64_t f, r;
        uint64_t h = hash_twobit(kmer, k, &f, &r);
        if (fwd) *fwd = f;
        if (rc) *rc = r;
        if (canon) *canon = h;
    });
}

int kh_reverse_hash(uint64_t h, int k, char *out) {
    return guard([&] {
        if (k < 0 || k > 32) fail(KH_EVALUE, "k-mer size must be <= 32");
        std::string s = revhash(h, k);
        memcpy(out, s.c_str(), (size_t)k + 1);
    });
}

int kh_hash_murmur(const char *kmer, int len, uint64_t *canon, uint64_t *fwd) {
    return guard([&] {
        if (canon) *canon = hash_murmur(kmer, len);
        if (fwd) *fwd = hash_murmur_fwd(kmer, len);
    });
}

int kh_reverse_complement(const char *s, size_t len, char *out) {
    return guard([&] {
        std::string r = revcomp(s, len);
        memcpy(out, r.data(), len);
        out[len] = 0;
    });
}

int kh_kmer_hashes(int hash_kind, int k, const char *seq, size_t len, uint64_t *out, uint64_t *n_out) {
    return guard([&] {
        std::vector<uint64_t> v;
        kmer_hashes_host(hash_kind, k, seq, len, v);
        if (out) memcpy(out, v.data(), v.size() * 8);
        *n_out = v.size();
    });
}

// ---------------- primes -----------------------------------------------------
int kh_is_prime(uint64_t n, int *out) {
    return guard([&] { *out = is_prime(n) ? 1 : 0; });
}

int kh_get_n_primes_near_x(uint32_t n, uint64_t x, uint64_t *out, uint32_t *found) {
    return guard([&] {
        std::vector<uint64_t> v = primes_near(n, x);
        memcpy(out, v.data(), v.size() * 8);
        *found = (uint32_t)v.size();
    });
}

// ---------------- parser ----------------------------------------------------
int kh_parser_open(const char *path, kh_parser **out) {
    return guard([&] {
        Parser *p = parser_open(path);
        *out = new kh_parser{p};
    });
}

int kh_parser_next_read(kh_parser *p, const char **name, size_t *name_len, const char **seq, size_t *seq_len,
                        const char **qual, size_t *qual_len) {
    int rc = KH_OK;
    int st = guard([&] {
        CHECK_PTR(p);
        ReadView rv;
        rc = parser_next_read(p->p, &rv);
        if (rc != KH_OK) return;
        *name = rv.name; *name_len = rv.name_len;
        *seq = rv.seq; *seq_len = rv.seq_len;
        *qual = rv.qual; *qual_len = rv.qual_len;
    });
    return st != KH_OK ? st : rc;
}

int kh_parser_num_reads(kh_parser *p, uint64_t *out) {
    return guard([&] { CHECK_PTR(p); *out = parser_num_reads(p->p); });
}

int kh_parser_is_complete(kh_parser *p, int *out) {
    return guard([&] { CHECK_PTR(p); *out = parser_is_complete(p->p) ? 1 : 0; });
}

void kh_parser_close(kh_parser *p) {
    if (!p) return;
    parser_close(p->p);
    delete p;
}

// ---------------- graph lifecycle -----------------------------------------------
int kh_graph_create(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int device,
                    kh_graph **out) {
    return guard([&] {
        Graph *g = graph_create(storage, hash_kind, k, sizes, n_tables, device);
        *out = new kh_graph{g};
    });
}

void kh_graph_destroy(kh_graph *g) {
    if (!g) return;
    if (g->owned) delete g->g;
    delete g;
}

int kh_graph_info(kh_graph *h, int *storage, int *hash_kind, int *k, int *n_tables) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        if (storage) *storage = g->kind;
        if (hash_kind) *hash_kind = g->hash;
        if (k) *k = g->k;
        if (n_tables) *n_tables = g->n;
    });
}

int kh_graph_tablesizes(kh_graph *h, uint64_t *out) {
    return guard([&] {
        CHECK_PTR(h);
        memcpy(out, h->g->sizes.data(), h->g->sizes.size() * 8);
    });
}

int kh_graph_set_use_bigcount(kh_graph *h, int on) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        // Storage::set_use_bigcount (src/oxli/storage.cc:50-56)
        if (g->kind != BYTE) fail(KH_EVALUE, "bigcount is not supported for this storage.");
        g->use_bigcount = on != 0;
        g->prm.use_bigcount = on ? 1 : 0;
    });
}

int kh_graph_get_use_bigcount(kh_graph *h, int *on) {
    return guard([&] { CHECK_PTR(h); *on = h->g->use_bigcount ? 1 : 0; });
}

int kh_graph_n_unique_kmers(kh_graph *h, uint64_t *out) {
    return guard([&] { CHECK_PTR(h); *out = h->g->n_unique; });
}

int kh_graph_n_occupied(kh_graph *h, uint64_t *out) {
    return guard([&] { CHECK_PTR(h); *out = h->g->n_occupied; });
}

int kh_graph_set_batch_kmers(kh_graph *h, uint64_t max_kmers) {
    return guard([&] {
        CHECK_PTR(h);
        if (max_kmers < 1024 || max_kmers > MAX_PASS_KMERS) fail(KH_EVALUE, "batch size out of range");
        h->g->batch_kmers = max_kmers;
    });
}

}  // extern "C"

// ---------------- consume helpers -------------------------------------------------
std::vector<uint64_t> TagSet::sorted() const {
    std::vector<uint64_t> v;
    v.reserve(size());
    for (uint64_t x : slot_)
        if (x != EMPTY) v.push_back(x);
    if (has_empty_) v.push_back(EMPTY);
    std::sort(v.begin(), v.end());
    return v;
}

// Hashgraph::consume_sequence_and_tag state machine (src/oxli/hashgraph.cc:200-271)
// over one batch: the is-new flags come from the device pass as a bitmap.  A
// k-mer's hash is needed only where the machine looks at it -- a k-mer that
// is not new (tag membership), a tag position, a read's last k-mer -- and is
// computed here from the batch's own reads (kh_device.h: the device's
// arithmetic), so no per-k-mer hash leaves the device.  Runs of new k-mers
// advance `since` arithmetically: a tag every density - 1 new k-mers.
static uint64_t tag_batch(Graph *g, const HostBatch &b, const uint32_t *nb) {
    const uint32_t density = 40;  // DEFAULT_TAG_DENSITY, include/oxli/oxli.hh:83
    const int k = g->k;
    auto hash_at = [&](uint64_t r, uint64_t j) -> uint64_t {
        const uint64_t pos = j + r * (uint64_t)(k - 1);
        return b.hash == MURMUR ? murmur_canonical(b.bytes.data() + pos, k) : canonical2(window2(b.words.data(), pos, k), k);
    };
    // first position >= j in [j, e) that is NOT new (e if none)
    auto next_old = [&](uint64_t j, uint64_t e) -> uint64_t {
        while (j < e) {
            uint32_t w = ~nb[j >> 5] >> (j & 31);   // old k-mers of this word from j on
            const uint64_t wend = (j | 31) + 1;
            if (w) {
                const uint64_t p = j + (uint64_t)__builtin_ctz(w);
                return p < e ? p : e;
            }
            j = wend;
        }
        return e;
    };
    // tags are inserted in prefetched groups: the pending ones go in before
    // any membership test (an old k-mer) and at the end of the batch
    g->tags.reserve(g->tags.size() + b.nkmers() / (density - 1) + b.nreads() + 64);
    uint64_t pend[64];
    uint32_t npend = 0;
    auto flush = [&] {
        g->tags.insert_batch(pend, npend);
        npend = 0;
    };
    auto add_tag = [&](uint64_t h) {
        pend[npend++] = h;
        if (npend == 64) flush();
    };
    uint64_t consumed = 0;
    for (uint64_t r = 0; r < b.nreads(); r++) {
        const uint64_t a = b.koff[r], e = b.koff[r + 1];
        uint32_t since = density / 2 + 1;
        for (uint64_t j = a; j < e;) {
            const uint64_t q = next_old(j, e);   // [j, q): new k-mers
            if (q > j) {
                const uint64_t t = q - j;
                consumed += t;
                // since + i for the i-th new k-mer (1-based); a tag at since
                // >= density resets it to 1, so tags fall on new k-mers
                // j + (density - since) - 1, then every density - 1 more
                uint64_t p = since >= density ? j : j + (density - since) - 1;
                uint64_t last_tag = ~0ull;
                for (; p < q; p += density - 1) {
                    add_tag(hash_at(r, p));
                    last_tag = p;
                }
                since = last_tag == ~0ull ? since + (uint32_t)t : (uint32_t)(q - last_tag);
                j = q;
            }
            if (j >= e) break;
            // an old k-mer: a tag already resets the count
            const uint64_t h = hash_at(r, j);
            if (npend) flush();
            since = g->tags.count(h) ? 1 : since + 1;
            if (since >= density) {
                add_tag(h);
                since = 1;
            }
            j++;
        }
        // every packed read holds >= 1 k-mer; the reference also tags the
        // (uninitialised) k-mer of reads shorter than k -- not reproduced
        if (e > a && since >= density / 2 - 1) add_tag(hash_at(r, e - 1));
    }
    flush();
    return consumed;
}

// The tag state machine of a consume_seqfile_and_tag call runs on its own
// host thread, batch by batch in stream order, while the calling thread
// already feeds the next batch to the device (the device pass needs no tag
// state).  Only that thread touches the tag set until finish().
struct TagPipe {
    Graph *g;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<HostBatch, std::vector<uint32_t>>> q;
    bool done = false;
    std::exception_ptr err;
    uint64_t consumed = 0;
    explicit TagPipe(Graph *g_) : g(g_) {
        th = std::thread([this] {
            for (;;) {
                std::pair<HostBatch, std::vector<uint32_t>> job;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return done || !q.empty(); });
                    if (q.empty()) return;
                    job = std::move(q.front());
                    q.pop_front();
                    cv.notify_all();
                }
                try {
                    if (!err) consumed += tag_batch(g, job.first, job.second.data());
                } catch (...) {
                    err = std::current_exception();
                }
            }
        });
    }
    // at most two batches wait (bounded host memory)
    void push(HostBatch &&b, std::vector<uint32_t> &&bits) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return q.size() < 2; });
        q.emplace_back(std::move(b), std::move(bits));
        cv.notify_all();
    }
    // every pushed batch tagged; the tagged k-mer count, or the tagger's error
    uint64_t finish() {
        {
            std::lock_guard<std::mutex> lk(mu);
            done = true;
            cv.notify_all();
        }
        if (th.joinable()) th.join();
        if (err) std::rethrow_exception(err);
        return consumed;
    }
    ~TagPipe() {
        if (th.joinable()) {
            {
                std::lock_guard<std::mutex> lk(mu);
                done = true;
                cv.notify_all();
            }
            th.join();
        }
    }
};
static thread_local TagPipe *t_tagpipe = nullptr;   // set by kh_consume_parser (mode 1)

// mode 0: count; 1: count and tag (through t_tagpipe when set: the batch is
// moved to the tagger, so callers must not use it afterwards)
static void consume_batch(Graph *g, HostBatch &b, int mode, uint64_t *consumed) {
    if (b.nkmers() == 0) return;
    if (mode == 0) {
        engine_consume_host(g, b, nullptr);
        *consumed += b.nkmers();
        return;
    }
    std::vector<uint32_t> bits((b.nkmers() + 31) / 32);
    PassOut out;
    out.h_newbits = bits.data();
    engine_consume_host(g, b, &out);
    if (t_tagpipe) t_tagpipe->push(std::move(b), std::move(bits));
    else *consumed += tag_batch(g, b, bits.data());
}

static uint64_t batch_bases_cap(Graph *g) { return g->batch_kmers * 2 + (1u << 20); }

// Host threads for the pipelined feed: OMP_NUM_THREADS (the job's CPU share
// on a shared node) or the hardware threads, at most 16.
static int feed_threads() {
    int n = (int)std::thread::hardware_concurrency();
    const char *e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) n = std::min(n > 0 ? n : 1, atoi(e));
    const char *f = getenv("KH_FEED_THREADS");   // development override
    if (f && atoi(f) > 0) n = atoi(f);
    return std::max(1, std::min(16, n));
}

// consume_seqfile (mode 0) as a pipeline: one reader thread runs the parser
// (FastxReader::get_next_read semantics, read_parsers.cc:329-372) into raw
// batches; packer threads clean and 2-bit pack them (_to_valid_dna,
// read_parsers.cc:53-69); the calling thread uploads and consumes them on the
// device in parse order, so tables and counters equal the serial path's.  A
// parse error stops the reader: every read before it is consumed, then the
// error is raised (as the reference does).
struct FeedSlot {
    RawBatch raw;
    HostBatch packed;
    bool ready = false;
};
static void pack_raw(const RawBatch &raw, HostBatch &b, int k, int hash) {
    b.hash = hash;
    const char *p = raw.seq.data();
    for (uint32_t n : raw.len) {
        b.append(p, n, k, true);
        p += n;
    }
}

// Chunk-parallel feed of a plain or BGZF file (kh_parser.cpp
// parser_plain_open): worker threads parse and pack chunks of ~64 MB of the
// (inflated) stream cut at record starts; the calling thread consumes them in
// file order after checking that each chunk starts where the previous one
// really ended and could be parsed on its own (otherwise it parses the rest
// of the input itself, serially).  Same reads, same order, same errors as the
// serial parser.
static bool consume_chunked(Graph *g, Parser *parser, PlainFile *pf, int mode, uint64_t *nreads_out,
                            uint64_t *consumed) {
    struct Chunk {
        std::vector<RawBatch> raw;
        std::vector<HostBatch> packed;
        uint64_t nreads = 0;
        size_t start = 0, end = 0;
        std::exception_ptr err;
        bool ready = false, redo = false;
    };
    const size_t n = plain_size(pf);
    const char *ce = getenv("KH_FEED_CHUNK");   // development / tests: chunk bytes
    const size_t CH = ce && atoll(ce) > 0 ? (size_t)atoll(ce) : (size_t)64 << 20;
    const size_t nch = (n + CH - 1) / CH;
    // no recognisable record start inside the second chunk (CRLF or wrapped
    // FASTQ): the streaming reader/packer pipeline instead
    if (nch > 1 && !plain_chunkable(pf, CH)) return false;
    parser_plain_commit(parser);
    const int T = std::max(1, feed_threads() - 1);
    const size_t depth = (size_t)T * 2;
    const uint64_t maxk = std::min<uint64_t>(g->batch_kmers, 1ull << 27);
    const int k = g->k, hash = g->hash;
    std::vector<std::unique_ptr<Chunk>> ch(nch);
    for (auto &c : ch) c.reset(new Chunk());
    std::mutex mu;
    std::condition_variable cv;
    size_t next = 0, taken_upto = 0;   // next chunk to parse; chunks below taken_upto are consumed
    bool stop = false;
    std::vector<std::thread> workers;
    for (int t = 0; t < T; t++)
        workers.emplace_back([&] {
            for (;;) {
                size_t c;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || next >= nch || next < taken_upto + depth; });
                    if (stop || next >= nch) return;
                    c = next++;
                }
                Chunk &C = *ch[c];
                try {
                    plain_parse_chunk(pf, c, CH, k, maxk, C.raw, &C.nreads, &C.start, &C.end, &C.redo);
                } catch (...) {
                    C.err = std::current_exception();
                }
                for (const RawBatch &r : C.raw) {
                    C.packed.emplace_back();
                    pack_raw(r, C.packed.back(), k, hash);
                }
                std::vector<RawBatch>().swap(C.raw);
                std::lock_guard<std::mutex> lk(mu);
                C.ready = true;
                cv.notify_all();
            }
        });
    auto finish = [&] {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        for (auto &t : workers) t.join();
    };
    uint64_t total = 0;
    size_t true_end = 0;   // where the reads consumed so far really end
    // after parser_plain_commit the parser's own source is stopped: every exit
    // (errors included) must mark it drained exactly once, or a later read
    // from it would wait forever for a producer that is gone
    bool drained = false;
    auto drain = [&] {
        if (drained) return;
        drained = true;
        *nreads_out = total;
        parser_mark_drained(parser, total);
    };
    bool serial_rest = false;
    // the chunks' packed batches go to the device merged up to `lim` k-mers
    // (a device pass per ~27M-k-mer chunk batch would cost its fixed
    // overheads 50 times per 1.3e9 k-mers)
    const uint64_t lim = std::min<uint64_t>(g->batch_kmers, 1ull << 30);
    HostBatch acc;
    acc.hash = hash;
    auto flush = [&] {
        if (acc.nkmers()) consume_batch(g, acc, mode, consumed);
        acc = HostBatch();
        acc.hash = hash;
    };
    auto take = [&](HostBatch &b) {
        if (acc.nkmers() && acc.nkmers() + b.nkmers() > lim) flush();
        if (!acc.nkmers()) acc = std::move(b);
        else acc.merge(b);
    };
    try {
        for (size_t c = 0; c < nch; c++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return ch[c]->ready; });
            }
            Chunk &C = *ch[c];
            // a chunk start that was not a record start, or a chunk that could
            // not be parsed on its own
            if (C.redo || (C.start != true_end && !(C.start >= n && true_end >= n))) {
                serial_rest = true;
                break;
            }
            for (HostBatch &b : C.packed) {
                take(b);
                HostBatch().words.swap(b.words);
            }
            total += C.nreads;
            true_end = C.end;
            if (C.err) {
                flush();
                drain();
                std::rethrow_exception(C.err);
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                taken_upto = c + 1;
                cv.notify_all();
            }
            C.packed.clear();
        }
    } catch (...) {
        finish();
        drain();
        throw;
    }
    finish();
    try {
        flush();
    } catch (...) {
        drain();
        throw;
    }
    // the rest of the input serially
    if (serial_rest && true_end < n) {
        try {
            plain_parse_rest(pf, true_end, CH, k, maxk, [&](RawBatch &r) {
                HostBatch b;
                pack_raw(r, b, k, hash);
                consume_batch(g, b, mode, consumed);
            }, &total);
        } catch (...) {
            drain();
            throw;
        }
    }
    drain();
    return true;
}

// mode 0: consume (count); 1: consume and tag (consume_batch)
static void consume_pipelined(Graph *g, Parser *parser, int mode, uint64_t *nreads_out, uint64_t *consumed) {
    if (PlainFile *pf = parser_plain_open(parser)) {
        std::unique_ptr<PlainFile, void (*)(PlainFile *)> hold(pf, parser_plain_close);
        if (consume_chunked(g, parser, pf, mode, nreads_out, consumed)) return;
    }
    const int T = feed_threads();
    const int npack = std::max(1, T - 1);
    const int depth = npack + 2;                       // batches in flight
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::unique_ptr<FeedSlot>> slots;       // parse order
    uint64_t seq_parsed = 0;                           // batches the reader produced
    bool reader_done = false, stop = false;
    std::exception_ptr reader_err;
    uint64_t taken = 0;
    std::deque<FeedSlot *> to_pack;
    // feed batches of at most 2^27 k-mers: host memory stays ~0.2 GB per batch in flight
    const uint64_t maxk = std::min<uint64_t>(g->batch_kmers, 1ull << 27), maxb = maxk * 2 + (1u << 20);
    const int k = g->k, hash = g->hash;
    std::thread reader([&] {
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || (int)slots.size() < depth; });
                if (stop) break;
            }
            std::unique_ptr<FeedSlot> sl(new FeedSlot());
            bool done = false;
            uint64_t t = 0;
            std::exception_ptr err;
            try {
                parser_fill_raw(parser, sl->raw, k, maxk, maxb, &done, &t);
            } catch (...) {
                err = std::current_exception();
            }
            std::lock_guard<std::mutex> lk(mu);
            taken += t;
            to_pack.push_back(sl.get());
            slots.push_back(std::move(sl));
            seq_parsed++;
            if (err) reader_err = err;
            if (err || done) reader_done = true;
            cv.notify_all();
            if (reader_done) break;
        }
        std::lock_guard<std::mutex> lk(mu);
        reader_done = true;
        cv.notify_all();
    });
    std::vector<std::thread> packers;
    for (int i = 0; i < npack; i++)
        packers.emplace_back([&] {
            for (;;) {
                FeedSlot *sl;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || !to_pack.empty() || reader_done; });
                    if (to_pack.empty()) {
                        if (stop || reader_done) return;
                        continue;
                    }
                    sl = to_pack.front();
                    to_pack.pop_front();
                }
                HostBatch &b = sl->packed;
                b.hash = hash;
                const char *p = sl->raw.seq.data();
                for (uint32_t n : sl->raw.len) {
                    b.append(p, n, k, true);
                    p += n;
                }
                std::vector<char>().swap(sl->raw.seq);
                std::lock_guard<std::mutex> lk(mu);
                sl->ready = true;
                cv.notify_all();
            }
        });
    auto finish = [&] {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        reader.join();
        for (auto &t : packers) t.join();
    };
    try {
        for (;;) {
            std::unique_ptr<FeedSlot> sl;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return (!slots.empty() && slots.front()->ready) || (reader_done && slots.empty()); });
                if (slots.empty()) break;
                sl = std::move(slots.front());
                slots.pop_front();
                cv.notify_all();
            }
            consume_batch(g, sl->packed, mode, consumed);
        }
    } catch (...) {
        finish();
        throw;
    }
    finish();
    *nreads_out = taken;
    if (reader_err) std::rethrow_exception(reader_err);
}

extern "C" {

int kh_consume_parser(kh_graph *h, kh_parser *ph, int mode, uint32_t *reads, uint64_t *kmers) {
    *reads = 0;
    *kmers = 0;
    return guard([&] {
        CHECK_PTR(h);
        CHECK_PTR(ph);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        uint64_t consumed = 0, nreads = 0;
        if (feed_threads() > 1) {
            std::unique_ptr<TagPipe> tp(mode == 1 ? new TagPipe(g) : nullptr);
            t_tagpipe = tp.get();
            try {
                consume_pipelined(g, ph->p, mode, &nreads, &consumed);
            } catch (...) {
                t_tagpipe = nullptr;
                // the reads before the error are consumed and tagged; the
                // caller sees the original error (a tagger failure of its
                // own would otherwise replace it and lose the counts)
                *reads = (uint32_t)nreads;
                *kmers = consumed;
                if (tp) {
                    try {
                        consumed += tp->finish();
                        *kmers = consumed;
                    } catch (...) {
                    }
                }
                throw;
            }
            t_tagpipe = nullptr;
            if (tp) consumed += tp->finish();
            *reads = (uint32_t)nreads;
            *kmers = consumed;
            return;
        }
        HostBatch b;
        b.hash = g->hash;
        bool done = false;
        while (!done) {
            b.clear();
            try {
                parser_fill_batch(ph->p, b, g->k, g->batch_kmers, batch_bases_cap(g), &done, &nreads);
            } catch (...) {
                // the reference consumed every read before the bad one, then throws
                consume_batch(g, b, mode, &consumed);
                *reads = (uint32_t)nreads;
                *kmers = consumed;
                throw;
            }
            consume_batch(g, b, mode, &consumed);
        }
        *reads = (uint32_t)nreads;
        *kmers = consumed;
    });
}

int kh_consume_parser_filtered(kh_graph *h, kh_parser *ph, uint32_t num_bands, uint32_t band, kh_graph *mh,
                               uint32_t threshold, int consume_masked, uint32_t *reads, uint64_t *kmers) {
    *reads = 0;
    *kmers = 0;
    return guard([&] {
        CHECK_PTR(h);
        CHECK_PTR(ph);
        Graph *g = h->g;
        BandMask f;
        if (num_bands) {
            // compute_band_interval: note the reference's check is band > num_bands,
            // and band == num_bands wraps to an empty interval in u64 arithmetic
            if (band > num_bands)
                fail(KH_EVALUE, "'band' must be in the interval [0, 'num_bands'), " + std::to_string(band) +
                                    " not in [0, " + std::to_string(num_bands) + ")");
            const uint64_t bs = UINT64_MAX / num_bands;
            f.num_bands = num_bands;
            f.band_lo = bs * band;
            f.band_hi = bs * (band + 1);
        }
        if (mh) {
            if (mh->g == g) fail(KH_EVALUE, "a table cannot be its own mask");
            if (mh->g->device != g->device) fail(KH_EVALUE, "mask table is on another device");
            f.mask = mh->g;
            f.threshold = threshold;
            f.consume_masked = consume_masked;
        }
        // table and mask locked together (no lock-order inversion between
        // two threads filtering each table by the other)
        std::unique_lock<std::recursive_mutex> lk(g->mu, std::defer_lock);
        std::unique_lock<std::recursive_mutex> mlk;
        if (f.mask) {
            mlk = std::unique_lock<std::recursive_mutex>(f.mask->mu, std::defer_lock);
            std::lock(lk, mlk);
        } else {
            lk.lock();
        }
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        b.hash = g->hash;
        bool done = false;
        uint64_t consumed = 0, nreads = 0;
        while (!done) {
            b.clear();
            try {
                parser_fill_batch(ph->p, b, g->k, g->batch_kmers, batch_bases_cap(g), &done, &nreads);
            } catch (...) {
                consumed += engine_consume_filtered(g, b, f);
                *reads = (uint32_t)nreads;
                *kmers = consumed;
                throw;
            }
            consumed += engine_consume_filtered(g, b, f);
        }
        *reads = (uint32_t)nreads;
        *kmers = consumed;
    });
}

int kh_consume_seqs(kh_graph *h, const char *seqs, const uint64_t *offsets, uint64_t nreads, int clean,
                    uint64_t *kmers) {
    *kmers = 0;
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        b.hash = g->hash;
        uint64_t consumed = 0;
        for (uint64_t r = 0; r < nreads; r++) {
            const char *s = seqs + offsets[r];
            // KmerIterator length = strlen (kmer_hash.cc:290)
            size_t len = strnlen(s, (size_t)(offsets[r + 1] - offsets[r]));
            if (len >= (size_t)g->k) b.append(s, len, g->k, clean != 0);
            if (b.nkmers() >= g->batch_kmers) {
                consume_batch(g, b, 0, &consumed);
                b.clear();
            }
        }
        consume_batch(g, b, 0, &consumed);
        *kmers = consumed;
    });
}

int kh_consume_packed_device(kh_graph *h, const uint64_t *d_words, const uint64_t *d_kmer_off, uint64_t nreads,
                             uint64_t nkmers) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        if (g->hash != TWOBIT) fail(KH_EVALUE, "packed 2-bit input requires a 2-bit hashing graph");
        engine_consume_twobit(g, d_words, d_kmer_off, nreads, nkmers, nullptr);
    });
}

int kh_consume_packed_fixed_device(kh_graph *h, const uint64_t *d_words, uint64_t nreads, uint32_t read_len) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        if (g->hash != TWOBIT) fail(KH_EVALUE, "packed 2-bit input requires a 2-bit hashing graph");
        engine_consume_twobit_fixed(g, d_words, nreads, read_len, nullptr);
    });
}

int kh_consume_bytes_fixed_device(kh_graph *h, const uint8_t *d_bytes, uint64_t nreads, uint32_t read_len) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        if (g->hash != MURMUR) fail(KH_EVALUE, "ASCII device input requires a Murmur hashing graph");
        engine_consume_bytes_fixed(g, d_bytes, nreads, read_len);
    });
}

int kh_median_counts_fixed_device(kh_graph *h, const void *d_reads, uint64_t nreads, uint32_t read_len,
                                  uint16_t *d_med, float *d_avg, float *d_stddev) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        engine_median_fixed_device(g, d_reads, nreads, read_len, d_med, d_avg, d_stddev);
    });
}

int kh_add_hashes(kh_graph *h, const uint64_t *hashes, uint64_t n, uint8_t *is_new) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        if (!n) return;
        DevBuf d(n * 8);
        KH_HIP(hipMemcpy(d.p, hashes, n * 8, hipMemcpyHostToDevice));
        PassOut out{is_new, nullptr};
        engine_consume_hashes(g, d.as<uint64_t>(), n, is_new ? &out : nullptr);
    });
}

int kh_get_counts(kh_graph *h, const uint64_t *hashes, uint64_t n, uint16_t *out) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        engine_get_counts(g, hashes, n, out);
    });
}

int kh_median_counts(kh_graph *h, const char *seqs, const uint64_t *offsets, uint64_t nreads, uint16_t *med,
                     float *avg, float *stddev, uint8_t *status) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        b.hash = g->hash;
        std::vector<uint64_t> idx;
        for (uint64_t r = 0; r < nreads; r++) {
            const char *s = seqs + offsets[r];
            size_t len = strnlen(s, (size_t)(offsets[r + 1] - offsets[r]));
            if (len >= (size_t)g->k) {
                b.append(s, len, g->k, false);
                idx.push_back(r);
                status[r] = 0;
            } else {
                status[r] = 1;
                med[r] = 0;
                avg[r] = 0;
                stddev[r] = 0;
            }
        }
        std::vector<uint16_t> m(idx.size());
        std::vector<float> a(idx.size()), s(idx.size());
        engine_median(g, b, m.data(), a.data(), s.data());
        for (size_t t = 0; t < idx.size(); t++) {
            med[idx[t]] = m[t];
            avg[idx[t]] = a[t];
            stddev[idx[t]] = s[t];
        }
    });
}

// a batch of raw (uncleaned) reads of >= k bases; the others get status 1
static void raw_batch(Graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads, HostBatch &b,
                      std::vector<uint64_t> &idx, uint8_t *status) {
    b.hash = g->hash;
    for (uint64_t r = 0; r < nreads; r++) {
        const char *s = seqs + offsets[r];
        const size_t len = strnlen(s, (size_t)(offsets[r + 1] - offsets[r]));
        const bool ok = len >= (size_t)g->k;
        if (ok) {
            b.append(s, len, g->k, false);
            idx.push_back(r);
        }
        if (status) status[r] = ok ? 0 : 1;
    }
}

int kh_graph_kmer_hashes(kh_graph *h, const char *seqs, const uint64_t *offsets, uint64_t nreads, uint64_t *out,
                         uint64_t *n_out) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        std::vector<uint64_t> idx;
        raw_batch(g, seqs, offsets, nreads, b, idx, nullptr);
        *n_out = b.nkmers();
        if (b.nkmers()) engine_hash_batch(g, b, out);
    });
}

int kh_graph_kmer_counts(kh_graph *h, const char *seqs, const uint64_t *offsets, uint64_t nreads, uint16_t *out,
                         uint64_t *n_out) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        std::vector<uint64_t> idx;
        raw_batch(g, seqs, offsets, nreads, b, idx, nullptr);
        *n_out = b.nkmers();
        if (b.nkmers()) engine_kmer_counts(g, b, out);
    });
}

int kh_median_at_least(kh_graph *h, const char *seqs, const uint64_t *offsets, uint64_t nreads, uint32_t cutoff,
                       uint8_t *out, uint8_t *status) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        HostBatch b;
        std::vector<uint64_t> idx;
        raw_batch(g, seqs, offsets, nreads, b, idx, status);
        for (uint64_t r = 0; r < nreads; r++) out[r] = 0;
        if (!b.nreads()) return;
        std::vector<uint8_t> res(b.nreads());
        engine_median_at_least(g, b, cutoff, res.data());
        for (size_t t = 0; t < idx.size(); t++) out[idx[t]] = res[t];
    });
}

int kh_abundance_distribution(kh_graph *h, kh_parser *ph, kh_graph *th, uint64_t *dist) {
    return guard([&] {
        CHECK_PTR(h);
        CHECK_PTR(ph);
        CHECK_PTR(th);
        Graph *g = h->g, *t = th->g;
        // both tables locked together (std::lock's deadlock avoidance): two
        // threads calling a.abundance_distribution(.., b) and
        // b.abundance_distribution(.., a) must not take them in opposite order
        std::unique_lock<std::recursive_mutex> lk(g->mu, std::defer_lock), lk2(t->mu, std::defer_lock);
        if (g == t) lk.lock();
        else std::lock(lk, lk2);
        KH_HIP(hipSetDevice(g->device));
        if (t->device != g->device) fail(KH_EVALUE, "tracking table must live on the same device");
        memset(dist, 0, 65536 * sizeof(uint64_t));
        HostBatch b;
        b.hash = g->hash;
        bool done = false;
        while (!done) {
            b.clear();
            uint64_t taken = 0;
            parser_fill_batch(ph->p, b, g->k, g->batch_kmers, batch_bases_cap(g), &done, &taken);
            const uint64_t nk = b.nkmers();
            if (!nk) continue;
            // self's iterator hashes (hashtable.cc:476-480), tracked in stream order
            std::vector<uint64_t> hs(nk);
            engine_hash_batch(g, b, hs.data());
            std::vector<uint8_t> isnew(nk);
            DevBuf d(nk * 8);
            KH_HIP(hipMemcpy(d.p, hs.data(), nk * 8, hipMemcpyHostToDevice));
            PassOut out{isnew.data(), nullptr};
            engine_consume_hashes(t, d.as<uint64_t>(), nk, &out);   // passes of t's batch size, in order
            std::vector<uint64_t> sel;
            for (uint64_t j = 0; j < nk; j++)
                if (isnew[j]) sel.push_back(hs[j]);
            std::vector<uint16_t> cnt(sel.size());
            engine_get_counts(g, sel.data(), sel.size(), cnt.data());
            for (uint16_t c : cnt) dist[c]++;
        }
    });
}

// ---------------- tables & files ------------------------------------------------
int kh_graph_table_nbytes(kh_graph *h, int i, uint64_t *out) {
    return guard([&] {
        CHECK_PTR(h);
        if (i < 0 || i >= h->g->n) fail(KH_EVALUE, "table index out of range");
        *out = h->g->nbytes[(size_t)i];
    });
}

int kh_graph_copy_table(kh_graph *h, int i, uint8_t *dst) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        if (i < 0 || i >= g->n) fail(KH_EVALUE, "table index out of range");
        KH_HIP(hipSetDevice(g->device));
        engine_download_table(g, i, dst);
    });
}

}  // extern "C"

// writer abstraction: plain or gzip (ByteStorageFile::save picks by extension,
// src/oxli/storage.cc:255-269).  The gzip writer advances through the table
// (the reference re-writes the table head for tables > INT_MAX bytes, F7).
struct Out {
    FILE *f = nullptr;
    gzFile gz = nullptr;
    void write(const void *p, size_t n) {
        const char *c = (const char *)p;
        while (n) {
            size_t chunk = std::min<size_t>(n, (size_t)INT_MAX / 2);
            if (gz) {
                if (gzwrite(gz, c, (unsigned)chunk) == 0) fail(KH_EFILE, "gzwrite failed while writing counting hash");
            } else if (fwrite(c, 1, chunk, f) != chunk) {
                fail(KH_EFILE, strerror(errno));
            }
            c += chunk;
            n -= chunk;
        }
    }
    void close() {
        if (gz) { gzclose(gz); gz = nullptr; }
        if (f) {
            if (fclose(f) != 0) { f = nullptr; fail(KH_EFILE, strerror(errno)); }
            f = nullptr;
        }
    }
    ~Out() {
        if (gz) gzclose(gz);
        if (f) fclose(f);
    }
};

static bool ends_with_gz(const std::string &s) {
    size_t dot = s.find_last_of('.');
    return dot != std::string::npos && s.substr(dot + 1) == "gz";
}

extern "C" int kh_graph_save(kh_graph *h, const char *path) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        Out o;
        const bool gz = g->kind == BYTE && ends_with_gz(path);
        if (gz) {
            o.gz = gzopen(path, "wb");
            if (!o.gz) fail(KH_EFILE, strerror(errno));
        } else {
            o.f = fopen(path, "wb");
            if (!o.f) fail(KH_EFILE, strerror(errno));
        }
        // header: doc/dev/binary-file-formats.rst; storage.cc:99-136 (bit),
        // 582-638 (byte), 772-803 (nibble)
        o.write("OXLI", 4);
        unsigned char version = 4, type = (unsigned char)g->kind;
        o.write(&version, 1);
        o.write(&type, 1);
        if (g->kind == BYTE) {
            unsigned char bc = g->use_bigcount ? 1 : 0;
            o.write(&bc, 1);
        }
        uint32_t k = (uint32_t)g->k;
        unsigned char n = (unsigned char)g->n;
        uint64_t occ = g->n_occupied;
        o.write(&k, 4);
        o.write(&n, 1);
        o.write(&occ, 8);
        std::vector<uint8_t> buf;
        for (int i = 0; i < g->n; i++) {
            uint64_t sz = g->sizes[(size_t)i];
            o.write(&sz, 8);
            buf.resize(g->nbytes[(size_t)i]);
            engine_download_table(g, i, buf.data());
            o.write(buf.data(), buf.size());
        }
        if (g->kind == BYTE) {
            std::vector<std::pair<uint64_t, uint16_t>> v(g->bigcounts.begin(), g->bigcounts.end());
            std::sort(v.begin(), v.end());
            uint64_t nb = v.size();
            o.write(&nb, 8);
            for (auto &kv : v) {
                o.write(&kv.first, 8);
                o.write(&kv.second, 2);
            }
        }
        o.close();
    });
}

// reader: plain or gzip (ByteStorageGzFileReader for *.gz countgraphs)
struct In {
    gzFile gz = nullptr;
    std::string path;
    void read(void *p, size_t n) {
        char *c = (char *)p;
        while (n) {
            unsigned chunk = (unsigned)std::min<size_t>(n, (size_t)INT_MAX / 2);
            int got = gzread(gz, c, chunk);
            if (got <= 0) fail(KH_EFILE, "Unexpected end of k-mer graph file: " + path);
            c += got;
            n -= (size_t)got;
        }
    }
    ~In() { if (gz) gzclose(gz); }
};

// raw header reader for khmer.extract_*_info (see include/khmer_hip.h)
extern "C" int kh_file_header(const char *path, int layout, int64_t *out) {
    return guard([&] {
        CHECK_PTR(path);
        CHECK_PTR(out);
        FILE *f = fopen(path, "rb");
        if (!f) fail(KH_EFILE, std::string("cannot open ") + path);
        unsigned char buf[32];
        const size_t got = fread(buf, 1, sizeof buf, f);
        fclose(f);
        size_t at = 0;
        auto take = [&](size_t n) -> uint64_t {
            if (at + n > got) fail(KH_EFILE, std::string("short header in ") + path);
            uint64_t v = 0;
            for (size_t b = 0; b < n; b++) v |= (uint64_t)buf[at + b] << (8 * b);
            at += n;
            return v;
        };
        take(4);
        if (memcmp(buf, "OXLI", 4) != 0) fail(KH_EFILE, std::string("missing OXLI signature in ") + path);
        out[0] = (int64_t)take(1);
        out[1] = (int64_t)take(1);
        out[2] = (layout == 1 && out[1] != NIBBLE) ? (int64_t)take(1) : -1;
        out[3] = (int64_t)take(4);
        out[4] = (int64_t)take(1);
        out[5] = (int64_t)take(8);
        out[6] = (int64_t)take(8);
    });
}

extern "C" int kh_graph_load(const char *path, int expected_storage, int hash_kind, int device, kh_graph **out) {
    return guard([&] {
        In in;
        in.path = path;
        in.gz = gzopen(path, "rb");
        if (!in.gz) fail(KH_EFILE, std::string("Cannot open k-mer graph file: ") + path);
        char sig[4];
        unsigned char version = 0, type = 0;
        in.read(sig, 4);
        in.read(&version, 1);
        in.read(&type, 1);
        if (memcmp(sig, "OXLI", 4) != 0) {
            char msg[128];
            snprintf(msg, sizeof msg, "Does not start with signature for a oxli file: 0x%x%x%x%x Should be: OXLI",
                     (unsigned char)sig[0], (unsigned char)sig[1], (unsigned char)sig[2], (unsigned char)sig[3]);
            fail(KH_EFILE, msg);
        }
        if (version != 4)
            fail(KH_EFILE, "Incorrect file format version " + std::to_string(version) + " while reading k-mer graph from " +
                               path + "; should be 4");
        if (type != (unsigned char)expected_storage)
            fail(KH_EFILE, "Incorrect file format type " + std::to_string(type) + " while reading k-mer graph from " + path);
        unsigned char bc = 0;
        if (type == BYTE) in.read(&bc, 1);
        uint32_t k = 0;
        unsigned char n = 0;
        uint64_t occ = 0;
        in.read(&k, 4);
        in.read(&n, 1);
        in.read(&occ, 8);
        if (n < 1) fail(KH_EFILE, std::string("Unexpected end of k-mer graph file: ") + path);
        if (n > MAXT) fail(KH_EFILE, std::string("too many tables in k-mer graph file: ") + path);
        std::vector<uint64_t> sizes;
        std::vector<std::vector<uint8_t>> tabs;
        for (int i = 0; i < n; i++) {
            uint64_t sz = 0;
            in.read(&sz, 8);
            if (sz == 0) fail(KH_EFILE, std::string("zero-sized table in k-mer graph file: ") + path);
            uint64_t nb = type == BIT ? sz / 8 + 1 : type == NIBBLE ? sz / 2 + 1 : sz;
            sizes.push_back(sz);
            tabs.emplace_back();
            // bounded chunks: a header that claims more than the file holds
            // fails at end of file rather than allocating the claimed size
            for (uint64_t a = 0; a < nb; a += (64u << 20)) {
                const uint64_t m = std::min<uint64_t>(64u << 20, nb - a);
                tabs.back().resize(a + m);
                in.read(tabs.back().data() + a, m);
            }
        }
        std::vector<std::pair<uint64_t, uint16_t>> bcs;
        if (type == BYTE) {
            uint64_t nbig = 0;
            in.read(&nbig, 8);
            for (uint64_t t = 0; t < nbig; t++) {
                uint64_t key;
                uint16_t val;
                in.read(&key, 8);
                in.read(&val, 2);
                bcs.emplace_back(key, val);
            }
        }
        int kk = (int)k;
        if (hash_kind == TWOBIT && kk > 32) fail(KH_EFILE, "k-mer size in file exceeds 32");
        Graph *g = graph_create(type, hash_kind, kk, sizes.data(), n, device);
        try {
            for (int i = 0; i < n; i++) engine_upload_table(g, i, tabs[(size_t)i].data());
            g->n_occupied = occ;
            g->n_unique = 0;  // not stored in the file (storage.hh:143-165)
            g->use_bigcount = bc != 0;
            g->prm.use_bigcount = bc ? 1 : 0;
            for (auto &kv : bcs) g->bigcounts[kv.first] = kv.second;
            g->bc_dirty = true;
        } catch (...) {
            delete g;
            throw;
        }
        *out = new kh_graph{g};
    });
}

// ---------------- tags ------------------------------------------------------------
extern "C" {

int kh_graph_n_tags(kh_graph *h, uint64_t *out) {
    return guard([&] {
        CHECK_PTR(h);
        std::lock_guard<std::recursive_mutex> lk(h->g->mu);
        *out = h->g->tags.size();
    });
}

int kh_graph_get_tags(kh_graph *h, uint64_t *out) {
    return guard([&] {
        CHECK_PTR(h);
        std::lock_guard<std::recursive_mutex> lk(h->g->mu);
        std::vector<uint64_t> v = h->g->tags.sorted();
        memcpy(out, v.data(), v.size() * 8);
    });
}

int kh_graph_add_tag(kh_graph *h, uint64_t t) {
    return guard([&] {
        CHECK_PTR(h);
        std::lock_guard<std::recursive_mutex> lk(h->g->mu);
        h->g->tags.insert(t);
    });
}

// Hashgraph::save_tagset (src/oxli/hashgraph.cc:55-88); std::set order = ascending
int kh_graph_save_tagset(kh_graph *h, const char *path) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        std::vector<uint64_t> v = g->tags.sorted();
        Out o;
        o.f = fopen(path, "wb");
        if (!o.f) fail(KH_EFILE, strerror(errno));
        o.write("OXLI", 4);
        unsigned char version = 4, type = 3;  // SAVED_TAGS
        o.write(&version, 1);
        o.write(&type, 1);
        uint32_t k = (uint32_t)g->k;
        uint64_t n = v.size();
        uint32_t density = 40;
        o.write(&k, 4);
        o.write(&n, 8);
        o.write(&density, 4);
        o.write(v.data(), n * 8);
        o.close();
    });
}

// Hashgraph::load_tagset (src/oxli/hashgraph.cc:90-152)
int kh_graph_load_tagset(kh_graph *h, const char *path, int clear) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        In in;
        in.path = path;
        in.gz = gzopen(path, "rb");
        if (!in.gz) fail(KH_EFILE, std::string("Cannot open tagset file: ") + path);
        char sig[4];
        unsigned char version = 0, type = 0;
        in.read(sig, 4);
        in.read(&version, 1);
        in.read(&type, 1);
        if (memcmp(sig, "OXLI", 4) != 0) fail(KH_EFILE, "Does not start with signature for a oxli file");
        if (version != 4) fail(KH_EFILE, "Incorrect file format version " + std::to_string(version) +
                                             " while reading tagset from " + path + "; should be 4");
        if (type != 3) fail(KH_EFILE, "Incorrect file format type " + std::to_string(type) + " while reading tagset from " + path);
        uint32_t k = 0, density = 0;
        uint64_t n = 0;
        in.read(&k, 4);
        in.read(&n, 8);
        in.read(&density, 4);
        if ((int)k != g->k) fail(KH_EFILE, "Incorrect k-mer size in tagset file");
        // read in bounded chunks: a corrupt count fails at end of file instead
        // of allocating whatever the header claims
        std::vector<uint64_t> v;
        for (uint64_t a = 0; a < n; a += (1u << 20)) {
            const uint64_t m = std::min<uint64_t>(1u << 20, n - a);
            const size_t old = v.size();
            v.resize(old + m);
            in.read(v.data() + old, m * 8);
        }
        if (clear) g->tags.clear();
        for (uint64_t t : v) g->tags.insert(t);
    });
}

}  // extern "C"

// ---------------- benchmark support -------------------------------------------------
extern "C" int kh_synth_packed_device(int device, uint64_t seed, uint64_t r0, uint64_t nreads, int read_len, int k,
                                      uint64_t *d_words, uint64_t *d_kmer_off) {
    return guard([&] {
        if (read_len < k || k < 1 || k > 32) fail(KH_EVALUE, "need 1 <= k <= read length and k <= 32");
        engine_synth_packed(device, seed, 0, r0, nreads, read_len, k, d_words, d_kmer_off);
    });
}

extern "C" int kh_synth_genomic_device(int device, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads,
                                       int read_len, int k, uint64_t *d_words, uint64_t *d_kmer_off) {
    return guard([&] {
        if (read_len < k || k < 1 || k > 32) fail(KH_EVALUE, "need 1 <= k <= read length and k <= 32");
        if (genome < (uint64_t)read_len) fail(KH_EVALUE, "genome shorter than a read");
        engine_synth_packed(device, seed, genome, r0, nreads, read_len, k, d_words, d_kmer_off);
    });
}

extern "C" int kh_unpack_ascii_device(int device, const uint64_t *d_words, uint64_t nbases, uint8_t *d_bytes) {
    return guard([&] { engine_unpack_ascii(device, d_words, nbases, d_bytes); });
}

extern "C" int kh_device_copy(int device, void *dst, const void *src, uint64_t nbytes) {
    return guard([&] {
        KH_HIP(hipSetDevice(device));
        KH_HIP(hipMemcpy(dst, src, nbytes, hipMemcpyDefault));
    });
}

extern "C" int kh_device_malloc(int device, uint64_t bytes, void **out) {
    return guard([&] {
        KH_HIP(hipSetDevice(device));
        KH_HIP(hipMalloc(out, bytes));
    });
}

extern "C" int kh_device_free(int device, void *p) {
    return guard([&] {
        KH_HIP(hipSetDevice(device));
        KH_HIP(hipFree(p));
    });
}

extern "C" int kh_device_synchronize(int device) {
    return guard([&] {
        KH_HIP(hipSetDevice(device));
        KH_HIP(hipDeviceSynchronize());
    });
}

extern "C" int kh_graph_set_profiling(kh_graph *h, int on) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        g->profile = on != 0;
        g->kstats.clear();
    });
}

extern "C" int kh_graph_set_schedule(kh_graph *h, int l1_chunk_tiles, int apply_dynamic) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        g->l1_chunk = l1_chunk_tiles < 0 ? -1 : l1_chunk_tiles;
        g->apply_dyn = apply_dynamic < 0 ? -1 : (apply_dynamic != 0);
    });
}

extern "C" int kh_graph_kernel_stats(kh_graph *h, char *buf, size_t cap, size_t *len) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        std::string s;
        char line[256];
        for (auto &kv : g->kstats) {
            snprintf(line, sizeof line, "%s\t%llu\t%.6f\n", kv.first.c_str(), (unsigned long long)kv.second.n,
                     kv.second.ms);
            s += line;
        }
        *len = s.size();
        if (buf && cap) {
            size_t n = std::min(cap - 1, s.size());
            memcpy(buf, s.data(), n);
            buf[n] = 0;
        }
    });
}

// reset a graph to its freshly constructed state (tables zeroed, counters,
// bigcounts and tags cleared) -- the benchmark's per-step reset
extern "C" int kh_graph_clear(kh_graph *h) {
    return guard([&] {
        CHECK_PTR(h);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        KH_HIP(hipSetDevice(g->device));
        dev_fill(g->d_tab, 0, g->arena_bytes, g->stream);
        KH_HIP(hipStreamSynchronize(g->stream));
        g->n_unique = g->n_occupied = 0;
        g->bigcounts.clear();
        g->bc_dirty = true;
        g->tags.clear();
    });
}

// ---------------------------------------------------------------------------
// sharded groups
extern "C" int kh_group_unique_id(unsigned char *out, size_t cap) {
    return guard([&] {
        CHECK_PTR(out);
        group_unique_id(out, cap);
    });
}

extern "C" int kh_group_create_mode(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables,
                                    int world, int rank, int nlocal, const int *devices, const unsigned char *uid,
                                    int mode, kh_group **out) {
    return guard([&] {
        CHECK_PTR(sizes);
        CHECK_PTR(devices);
        CHECK_PTR(out);
        *out = nullptr;
        if (mode != KH_GROUP_BROADCAST && mode != KH_GROUP_EXCHANGE && mode != KH_GROUP_DELTA)
            fail(KH_EVALUE, "unknown group mode");
        ShardGroup *G = group_create(storage, hash_kind, k, sizes, n_tables, world, rank, nlocal, devices, uid, mode);
        *out = new kh_group{G};
    });
}

extern "C" int kh_group_create(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int world,
                               int rank, int nlocal, const int *devices, const unsigned char *uid, kh_group **out) {
    return kh_group_create_mode(storage, hash_kind, k, sizes, n_tables, world, rank, nlocal, devices, uid,
                                KH_GROUP_BROADCAST, out);
}

extern "C" int kh_group_create_hosted_mode(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables,
                                           int world, int rank, int device, const kh_transport *transport, int mode,
                                           kh_group **out) {
    return guard([&] {
        CHECK_PTR(sizes);
        CHECK_PTR(transport);
        CHECK_PTR(out);
        *out = nullptr;
        if (mode != KH_GROUP_BROADCAST && mode != KH_GROUP_EXCHANGE && mode != KH_GROUP_DELTA)
            fail(KH_EVALUE, "unknown group mode");
        ShardGroup *G = group_create_hosted(storage, hash_kind, k, sizes, n_tables, world, rank, device, transport,
                                            mode);
        *out = new kh_group{G};
    });
}

extern "C" int kh_group_create_hosted(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables,
                                      int world, int rank, int device, const kh_transport *transport,
                                      kh_group **out) {
    return kh_group_create_hosted_mode(storage, hash_kind, k, sizes, n_tables, world, rank, device, transport,
                                       KH_GROUP_BROADCAST, out);
}

extern "C" int kh_group_comm_info(kh_group *grp, int *nranks, int *device) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(nranks);
        CHECK_PTR(device);
        group_comm_info(grp->G, nranks, device);
    });
}

extern "C" void kh_group_destroy(kh_group *grp) {
    if (!grp) return;
    group_destroy(grp->G);
    delete grp;
}

extern "C" int kh_group_shard(kh_group *grp, int l, kh_graph **out) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(out);
        *out = new kh_graph{group_shard(grp->G, l), false};
    });
}

extern "C" int kh_group_info(kh_group *grp, int *world, int *nlocal, int *rank0) {
    return guard([&] {
        CHECK_PTR(grp);
        *world = group_world(grp->G);
        *nlocal = group_nlocal(grp->G);
        *rank0 = group_rank(grp->G, 0);
    });
}

extern "C" int kh_group_slice(kh_group *grp, int l, int table, uint64_t *lo, uint64_t *size) {
    return guard([&] {
        CHECK_PTR(grp);
        Graph *g = group_shard(grp->G, l);
        if (table < 0 || table >= g->n) fail(KH_EVALUE, "no such table");
        *lo = g->lo[(size_t)table];
        *size = g->lsz[(size_t)table];
    });
}

extern "C" int kh_group_rank_slice(kh_group *grp, int rank, int table, uint64_t *lo, uint64_t *size) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(lo);
        CHECK_PTR(size);
        group_rank_slice(grp->G, rank, table, lo, size);
    });
}

extern "C" int kh_group_mode(kh_group *grp, int *mode) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(mode);
        *mode = group_exchange(grp->G);
    });
}

extern "C" int kh_group_consume_packed_fixed_device(kh_group *grp, const uint64_t *const *d_words, uint64_t nreads,
                                                    uint64_t read_len) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(d_words);
        std::vector<std::unique_lock<std::recursive_mutex>> locks;
        for (int l = 0; l < group_nlocal(grp->G); l++) locks.emplace_back(group_shard(grp->G, l)->mu);
        group_consume_fixed(grp->G, d_words, nreads, read_len);
    });
}

extern "C" int kh_group_consume_bytes_fixed_device(kh_group *grp, const uint8_t *const *d_bytes, uint64_t nreads,
                                                   uint64_t read_len) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(d_bytes);
        std::vector<std::unique_lock<std::recursive_mutex>> locks;
        for (int l = 0; l < group_nlocal(grp->G); l++) locks.emplace_back(group_shard(grp->G, l)->mu);
        group_consume_bytes_fixed(grp->G, d_bytes, nreads, read_len);
    });
}

extern "C" int kh_group_median_fixed_device(kh_group *grp, const void *const *d_reads, uint64_t nreads,
                                            uint64_t read_len, uint16_t *const *d_med, float *const *d_avg,
                                            float *const *d_sd) {
    return guard([&] {
        CHECK_PTR(grp);
        CHECK_PTR(d_reads);
        CHECK_PTR(d_med);
        CHECK_PTR(d_avg);
        CHECK_PTR(d_sd);
        std::vector<std::unique_lock<std::recursive_mutex>> locks;
        for (int l = 0; l < group_nlocal(grp->G); l++) locks.emplace_back(group_shard(grp->G, l)->mu);
        group_median_fixed(grp->G, d_reads, nreads, read_len, d_med, d_avg, d_sd);
    });
}

extern "C" int kh_group_counters(kh_group *grp, uint64_t *n_unique, uint64_t *n_occupied) {
    return guard([&] {
        CHECK_PTR(grp);
        group_counters(grp->G, n_unique, n_occupied);
    });
}

extern "C" int kh_group_wire_stats(kh_group *grp, uint64_t *dense_bytes, uint64_t *sent_bytes) {
    return guard([&] {
        CHECK_PTR(grp);
        group_wire_stats(grp->G, dense_bytes, sent_bytes);
    });
}

extern "C" int kh_graph_get_bigcounts(kh_graph *h, uint64_t *keys, uint16_t *vals, uint64_t cap, uint64_t *n) {
    return guard([&] {
        CHECK_PTR(h);
        CHECK_PTR(n);
        Graph *g = h->g;
        std::lock_guard<std::recursive_mutex> lk(g->mu);
        std::vector<std::pair<uint64_t, uint16_t>> v(g->bigcounts.begin(), g->bigcounts.end());
        std::sort(v.begin(), v.end());
        *n = v.size();
        if (cap >= v.size() && keys && vals)
            for (size_t i = 0; i < v.size(); i++) {
                keys[i] = v[i].first;
                vals[i] = v[i].second;
            }
    });
}
