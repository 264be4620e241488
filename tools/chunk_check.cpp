// Development: the chunk-parallel parse (kh_parser.cpp plain_parse_chunk /
// plain_parse_rest, in consume_chunked's order, one thread) against the
// streaming parser over the same file: reads parsed, a digest of the reads
// of >= k bases, and the error.  Host only (no device).
// Build: see tools/chunk_check.sh.  Usage: chunk_check <file> <chunk bytes> [k]
// Timing: chunk_check <file> <chunk bytes> <k> <threads> -- the chunks parsed
// on <threads> threads (no ordering or fallback), against the streaming
// parser, wall-clock rates.
#include <stdio.h>
#include <stdlib.h>
#include <atomic>
#include <chrono>
#include <functional>
#include <thread>
#include <string>
#include <vector>
#include "../khmer_amd/csrc/kh_internal.h"

namespace kh {
struct Parser;
struct PlainFile;
Parser *parser_open(const char *path);
void parser_close(Parser *p);
void parser_fill_raw(Parser *p, RawBatch &b, int k, uint64_t max_kmers, uint64_t max_bases, bool *done, uint64_t *taken);
PlainFile *parser_plain_open(Parser *pr);
void parser_plain_commit(Parser *pr);
void parser_plain_close(PlainFile *f);
size_t plain_size(const PlainFile *f);
bool plain_chunkable(const PlainFile *f, size_t CH);
void plain_parse_chunk(const PlainFile *f, size_t c, size_t CH, int k, uint64_t max_kmers, std::vector<RawBatch> &out,
                       uint64_t *nreads, size_t *start, size_t *end, bool *redo);
void plain_parse_rest(const PlainFile *f, size_t from, size_t CH, int k, uint64_t max_kmers,
                      const std::function<void(RawBatch &)> &sink, uint64_t *nreads);
}  // namespace kh

struct Out {
    uint64_t reads = 0, kept = 0, h = 1469598103934665603ull;
    std::string err;
    void add(const kh::RawBatch &b) {
        const char *p = b.seq.data();
        for (uint32_t n : b.len) {
            h = (h ^ n) * 1099511628211ull;
            for (uint32_t i = 0; i < n; i++) h = (h ^ (unsigned char)p[i]) * 1099511628211ull;
            p += n;
            kept++;
        }
    }
};

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int timing(const char *path, size_t CH, int k, int T) {
    const uint64_t maxk = 1 << 20;
    double t0 = now();
    uint64_t r0 = 0;
    {
        kh::Parser *p = kh::parser_open(path);
        for (bool done = false; !done;) {
            kh::RawBatch r;
            kh::parser_fill_raw(p, r, k, maxk, maxk * 2 + 4096, &done, &r0);
        }
        kh::parser_close(p);
    }
    const double ts = now() - t0;
    t0 = now();
    kh::Parser *p = kh::parser_open(path);
    kh::PlainFile *f = kh::parser_plain_open(p);
    if (!f) { printf("{\"chunked\": false}\n"); return 3; }
    kh::parser_plain_commit(p);
    const size_t n = kh::plain_size(f), nch = (n + CH - 1) / CH;
    std::atomic<size_t> next{0};
    std::atomic<uint64_t> reads{0}, redo{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&] {
            for (size_t c; (c = next++) < nch;) {
                std::vector<kh::RawBatch> raw;
                uint64_t nr = 0;
                size_t s = 0, e = 0;
                bool rd = false;
                kh::plain_parse_chunk(f, c, CH, k, maxk, raw, &nr, &s, &e, &rd);
                reads += nr;
                redo += rd;
            }
        });
    for (auto &x : th) x.join();
    const double tc = now() - t0;
    printf("{\"file\": \"%s\", \"stream_bytes\": %zu, \"threads\": %d, \"streaming_s\": %.3f, \"streaming_GBps\": %.3f, "
           "\"chunked_s\": %.3f, \"chunked_GBps\": %.3f, \"reads\": [%llu, %llu], \"redo\": %llu}\n",
           path, n, T, ts, n / ts / 1e9, tc, n / tc / 1e9, (unsigned long long)r0, (unsigned long long)reads.load(),
           (unsigned long long)redo.load());
    kh::parser_plain_close(f);
    kh::parser_close(p);
    return 0;
}

// pack check: HostBatch::append(clean) against a scalar restatement of
// _to_valid_dna + twobit_repr on random reads over all byte values
static int pack_check(uint64_t seed, int nreads) {
    auto rnd = [&]() { seed ^= seed << 13; seed ^= seed >> 7; seed ^= seed << 17; return seed; };
    const char alpha[] = "ACGTACGTACGTacgtNnXx \t\n@+";
    kh::HostBatch b;
    std::vector<uint8_t> codes;
    for (int r = 0; r < nreads; r++) {
        const size_t len = 21 + rnd() % 300;
        std::string s(len, 'A');
        for (auto &c : s) c = (rnd() % 8) ? alpha[rnd() % (sizeof alpha - 1)] : (char)(rnd() & 0xFF);
        b.append(s.data(), s.size(), 21, true);
        for (unsigned char c : s) {
            char cc = (c == 'A' || c == 'C' || c == 'G' || c == 'T') ? (char)c
                      : (c == 'a' || c == 'c' || c == 'g' || c == 't') ? (char)(c - 32) : 'A';
            codes.push_back(cc == 'A' ? 0 : cc == 'T' ? 1 : cc == 'C' ? 2 : 3);
        }
    }
    uint64_t bad = 0;
    for (size_t i = 0; i < codes.size(); i++) {
        const uint32_t got = (uint32_t)(b.words[i >> 5] >> (62 - 2 * (i & 31))) & 3;
        bad += got != codes[i];
    }
    // merge: batches of random sizes merged in order equal one batch
    kh::HostBatch m, part;
    uint64_t seed2 = seed;
    seed = 0x9E3779B97F4A7C15ull;
    for (int r = 0; r < nreads; r++) {
        const size_t len = 21 + rnd() % 300;
        std::string s(len, 'A');
        for (auto &c : s) c = (rnd() % 8) ? alpha[rnd() % (sizeof alpha - 1)] : (char)(rnd() & 0xFF);
        part.append(s.data(), s.size(), 21, true);
        if ((r * 2654435761u) % 7 == 0 || r + 1 == nreads) {
            m.merge(part);
            part = kh::HostBatch();
        }
    }
    (void)seed2;
    uint64_t mbad = (m.nbases != b.nbases) * 1 + (m.koff != b.koff) * 2 + (m.read_kmers != b.read_kmers) * 4 + (m.uniform != b.uniform) * 8;
    for (uint64_t i = 0; i < (b.nbases + 31) / 32 && !mbad; i++) mbad += m.words[i] != b.words[i];
    printf("{\"pack_bases\": %zu, \"mismatches\": %llu, \"merge_mismatch\": %llu}\n", codes.size(),
           (unsigned long long)bad, (unsigned long long)mbad);
    return bad || mbad ? 1 : 0;
}

int main(int argc, char **argv) {
    if (argc == 3 && std::string(argv[1]) == "--pack") return pack_check(0x9E3779B97F4A7C15ull, atoi(argv[2]));
    if (argc < 3) return 2;
    const char *path = argv[1];
    const size_t CH = strtoull(argv[2], nullptr, 10);
    const int k = argc > 3 ? atoi(argv[3]) : 21;
    if (argc > 4) return timing(path, CH, k, atoi(argv[4]));
    const uint64_t maxk = 1 << 20;
    Out a, b;
    try {   // streaming
        kh::Parser *p = kh::parser_open(path);
        for (bool done = false; !done;) {
            kh::RawBatch r;
            uint64_t t = 0;
            try {
                kh::parser_fill_raw(p, r, k, maxk, maxk * 2 + 4096, &done, &t);
            } catch (const std::exception &e) {
                a.reads += t;
                a.add(r);
                throw;
            }
            a.reads += t;
            a.add(r);
        }
        kh::parser_close(p);
    } catch (const std::exception &e) {
        a.err = e.what();
    }
    int mode = 0;   // 0 chunked, 1 not chunkable, 2 serial rest taken
    try {   // chunked, in consume_chunked's order
        kh::Parser *p = kh::parser_open(path);
        kh::PlainFile *f = kh::parser_plain_open(p);
        if (!f) { printf("{\"chunked\": false}\n"); return 3; }
        const size_t n = kh::plain_size(f), nch = (n + CH - 1) / CH;
        if (nch > 1 && !kh::plain_chunkable(f, CH)) mode = 1;
        size_t true_end = 0;
        bool serial = mode == 1;
        for (size_t c = 0; c < nch && !serial; c++) {
            std::vector<kh::RawBatch> raw;
            uint64_t nr = 0;
            size_t s = 0, e = 0;
            bool redo = false;
            std::string err;
            try {
                kh::plain_parse_chunk(f, c, CH, k, maxk, raw, &nr, &s, &e, &redo);
            } catch (const std::exception &x) {
                err = x.what();
            }
            if (redo || (s != true_end && !(s >= n && true_end >= n))) { serial = true; mode = 2; break; }
            for (auto &r : raw) b.add(r);
            b.reads += nr;
            true_end = e;
            if (!err.empty()) throw std::runtime_error(err);
        }
        if (serial && true_end < n)
            kh::plain_parse_rest(f, true_end, CH, k, maxk, [&](kh::RawBatch &r) { b.add(r); }, &b.reads);
        kh::parser_plain_close(f);
        kh::parser_close(p);
    } catch (const std::exception &e) {
        b.err = e.what();
    }
    const bool same = a.reads == b.reads && a.kept == b.kept && a.h == b.h && a.err == b.err;
    printf("{\"same\": %s, \"mode\": %d, \"reads\": [%llu, %llu], \"kept\": [%llu, %llu], \"err\": [\"%s\", \"%s\"]}\n",
           same ? "true" : "false", mode, (unsigned long long)a.reads, (unsigned long long)b.reads,
           (unsigned long long)a.kept, (unsigned long long)b.kept, a.err.c_str(), b.err.c_str());
    return same ? 0 : 1;
}
