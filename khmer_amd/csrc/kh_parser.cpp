// kh_parser.cpp -- FASTA/FASTQ reader of libkhmer_hip.so.
//
// Replaces oxli::read_parsers::FastxReader (src/oxli/read_parsers.cc:257-372),
// which wraps the vendored seqan record reader
// (third-party/seqan/core/include/seqan/seq_io/read_fasta_fastq.h:300-650).
// Record semantics kept:
//   * format fixed by the first byte of the (decompressed) file: '>' FASTA,
//     '@' FASTQ; anything else -> "badly formatted", empty -> "does not contain
//     any sequences!" (read_parsers.cc:257-272);
//   * name = rest of the header line (seqan readLine: \n, \r\n, \r);
//   * sequence = non-space characters of the following lines up to a line that
//     starts with '>' (FASTA) / '+' (FASTQ); the first line after the header
//     is never a stop line;
//   * FASTQ: the '+' line is empty or repeats the name; then exactly
//     len(sequence) non-space quality characters (EOF earlier is tolerated),
//     the rest of that line skipped;
//   * a read with an empty sequence -> InvalidRead "Sequence is empty"; after
//     the first read carried qualities, a length mismatch -> "Sequence and
//     quality lengths differ"; num_reads counts good reads only
//     (read_parsers.cc:337-353).
// The parser is shared by threads: one mutex serialises record extraction,
// like the reference's spin lock (read_parsers.cc:334).
//
// Input bytes come from a Source: plain and gzip files through zlib, bzip2
// files ("BZh" magic) through the system libbz2 -- the formats seqan's
// stream autodetection accepts (read_parsers.cc:257-272).  A stream that ends
// inside a compressed block (truncated .gz / .bz2) or carries corrupt data
// raises KH_EFILE (OSError), as the reference's tests expect
// (tests/test_read_parsers.py:183-255).
//
// Decompression runs off the parsing thread: BGZF files (chains of
// independent gzip members, htslib's bgzip format) are inflated member group
// by member group on worker threads, every other compressed stream on one
// read-ahead thread; either way the parser sees the same bytes in the same
// order, and a corrupt stream raises after the bytes before the damage.
#include <ctype.h>
#include <stdio.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>
#include <emmintrin.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <string>
#include <thread>

#include "kh_internal.h"

// libbz2's public decompression ABI (bzlib.h of bzip2 1.0.x; the image ships
// the runtime library without its header).
extern "C" {
struct kh_bz_stream {
    char *next_in;
    unsigned int avail_in, total_in_lo32, total_in_hi32;
    char *next_out;
    unsigned int avail_out, total_out_lo32, total_out_hi32;
    void *state;
    void *(*bzalloc)(void *, int, int);
    void (*bzfree)(void *, void *);
    void *opaque;
};
int BZ2_bzDecompressInit(kh_bz_stream *strm, int verbosity, int small);
int BZ2_bzDecompress(kh_bz_stream *strm);
int BZ2_bzDecompressEnd(kh_bz_stream *strm);
}

namespace kh {

namespace {
constexpr int BZ_OK_ = 0, BZ_STREAM_END_ = 4;

struct Source {
    std::string path;
    virtual ~Source() {}
    virtual bool plain() const { return false; }   // uncompressed file read as is
    // up to n bytes into dst; 0 at the clean end of the stream; throws on a
    // corrupt or truncated stream
    virtual size_t read(unsigned char *dst, size_t n) = 0;
    [[noreturn]] void corrupt(const char *what) {
        fail(KH_EFILE, std::string("File ") + path + ": " + what);
    }
};

struct GzSource : Source {
    gzFile gz = nullptr;
    ~GzSource() override { if (gz) gzclose(gz); }
    bool plain() const override { return gz && gzdirect(gz) == 1; }
    size_t read(unsigned char *dst, size_t n) override {
        int got = gzread(gz, dst, (unsigned)n);
        if (got > 0) return (size_t)got;
        int err = Z_OK;
        const char *msg = gzerror(gz, &err);
        if (got < 0 || (err != Z_OK && err != Z_STREAM_END)) corrupt(msg && *msg ? msg : "gzip stream error");
        return 0;
    }
};

struct Bz2Source : Source {
    FILE *f = nullptr;
    kh_bz_stream s;
    bool live = false, done = false;
    std::vector<char> in = std::vector<char>(1 << 20);
    ~Bz2Source() override {
        if (live) BZ2_bzDecompressEnd(&s);
        if (f) fclose(f);
    }
    void start() {
        memset(&s, 0, sizeof s);
        if (BZ2_bzDecompressInit(&s, 0, 0) != BZ_OK_) corrupt("cannot start bzip2 decoder");
        live = true;
    }
    unsigned refill() {
        size_t n = fread(in.data(), 1, in.size(), f);
        if (n == 0 && ferror(f)) corrupt("read error");
        s.next_in = in.data();
        s.avail_in = (unsigned)n;
        return (unsigned)n;
    }
    size_t read(unsigned char *dst, size_t n) override {
        size_t got = 0;
        while (got == 0 && !done) {
            if (s.avail_in == 0 && !refill()) corrupt("bzip2 stream is truncated");
            s.next_out = (char *)dst;
            s.avail_out = (unsigned)n;
            int rc = BZ2_bzDecompress(&s);
            got = n - s.avail_out;
            if (rc == BZ_STREAM_END_) {
                // concatenated streams (pbzip2 output) continue with a fresh decoder
                char *rest = s.next_in;
                unsigned rest_n = s.avail_in;
                BZ2_bzDecompressEnd(&s);
                live = false;
                if (rest_n) memmove(in.data(), rest, rest_n);
                else rest_n = refill();
                if (!rest_n) { done = true; break; }
                start();
                s.next_in = in.data();
                s.avail_in = rest_n;
            } else if (rc != BZ_OK_) {
                corrupt("bzip2 data error");
            }
        }
        return got;
    }
};

// bytes [pos, n) of a mapped file, read on demand (chunk parsers)
struct MemSource : Source {
    const unsigned char *p = nullptr;
    size_t n = 0, pos = 0;
    size_t read(unsigned char *dst, size_t m) override {
        const size_t k = std::min(m, n - pos);
        memcpy(dst, p + pos, k);
        pos += k;
        return k;
    }
};

// Worker threads for decompression: the job's CPU share (OMP_NUM_THREADS,
// as the feed's packers) halved, 2..8; KH_INFLATE_THREADS overrides.
int inflate_threads() {
    int n = (int)std::thread::hardware_concurrency();
    const char *e = getenv("OMP_NUM_THREADS");
    if (e && atoi(e) > 0) n = std::min(n > 0 ? n : 1, atoi(e));
    n = std::max(2, std::min(8, n / 2));
    const char *f = getenv("KH_INFLATE_THREADS");
    if (f && atoi(f) > 0) n = std::min(64, atoi(f));
    return n;
}

// Decompressed bytes handed over in file order through a ring of R slots:
// producers fill slot g % R with group g once group g - R has been read.
// A producer that meets damage stores the bytes it could decode and the
// error; the consumer returns those bytes, then raises.
struct RingSource : Source {
    struct Slot {
        std::vector<unsigned char> out;
        size_t len = 0, pos = 0;
        bool ready = false, last = false;
        std::string err;   // the complete message (KH_EFILE) raised after the bytes
    };
    std::vector<Slot> ring;
    std::mutex mu;
    std::condition_variable cv_free, cv_ready;
    uint64_t cur = 0;        // the group the consumer reads
    bool stop = false, ended = false;
    std::vector<std::thread> th;

    void start_ring(int R) { ring.resize((size_t)R); }
    void stop_threads() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_free.notify_all();
        for (auto &t : th) t.join();
        th.clear();
    }
    // producer side: wait until group g's slot is free (false: stopping)
    bool wait_free(uint64_t g) {
        std::unique_lock<std::mutex> lk(mu);
        cv_free.wait(lk, [&] { return stop || g < cur + ring.size(); });
        return !stop;
    }
    void publish(uint64_t g) {
        {
            std::lock_guard<std::mutex> lk(mu);
            ring[g % ring.size()].ready = true;
        }
        cv_ready.notify_all();
    }
    size_t read(unsigned char *dst, size_t n) override {
        for (;;) {
            if (ended) return 0;
            Slot &s = ring[cur % ring.size()];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_ready.wait(lk, [&] { return s.ready; });
            }
            if (s.pos < s.len) {
                const size_t k = std::min(n, s.len - s.pos);
                memcpy(dst, s.out.data() + s.pos, k);
                s.pos += k;
                return k;
            }
            if (!s.err.empty()) fail(KH_EFILE, s.err);
            if (s.last) { ended = true; return 0; }
            {
                std::lock_guard<std::mutex> lk(mu);
                s.ready = false;
                s.pos = s.len = 0;
                cur++;
            }
            cv_free.notify_all();
        }
    }
};

// BGZF (SAM/BAM format specification 4.1): gzip members with FLG.FEXTRA whose
// 'BC' subfield holds the member size - 1, each inflating to <= 64 KiB.  The
// whole file is checked to be such a chain up front (headers only); a file
// that is not (one member, other flags, a truncated tail) takes zlib's gzread
// path instead, so its bytes and errors are zlib's.
struct BgzfMember { uint64_t cdata; uint32_t clen, crc, isize; };

static uint32_t le32(const unsigned char *q) {
    return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
}
bool bgzf_scan(const unsigned char *p, size_t n, std::vector<BgzfMember> &mem) {
    size_t off = 0;
    while (off < n) {
        const unsigned char *h = p + off;
        if (n - off < 12 + 6 + 8 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4) return false;
        const size_t xlen = (size_t)h[10] | (size_t)h[11] << 8;
        if (off + 12 + xlen > n) return false;
        long bsize = -1;
        for (size_t x = 12; x + 4 <= 12 + xlen;) {
            const size_t slen = (size_t)h[x + 2] | (size_t)h[x + 3] << 8;
            if (h[x] == 'B' && h[x + 1] == 'C' && slen == 2 && x + 6 <= 12 + xlen)
                bsize = (long)h[x + 4] | (long)h[x + 5] << 8;
            x += 4 + slen;
        }
        if (bsize < 0) return false;
        const size_t total = (size_t)bsize + 1;
        if (total < 12 + xlen + 8 || off + total > n) return false;
        BgzfMember m;
        m.cdata = off + 12 + xlen;
        m.clen = (uint32_t)(total - 12 - xlen - 8);
        m.crc = le32(h + total - 8);
        m.isize = le32(h + total - 4);
        if (m.isize > 65536) return false;
        mem.push_back(m);
        off += total;
    }
    return mem.size() >= 2;
}
// inflate member m of the mapped file p into dst (m.isize bytes of room):
// the bytes decoded (all of them, or those before the damage) and, on
// damage, zlib's message in *err
size_t bgzf_inflate(z_stream &z, const unsigned char *p, const BgzfMember &m, unsigned char *dst, std::string *err) {
    inflateReset(&z);
    z.next_in = (Bytef *)(p + m.cdata);
    z.avail_in = m.clen;
    // an empty member (ISIZE 0, e.g. the 28-byte EOF marker alone in a member
    // group) may come with no output buffer at all: zlib refuses a null
    // next_out (Z_STREAM_ERROR) even when there is nothing to write
    unsigned char none = 0;
    z.next_out = dst ? dst : &none;
    z.avail_out = m.isize;
    const int rc = inflate(&z, Z_FINISH);
    const size_t got = m.isize - z.avail_out;
    if (rc != Z_STREAM_END)
        *err = z.msg ? z.msg : (rc == Z_BUF_ERROR ? "incorrect length check" : "invalid compressed data");
    else if (z.avail_in != 0 || got != m.isize)
        *err = "incorrect length check";
    else if (crc32(0, dst, (uInt)got) != m.crc)
        *err = "incorrect data check";
    return got;
}
// a raw-deflate decoder for bgzf_inflate
struct Inflater {
    z_stream z;
    bool ok = false;
    Inflater() {
        memset(&z, 0, sizeof z);
        ok = inflateInit2(&z, -15) == Z_OK;
    }
    ~Inflater() { if (ok) inflateEnd(&z); }
};
// a read-only mapping of a whole file
bool map_file(const char *path, int *fd, const unsigned char **p, size_t *n, size_t min_size) {
    *fd = ::open(path, O_RDONLY);
    if (*fd < 0) return false;
    struct stat st;
    if (fstat(*fd, &st) != 0 || st.st_size <= 0 || (size_t)st.st_size < min_size) return false;
    void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, *fd, 0);
    if (m == MAP_FAILED) return false;
    *p = (const unsigned char *)m;
    *n = (size_t)st.st_size;
    madvise(m, *n, MADV_SEQUENTIAL);
    return true;
}

// The BGZF stream, member groups inflated by worker threads into the ring.
struct BgzfSource : RingSource {
    int fd = -1;
    const unsigned char *p = nullptr;
    size_t n = 0;
    std::vector<BgzfMember> mem;
    std::vector<size_t> gfirst;   // group g = members [gfirst[g], gfirst[g + 1])
    uint64_t next_g = 0;          // next group a worker takes (under mu)
    static constexpr size_t GROUP = 64;   // members per group (<= 4 MiB)

    ~BgzfSource() override {
        stop_threads();
        if (p) munmap((void *)p, n);
        if (fd >= 0) close(fd);
    }
    void worker() {
        Inflater inf;
        if (!inf.ok) return;
        for (;;) {
            uint64_t g;
            {
                std::unique_lock<std::mutex> lk(mu);
                if (stop || next_g + 1 >= gfirst.size()) break;
                g = next_g++;
            }
            if (!wait_free(g)) break;
            Slot &s = ring[g % ring.size()];
            size_t need = 0;
            for (size_t i = gfirst[g]; i < gfirst[g + 1]; i++) need += mem[i].isize;
            if (s.out.size() < need) s.out.resize(need);
            size_t len = 0;
            std::string err;
            for (size_t i = gfirst[g]; i < gfirst[g + 1] && err.empty(); i++)
                len += bgzf_inflate(inf.z, p, mem[i], s.out.data() + len, &err);
            s.len = len;
            s.pos = 0;
            s.err = err.empty() ? err : "File " + path + ": " + err;
            s.last = g + 2 == gfirst.size() || !err.empty();
            publish(g);
            if (!err.empty()) break;   // nothing after the damage is read
        }
    }
    bool open(const char *path_) {
        path = path_;
        // small files: zlib (KH_BGZF_MIN_BYTES: development / tests)
        const char *e = getenv("KH_BGZF_MIN_BYTES");
        const size_t min_bytes = e ? (size_t)atoll(e) : (size_t)1 << 20;
        if (!map_file(path_, &fd, &p, &n, std::max<size_t>(1, min_bytes))) return false;
        if (!bgzf_scan(p, n, mem)) return false;
        for (size_t i = 0; i < mem.size(); i += GROUP) gfirst.push_back(i);
        gfirst.push_back(mem.size());
        const int nw = inflate_threads();
        start_ring(2 * nw);
        for (int t = 0; t < nw; t++) th.emplace_back([this] { worker(); });
        return true;
    }
};

// Any other compressed stream: the inner source (zlib gzread, libbz2) runs
// on one thread that fills 4 MiB slots ahead of the parser.
struct ReadAheadSource : RingSource {
    std::unique_ptr<Source> in;
    static constexpr size_t CHUNK = 4 << 20;
    ~ReadAheadSource() override { stop_threads(); }
    void producer() {
        for (uint64_t g = 0;; g++) {
            if (!wait_free(g)) return;
            Slot &s = ring[g % ring.size()];
            if (s.out.size() < CHUNK) s.out.resize(CHUNK);
            size_t len = 0;
            bool end = false;
            std::string err;
            try {
                while (len < CHUNK) {
                    const size_t k = in->read(s.out.data() + len, CHUNK - len);
                    if (k == 0) { end = true; break; }
                    len += k;
                }
            } catch (const std::exception &e) {   // the inner source's "File <path>: ..."
                err = e.what();
                if (err.empty()) err = "File " + path + ": read error";
            }
            s.len = len;
            s.pos = 0;
            s.err = err;
            s.last = end || !err.empty();
            publish(g);
            if (s.last) return;
        }
    }
    void begin(std::unique_ptr<Source> inner) {
        in = std::move(inner);
        path = in->path;
        start_ring(3);
        th.emplace_back([this] { producer(); });
    }
};

static bool async_off() {
    static const bool v = [] { const char *e = dev_getenv("KH_ASYNC_INFLATE"); return e && atoi(e) == 0; }();
    return v;
}

std::unique_ptr<Source> open_source(const char *path) {
    unsigned char magic[3] = {0, 0, 0};
    FILE *f = fopen(path, "rb");
    if (!f) return nullptr;
    size_t m = fread(magic, 1, 3, f);
    if (m == 3 && magic[0] == 'B' && magic[1] == 'Z' && magic[2] == 'h') {
        rewind(f);
        std::unique_ptr<Bz2Source> b(new Bz2Source());
        b->path = path;
        b->f = f;
        b->start();
        if (async_off()) return std::move(b);
        std::unique_ptr<ReadAheadSource> r(new ReadAheadSource());
        r->begin(std::move(b));
        return std::move(r);
    }
    fclose(f);
    const bool gzip_magic = m == 3 && magic[0] == 0x1f && magic[1] == 0x8b;
    if (gzip_magic && !async_off()) {
        std::unique_ptr<BgzfSource> bg(new BgzfSource());
        if (bg->open(path)) return std::move(bg);
    }
    gzFile gz = gzopen(path, "rb");
    if (!gz) return nullptr;
    gzbuffer(gz, 1 << 20);
    std::unique_ptr<GzSource> g(new GzSource());
    g->path = path;
    g->gz = gz;
    if (g->plain() || async_off()) return std::move(g);
    std::unique_ptr<ReadAheadSource> r(new ReadAheadSource());
    r->begin(std::move(g));
    return std::move(r);
}
}  // namespace

// isspace() of the C locale as a table (space, \t, \n, \v, \f, \r)
struct WsTab {
    unsigned char t[256];
    WsTab() {
        for (int c = 0; c < 256; c++) t[c] = isspace(c) ? 1 : 0;
    }
};
static const WsTab g_ws;

// The first whitespace byte in [q, e) (e if none): 16 bytes a step with SSE2
// (x86-64 baseline) -- every whitespace byte is <= 0x20, so only the bytes
// <= 0x20 of a block are checked against the table.
static inline const unsigned char *find_ws(const unsigned char *q, const unsigned char *e) {
    const __m128i lim = _mm_set1_epi8(0x20);
    while (e - q >= 16) {
        const __m128i x = _mm_loadu_si128((const __m128i *)q);
        unsigned m = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(_mm_max_epu8(x, lim), lim));
        while (m) {
            const int b = __builtin_ctz(m);
            if (g_ws.t[q[b]]) return q + b;
            m &= m - 1;
        }
        q += 16;
    }
    while (q < e && !g_ws.t[*q]) q++;
    return q;
}
// The first '\n' or '\r' in [q, e) (e if none)
static inline const unsigned char *find_eol(const unsigned char *q, const unsigned char *e) {
    const __m128i nl = _mm_set1_epi8('\n'), cr = _mm_set1_epi8('\r');
    while (e - q >= 16) {
        const __m128i x = _mm_loadu_si128((const __m128i *)q);
        const unsigned m = (unsigned)_mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, nl), _mm_cmpeq_epi8(x, cr)));
        if (m) return q + __builtin_ctz(m);
        q += 16;
    }
    while (q < e && *q != '\n' && *q != '\r') q++;
    return q;
}

struct Parser {
    std::unique_ptr<Source> src;
    std::string path;
    std::vector<unsigned char> buf;
    size_t pos = 0, len = 0;
    bool eof = false;
    bool fastq = false;
    bool have_qualities = false;
    uint64_t num_reads = 0;
    std::string name, seq, qual, tmp;
    std::mutex mu;

    std::string broken;   // a corrupt stream met while opening, raised on first use

    uint64_t src_bytes = 0;   // bytes taken from src so far
    // offset of the next unparsed byte in the source's stream
    uint64_t offset() const { return src_bytes - (len - pos); }
    int peek() {
        if (pos < len) return buf[pos];
        if (!broken.empty()) fail(KH_EFILE, broken);
        if (eof) return -1;
        size_t n = src->read(buf.data(), buf.size());
        if (n == 0) { eof = true; len = pos = 0; return -1; }
        src_bytes += n;
        len = n; pos = 0;
        return buf[0];
    }
    void next() { pos++; }
    bool at_end() { return peek() < 0; }

    void read_line(std::string &out) {
        out.clear();
        for (;;) {
            if (pos >= len && peek() < 0) return;
            // fast scan of the buffered chunk
            unsigned char *s = buf.data() + pos, *e = buf.data() + len;
            unsigned char *q = (unsigned char *)find_eol(s, e);
            out.append((const char *)s, (size_t)(q - s));
            pos += (size_t)(q - s);
            if (q < e) {
                if (*q == '\n') { pos++; return; }
                pos++;  // '\r'
                if (peek() == '\n') pos++;
                return;
            }
        }
    }
    void skip_line() {
        int c;
        while ((c = peek()) >= 0 && c != '\n') pos++;
        if (c == '\n') pos++;
    }

    // seqan readRecord; returns false on INVALID_FORMAT
    bool read_record() {
        name.clear(); seq.clear(); qual.clear();
        const int marker = fastq ? '@' : '>';
        const int stop = fastq ? '+' : '>';
        if (peek() != marker) return false;
        next();
        if (at_end()) return true;
        read_line(name);
        if (at_end()) return true;
        bool after_eol = false;
        for (;;) {
            if (pos >= len && peek() < 0) break;
            int c = buf[pos];
            if (c == '\r' || c == '\n') { after_eol = true; pos++; continue; }
            if (after_eol && c == stop) break;
            // fast path: copy a run of sequence characters
            unsigned char *s = buf.data() + pos, *e = buf.data() + len;
            unsigned char *q = (unsigned char *)find_ws(s, e);
            if (q == s) { pos++; after_eol = false; continue; }  // isolated space
            seq.append((const char *)s, (size_t)(q - s));
            pos += (size_t)(q - s);
            after_eol = false;
        }
        if (!fastq) return true;
        if (at_end()) return true;
        if (peek() != '+') return false;
        next();
        if (at_end()) return true;
        read_line(tmp);
        if (!tmp.empty() && tmp != name) return false;
        if (at_end()) return true;
        // qualities: runs of non-space characters copied in bulk, whitespace
        // (line breaks of multi-line records) skipped, until len(seq) are read
        while (qual.size() < seq.size()) {
            if (pos >= len && peek() < 0) break;
            unsigned char *s = buf.data() + pos, *e = buf.data() + len;
            const size_t need = seq.size() - qual.size();
            unsigned char *lim = (size_t)(e - s) > need ? s + need : e;
            unsigned char *q = (unsigned char *)find_ws(s, lim);
            if (q == s) { pos++; continue; }   // a whitespace character
            qual.append((const char *)s, (size_t)(q - s));
            pos += (size_t)(q - s);
        }
        if (qual.size() == seq.size()) skip_line();
        return true;
    }

    // FastxReader::get_next_read (read_parsers.cc:329-372); caller holds mu.
    // returns KH_OK with a read, KH_END, or throws
    int next_read_locked() {
        if (at_end()) return KH_END;
        if (!read_record()) fail(KH_EFILE, "Generic StreamReadError error");
        if (num_reads == 0 && !qual.empty()) have_qualities = true;
        if (seq.empty()) fail(KH_EVALUE, "Sequence is empty");
        if (have_qualities && seq.size() != qual.size()) fail(KH_EVALUE, "Sequence and quality lengths differ");
        num_reads++;
        return KH_OK;
    }
};

Parser *parser_open(const char *path) {
    std::unique_ptr<Source> src = open_source(path);
    if (!src) fail(KH_EFILE, std::string("File ") + path + " contains badly formatted sequence or does not exist.");
    std::unique_ptr<Parser> p(new Parser());
    p->src = std::move(src);
    p->path = path;
    p->buf.resize(1 << 22);
    int c;
    try {
        c = p->peek();
    } catch (const Error &e) {
        // the reference opens a truncated .bz2 and fails on the first read
        // (tests/test_read_parsers.py:218-228)
        p->broken = e.what();
        return p.release();
    }
    if (c < 0) fail(KH_EFILE, std::string("File ") + path + " does not contain any sequences!");
    if (c != '>' && c != '@')
        fail(KH_EFILE, std::string("File ") + path + " contains badly formatted sequence or does not exist.");
    p->fastq = (c == '@');
    return p.release();
}

void parser_close(Parser *p) { delete p; }

// thread-local copies handed to the C ABI (pointers valid until the next call)
struct TLRead { std::string name, seq, qual; };
static thread_local TLRead tl_read;

int parser_next_read(Parser *p, ReadView *rv) {
    std::lock_guard<std::mutex> lk(p->mu);
    int rc = p->next_read_locked();
    if (rc != KH_OK) return rc;
    tl_read.name = p->name; tl_read.seq = p->seq; tl_read.qual = p->qual;
    rv->name = tl_read.name.data(); rv->name_len = tl_read.name.size();
    rv->seq = tl_read.seq.data(); rv->seq_len = tl_read.seq.size();
    rv->qual = tl_read.qual.data(); rv->qual_len = tl_read.qual.size();
    return KH_OK;
}

uint64_t parser_num_reads(Parser *p) {
    std::lock_guard<std::mutex> lk(p->mu);
    return p->num_reads;
}

bool parser_is_complete(Parser *p) {
    std::lock_guard<std::mutex> lk(p->mu);
    return p->at_end();
}

// Fill a batch (cleaned, packed) with up to max_kmers k-mers.  Reads shorter
// than k are counted but not packed.  *taken counts the reads parsed so far
// (also when a malformed read throws); sets *done at end of input.
void parser_fill_batch(Parser *p, HostBatch &b, int k, uint64_t max_kmers, uint64_t max_bases, bool *done,
                       uint64_t *taken) {
    std::lock_guard<std::mutex> lk(p->mu);
    *done = false;
    while (b.nkmers() < max_kmers && b.nbases < max_bases) {
        int rc = p->next_read_locked();  // may throw
        if (rc == KH_END) { *done = true; break; }
        (*taken)++;
        if (p->seq.size() >= (size_t)k) b.append(p->seq.data(), p->seq.size(), k, true);
    }
}

// ---- chunk-parallel parsing (kh_capi.cpp consume_chunked) ----
// A plain FASTA/FASTQ file, or a BGZF file, that no read has been taken from
// yet is cut into chunks at record starts; each chunk is parsed by its own
// Parser over its bytes (the same record semantics), so parsing scales with
// threads.  A chunk start is a line beginning with '>' (FASTA: unambiguous) or
// with '@' that begins two consecutive well-formed four-line records (FASTQ).
// Chunk c's parser stops at the first record boundary at or past chunk c+1's
// start; the consumer checks that they coincide and otherwise re-parses the
// rest of the input serially from where chunk c really ended (exact either
// way).  A plain file is mapped whole.  A BGZF file is a stream of known
// length (the members' ISIZE) whose members can be inflated independently:
// chunk c inflates only the members under its window, [c*CH - 1, (c+1)*CH +
// BGZF_EXTRA); a record that runs past the window, or damage inside it,
// makes the chunk "redo" and the consumer continues serially from there
// through a sequential member reader (the streaming source's bytes, order and
// errors).
struct PlainFile {
    std::string path;
    int fd = -1;
    const unsigned char *p = nullptr;   // the mapped file
    size_t mapped = 0;
    size_t n = 0;                        // stream bytes (BGZF: inflated)
    bool fastq = false;
    bool bgzf = false;
    std::vector<BgzfMember> mem;         // BGZF members
    std::vector<uint64_t> uoff;          // BGZF: stream offset of member i (size + 1)
    ~PlainFile() {
        if (p) munmap((void *)p, mapped);
        if (fd >= 0) close(fd);
    }
};

constexpr size_t BGZF_LIM = 1 << 20;     // record-start search span in a BGZF window
constexpr size_t BGZF_EXTRA = 4 << 20;   // window bytes past the chunk's end

// bytes [lo, hi) of an n-byte stream, b[0] being byte lo
struct View {
    const unsigned char *b;
    size_t lo, hi, n;
};

static bool chunk_bgzf_on() {
    const char *e = getenv("KH_BGZF_CHUNKED");   // development / tests: 0 streams BGZF through one parser
    return !(e && atoi(e) == 0);
}

PlainFile *parser_plain_open(Parser *pr) {
    std::lock_guard<std::mutex> lk(pr->mu);
    if (pr->num_reads != 0 || pr->offset() != 0 || !pr->broken.empty()) return nullptr;
    const bool bg = dynamic_cast<BgzfSource *>(pr->src.get()) != nullptr;
    if (!pr->src->plain() && !(bg && chunk_bgzf_on())) return nullptr;
    std::unique_ptr<PlainFile> f(new PlainFile());
    f->path = pr->path;
    f->fastq = pr->fastq;
    if (!map_file(pr->path.c_str(), &f->fd, &f->p, &f->mapped, 1)) return nullptr;
    f->n = f->mapped;
    if (bg) {
        if (!bgzf_scan(f->p, f->mapped, f->mem)) return nullptr;
        f->bgzf = true;
        f->uoff.resize(f->mem.size() + 1);
        f->uoff[0] = 0;
        for (size_t i = 0; i < f->mem.size(); i++) f->uoff[i + 1] = f->uoff[i] + f->mem[i].isize;
        f->n = f->uoff.back();
    }
    return f.release();
}
// the chunk path takes the file: a BGZF parser's own inflate workers stop
// (they would inflate groups nobody reads); the parser is drained afterwards
void parser_plain_commit(Parser *pr) {
    std::lock_guard<std::mutex> lk(pr->mu);
    if (BgzfSource *b = dynamic_cast<BgzfSource *>(pr->src.get())) b->stop_threads();
}
void parser_plain_close(PlainFile *f) { delete f; }
size_t plain_size(const PlainFile *f) { return f->n; }

// first member whose bytes reach past offset x
static size_t bgzf_member_at(const PlainFile *f, size_t x) {
    return (size_t)(std::upper_bound(f->uoff.begin(), f->uoff.end(), (uint64_t)x) - f->uoff.begin()) - 1;
}
// inflate the members under stream bytes [lo, hi) into buf; the view covers
// whole members; false on damage
static bool bgzf_window(const PlainFile *f, size_t lo, size_t hi, std::vector<unsigned char> &buf, View *v) {
    const size_t ma = bgzf_member_at(f, lo);
    size_t mb = ma;
    while (mb < f->mem.size() && f->uoff[mb] < hi) mb++;
    buf.resize((size_t)(f->uoff[mb] - f->uoff[ma]));
    Inflater inf;
    if (!inf.ok) return false;
    size_t len = 0;
    for (size_t i = ma; i < mb; i++) {
        std::string err;
        len += bgzf_inflate(inf.z, f->p, f->mem[i], buf.data() + len, &err);
        if (!err.empty()) return false;
    }
    *v = View{buf.data(), (size_t)f->uoff[ma], (size_t)f->uoff[mb], f->n};
    return true;
}
static View whole(const PlainFile *f) { return View{f->p, 0, f->n, f->n}; }

// the first record start in [from, from + limit) (v.n if none there): the
// search is bounded, so a file whose records the heuristic cannot recognise
// (CRLF or line-wrapped FASTQ) costs each chunk at most `limit` bytes of scan.
// Needs from - 1 >= v.lo.
static size_t record_start(const View &v, bool fastq, size_t from, size_t limit) {
    if (from == 0) return 0;
    if (from >= v.n || from >= v.hi) return v.n;
    const unsigned char *B = v.b, *e = v.b + (v.hi - v.lo);
    const unsigned char *q = B + (from - v.lo);
    const unsigned char *lim = limit < v.hi - from ? q + limit : e;
    auto line_end = [&](const unsigned char *x) -> const unsigned char * {
        const void *m = memchr(x, '\n', (size_t)(e - x));
        return m ? (const unsigned char *)m : e;
    };
    // start of the first line beginning at or after from
    if (q[-1] != '\n') {
        q = line_end(q);
        if (q < e) q++;
    }
    auto record4 = [&](const unsigned char *r, const unsigned char **next) -> bool {
        if (r >= e || *r != '@') return false;
        const unsigned char *l1 = line_end(r);
        if (l1 >= e) return false;
        const unsigned char *s0 = l1 + 1, *s1 = line_end(s0);
        if (s1 >= e || s1 == s0) return false;
        const unsigned char *p0 = s1 + 1;
        if (p0 >= e || *p0 != '+') return false;
        const unsigned char *p1 = line_end(p0);
        if (p1 >= e) return false;
        const unsigned char *q0 = p1 + 1, *q1 = line_end(q0);
        if (q1 - q0 != s1 - s0) return false;
        for (const unsigned char *c = s0; c < s1; c++)
            if (*c == '\r' || *c == ' ' || *c == '\t') return false;
        for (const unsigned char *c = q0; c < q1; c++)
            if (*c == '\r' || *c == ' ' || *c == '\t') return false;
        *next = q1 < e ? q1 + 1 : e;
        return true;
    };
    while (q < lim) {
        if (!fastq) {
            if (*q == '>') return v.lo + (size_t)(q - B);
        } else if (*q == '@') {
            const unsigned char *n1, *n2;
            if (record4(q, &n1) && (n1 >= e || record4(n1, &n2))) return v.lo + (size_t)(q - B);
        }
        q = line_end(q);
        if (q < e) q++;
    }
    return v.n;
}
size_t plain_record_start(const PlainFile *f, size_t from, size_t limit) {
    return record_start(whole(f), f->fastq, from, limit);
}

// a chunk parser over stream bytes from `start` (same record rules as the
// file's own parser; the first-read rule was settled by the file's first record)
static void chunk_parser(Parser &pr, const PlainFile *f, const unsigned char *p, size_t nbytes) {
    std::unique_ptr<MemSource> ms(new MemSource());
    ms->path = f->path;
    ms->p = p;
    ms->n = nbytes;
    ms->pos = 0;
    pr.src = std::move(ms);
    pr.path = f->path;
    pr.buf.resize(std::min<size_t>(1 << 22, std::max<size_t>(nbytes, 4096)));
    pr.fastq = f->fastq;
    pr.have_qualities = f->fastq;
    pr.num_reads = 1;
}
static void add_raw(std::vector<RawBatch> &out, const std::string &seq, int k, uint64_t max_kmers) {
    const size_t n = seq.size();
    if (n < (size_t)k) return;
    RawBatch *b = &out.back();
    if (b->nkmers >= max_kmers) {
        out.emplace_back();
        b = &out.back();
    }
    b->seq.insert(b->seq.end(), seq.begin(), seq.end());
    b->len.push_back((uint32_t)n);
    b->nkmers += n - (size_t)k + 1;
    b->nreads_parsed++;
}

// Parse records starting at byte `start` until the next record would start at
// or past `stop`; returns the offset where parsing stopped.  Reads >= k bases
// go into raw batches of <= max_kmers k-mers (out grows by one batch at a
// time).  *nreads counts good reads; a malformed record throws after the
// reads before it are in out.  *overrun: the parse needed bytes past the
// view that the stream has (its result is void; nothing thrown).
static uint64_t parse_range(const View &v, const PlainFile *f, size_t start, size_t stop, int k, uint64_t max_kmers,
                            std::vector<RawBatch> &out, uint64_t *nreads, bool *overrun) {
    Parser pr;
    chunk_parser(pr, f, v.b + (start - v.lo), v.hi - start);
    if (out.empty()) out.emplace_back();
    *overrun = false;
    try {
        for (;;) {
            if (start + pr.offset() >= stop) break;
            if (pr.next_read_locked() == KH_END) break;
            (*nreads)++;
            add_raw(out, pr.seq, k, max_kmers);
        }
    } catch (...) {
        if (pr.eof && v.hi < v.n) { *overrun = true; return start + pr.offset(); }
        throw;
    }
    if (pr.eof && v.hi < v.n) *overrun = true;
    return start + pr.offset();
}
uint64_t plain_parse_range(const PlainFile *f, size_t start, size_t stop, int k, uint64_t max_kmers,
                           std::vector<RawBatch> &out, uint64_t *nreads) {
    bool overrun;
    return parse_range(whole(f), f, start, stop, k, max_kmers, out, nreads, &overrun);
}

// Is a chunked parse worth starting (a record start recognised inside the
// second chunk)?  Single-chunk inputs always are.
bool plain_chunkable(const PlainFile *f, size_t CH) {
    if (f->n <= CH) return true;
    if (!f->bgzf) return record_start(whole(f), f->fastq, CH, CH) < f->n;
    std::vector<unsigned char> buf;
    View v;
    if (!bgzf_window(f, CH - 1, std::min(f->n, CH + BGZF_EXTRA), buf, &v)) return false;
    return record_start(v, f->fastq, CH, BGZF_LIM) < f->n;
}

// Chunk c of CH bytes: where its first record starts (n: none recognised),
// where its parse really ended, its reads; *redo: the chunk could not be
// parsed on its own (the consumer continues serially from its start).  A
// malformed record throws after the reads before it are in out.
void plain_parse_chunk(const PlainFile *f, size_t c, size_t CH, int k, uint64_t max_kmers, std::vector<RawBatch> &out,
                       uint64_t *nreads, size_t *start, size_t *end, bool *redo) {
    const size_t n = f->n, nch = (n + CH - 1) / CH;
    *redo = false;
    std::vector<unsigned char> buf;
    View v = whole(f);
    size_t lim = CH;
    if (f->bgzf) {
        lim = BGZF_LIM;
        const size_t lo = c ? c * CH - 1 : 0, hi = std::min(n, (c + 1) * CH + BGZF_EXTRA);
        if (!bgzf_window(f, lo, hi, buf, &v)) {   // damage: the serial rest meets it in order
            *start = *end = n;
            *redo = true;
            return;
        }
    }
    // a chunk without a recognised record start parses nothing (the consumer
    // then continues serially); a chunk whose successor has none stops at the
    // first record boundary past its own end, so no chunk holds much more than CH
    *start = record_start(v, f->fastq, c * CH, lim);
    size_t stop_at = n;
    if (c + 1 < nch) {
        stop_at = record_start(v, f->fastq, (c + 1) * CH, lim);
        if (stop_at >= n) stop_at = (c + 1) * CH;
    }
    *end = n;
    if (*start < n) {
        bool overrun = false;
        *end = parse_range(v, f, *start, stop_at, k, max_kmers, out, nreads, &overrun);
        if (overrun) {
            out.clear();
            *nreads = 0;
            *redo = true;
        }
    }
}

// BGZF members in order from stream offset `from` (the streaming source's
// bytes, with its damage messages), for the serial rest
struct BgzfSeqSource : Source {
    const PlainFile *f;
    size_t m, skip;
    Inflater inf;
    std::vector<unsigned char> buf = std::vector<unsigned char>(65536);
    size_t pos = 0, len = 0;
    std::string err;
    size_t read(unsigned char *dst, size_t want) override {
        while (pos >= len) {
            if (!err.empty()) fail(KH_EFILE, "File " + path + ": " + err);
            if (m >= f->mem.size()) return 0;
            len = bgzf_inflate(inf.z, f->p, f->mem[m++], buf.data(), &err);
            pos = std::min(skip, len);
            skip -= pos;
        }
        const size_t k = std::min(want, len - pos);
        memcpy(dst, buf.data() + pos, k);
        pos += k;
        return k;
    }
};

// The rest of the input from `from`, serially, batch by batch to sink; *nreads
// counts the reads parsed (a malformed record or damage throws after the
// reads before it are sunk and counted).
void plain_parse_rest(const PlainFile *f, size_t from, size_t CH, int k, uint64_t max_kmers,
                      const std::function<void(RawBatch &)> &sink, uint64_t *nreads) {
    if (!f->bgzf) {
        // in pieces of about CH bytes (each piece ends on a real record
        // boundary), so host memory stays bounded
        while (from < f->n) {
            std::vector<RawBatch> raw;
            uint64_t nr = 0;
            std::exception_ptr err;
            size_t end = f->n;
            try {
                end = plain_parse_range(f, from, std::min(f->n, from + CH), k, max_kmers, raw, &nr);
            } catch (...) {
                err = std::current_exception();
            }
            for (RawBatch &r : raw) sink(r);
            *nreads += nr;
            if (err) std::rethrow_exception(err);
            if (end <= from) break;   // no progress: end of input
            from = end;
        }
        return;
    }
    if (from >= f->n) return;
    Parser pr;
    std::unique_ptr<BgzfSeqSource> src(new BgzfSeqSource());
    src->path = f->path;
    src->f = f;
    src->m = bgzf_member_at(f, from);
    src->skip = from - (size_t)f->uoff[src->m];
    pr.src = std::move(src);
    pr.path = f->path;
    pr.buf.resize(1 << 22);
    pr.fastq = f->fastq;
    pr.have_qualities = f->fastq;
    pr.num_reads = 1;
    for (;;) {
        RawBatch b;
        std::exception_ptr err;
        bool done = false;
        uint64_t nr = 0;
        try {
            while (b.nkmers < max_kmers) {
                if (pr.next_read_locked() == KH_END) { done = true; break; }
                nr++;
                b.nreads_parsed++;
                const size_t n = pr.seq.size();
                if (n < (size_t)k) continue;
                b.seq.insert(b.seq.end(), pr.seq.begin(), pr.seq.end());
                b.len.push_back((uint32_t)n);
                b.nkmers += n - (size_t)k + 1;
            }
        } catch (...) {
            err = std::current_exception();
        }
        sink(b);
        *nreads += nr;
        if (err) std::rethrow_exception(err);
        if (done) return;
    }
}

// the parser has been drained by the chunk path: reads counted, nothing left
void parser_mark_drained(Parser *pr, uint64_t nreads) {
    std::lock_guard<std::mutex> lk(pr->mu);
    pr->num_reads += nreads;
    pr->eof = true;
    pr->pos = pr->len = 0;
    pr->src.reset(new MemSource());
}

// Raw reads (uncleaned sequence bytes) of up to max_kmers k-mers for the
// pipelined feed (kh_consume_parser): the same record semantics as
// parser_fill_batch; cleaning and packing happen on the packer threads.
void parser_fill_raw(Parser *p, RawBatch &b, int k, uint64_t max_kmers, uint64_t max_bases, bool *done,
                     uint64_t *taken) {
    std::lock_guard<std::mutex> lk(p->mu);
    *done = false;
    while (b.nkmers < max_kmers && b.seq.size() < max_bases) {
        int rc = p->next_read_locked();  // may throw
        if (rc == KH_END) { *done = true; break; }
        (*taken)++;
        b.nreads_parsed++;
        const size_t n = p->seq.size();
        if (n < (size_t)k) continue;
        b.seq.insert(b.seq.end(), p->seq.begin(), p->seq.end());
        b.len.push_back((uint32_t)n);
        b.nkmers += n - (size_t)k + 1;
    }
}

}  // namespace kh
