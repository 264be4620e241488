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
#include <ctype.h>
#include <string.h>
#include <zlib.h>

#include <string>

#include "kh_internal.h"

namespace kh {

struct Parser {
    gzFile gz = nullptr;
    std::string path;
    std::vector<unsigned char> buf;
    size_t pos = 0, len = 0;
    bool eof = false;
    bool fastq = false;
    bool have_qualities = false;
    uint64_t num_reads = 0;
    std::string name, seq, qual, tmp;
    std::mutex mu;

    ~Parser() { if (gz) gzclose(gz); }

    int peek() {
        if (pos < len) return buf[pos];
        if (eof) return -1;
        int n = gzread(gz, buf.data(), (unsigned)buf.size());
        if (n <= 0) { eof = true; len = pos = 0; return -1; }
        len = (size_t)n; pos = 0;
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
            unsigned char *q = s;
            while (q < e && *q != '\n' && *q != '\r') q++;
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
            unsigned char *s = buf.data() + pos, *e = buf.data() + len, *q = s;
            while (q < e && *q != '\n' && *q != '\r' && !isspace(*q)) q++;
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
        int c;
        while (qual.size() < seq.size() && (c = peek()) >= 0) {
            if (!isspace(c)) qual.push_back((char)c);
            pos++;
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
    gzFile gz = gzopen(path, "rb");
    if (!gz) fail(KH_EFILE, std::string("File ") + path + " contains badly formatted sequence or does not exist.");
    gzbuffer(gz, 1 << 20);
    Parser *p = new Parser();
    p->gz = gz;
    p->path = path;
    p->buf.resize(1 << 22);
    int c = p->peek();
    if (c < 0) {
        delete p;
        fail(KH_EFILE, std::string("File ") + path + " does not contain any sequences!");
    }
    if (c != '>' && c != '@') {
        delete p;
        fail(KH_EFILE, std::string("File ") + path + " contains badly formatted sequence or does not exist.");
    }
    p->fastq = (c == '@');
    return p;
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

}  // namespace kh
