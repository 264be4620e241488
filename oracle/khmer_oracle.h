/*
 * khmer_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference (ctb/khmer, oxli)
 * k-mer counting hot path.  It is the parity checker for the HIP product path
 * and the CPU baseline ("port") in bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never does.
 *
 * Parity pinning: the reference could not be built or run in this environment
 * (execution denied).  This restatement is pinned by the
 * reference's own known-answer tests and fixture results, transcribed into
 * tests/test_oracle_kats.py (see DESIGN.md "Oracle").
 *
 * Semantics = the reference's single-threaded stream order.
 */
#ifndef KHMER_ORACLE_H
#define KHMER_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* storage kinds == reference file-type codes (include/oxli/oxli.hh:91-97) */
#define OR_BYTE   1  /* ByteStorage   (Countgraph)      */
#define OR_BIT    2  /* BitStorage    (Nodegraph)       */
#define OR_NIBBLE 7  /* NibbleStorage (SmallCountgraph) */

/* hash families */
#define OR_HASH_TWOBIT 0  /* Hashgraph classes: reversible 2-bit (kmer_hash.cc:65-95) */
#define OR_HASH_MURMUR 1  /* *table classes: MurmurHash3 canonical (kmer_hash.cc:177-198) */

typedef struct or_table or_table;
typedef struct or_parser or_parser;

/* ---- hashing (include/oxli/kmer_hash.hh:62-96, src/oxli/kmer_hash.cc) ---- */
int      or_hash2bit(const char *kmer, int k, uint64_t *fwd, uint64_t *rc, uint64_t *out);
void     or_revhash(uint64_t h, int k, char *out /* k+1 bytes */);
void     or_revcomp(const char *in, size_t len, char *out);
void     or_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t out[2]);
uint64_t or_hash_murmur(const char *kmer, int k);
uint64_t or_hash_murmur_forward(const char *kmer, int k);

/* ---- primes (include/oxli/hashtable.hh:79-123) ---- */
int      or_is_prime(uint64_t n);
int      or_get_n_primes_near_x(uint32_t n, uint64_t x, uint64_t *out);

/* ---- tables (include/oxli/storage.hh) ---- */
or_table *or_table_new(int kind, int hash, int k, const uint64_t *sizes, int n);
void      or_table_free(or_table *t);
int       or_add(or_table *t, uint64_t h);             /* Storage::add -> is_new */
int       or_test_and_set(or_table *t, uint64_t h);    /* Storage::test_and_set_bits */
int       or_get(const or_table *t, uint64_t h);       /* Storage::get_count */
void      or_set_bigcount(or_table *t, int on);
uint64_t  or_n_unique(const or_table *t);
uint64_t  or_n_occupied(const or_table *t);
uint64_t  or_table_nbytes(const or_table *t, int i);
const uint8_t *or_table_data(const or_table *t, int i);
uint64_t  or_bigcount_size(const or_table *t);
void      or_bigcount_export(const or_table *t, uint64_t *keys, uint16_t *vals); /* ascending keys */

/* ---- consume (src/oxli/hashtable.cc:125-150, 280-294) ---- */
uint32_t  or_consume_string(or_table *t, const char *s, size_t len); /* raw string, no cleaning */
uint64_t  or_kmer_hashes(const or_table *t, const char *s, size_t len, uint64_t *out);
/* consume a FASTA/FASTQ(.gz) file with read cleaning; mode 0 = consume_seqfile,
 * 1 = consume_seqfile_and_tag.  Returns 0 ok, <0 error (message via or_last_error). */
int       or_consume_fastx(or_table *t, const char *path, int mode,
                           uint32_t *reads, uint64_t *kmers);
/* consume_seqfile_with_mask / _banding / _banding_with_mask (hashtable.cc:152-274) */
int       or_consume_fastx_filtered(or_table *t, const char *path, uint32_t num_bands, uint32_t band,
                                    const or_table *mask, uint32_t threshold, int consume_masked,
                                    uint32_t *reads, uint64_t *kmers);
/* consume an in-memory batch: seqs concatenated, offs[nreads+1]; cleaned per read */
uint64_t  or_consume_batch(or_table *t, const char *seqs, const uint64_t *offs, uint64_t nreads);

/* ---- queries (src/oxli/hashtable.cc:299-328) ---- */
int       or_median(const or_table *t, const char *s, size_t len,
                    uint16_t *med, float *avg, float *sd);

int       or_abundance_distribution(or_table *t, or_table *tracking, const char *path,
                                    uint64_t *dist /* 65536 */);

/* ---- tags (src/oxli/hashgraph.cc:200-271) ---- */
uint64_t  or_n_tags(const or_table *t);
void      or_tags_export(const or_table *t, uint64_t *out); /* ascending */

/* ---- files (src/oxli/storage.cc) ---- */
int       or_save(const or_table *t, const char *path);
int       or_save_tagset(const or_table *t, const char *path);

/* ---- FASTA/FASTQ reader (src/oxli/read_parsers.cc:329-372 semantics) ---- */
or_parser *or_parser_open(const char *path);
/* returns 1 = read, 0 = end, <0 = error; pointers valid until next call */
int        or_parser_next(or_parser *p, const char **name, const char **seq,
                          const char **qual, size_t *seqlen, size_t *quallen);
uint64_t   or_parser_num_reads(const or_parser *p);
void       or_parser_close(or_parser *p);

const char *or_last_error(void);

/* ---- CPU baseline: multi-threaded consume of an in-memory batch, with the
 * reference's -T>1 atomic semantics (storage.hh:571-624).  Table bytes equal the
 * single-stream result unless bins saturate concurrently. ---- */
uint64_t  or_consume_batch_mt(or_table *t, const char *seqs, const uint64_t *offs,
                              uint64_t nreads, int nthreads);

/* ---- synthetic streams of khmer_amd/synth.py (NOT reference functions; they
 * let the oracle consume the benchmark's exact workload for golden fixtures) ---- */
void      or_synth_read(uint64_t seed, uint64_t r, int L, char *out /* L+1 */);
void      or_synth_genomic_read(uint64_t seed, uint64_t genome, uint64_t r, int L, char *out /* L+1 */);
uint64_t  or_consume_synth(or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L);
uint64_t  or_consume_synth_mt(or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L,
                              int nthreads);
int       or_median_synth(const or_table *t, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int L,
                          uint16_t *med, float *avg, float *sd);

#ifdef __cplusplus
}
#endif
#endif
