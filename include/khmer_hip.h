/*
 * khmer_hip.h -- C ABI of libkhmer_hip.so, the MI355X-native k-mer counting
 * engine behind the khmer_amd Python package.
 *
 * Plain pointers and sizes only; no torch types.  Each entry point names the
 * reference interface it replaces (paths under ctb/khmer).  Every function
 * returns a status code (KH_OK on success); on failure kh_last_error() holds a
 * thread-local message and the code selects the Python exception class the
 * reference raises for the same failure
 * (khmer/_oxli/oxli_exception_convert.cc:9-31).
 *
 * Threading: calls on one graph are serialised by the library (the reference's
 * atomic/spin-locked table updates, include/oxli/storage.hh:571-624); a parser
 * may be drained by several threads, each read is consumed exactly once
 * (src/oxli/read_parsers.cc:329-372).  ctypes releases the GIL around calls.
 */
#ifndef KHMER_HIP_H
#define KHMER_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KH_ABI_VERSION 1

/* status codes -> Python exceptions */
#define KH_OK       0
#define KH_EVALUE   1  /* ValueError    (oxli_value_exception, InvalidValue, InvalidRead) */
#define KH_EFILE    2  /* OSError       (oxli_file_exception, InvalidStream, StreamReadError) */
#define KH_EATTR    3  /* AttributeError (ReadOnlyAttribute) */
#define KH_ENOMEM   4  /* MemoryError   (std::bad_alloc, hipErrorOutOfMemory) */
#define KH_EDEVICE  5  /* RuntimeError  (HIP runtime failure / no device) */
#define KH_ERUNTIME 6  /* RuntimeError  (generic oxli_exception in helpers) */
#define KH_END      7  /* not an error: parser exhausted (NoMoreReadsAvailable) */

/* storage kinds == on-disk type codes (include/oxli/oxli.hh:91-97) */
#define KH_STORAGE_BYTE   1  /* ByteStorage   -> Countgraph / Counttable           */
#define KH_STORAGE_BIT    2  /* BitStorage    -> Nodegraph / Nodetable             */
#define KH_STORAGE_NIBBLE 7  /* NibbleStorage -> SmallCountgraph / SmallCounttable */

/* hash families */
#define KH_HASH_TWOBIT 0  /* Hashgraph: reversible 2-bit (include/oxli/kmer_hash.hh:62-96) */
#define KH_HASH_MURMUR 1  /* MurmurHashtable (include/oxli/hashtable.hh:494-534)           */

typedef struct kh_graph kh_graph;
typedef struct kh_parser kh_parser;
typedef struct kh_group kh_group;

const char *kh_last_error(void);
int kh_abi_version(void);
/* number of visible HIP devices (0 when none; never an error) */
int kh_device_count(int *n);

/* ---------------- hashing helpers ------------------------------------------
 * replaces khmer._khmer.forward_hash / forward_hash_no_rc / reverse_hash /
 * hash_murmur3 / hash_no_rc_murmur3 / reverse_complement
 * (src/khmer/_cpy_khmer.cc:63-190 over src/oxli/kmer_hash.cc:65-207) */
int kh_hash_twobit(const char *kmer, int k, uint64_t *fwd, uint64_t *rc, uint64_t *canon);
int kh_reverse_hash(uint64_t h, int k, char *out /* k+1 */);
int kh_hash_murmur(const char *kmer, int len, uint64_t *canon, uint64_t *fwd);
int kh_reverse_complement(const char *s, size_t len, char *out /* len+1 */);
/* all k-mer hashes of a string, reference iterator semantics
 * (Hashtable::get_kmer_hashes, src/oxli/hashtable.cc:378-388) */
int kh_kmer_hashes(int hash_kind, int k, const char *seq, size_t len,
                   uint64_t *out, uint64_t *n_out);

/* ---------------- primes ----------------------------------------------------
 * replaces khmer._oxli.utils.get_n_primes_near_x / is_prime
 * (khmer/_oxli/utils.pyx:12-17 over include/oxli/hashtable.hh:79-123) */
int kh_is_prime(uint64_t n, int *out);
int kh_get_n_primes_near_x(uint32_t n, uint64_t x, uint64_t *out, uint32_t *found);

/* ---------------- read parser -----------------------------------------------
 * replaces oxli::read_parsers::ReadParser<FastxReader> and the CPython
 * khmer.ReadParser (include/oxli/read_parsers.hh:138-178,
 * src/oxli/read_parsers.cc:257-382, src/khmer/_cpy_readparsers.cc:392-550).
 * FASTA/FASTQ: plain, gzip (incl. BGZF / concatenated members) or bzip2. */
int  kh_parser_open(const char *path, kh_parser **out);
/* next read; returns KH_END when exhausted.  Pointers stay valid until the
 * next call on this parser from the same thread. */
int  kh_parser_next_read(kh_parser *p, const char **name, size_t *name_len,
                         const char **seq, size_t *seq_len,
                         const char **qual, size_t *qual_len);
int  kh_parser_num_reads(kh_parser *p, uint64_t *out);
int  kh_parser_is_complete(kh_parser *p, int *out);
void kh_parser_close(kh_parser *p);

/* ---------------- graph lifecycle -------------------------------------------
 * replaces the Countgraph / SmallCountgraph / Nodegraph (and Counttable /
 * SmallCounttable / Nodetable) constructors, khmer/_oxli/graphs.pyx:817-900 ->
 * include/oxli/hashgraph.hh:273-296, include/oxli/hashtable.hh:591-627.
 * Tables live in HBM of `device`; they are zero-initialised. */
int  kh_graph_create(int storage, int hash_kind, int k, const uint64_t *sizes,
                     int n_tables, int device, kh_graph **out);
void kh_graph_destroy(kh_graph *g);
int  kh_graph_info(kh_graph *g, int *storage, int *hash_kind, int *k, int *n_tables);
int  kh_graph_tablesizes(kh_graph *g, uint64_t *out);          /* hashsizes() */
int  kh_graph_set_use_bigcount(kh_graph *g, int on);           /* storage.cc:50-56 */
int  kh_graph_get_use_bigcount(kh_graph *g, int *on);
/* the bigcount map (storage.hh:498 KmerCountMap) sorted by hash: n entries
 * are written when cap >= n; *n always receives the map size */
int  kh_graph_get_bigcounts(kh_graph *g, uint64_t *keys, uint16_t *vals, uint64_t cap, uint64_t *n);
int  kh_graph_n_unique_kmers(kh_graph *g, uint64_t *out);      /* storage.hh:143-165 */
int  kh_graph_n_occupied(kh_graph *g, uint64_t *out);
/* largest k-mer batch processed per device pipeline pass (memory knob) */
int  kh_graph_set_batch_kmers(kh_graph *g, uint64_t max_kmers);
/* back to the freshly constructed state (zero tables, counters, bigcounts, tags) */
int  kh_graph_clear(kh_graph *g);

/* ---------------- hot path: consume ----------------------------------------
 * Hashtable::consume_seqfile<FastxReader> (src/oxli/hashtable.cc:125-150):
 * drains `p`, cleans every read (read_parsers.cc:53-69), counts every k-mer.
 * Returns this call's share of (reads, k-mers).  mode 1 = consume_seqfile_and_tag
 * (src/oxli/hashgraph.cc:290-320). */
int kh_consume_parser(kh_graph *g, kh_parser *p, int mode, uint32_t *reads, uint64_t *kmers);

/* Hashtable::consume_seqfile_with_mask / _banding / _banding_with_mask
 * (src/oxli/hashtable.cc:152-274; khmer/_oxli/graphs.pyx:241-280).  Counts a
 * k-mer only if its hash lies in band `band` of `num_bands`
 * (compute_band_interval, src/oxli/kmer_hash.cc:262-276) and, when `mask` is
 * not NULL, mask's count c of the hash satisfies c >= threshold
 * (consume_masked) or c <= threshold.  num_bands == 0 disables banding.
 * *kmers = k-mers counted.  KH_EVALUE if band > num_bands or mask == g. */
int kh_consume_parser_filtered(kh_graph *g, kh_parser *p, uint32_t num_bands, uint32_t band, kh_graph *mask,
                               uint32_t threshold, int consume_masked, uint32_t *reads, uint64_t *kmers);
/* Hashtable::consume_string over a batch of reads (src/oxli/hashtable.cc:280-294).
 * seqs = concatenated reads, offsets[nreads+1]; clean != 0 applies
 * _to_valid_dna first (consume_seqfile semantics), 0 hashes raw (consume()). */
int kh_consume_seqs(kh_graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads,
                    int clean, uint64_t *kmers);
/* device-resident packed reads (bench / multi-GPU path): `d_words` 2-bit
 * packed bases (kh_device.h layout) and `d_kmer_off[nreads+1]` k-mer prefix
 * offsets (d_kmer_off[0] == 0), both already in this graph's device memory.
 * Every read must hold at least one k-mer.  Processed in device batches of
 * kh_graph_set_batch_kmers() k-mers; returns when the tables are updated. */
int kh_consume_packed_device(kh_graph *g, const uint64_t *d_words, const uint64_t *d_kmer_off,
                             uint64_t nreads, uint64_t nkmers);
/* the same for reads of one length (read_len >= k): no offset array, read r
 * starts at base r*read_len (the common fixed-length sequencing case). */
int kh_consume_packed_fixed_device(kh_graph *g, const uint64_t *d_words, uint64_t nreads, uint32_t read_len);
/* Murmur graphs (Counttable family, include/oxli/hashtable.hh:494-627): ASCII
 * reads of one length already in device memory, read r at byte r*read_len;
 * MurmurKmerHashIterator over each (src/oxli/kmer_hash.cc:177-198).
 * The kernels read every k-mer as aligned 8-byte words, up to 64 bytes past
 * the last read: when the allocation holding d_bytes ends less than 64 bytes
 * after nreads*read_len, the library first copies the reads into a padded
 * buffer of its own (correct for any buffer; allocate +64 bytes to avoid the
 * copy). */
int kh_consume_bytes_fixed_device(kh_graph *g, const uint8_t *d_bytes, uint64_t nreads, uint32_t read_len);
/* explicit hashes: Hashtable::count/add(HashIntoType) (include/oxli/hashtable.hh:222-243);
 * is_new[n] (nullable) receives Storage::add's return per hash, in order. */
int kh_add_hashes(kh_graph *g, const uint64_t *hashes, uint64_t n, uint8_t *is_new);

/* ---------------- queries --------------------------------------------------- */
/* Storage::get_count per hash (storage.hh:206-219, 362-379, 627-649) */
int kh_get_counts(kh_graph *g, const uint64_t *hashes, uint64_t n, uint16_t *out);
/* Hashtable::get_median_count per read (src/oxli/hashtable.cc:299-328); reads
 * with no k-mer get status[r] = 1 (the reference throws for them). */
int kh_median_counts(kh_graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads,
                     uint16_t *med, float *avg, float *stddev, uint8_t *status);
/* get_median_count per read of device-resident fixed-length reads (2-bit
 * packed words for 2-bit graphs, ASCII bytes for Murmur graphs), outputs in
 * device memory; read_len - k + 1 <= 256.  ASCII input: the padding rule of
 * kh_consume_bytes_fixed_device applies (2-bit input: the packed layout's
 * trailing word, as kh_synth_packed_device writes it).  Same values as kh_median_counts
 * (src/oxli/hashtable.cc:299-328; scripts/count-median.py:123 is the caller). */
int kh_median_counts_fixed_device(kh_graph *g, const void *d_reads, uint64_t nreads, uint32_t read_len,
                                  uint16_t *d_med, float *d_avg, float *d_stddev);
/* Hashtable::get_kmer_hashes / get_kmer_counts (src/oxli/hashtable.cc:378-388,
 * 403-413) over a batch of reads (raw, no cleaning: the table's own k-mer
 * iterator), on the device.  Reads shorter than k contribute nothing; out
 * receives the k-mers of the remaining reads back to back (*n_out of them;
 * out must hold sum(len - k + 1) entries). */
int kh_graph_kmer_hashes(kh_graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads,
                         uint64_t *out, uint64_t *n_out);
int kh_graph_kmer_counts(kh_graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads,
                         uint16_t *out, uint64_t *n_out);
/* Hashtable::median_at_least per read (src/oxli/hashtable.cc:333-364; the
 * normalize-by-median filter, khmer/trimming.py:45): out[r] = 1 when at least
 * unsigned(0.5 + float(n)/2) of the read's n k-mers have a count >= cutoff.
 * Reads shorter than k get status[r] = 1 and out[r] = 0 (the reference's
 * Python binding raises ValueError for them, graphs.pyx:182-185). */
int kh_median_at_least(kh_graph *g, const char *seqs, const uint64_t *offsets, uint64_t nreads, uint32_t cutoff,
                       uint8_t *out, uint8_t *status);
/* Hashtable::abundance_distribution (src/oxli/hashtable.cc:451-493);
 * dist[65536]. */
int kh_abundance_distribution(kh_graph *g, kh_parser *p, kh_graph *tracking, uint64_t *dist);

/* ---------------- tables, files, tags ---------------------------------------- */
int kh_graph_table_nbytes(kh_graph *g, int i, uint64_t *out);
int kh_graph_copy_table(kh_graph *g, int i, uint8_t *dst);      /* get_raw_tables() */
int kh_graph_save(kh_graph *g, const char *path);               /* storage.cc:99-136,582-803 */
/* Countgraph/Nodegraph/SmallCountgraph .load (graphs.pyx:302-307);
 * expected_storage checks the file type code like the reference readers. */
int kh_graph_load(const char *path, int expected_storage, int hash_kind, int device,
                  kh_graph **out);

/* header fields of a saved table file, read as raw bytes like the reference's
 * Python readers (khmer/__init__.py:95-178 extract_nodegraph_info /
 * extract_countgraph_info).  layout 0: no bigcount byte (nodegraph reader);
 * layout 1: a bigcount byte unless the type is SMALLCOUNT (countgraph reader).
 * out[7] = {version, type, use_bigcount (-1 when absent), k, n_tables,
 * n_occupied, first table size}.  KH_EFILE when the file is short or does not
 * start with "OXLI". */
int kh_file_header(const char *path, int layout, int64_t *out);
int kh_graph_n_tags(kh_graph *g, uint64_t *out);
int kh_graph_get_tags(kh_graph *g, uint64_t *out);              /* ascending */
int kh_graph_add_tag(kh_graph *g, uint64_t h);
int kh_graph_save_tagset(kh_graph *g, const char *path);        /* hashgraph.cc:55-88 */
int kh_graph_load_tagset(kh_graph *g, const char *path, int clear);

/* ---------------- benchmark support -----------------------------------------
 * seeded synthetic 2-bit reads (khmer_amd/synth.py's definition) generated
 * straight into HBM: reads r0 .. r0+nreads-1 of length read_len, packed
 * contiguously (nreads*read_len/32 + 2 words), k-mer offsets r*(read_len-k+1). */
int kh_synth_packed_device(int device, uint64_t seed, uint64_t r0, uint64_t nreads, int read_len, int k,
                           uint64_t *d_words, uint64_t *d_kmer_off);
/* the skewed "genomic" stream of SURVEY.md §8(d) (khmer_amd/synth.py
 * genomic_codes): reads sampled from a random genome of `genome` bases, either
 * strand, 1% substitutions; same packing as kh_synth_packed_device. */
int kh_synth_genomic_device(int device, uint64_t seed, uint64_t genome, uint64_t r0, uint64_t nreads, int read_len,
                            int k, uint64_t *d_words, uint64_t *d_kmer_off);
/* 2-bit packed bases -> ASCII bytes (A/T/C/G), both in device memory */
int kh_unpack_ascii_device(int device, const uint64_t *d_words, uint64_t nbases, uint8_t *d_bytes);
int kh_device_malloc(int device, uint64_t bytes, void **out);
/* synchronous copy between host and/or device memory of `device` */
int kh_device_copy(int device, void *dst, const void *src, uint64_t nbytes);
int kh_device_free(int device, void *p);
int kh_device_synchronize(int device);
/* per-kernel HIP-event timing on the graph's stream: on=1 resets and enables;
 * stats are text lines "kernel<TAB>launches<TAB>total_ms" */
int kh_graph_set_profiling(kh_graph *g, int on);
/* work distribution of the fixed-capacity level 1 and of apply (no reference
 * counterpart; results are identical either way): l1_chunk_tiles = tiles per
 * dynamically scheduled level-1 chunk (0: one fixed share per workgroup),
 * apply_dynamic = 1 regions from a queue / 0 fixed stride; -1 keeps the
 * default (KH_L1_CHUNK / KH_APPLY_DYN, else 32 and 1) */
int kh_graph_set_schedule(kh_graph *g, int l1_chunk_tiles, int apply_dynamic);
int kh_graph_kernel_stats(kh_graph *g, char *buf, size_t cap, size_t *len);

/* ---------------- multi-GPU sharded groups ----------------------------------
 * SURVEY.md §8(e).  The reference has no multi-device path; its hash-space
 * sharding precedent is k-mer banding (src/oxli/hashtable.cc:192-228), which
 * yields byte-identical tables.  Here rank r of a G-rank group owns bins
 * [lo_r, lo_{r+1}) of every table (contiguous, 8-bin aligned slices); input
 * reads are consumed as one stream in rank order (source reads broadcast over
 * RCCL/xGMI, each rank applies the updates of the bins it owns); n_unique,
 * n_occupied and bigcounts are exact (winners routed to k-mer-window owners,
 * bigcount tallies all-gathered).  One process per GPU (nlocal = 1, uid from
 * rank 0's kh_group_unique_id), or all shards in one process on one device
 * (nlocal = world, uid = NULL: loopback, for testing).  Consume calls are
 * collective: every rank calls them in the same order with the same shape. */
int kh_group_unique_id(unsigned char *out, size_t cap);   /* cap >= 128 */
int kh_group_create(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int world, int rank,
                    int nlocal, const int *devices, const unsigned char *uid, kh_group **out);
void kh_group_destroy(kh_group *grp);
/* A one-shard-per-process group whose collectives run through host callbacks
 * instead of RCCL (a "host transport"): every call is collective over the
 * group, buffers are host memory, a nonzero return is an error.  Used to run
 * the multi-process protocol where RCCL cannot (several ranks on one device,
 * CPU-side plumbing such as gloo or a TCP rendezvous).
 *   allgather: recv[world * bytes] = every rank's `bytes` bytes, in rank order
 *   broadcast: buf (bytes) of rank `root` to every rank
 *   alltoallv: rank r's send holds the blocks for ranks 0..world-1 back to
 *              back (send_bytes[d] each); recv gets the blocks from ranks
 *              0..world-1 back to back (recv_bytes[s] each) */
typedef struct kh_transport {
    void *ctx;
    int (*allgather)(void *ctx, const void *send, void *recv, uint64_t bytes);
    int (*broadcast)(void *ctx, void *buf, uint64_t bytes, int root);
    int (*alltoallv)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv,
                     const uint64_t *recv_bytes);
} kh_transport;
int kh_group_create_hosted(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int world,
                           int rank, int device, const kh_transport *transport, kh_group **out);
/* RCCL view of a one-shard-per-process group: ncclCommCount / ncclCommCuDevice
 * (nranks = 0 and device = -1 for loopback and host-transport groups) */
int kh_group_comm_info(kh_group *grp, int *nranks, int *device);
/* local shard l as a graph handle (view: valid while the group lives; its
 * tables are the slices [lo, lo + size) reported by kh_group_slice) */
int kh_group_shard(kh_group *grp, int l, kh_graph **out);
int kh_group_info(kh_group *grp, int *world, int *nlocal, int *rank0);
int kh_group_slice(kh_group *grp, int l, int table, uint64_t *lo, uint64_t *size);
/* replaces the per-rank consume loop (hashtable.cc:106-133) over 2-bit packed
 * fixed-length reads: d_words[l] = local shard l's own reads (nlocal pointers) */
int kh_group_consume_packed_fixed_device(kh_group *grp, const uint64_t *const *d_words, uint64_t nreads,
                                         uint64_t read_len);
/* Group modes.  KH_GROUP_BROADCAST (kh_group_create): the
 * slices above, every rank hashes every source's reads (Option B).
 * KH_GROUP_EXCHANGE (Option A): every rank hashes only its own reads into the
 * unsharded level-1 buckets and sends each bucket to its owner (grouped
 * ncclSend/ncclRecv; host transport: alltoallv); rank r owns a contiguous
 * range of level-1 buckets, i.e. bucket-aligned slices reported by
 * kh_group_rank_slice.  A consume call's stream is taken pass by pass: pass p
 * holds the p-th chunk of every rank's reads in rank order, and n_unique /
 * bigcounts are exact for that order (tables and n_occupied do not depend on
 * the order). */
/* KH_GROUP_DELTA: the exchange-mode ownership, but no per-k-mer records
 * travel.  Every rank partitions and counts its own chunk of a pass into
 * full-size "delta" tables (the tables that chunk alone would give from
 * empty tables); each owner receives every rank's delta of its slice
 * (all-to-all), turns them into per-rank prefixes (the owned bytes as the
 * stream saw them when that rank's chunk began: table before the pass plus
 * the deltas of the lower ranks, saturating) and its updated slice, and
 * sends the prefixes back (all-to-all); every rank then applies its chunk
 * over its prefix tables with the single-GPU pipeline, which gives the
 * exact is_new winners, occupancy and bigcount events of its own k-mers.
 * Wire bytes per pass: 2 x the table bytes x (world - 1) / world per rank,
 * against exchange mode's 8 bytes per (k-mer, table).  A pass takes up to
 * the graph's batch of every rank's reads, in rank order (passes of
 * khmer_amd.parallel.delta_passes); n_unique and bigcounts are exact for
 * that order (src/oxli/hashtable.cc:192-228 is the reference's own
 * partitioned consume). */
enum { KH_GROUP_BROADCAST = 0, KH_GROUP_EXCHANGE = 1, KH_GROUP_DELTA = 2 };
int kh_group_create_mode(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int world, int rank,
                         int nlocal, const int *devices, const unsigned char *uid, int mode, kh_group **out);
int kh_group_create_hosted_mode(int storage, int hash_kind, int k, const uint64_t *sizes, int n_tables, int world,
                                int rank, int device, const kh_transport *transport, int mode, kh_group **out);
int kh_group_mode(kh_group *grp, int *mode);
/* bins [lo, lo + size) of table `table` held by rank `rank` (any rank) */
int kh_group_rank_slice(kh_group *grp, int rank, int table, uint64_t *lo, uint64_t *size);
int kh_group_counters(kh_group *grp, uint64_t *n_unique, uint64_t *n_occupied);   /* collective */
/* delta mode: bytes of the table pieces this process's ranks exchanged with
 * other ranks so far, as dense slices and as sent (sparse pieces: a bitmap of
 * the nonzero bytes plus those bytes; KH_DELTA_SPARSE=0 sends them dense).
 * No reference counterpart: the wire accounting of the MI355X group modes. */
int kh_group_wire_stats(kh_group *grp, uint64_t *dense_bytes, uint64_t *sent_bytes);
/* The Counttable family (MurmurHash3) in a group: the same
 * collective consume over ASCII fixed-length reads (d_bytes[l] = local shard
 * l's own reads; hash_kind KH_HASH_MURMUR at group creation).  Replaces the
 * per-rank consume loop (src/oxli/hashtable.cc:106-133) of
 * MurmurHashtable / SmallCounttable (include/oxli/hashtable.hh:494-534,
 * 606-620). */
int kh_group_consume_bytes_fixed_device(kh_group *grp, const uint8_t *const *d_bytes, uint64_t nreads,
                                        uint64_t read_len);
/* Hashtable::get_median_count (src/oxli/hashtable.cc:299-328) over every
 * rank's own fixed-length reads (collective; 2-bit groups: packed words,
 * Murmur groups: ASCII bytes; read_len - k + 1 <= 256).  A k-mer's bins live
 * on several ranks: exchange mode routes each (k-mer, table) lookup to the
 * bin's owner with the consume's level-1 partition and reduces the per-k-mer
 * minima back (MIN reduce-scatter); broadcast mode has every rank take the
 * minimum over its own bins of every source's k-mers (MIN reduce to the
 * source).  The read's home rank computes median / average / stddev
 * (float32 bit-exact as kh_median_counts_fixed_device) into d_med[l] /
 * d_avg[l] / d_sd[l] (device, one entry per read of local shard l). */
int kh_group_median_fixed_device(kh_group *grp, const void *const *d_reads, uint64_t nreads, uint64_t read_len,
                                 uint16_t *const *d_med, float *const *d_avg, float *const *d_sd);

#ifdef __cplusplus
}
#endif
#endif
