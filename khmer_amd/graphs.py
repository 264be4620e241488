"""Countgraph / Nodegraph / SmallCountgraph and the *table family on MI355X.

Python mirror of the reference's Cython API (khmer/_oxli/graphs.pyx:31-347,
817-900): same class names, constructor arguments, method names, return types
and exception classes.  Every table lives in HBM; every k-mer update and query
runs in libkhmer_hip.so's HIP kernels (no CPU fallback).  Scalar helpers that
the reference also computes on the host (hash(), reverse_hash()) stay on the
host.
"""
import ctypes

from . import _lib
from ._lib import lib, check
from .parsing import ReadParser
from .utils import get_n_primes_near_x

MAX_BIGCOUNT = 65535  # include/oxli/oxli.hh:82


def _is_str(o):
    return isinstance(o, str)


def _is_num(o):
    return isinstance(o, int) and not isinstance(o, bool)


def _u64_array(values):
    return (ctypes.c_uint64 * max(len(values), 1))(*values)


class Hashtable(object):
    """Base of every table class (khmer/_oxli/graphs.pyx:31-347)."""

    _storage = _lib.STORAGE_BYTE
    _hash_kind = _lib.HASH_TWOBIT

    def __init__(self, k, starting_size, n_tables, primes=None):
        self._g = None
        self._mirrors = None
        self._views = []
        if primes:
            sizes = [int(p) for p in primes]
        else:
            sizes = get_n_primes_near_x(int(n_tables), int(starting_size))
        h = ctypes.c_void_p()
        check(lib.kh_graph_create(self._storage, self._hash_kind, int(k), _u64_array(sizes),
                                  len(sizes), _lib.default_device(), ctypes.byref(h)))
        self._g = h
        self._k = int(k)

    @classmethod
    def _from_handle(cls, h):
        self = cls.__new__(cls)
        self._g = h
        self._mirrors = None
        self._views = []
        k = ctypes.c_int()
        check(lib.kh_graph_info(h, None, None, ctypes.byref(k), None))
        self._k = k.value
        return self

    def __del__(self):
        g = getattr(self, "_g", None)
        if g is not None:
            lib.kh_graph_destroy(g)
            self._g = None

    # ---- k-mer sanitising (graphs.pyx:33-83) ----
    def sanitize_seq_kmer(self, kmer):
        if len(kmer) != self.ksize():
            raise ValueError("Expected k-mer length {} but got {}.".format(self.ksize(), len(kmer)))
        return kmer.encode("latin-1") if isinstance(kmer, str) else bytes(kmer)

    def _kmer_type_error(self, kmer):
        raise TypeError("Object of type {0} can not be interpretted as  a k-mer".format(type(kmer)))

    def _valid_sequence(self, sequence):
        if len(sequence) < self.ksize():
            raise ValueError("sequence length ({}) must >= the hashtable k-mer size ({})".format(
                len(sequence), self.ksize()))
        return sequence.encode("latin-1")

    def _hash_bytes(self, b):
        out = ctypes.c_uint64()
        if self._hash_kind == _lib.HASH_MURMUR:
            check(lib.kh_hash_murmur(b, self._k, ctypes.byref(out), None))
        else:
            check(lib.kh_hash_twobit(b, self._k, None, None, ctypes.byref(out)))
        return out.value

    # Host mirrors behind get_raw_tables(): up to this many bytes they are
    # re-copied after every mutating call, so views handed out earlier track
    # the device tables like the reference's aliasing views
    # (graphs.pyx:333-347).  Larger tables are not re-copied per call (a
    # GB-sized copy per add() would cost seconds): the views handed out are
    # released instead, so reading one after a mutating call raises
    # ValueError rather than returning stale bytes; get_raw_tables() again
    # gives fresh ones.
    _MIRROR_EAGER_BYTES = 256 << 20

    def _refresh_mirrors(self, force=False):
        if not self._mirrors:
            return
        if not force and sum(len(b) for b in self._mirrors) > self._MIRROR_EAGER_BYTES:
            for v in self._views:
                try:
                    v.release()
                except BufferError:   # re-exported (e.g. numpy.frombuffer): leave it
                    pass
            self._views = []
            return
        for i, buf in enumerate(self._mirrors):
            ptr = (ctypes.c_char * len(buf)).from_buffer(buf)
            check(lib.kh_graph_copy_table(self._g, i, ptr))

    # ---- single k-mer operations (graphs.pyx:85-132) ----
    def count(self, kmer):
        """Increment the count of this k-mer (synonym for add)."""
        self.add(kmer)

    def add(self, kmer):
        """Increment the count of this k-mer; returns True if it was new."""
        if _is_str(kmer):
            h = self._hash_bytes(self.sanitize_seq_kmer(kmer))
        elif _is_num(kmer):
            h = int(kmer)
        else:
            self._kmer_type_error(kmer)
        arr = (ctypes.c_uint64 * 1)(h)
        isnew = (ctypes.c_uint8 * 1)()
        check(lib.kh_add_hashes(self._g, arr, 1, isnew))
        self._refresh_mirrors()
        return bool(isnew[0])

    def hash(self, kmer):
        """Compute the hash of this k-mer."""
        if _is_num(kmer):
            return kmer
        return self._hash_bytes(self.sanitize_seq_kmer(kmer))

    def reverse_hash(self, kmer_hash):
        """Turn a k-mer hash back into a DNA k-mer, if possible."""
        if self._hash_kind == _lib.HASH_MURMUR:
            raise ValueError("not implemented")
        buf = ctypes.create_string_buffer(self._k + 1)
        check(lib.kh_reverse_hash(int(kmer_hash), self._k, buf))
        return buf.value.decode()

    def get(self, kmer):
        """Retrieve the count for the given k-mer (string or hash)."""
        if _is_str(kmer):
            h = self._hash_bytes(self.sanitize_seq_kmer(kmer))
        elif _is_num(kmer):
            h = int(kmer)
        else:
            self._kmer_type_error(kmer)
        return self._get_counts([h])[0]

    def _get_counts(self, hashes):
        n = len(hashes)
        out = (ctypes.c_uint16 * max(n, 1))()
        if n:
            check(lib.kh_get_counts(self._g, _u64_array(hashes), n, out))
        return list(out[:n])

    # ---- table info ----
    def ksize(self):
        return self._k

    def hashsizes(self):
        n = self.n_tables()
        out = (ctypes.c_uint64 * n)()
        check(lib.kh_graph_tablesizes(self._g, out))
        return list(out)

    def n_tables(self):
        n = ctypes.c_int()
        check(lib.kh_graph_info(self._g, None, None, None, ctypes.byref(n)))
        return n.value

    def n_unique_kmers(self):
        """Estimate of the number of unique kmers stored."""
        out = ctypes.c_uint64()
        check(lib.kh_graph_n_unique_kmers(self._g, ctypes.byref(out)))
        return out.value

    def n_occupied(self):
        """Estimate of the number of occupied slots in the storage."""
        out = ctypes.c_uint64()
        check(lib.kh_graph_n_occupied(self._g, ctypes.byref(out)))
        return out.value

    def set_use_bigcount(self, bigcount):
        check(lib.kh_graph_set_use_bigcount(self._g, 1 if bigcount else 0))

    def get_use_bigcount(self):
        out = ctypes.c_int()
        check(lib.kh_graph_get_use_bigcount(self._g, ctypes.byref(out)))
        return bool(out.value)

    # ---- sequences (graphs.pyx:134-214) ----
    def get_kmers(self, sequence):
        """Generate an ordered list of all k-mers in sequence."""
        self._valid_sequence(sequence)
        k = self.ksize()
        return [sequence[i:i + k] for i in range(len(sequence) - k + 1)]

    def consume(self, sequence):
        """Increment the counts of all of the k-mers in the sequence."""
        data = self._valid_sequence(sequence)
        offs = (ctypes.c_uint64 * 2)(0, len(data))
        out = ctypes.c_uint64()
        check(lib.kh_consume_seqs(self._g, data, offs, 1, 0, ctypes.byref(out)))
        self._refresh_mirrors()
        return out.value

    def get_kmer_hashes(self, sequence):
        """Hashes of all k-mers in sequence, in order (hashed on the device,
        Hashtable::get_kmer_hashes, src/oxli/hashtable.cc:378-388)."""
        data = self._valid_sequence(sequence)
        out = (ctypes.c_uint64 * max(len(data), 1))()
        n = ctypes.c_uint64()
        offs = (ctypes.c_uint64 * 2)(0, len(data))
        check(lib.kh_graph_kmer_hashes(self._g, data, offs, 1, out, ctypes.byref(n)))
        return list(out[:n.value])

    def get_kmer_counts(self, sequence):
        """Retrieve an ordered list of the counts of all k-mers in sequence
        (hashed and counted on the device, src/oxli/hashtable.cc:403-413)."""
        data = self._valid_sequence(sequence)
        out = (ctypes.c_uint16 * max(len(data), 1))()
        n = ctypes.c_uint64()
        offs = (ctypes.c_uint64 * 2)(0, len(data))
        check(lib.kh_graph_kmer_counts(self._g, data, offs, 1, out, ctypes.byref(n)))
        return list(out[:n.value])

    def get_min_count(self, sequence):
        counts = self.get_kmer_counts(sequence)
        return min([255] + counts) if counts else 255

    def get_max_count(self, sequence):
        counts = self.get_kmer_counts(sequence)
        return max([0] + counts)

    def get_median_count(self, sequence):
        """median, average, and stddev of the k-mer counts in sequence."""
        data = self._valid_sequence(sequence)
        res = self.get_median_counts_batch([data])[0]
        if res is None:
            raise ValueError("no k-mer counts for this string; too short?")
        return res

    def get_median_counts_batch(self, sequences):
        """Batched get_median_count over many reads (one device pass).
        Returns a list of (median, average, stddev) or None for reads without
        a k-mer."""
        datas = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in sequences]
        n = len(datas)
        if not n:
            return []
        offs = [0]
        for d in datas:
            offs.append(offs[-1] + len(d))
        med = (ctypes.c_uint16 * n)()
        avg = (ctypes.c_float * n)()
        sd = (ctypes.c_float * n)()
        st = (ctypes.c_uint8 * n)()
        check(lib.kh_median_counts(self._g, b"".join(datas), _u64_array(offs), n, med, avg, sd, st))
        return [None if st[i] else (med[i], avg[i], sd[i]) for i in range(n)]

    def median_at_least(self, sequence, median):
        """Check if median k-mer count is at least the given value
        (Hashtable::median_at_least, src/oxli/hashtable.cc:333-364, on the
        device)."""
        self._valid_sequence(sequence)
        return self.median_at_least_batch([sequence], median)[0]

    def median_at_least_batch(self, sequences, median):
        """median_at_least over many reads in one device pass (the
        normalize-by-median filter over a batch).  `median` is converted as
        the reference's `unsigned int cutoff`.  Reads shorter than k give
        None (median_at_least raises ValueError for them)."""
        datas = [s.encode("latin-1") if isinstance(s, str) else bytes(s) for s in sequences]
        n = len(datas)
        if not n:
            return []
        offs = [0]
        for d in datas:
            offs.append(offs[-1] + len(d))
        out = (ctypes.c_uint8 * n)()
        st = (ctypes.c_uint8 * n)()
        check(lib.kh_median_at_least(self._g, b"".join(datas), _u64_array(offs), n, int(median) & 0xFFFFFFFF,
                                     out, st))
        return [None if st[i] else bool(out[i]) for i in range(n)]

    # ---- files of reads (graphs.pyx:216-296) ----
    def _get_parser(self, parser_or_filename):
        if isinstance(parser_or_filename, ReadParser):
            return parser_or_filename, None
        if _is_str(parser_or_filename):
            p = ReadParser(parser_or_filename)
            return p, p
        raise TypeError("argument does not appear to be a parser or a filename: {}".format(
            parser_or_filename))

    def _consume_parser(self, parser_or_filename, mode):
        parser, owned = self._get_parser(parser_or_filename)
        reads, kmers = ctypes.c_uint32(), ctypes.c_uint64()
        try:
            rc = lib.kh_consume_parser(self._g, parser.handle, mode, ctypes.byref(reads),
                                       ctypes.byref(kmers))
            self._refresh_mirrors()
            check(rc)
        finally:
            if owned is not None:
                owned.close()
        return reads.value, kmers.value

    def consume_seqfile(self, parser_or_filename):
        """Count all k-mers from file_name (or a shared ReadParser)."""
        return self._consume_parser(parser_or_filename, 0)

    def _consume_filtered(self, parser_or_filename, num_bands, band, mask, threshold, consume_masked):
        if mask is not None and not isinstance(mask, Hashtable):
            raise TypeError("mask must be a table")
        if num_bands == 0 and mask is None:
            return self.consume_seqfile(parser_or_filename)
        if num_bands < 0 or band < 0:
            raise OverflowError("can't convert negative value to unsigned int")
        parser, owned = self._get_parser(parser_or_filename)
        reads, kmers = ctypes.c_uint32(), ctypes.c_uint64()
        try:
            rc = lib.kh_consume_parser_filtered(
                self._g, parser.handle, int(num_bands), int(band),
                None if mask is None else mask._g, int(threshold) & 0xFFFFFFFF,
                1 if consume_masked else 0, ctypes.byref(reads), ctypes.byref(kmers))
            self._refresh_mirrors()
            check(rc)
        finally:
            if owned is not None:
                owned.close()
        return reads.value, kmers.value

    def consume_seqfile_with_mask(self, parser_or_filename, mask, threshold=0, consume_masked=False):
        """Count the k-mers whose count in `mask` is <= threshold (or >= with
        consume_masked) (graphs.pyx:241-252)."""
        if not isinstance(mask, Hashtable):
            raise TypeError("mask must be a table")
        return self._consume_filtered(parser_or_filename, 0, 0, mask, threshold, consume_masked)

    def consume_seqfile_banding(self, parser_or_filename, num_bands, band):
        """Count the k-mers whose hash falls in band `band` of `num_bands`
        (graphs.pyx:254-264)."""
        if int(num_bands) == 0:
            raise ValueError("num_bands must be > 0")
        return self._consume_filtered(parser_or_filename, num_bands, band, None, 0, False)

    def consume_seqfile_banding_with_mask(self, parser_or_filename, num_bands, band, mask, threshold=0,
                                          consume_masked=False):
        """Banding and mask together (graphs.pyx:266-280)."""
        if int(num_bands) == 0:
            raise ValueError("num_bands must be > 0")
        if not isinstance(mask, Hashtable):
            raise TypeError("mask must be a table")
        return self._consume_filtered(parser_or_filename, num_bands, band, mask, threshold, consume_masked)

    def abundance_distribution(self, parser_or_filename, tracking):
        """Calculate the k-mer abundance distribution over input reads."""
        if not isinstance(tracking, Hashtable):
            raise TypeError("tracking must be a table")
        parser, owned = self._get_parser(parser_or_filename)
        dist = (ctypes.c_uint64 * 65536)()
        try:
            check(lib.kh_abundance_distribution(self._g, parser.handle, tracking._g, dist))
        finally:
            if owned is not None:
                owned.close()
        tracking._refresh_mirrors()
        return list(dist[:MAX_BIGCOUNT])

    # ---- persistence (graphs.pyx:298-307) ----
    def save(self, file_name):
        """Save the graph to the specified file."""
        check(lib.kh_graph_save(self._g, str(file_name).encode()))

    @classmethod
    def load(cls, file_name):
        """Load the graph from the specified file."""
        h = ctypes.c_void_p()
        check(lib.kh_graph_load(str(file_name).encode(), cls._storage, cls._hash_kind,
                                _lib.default_device(), ctypes.byref(h)))
        return cls._from_handle(h)

    # ---- raw tables (graphs.pyx:333-347) ----
    def _raw_sizes(self):
        sizes = []
        for i in range(self.n_tables()):
            out = ctypes.c_uint64()
            check(lib.kh_graph_table_nbytes(self._g, i, ctypes.byref(out)))
            sizes.append(out.value)
        return sizes

    def get_raw_tables(self):
        """Read-only memoryviews of the tables.  The views are host mirrors.
        Up to 256 MiB of tables, every later mutating call on this object
        refreshes them, so they track the device tables like the reference's
        aliasing views (graphs.pyx:333-347).  Above that, a mutating call
        releases them (reading one raises ValueError); call get_raw_tables()
        again for current bytes."""
        if self._mirrors is None:
            self._mirrors = [bytearray(n) for n in self._raw_sizes()]
        self._refresh_mirrors(force=True)
        views = [memoryview(b).toreadonly() for b in self._mirrors]
        if sum(len(b) for b in self._mirrors) > self._MIRROR_EAGER_BYTES:
            self._views.extend(views)
        return views


class Hashgraph(Hashtable):
    """2-bit hashed graph classes with a tag set (khmer/_oxli/graphs.pyx:350-815)."""

    def consume_seqfile_and_tag(self, parser_or_filename):
        """Consume all sequences in a FASTA/FASTQ file and tag the graph."""
        return self._consume_parser(parser_or_filename, 1)

    def add_tag(self, kmer):
        h = kmer if _is_num(kmer) else self.hash(kmer)
        check(lib.kh_graph_add_tag(self._g, int(h)))

    def _tag_hashes(self):
        n = ctypes.c_uint64()
        check(lib.kh_graph_n_tags(self._g, ctypes.byref(n)))
        out = (ctypes.c_uint64 * max(n.value, 1))()
        check(lib.kh_graph_get_tags(self._g, out))
        return list(out[:n.value])

    def get_tagset(self):
        return [self.reverse_hash(t) for t in self._tag_hashes()]

    def tags(self):
        for t in self._tag_hashes():
            yield self.reverse_hash(t)

    @property
    def n_tags(self):
        n = ctypes.c_uint64()
        check(lib.kh_graph_n_tags(self._g, ctypes.byref(n)))
        return n.value

    def save_tagset(self, filename):
        check(lib.kh_graph_save_tagset(self._g, str(filename).encode()))

    def load_tagset(self, filename, clear_tags=True):
        check(lib.kh_graph_load_tagset(self._g, str(filename).encode(), 1 if clear_tags else 0))


class Countgraph(Hashgraph):
    """Count-Min sketch of 8-bit counters, 2-bit hashing (graphs.pyx:817-831)."""
    _storage = _lib.STORAGE_BYTE


class SmallCountgraph(Hashgraph):
    """Count-Min sketch of 4-bit counters, 2-bit hashing (graphs.pyx:858-879)."""
    _storage = _lib.STORAGE_NIBBLE


class Nodegraph(Hashgraph):
    """Bloom filter, 2-bit hashing (graphs.pyx:883-900)."""
    _storage = _lib.STORAGE_BIT


class Counttable(Hashtable):
    """Count-Min sketch of 8-bit counters, MurmurHash3 (hashtable.hh:591-596)."""
    _storage = _lib.STORAGE_BYTE
    _hash_kind = _lib.HASH_MURMUR


class SmallCounttable(Hashtable):
    """Count-Min sketch of 4-bit counters, MurmurHash3 (hashtable.hh:605-610)."""
    _storage = _lib.STORAGE_NIBBLE
    _hash_kind = _lib.HASH_MURMUR


class Nodetable(Hashtable):
    """Bloom filter, MurmurHash3 (hashtable.hh:620-625)."""
    _storage = _lib.STORAGE_BIT
    _hash_kind = _lib.HASH_MURMUR
