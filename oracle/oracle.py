"""ctypes wrapper over oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's k-mer counting path (see
oracle/khmer_oracle.c).  Imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, always as the checker, never as the product.
Parity is pinned by the reference's own known-answer tests
(tests/test_oracle_kats.py); the reference could not be executed here.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

BYTE, BIT, NIBBLE = 1, 2, 7
TWOBIT, MURMUR = 0, 1

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, u32, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        P = ctypes.c_void_p
        sig = {
            "or_hash2bit": (i32, [ctypes.c_char_p, i32, ctypes.POINTER(u64),
                                  ctypes.POINTER(u64), ctypes.POINTER(u64)]),
            "or_revhash": (None, [u64, i32, ctypes.c_char_p]),
            "or_revcomp": (None, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
            "or_hash_murmur": (u64, [ctypes.c_char_p, i32]),
            "or_hash_murmur_forward": (u64, [ctypes.c_char_p, i32]),
            "or_is_prime": (i32, [u64]),
            "or_get_n_primes_near_x": (i32, [u32, u64, ctypes.POINTER(u64)]),
            "or_table_new": (P, [i32, i32, i32, ctypes.POINTER(u64), i32]),
            "or_table_free": (None, [P]),
            "or_add": (i32, [P, u64]),
            "or_test_and_set": (i32, [P, u64]),
            "or_get": (i32, [P, u64]),
            "or_set_bigcount": (None, [P, i32]),
            "or_n_unique": (u64, [P]),
            "or_n_occupied": (u64, [P]),
            "or_table_nbytes": (u64, [P, i32]),
            "or_table_data": (ctypes.POINTER(ctypes.c_uint8), [P, i32]),
            "or_bigcount_size": (u64, [P]),
            "or_bigcount_export": (None, [P, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint16)]),
            "or_consume_string": (u32, [P, ctypes.c_char_p, ctypes.c_size_t]),
            "or_kmer_hashes": (u64, [P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(u64)]),
            "or_consume_fastx": (i32, [P, ctypes.c_char_p, i32, ctypes.POINTER(u32), ctypes.POINTER(u64)]),
            "or_consume_fastx_filtered": (i32, [P, ctypes.c_char_p, u32, u32, P, u32, i32,
                                                ctypes.POINTER(u32), ctypes.POINTER(u64)]),
            "or_consume_batch": (u64, [P, ctypes.c_char_p, ctypes.POINTER(u64), u64]),
            "or_consume_batch_mt": (u64, [P, ctypes.c_char_p, ctypes.POINTER(u64), u64, i32]),
            "or_median": (i32, [P, ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint16),
                                ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
            "or_abundance_distribution": (i32, [P, P, ctypes.c_char_p, ctypes.POINTER(u64)]),
            "or_n_tags": (u64, [P]),
            "or_tags_export": (None, [P, ctypes.POINTER(u64)]),
            "or_save": (i32, [P, ctypes.c_char_p]),
            "or_save_tagset": (i32, [P, ctypes.c_char_p]),
            "or_parser_open": (P, [ctypes.c_char_p]),
            "or_parser_next": (i32, [P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_size_t)]),
            "or_parser_num_reads": (u64, [P]),
            "or_parser_close": (None, [P]),
            "or_last_error": (ctypes.c_char_p, []),
            "or_synth_read": (None, [u64, u64, i32, ctypes.c_char_p]),
            "or_synth_genomic_read": (None, [u64, u64, u64, i32, ctypes.c_char_p]),
            "or_consume_synth": (u64, [P, u64, u64, u64, u64, i32]),
            "or_consume_synth_mt": (u64, [P, u64, u64, u64, u64, i32, i32]),
            "or_median_synth": (i32, [P, u64, u64, u64, u64, i32, P, P, P]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _b(s):
    return s.encode("latin-1") if isinstance(s, str) else s


def err():
    return lib().or_last_error().decode()


def forward_hash(kmer, k):
    out = ctypes.c_uint64()
    if lib().or_hash2bit(_b(kmer), k, None, None, ctypes.byref(out)) != 0:
        raise ValueError(err())
    return out.value


def forward_hash_no_rc(kmer, k):
    f = ctypes.c_uint64()
    if lib().or_hash2bit(_b(kmer), k, ctypes.byref(f), None, None) != 0:
        raise ValueError(err())
    return f.value


def reverse_hash(h, k):
    buf = ctypes.create_string_buffer(k + 1)
    lib().or_revhash(h, k, buf)
    return buf.value.decode()


def reverse_complement(s):
    buf = ctypes.create_string_buffer(len(s) + 1)
    lib().or_revcomp(_b(s), len(s), buf)
    return buf.raw[:len(s)].decode("latin-1")


def hash_murmur3(s):
    return lib().or_hash_murmur(_b(s), len(s))


def hash_no_rc_murmur3(s):
    return lib().or_hash_murmur_forward(_b(s), len(s))


def is_prime(n):
    return bool(lib().or_is_prime(n))


def get_n_primes_near_x(n, x):
    out = (ctypes.c_uint64 * max(n, 1))()
    got = lib().or_get_n_primes_near_x(n, int(x), out)
    if got != n:
        raise RuntimeError("unable to find %d prime numbers < %d" % (n, int(x)))
    return list(out[:n])


class Table:
    """Oracle table (Countgraph/Nodegraph/SmallCountgraph or *table family)."""

    def __init__(self, kind, k, sizes, hash=TWOBIT):
        arr = (ctypes.c_uint64 * len(sizes))(*sizes)
        self._h = lib().or_table_new(kind, hash, k, arr, len(sizes))
        if not self._h:
            raise MemoryError(err())
        self.kind, self.k, self.sizes, self.hashfn = kind, k, list(sizes), hash

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_table_free(self._h)
            self._h = None

    def set_use_bigcount(self, on):
        lib().or_set_bigcount(self._h, 1 if on else 0)

    def add(self, h):
        return lib().or_add(self._h, h)

    def test_and_set(self, h):
        return lib().or_test_and_set(self._h, h)

    def get(self, h):
        return lib().or_get(self._h, h)

    def hash(self, kmer):
        if self.hashfn == MURMUR:
            return hash_murmur3(kmer[:self.k])
        return forward_hash(kmer[:self.k], self.k)

    def consume(self, seq):
        return lib().or_consume_string(self._h, _b(seq), len(seq))

    def kmer_hashes(self, seq):
        out = (ctypes.c_uint64 * max(len(seq), 1))()
        n = lib().or_kmer_hashes(self._h, _b(seq), len(seq), out)
        return list(out[:n])

    def consume_fastx(self, path, tag=False):
        r, k = ctypes.c_uint32(), ctypes.c_uint64()
        rc = lib().or_consume_fastx(self._h, _b(path), 1 if tag else 0,
                                    ctypes.byref(r), ctypes.byref(k))
        if rc in (-1, -3):
            raise OSError(err())
        if rc < 0:
            raise ValueError(err())
        return r.value, k.value

    def consume_fastx_filtered(self, path, num_bands=0, band=0, mask=None, threshold=0, consume_masked=False):
        r, k = ctypes.c_uint32(), ctypes.c_uint64()
        rc = lib().or_consume_fastx_filtered(self._h, _b(path), num_bands, band,
                                             None if mask is None else mask._h, threshold & 0xFFFFFFFF,
                                             1 if consume_masked else 0, ctypes.byref(r), ctypes.byref(k))
        if rc in (-1, -3):
            raise OSError(err())
        if rc < 0:
            raise ValueError(err())
        return r.value, k.value

    def consume_batch(self, seqs, offs, threads=0):
        """seqs: bytes; offs: sequence of nreads+1 offsets."""
        arr = (ctypes.c_uint64 * len(offs))(*offs)
        if threads:
            return lib().or_consume_batch_mt(self._h, seqs, arr, len(offs) - 1, threads)
        return lib().or_consume_batch(self._h, seqs, arr, len(offs) - 1)

    def consume_synth(self, seed, r0, nreads, length, genome=0, threads=1):
        """Consume reads r0.. of the benchmark's synthetic stream (khmer_amd/synth.py),
        in stream order; genome > 0 selects the genomic stream.  threads > 1
        hashes on worker threads, the adds stay in stream order (same result)."""
        if threads > 1:
            return lib().or_consume_synth_mt(self._h, seed, genome, r0, nreads, length, threads)
        return lib().or_consume_synth(self._h, seed, genome, r0, nreads, length)

    def median_synth(self, seed, r0, nreads, length, genome=0):
        """get_median_count of reads r0.. of the synthetic stream: numpy
        (median u16, average f32, stddev f32) arrays."""
        import numpy as np
        med = np.zeros(nreads, np.uint16)
        avg = np.zeros(nreads, np.float32)
        sd = np.zeros(nreads, np.float32)
        if lib().or_median_synth(self._h, seed, genome, r0, nreads, length, med.ctypes.data, avg.ctypes.data,
                                 sd.ctypes.data) != 0:
            raise ValueError(err())
        return med, avg, sd

    def table_view(self, i):
        """Zero-copy read-only view of table i (for digests of GB tables)."""
        n = lib().or_table_nbytes(self._h, i)
        p = lib().or_table_data(self._h, i)
        return memoryview((ctypes.c_uint8 * n).from_address(ctypes.addressof(p.contents))).cast("B")

    def median(self, seq):
        m, a, s = ctypes.c_uint16(), ctypes.c_float(), ctypes.c_float()
        if lib().or_median(self._h, _b(seq), len(seq), ctypes.byref(m), ctypes.byref(a),
                           ctypes.byref(s)) != 0:
            raise ValueError(err())
        return m.value, a.value, s.value

    def abundance_distribution(self, path, tracking):
        dist = (ctypes.c_uint64 * 65536)()
        rc = lib().or_abundance_distribution(self._h, tracking._h, _b(path), dist)
        if rc in (-1, -3):
            raise OSError(err())
        if rc < 0:
            raise ValueError(err())
        return list(dist[:65535])

    def n_unique_kmers(self):
        return lib().or_n_unique(self._h)

    def n_occupied(self):
        return lib().or_n_occupied(self._h)

    def set_table_bytes(self, i, data):
        """Overwrite table i's bytes (the storage half of Hashtable::load,
        src/oxli/storage.cc:272-404; counters are left as they are)."""
        n = lib().or_table_nbytes(self._h, i)
        if len(data) != n:
            raise ValueError("table %d holds %d bytes, got %d" % (i, n, len(data)))
        p = lib().or_table_data(self._h, i)
        ctypes.memmove(ctypes.addressof(p.contents), bytes(data), n)

    def table_bytes(self, i):
        n = lib().or_table_nbytes(self._h, i)
        p = lib().or_table_data(self._h, i)
        return ctypes.string_at(p, n)

    def bigcounts(self):
        n = lib().or_bigcount_size(self._h)
        keys = (ctypes.c_uint64 * max(n, 1))()
        vals = (ctypes.c_uint16 * max(n, 1))()
        lib().or_bigcount_export(self._h, keys, vals)
        return dict(zip(keys[:n], vals[:n]))

    def tags(self):
        n = lib().or_n_tags(self._h)
        out = (ctypes.c_uint64 * max(n, 1))()
        lib().or_tags_export(self._h, out)
        return list(out[:n])

    def save(self, path):
        if lib().or_save(self._h, _b(path)) != 0:
            raise OSError(err())

    def save_tagset(self, path):
        if lib().or_save_tagset(self._h, _b(path)) != 0:
            raise OSError(err())


def synth_read(seed, r, length, genome=0):
    buf = ctypes.create_string_buffer(length + 1)
    if genome:
        lib().or_synth_genomic_read(seed, genome, r, length, buf)
    else:
        lib().or_synth_read(seed, r, length, buf)
    return buf.raw[:length]


def read_fastx(path):
    """Yield (name, sequence, quality) with the reference's record semantics."""
    L = lib()
    p = L.or_parser_open(_b(path))
    if not p:
        raise OSError(err())
    try:
        n, s, q = ctypes.c_char_p(), ctypes.c_char_p(), ctypes.c_char_p()
        sl, ql = ctypes.c_size_t(), ctypes.c_size_t()
        while True:
            rc = L.or_parser_next(p, ctypes.byref(n), ctypes.byref(s), ctypes.byref(q),
                                  ctypes.byref(sl), ctypes.byref(ql))
            if rc == 0:
                return
            if rc == -3:
                raise OSError(err())
            if rc < 0:
                raise ValueError(err())
            yield n.value.decode("latin-1"), s.value.decode("latin-1"), q.value.decode("latin-1")
    finally:
        L.or_parser_close(p)
