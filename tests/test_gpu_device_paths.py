"""Device-resident benchmark paths against the oracle: the ASCII unpack of the
synthetic stream, Murmur (Counttable family) consume of fixed-length device
reads, and get_median_count over device reads (one wave per read).

Reference semantics: MurmurKmerHashIterator / MurmurHashtable
(include/oxli/hashtable.hh:436-534, src/oxli/kmer_hash.cc:177-198) and
Hashtable::get_median_count (src/oxli/hashtable.cc:299-328; float32 average and
stddev bit-exact, median = sorted[n/2])."""
import ctypes
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6b686d6572


class _Dev(object):
    def __init__(self):
        from khmer_amd import _lib
        self.lib, self.dev, self.bufs = _lib.lib, _lib.default_device(), []

    def alloc(self, n):
        from khmer_amd._lib import check
        p = ctypes.c_void_p()
        check(self.lib.kh_device_malloc(self.dev, n, ctypes.byref(p)))
        self.bufs.append(p)
        return p

    def get(self, p, n):
        from khmer_amd._lib import check
        out = ctypes.create_string_buffer(n)
        check(self.lib.kh_device_copy(self.dev, out, p, n))
        return out.raw

    def free(self):
        for p in self.bufs:
            self.lib.kh_device_free(self.dev, p)
        self.bufs = []


def _reads(d, nreads, L, genome):
    from khmer_amd._lib import check
    words = d.alloc((nreads * L // 32 + 2) * 8)
    koff = d.alloc((nreads + 1) * 8)
    if genome:
        check(d.lib.kh_synth_genomic_device(d.dev, SEED, genome, 0, nreads, L, 21, words, koff))
    else:
        check(d.lib.kh_synth_packed_device(d.dev, SEED, 0, nreads, L, 21, words, koff))
    return words


def _host_reads(nreads, L, genome):
    from khmer_amd import synth
    if genome:
        return synth.genomic_batch(0, nreads, L, genome)[0]
    return synth.batch(0, nreads, L)[0]


@pytest.mark.parametrize("genome", [0, 5000])
def test_unpack_ascii(genome):
    from khmer_amd._lib import check
    d = _Dev()
    try:
        n, L = 777, 150
        words = _reads(d, n, L, genome)
        out = d.alloc(n * L + 64)
        check(d.lib.kh_unpack_ascii_device(d.dev, words, n * L, out))
        assert d.get(out, n * L) == _host_reads(n, L, genome)
    finally:
        d.free()


@pytest.mark.parametrize("k,x,genome", [(51, 1e5, 0), (51, 2e4, 3000), (23, 5e4, 3000)])
def test_murmur_fixed_device_consume(k, x, genome):
    import khmer_amd
    from khmer_amd._lib import check
    from oracle import oracle as O
    d = _Dev()
    try:
        n, L = 3000, 150
        words = _reads(d, n, L, genome)
        asc = d.alloc(n * L + 64)
        check(d.lib.kh_unpack_ascii_device(d.dev, words, n * L, asc))
        g = khmer_amd.SmallCounttable(k, x, 4)
        check(d.lib.kh_graph_set_batch_kmers(g._g, 50000))   # several device passes
        check(d.lib.kh_consume_bytes_fixed_device(g._g, asc, n, L))
        o = O.Table(O.NIBBLE, k, g.hashsizes(), O.MURMUR)
        seqs = _host_reads(n, L, genome)
        o.consume_batch(seqs, [i * L for i in range(n + 1)])
        tabs = g.get_raw_tables()
        for i in range(4):
            assert bytes(tabs[i]) == o.table_bytes(i)
        assert (g.n_unique_kmers(), g.n_occupied()) == (o.n_unique_kmers(), o.n_occupied())
    finally:
        d.free()


@pytest.mark.parametrize("cls,k,x,genome,bigcount", [
    ("SmallCountgraph", 31, 1e5, 0, False),
    ("SmallCountgraph", 31, 3e4, 4000, False),
    ("Countgraph", 21, 5e4, 1000, True),      # counts past 255: bigcount values
    ("Countgraph", 21, 5e4, 3000, False),
    ("Nodegraph", 25, 5e4, 3000, False),
    ("SmallCounttable", 51, 4e4, 3000, False),
])
def test_median_fixed_device(cls, k, x, genome, bigcount):
    import khmer_amd
    from khmer_amd._lib import check
    from oracle import oracle as O
    d = _Dev()
    try:
        n, L = 2500, 150
        words = _reads(d, n, L, genome)
        g = getattr(khmer_amd, cls)(k, x, 4)
        if bigcount:
            g.set_use_bigcount(True)
        murmur = cls == "SmallCounttable"
        src = words
        if murmur:
            src = d.alloc(n * L + 64)
            check(d.lib.kh_unpack_ascii_device(d.dev, words, n * L, src))
            check(d.lib.kh_consume_bytes_fixed_device(g._g, src, n, L))
        else:
            check(d.lib.kh_consume_packed_fixed_device(g._g, words, n, L))
        med, avg, sd = d.alloc(n * 2 + 64), d.alloc(n * 4 + 64), d.alloc(n * 4 + 64)
        check(d.lib.kh_median_counts_fixed_device(g._g, src, n, L, med, avg, sd))
        m = np.frombuffer(d.get(med, n * 2), dtype=np.uint16)
        a = np.frombuffer(d.get(avg, n * 4), dtype=np.uint32)
        s = np.frombuffer(d.get(sd, n * 4), dtype=np.uint32)
        kind = {"SmallCountgraph": O.NIBBLE, "Countgraph": O.BYTE, "Nodegraph": O.BIT,
                "SmallCounttable": O.NIBBLE}[cls]
        o = O.Table(kind, k, g.hashsizes(), O.MURMUR if murmur else O.TWOBIT)
        o.set_use_bigcount(bigcount)
        seqs = _host_reads(n, L, genome)
        o.consume_batch(seqs, [i * L for i in range(n + 1)])
        if bigcount:
            assert max(m) > 255, "the case should reach bigcount values"
        for r in range(n):
            em, ea, es = o.median(seqs[r * L:(r + 1) * L])
            assert int(m[r]) == em, r
            assert int(a[r]) == struct.unpack("<I", struct.pack("<f", ea))[0], r
            assert int(s[r]) == struct.unpack("<I", struct.pack("<f", es))[0], r
    finally:
        d.free()


def test_median_fixed_device_errors():
    import khmer_amd
    from khmer_amd._lib import check, lib
    d = _Dev()
    try:
        g = khmer_amd.Countgraph(21, 1e4, 2)
        buf = d.alloc(4096)
        with pytest.raises(ValueError):
            check(lib.kh_median_counts_fixed_device(g._g, buf, 1, 20, buf, buf, buf))   # read shorter than k
        with pytest.raises(ValueError):
            check(lib.kh_median_counts_fixed_device(g._g, buf, 1, 300, buf, buf, buf))  # > 256 k-mers per read
        with pytest.raises(ValueError):
            check(lib.kh_consume_bytes_fixed_device(g._g, buf, 1, 30))   # 2-bit graph
    finally:
        d.free()
