"""HIP path vs the oracle: bit-exact tables and counters (GPU).

Each case consumes the same input through khmer_amd (HIP kernels in
libkhmer_hip.so) and through the CPU restatement (oracle/), then compares every
table byte, n_occupied, n_unique_kmers and bigcounts.  Inputs: the reference's
own fixtures (tests/golden/data) and seeded synthetic reads.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import data

pytestmark = pytest.mark.gpu

khmer = pytest.importorskip("khmer_amd")
from khmer_amd import synth  # noqa: E402

KIND = {"Countgraph": O.BYTE, "SmallCountgraph": O.NIBBLE, "Nodegraph": O.BIT,
        "Counttable": O.BYTE, "SmallCounttable": O.NIBBLE, "Nodetable": O.BIT}
HASH = {"Countgraph": O.TWOBIT, "SmallCountgraph": O.TWOBIT, "Nodegraph": O.TWOBIT,
        "Counttable": O.MURMUR, "SmallCounttable": O.MURMUR, "Nodetable": O.MURMUR}


def make_pair(cls, k, sizes, bigcount=False):
    g = getattr(khmer, cls)(k, 1, 1, primes=sizes)
    o = O.Table(KIND[cls], k, sizes, hash=HASH[cls])
    if bigcount:
        g.set_use_bigcount(True)
        o.set_use_bigcount(True)
    return g, o


def assert_same(g, o, msg=""):
    tabs = g.get_raw_tables()
    for i in range(len(o.sizes)):
        a, b = bytes(tabs[i]), o.table_bytes(i)
        assert len(a) == len(b), msg
        if a != b:
            diff = np.nonzero(np.frombuffer(a, np.uint8) != np.frombuffer(b, np.uint8))[0]
            raise AssertionError("%s table %d differs at %d bytes (first %s)" % (msg, i, len(diff), diff[:8]))
    assert g.n_occupied() == o.n_occupied(), (msg, g.n_occupied(), o.n_occupied())
    assert g.n_unique_kmers() == o.n_unique_kmers(), (msg, g.n_unique_kmers(), o.n_unique_kmers())


FIXTURES = ["random-20-a.fa", "test-abund-read-2.fa", "valid-read-testing.fq", "25k.fq.gz",
            "random-31-c.fa", "all-A.fa"]


@pytest.mark.parametrize("cls", ["Countgraph", "SmallCountgraph", "Nodegraph"])
@pytest.mark.parametrize("fname", FIXTURES)
@pytest.mark.parametrize("k,x,n", [(12, 1e5, 4), (21, 1e7, 4), (20, 1e3, 2), (31, 123457, 3)])
def test_fixture_consume(cls, fname, k, x, n):
    sizes = O.get_n_primes_near_x(n, x)
    g, o = make_pair(cls, k, sizes, bigcount=(cls == "Countgraph"))
    got = g.consume_seqfile(data(fname))
    want = o.consume_fastx(data(fname))
    assert got == want
    assert_same(g, o, "%s %s k=%d" % (cls, fname, k))
    if cls == "Countgraph":
        assert g.n_unique_kmers() == o.n_unique_kmers()


@pytest.mark.parametrize("cls", ["Countgraph", "SmallCountgraph", "Nodegraph"])
@pytest.mark.parametrize("fname", ["100-reads.fq.bz2", "random-20-a.fq.bz2", "test-abund-read-2.fa.bz2"])
def test_bzip2_consume(tmp_path, cls, fname):
    """bzip2 input straight to the device; the oracle reads Python's
    bz2-decompressed copy."""
    import bz2
    plain = tmp_path / fname[:-4]
    plain.write_bytes(bz2.decompress(open(data(fname), "rb").read()))
    sizes = O.get_n_primes_near_x(4, 100003)
    g, o = make_pair(cls, 20, sizes, bigcount=(cls == "Countgraph"))
    assert g.consume_seqfile(data(fname)) == o.consume_fastx(str(plain))
    assert_same(g, o, "%s %s" % (cls, fname))


@pytest.mark.parametrize("fname", ["100-reads.fq.truncated.bz2", "100-reads.fq.truncated.gz"])
def test_truncated_compressed_consume_raises(fname):
    g = khmer.Countgraph(20, 1e5, 4)
    with pytest.raises(OSError):
        g.consume_seqfile(data(fname))


@pytest.mark.parametrize("cls", ["Counttable", "SmallCounttable", "Nodetable"])
@pytest.mark.parametrize("fname", ["random-20-a.fa", "test-abund-read-2.fa", "valid-read-testing.fq"])
@pytest.mark.parametrize("k", [4, 15, 51])
def test_murmur_consume(cls, fname, k):
    sizes = O.get_n_primes_near_x(3, 99991)
    g, o = make_pair(cls, k, sizes)
    assert g.consume_seqfile(data(fname)) == o.consume_fastx(data(fname))
    assert_same(g, o, "%s %s k=%d" % (cls, fname, k))


def test_multi_batch_equals_single(tmp_path):
    """Small device batches (many pipeline passes) give the single-stream result."""
    path = str(tmp_path / "syn.fq")
    synth.write_fastq(path, 3000, 150)
    sizes = O.get_n_primes_near_x(4, 200003)
    g, o = make_pair("Countgraph", 21, sizes, bigcount=True)
    from khmer_amd._lib import lib
    lib.kh_graph_set_batch_kmers(g._g, 4096)
    assert g.consume_seqfile(path) == o.consume_fastx(path)
    assert_same(g, o, "multi-batch")


@pytest.mark.parametrize("cls,k", [("Countgraph", 21), ("Nodegraph", 31), ("SmallCountgraph", 21)])
def test_synthetic_1m_reads(tmp_path, cls, k):
    """200k x 150 bp synthetic reads, tables sized so bins collide heavily."""
    seqs, offs = synth.batch(0, 200000, 150)
    sizes = O.get_n_primes_near_x(4, 4000037)
    g, o = make_pair(cls, k, sizes, bigcount=(cls == "Countgraph"))
    import ctypes
    from khmer_amd._lib import lib, check
    out = ctypes.c_uint64()
    arr = (ctypes.c_uint64 * len(offs))(*[int(v) for v in offs])
    check(lib.kh_consume_seqs(g._g, seqs, arr, len(offs) - 1, 1, ctypes.byref(out)))
    assert out.value == o.consume_batch(seqs, [int(v) for v in offs])
    assert_same(g, o, "synthetic %s" % cls)


def test_saturation_and_bigcount():
    """Bins crossing 255 inside one batch: exact stream-order bigcounts."""
    g, o = make_pair("Countgraph", 4, O.get_n_primes_near_x(4, 4 ** 4), bigcount=True)
    seqs = ["A" * 10000, "ACGT" * 700 + "TTTT" * 300, "G" * 4000, "CAGTTT" * 500]
    for s in seqs:
        assert g.consume(s) == o.consume(s)
    assert_same(g, o, "saturation")
    for kmer in ("AAAA", "ACGT", "TTTT", "GGGG", "CAGT", "AGTT"):
        assert g.get(kmer) == o.get(o.hash(kmer)), kmer


def test_saturation_many_kmers_one_batch(tmp_path):
    """Low-complexity reads: thousands of bins saturate in one device batch."""
    rng = np.random.default_rng(7)
    motifs = ["".join(rng.choice(list("ACGT"), 25)) for _ in range(40)]
    reads = [(motifs[i % 40] * 8)[: 150] for i in range(6000)]
    path = str(tmp_path / "lowc.fa")
    with open(path, "w") as fh:
        for i, r in enumerate(reads):
            fh.write(">%d\n%s\n" % (i, r))
    g, o = make_pair("Countgraph", 21, O.get_n_primes_near_x(3, 70001), bigcount=True)
    assert g.consume_seqfile(path) == o.consume_fastx(path)
    assert_same(g, o, "low complexity")
    f1, f2 = str(tmp_path / "g.ct"), str(tmp_path / "o.ct")
    g.save(f1)
    o.save(f2)
    assert open(f1, "rb").read() == open(f2, "rb").read()


def test_add_hash_is_new_sequence():
    """add() returns Storage::add's is_new in stream order (storage.hh:571-624)."""
    for cls in ("Countgraph", "Nodegraph", "SmallCountgraph"):
        g, o = make_pair(cls, 4, [11, 13])
        for s in ("AAAA", "ACTG", "AACG", "AGAC", "AAAA", "GTTT"):
            h = o.hash(s)
            assert g.add(h) == bool(o.add(h)), (cls, s)
        assert_same(g, o, cls)


def test_median_counts_bit_exact():
    g, o = make_pair("Countgraph", 12, O.get_n_primes_near_x(4, 1e5), bigcount=True)
    g.consume_seqfile(data("test-abund-read-2.fa"))
    o.consume_fastx(data("test-abund-read-2.fa"))
    seqs = [s for _, s, _ in O.read_fastx(data("random-20-a.fa"))]
    seqs += [s for _, s, _ in O.read_fastx(data("test-abund-read-2.fa"))][:200]
    got = g.get_median_counts_batch(seqs)
    for s, gm in zip(seqs, got):
        om = o.median(s)
        assert gm is not None
        assert gm[0] == om[0]
        assert np.float32(gm[1]).tobytes() == np.float32(om[1]).tobytes()
        assert np.float32(gm[2]).tobytes() == np.float32(om[2]).tobytes()


@pytest.mark.parametrize("x,expect", [(1e7, 3960), (1e5, 3959)])
def test_tagging_path(tmp_path, x, expect):
    sizes = O.get_n_primes_near_x(2, x)
    g, o = make_pair("Nodegraph", 20, sizes)
    got = g.consume_seqfile_and_tag(data("random-20-a.fa"))
    want = o.consume_fastx(data("random-20-a.fa"), tag=True)
    assert got == want
    assert g.n_unique_kmers() == expect
    assert_same(g, o, "tag")
    f1, f2 = str(tmp_path / "g.tagset"), str(tmp_path / "o.tagset")
    g.save_tagset(f1)
    o.save_tagset(f2)
    assert open(f1, "rb").read() == open(f2, "rb").read()


def test_abundance_distribution():
    sizes = [1000003, 1009837, 1000005]
    g = khmer.Countgraph(12, 1, 1, primes=sizes)
    g.consume_seqfile(data("random-20-a.fa"))
    tracking = khmer.Nodegraph(12, 1, 1, primes=sizes)
    dist = g.abundance_distribution(data("random-20-a.fa"), tracking)
    assert sum(dist) == 3966
    o = O.Table(O.BYTE, 12, sizes)
    o.consume_fastx(data("random-20-a.fa"))
    assert dist == o.abundance_distribution(data("random-20-a.fa"), O.Table(O.BIT, 12, sizes))


@pytest.mark.parametrize("batch", [(1024, 1024), (1024, 4096), (4096, 1024)])
def test_abundance_distribution_many_passes(batch):
    """Parser batches larger than the tracking table's device pass:
    is-new flags come from several in-order passes and must stay exact."""
    from khmer_amd._lib import lib, check
    sizes = [1000003, 1009837, 1000005]
    g = khmer.Countgraph(12, 1, 1, primes=sizes)
    g.consume_seqfile(data("random-20-a.fa"))
    tracking = khmer.Nodegraph(12, 1, 1, primes=sizes)
    check(lib.kh_graph_set_batch_kmers(g._g, batch[0]))
    check(lib.kh_graph_set_batch_kmers(tracking._g, batch[1]))
    dist = g.abundance_distribution(data("random-20-a.fa"), tracking)
    o = O.Table(O.BYTE, 12, sizes)
    o.consume_fastx(data("random-20-a.fa"))
    assert sum(dist) == 3966
    assert dist == o.abundance_distribution(data("random-20-a.fa"), O.Table(O.BIT, 12, sizes))


def test_add_hashes_is_new_many_passes():
    """kh_add_hashes with per-hash is_new over more hashes than one pass."""
    import ctypes
    import random
    from khmer_amd._lib import lib, check
    sizes = [10007, 10009]
    g = khmer.Countgraph(12, 1, 1, primes=sizes)
    check(lib.kh_graph_set_batch_kmers(g._g, 1024))
    rng = random.Random(7)
    hs = [rng.randrange(1 << 24) for _ in range(5000)]
    arr = (ctypes.c_uint64 * len(hs))(*hs)
    isnew = (ctypes.c_uint8 * len(hs))()
    check(lib.kh_add_hashes(g._g, arr, len(hs), isnew))
    o = O.Table(O.BYTE, 12, sizes)
    assert list(isnew) == [o.add(h) for h in hs]
    assert g.n_unique_kmers() == o.n_unique_kmers()


@pytest.mark.parametrize("cls", ["Countgraph", "SmallCountgraph", "Nodegraph"])
@pytest.mark.parametrize("suffix", ["", ".gz"])
def test_save_matches_oracle_and_loads(tmp_path, cls, suffix):
    sizes = O.get_n_primes_near_x(4, 1e5)
    g, o = make_pair(cls, 12, sizes, bigcount=(cls == "Countgraph"))
    g.consume_seqfile(data("random-20-a.fa"))
    o.consume_fastx(data("random-20-a.fa"))
    f1, f2 = str(tmp_path / ("g.ct" + suffix)), str(tmp_path / "o.ct")
    g.save(f1)
    o.save(f2)
    import gzip
    raw = gzip.open(f1).read() if (suffix and cls == "Countgraph") else open(f1, "rb").read()
    assert raw == open(f2, "rb").read()
    h = getattr(khmer, cls).load(f1)
    assert h.n_occupied() == o.n_occupied()
    for i, t in enumerate(h.get_raw_tables()):
        assert bytes(t) == o.table_bytes(i)


def test_device_synth_matches_host_synth():
    """kh_synth_packed_device generates exactly khmer_amd.synth's reads."""
    import ctypes
    from khmer_amd._lib import lib, check
    n, L, k = 5000, 150, 21
    sizes = O.get_n_primes_near_x(4, 1000003)
    g = khmer.Countgraph(k, 1, 1, primes=sizes)
    dev = khmer._lib.default_device()
    nwords = n * L // 32 + 2
    w, ko = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(dev, nwords * 8, ctypes.byref(w)))
    check(lib.kh_device_malloc(dev, (n + 1) * 8, ctypes.byref(ko)))
    check(lib.kh_synth_packed_device(dev, synth.SEED, 0, n, L, k, w, ko))
    check(lib.kh_consume_packed_device(g._g, w, ko, n, n * (L - k + 1)))
    lib.kh_device_free(dev, w)
    lib.kh_device_free(dev, ko)
    seqs, offs = synth.batch(0, n, L)
    o = O.Table(O.BYTE, k, sizes)
    o.consume_batch(seqs, [int(v) for v in offs])
    assert_same(g, o, "device synth")


@pytest.mark.parametrize("fixed", [True, False])
@pytest.mark.parametrize("batch", [1 << 20, 50000])
def test_device_packed_paths_batched(fixed, batch):
    """Fixed- and variable-length device paths, one and many device batches."""
    import ctypes
    from khmer_amd._lib import lib, check
    n, L, k = 20000, 150, 21
    sizes = O.get_n_primes_near_x(4, 1000003)
    g = khmer.Countgraph(k, 1, 1, primes=sizes)
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, batch))
    dev = khmer._lib.default_device()
    w, ko = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(dev, (n * L // 32 + 2) * 8, ctypes.byref(w)))
    check(lib.kh_device_malloc(dev, (n + 1) * 8, ctypes.byref(ko)))
    check(lib.kh_synth_packed_device(dev, synth.SEED, 0, n, L, k, w, ko))
    if fixed:
        check(lib.kh_consume_packed_fixed_device(g._g, w, n, L))
    else:
        check(lib.kh_consume_packed_device(g._g, w, ko, n, n * (L - k + 1)))
    lib.kh_device_free(dev, w)
    lib.kh_device_free(dev, ko)
    seqs, offs = synth.batch(0, n, L)
    o = O.Table(O.BYTE, k, sizes)
    o.set_use_bigcount(True)
    o.consume_batch(seqs, [int(v) for v in offs])
    assert_same(g, o, "device packed fixed=%s batch=%d" % (fixed, batch))


def test_variable_length_reads_multi_batch(tmp_path):
    """Ragged reads (1..300 bp) through several device batches."""
    rng = np.random.default_rng(11)
    path = str(tmp_path / "ragged.fa")
    with open(path, "w") as fh:
        for i in range(4000):
            L = int(rng.integers(1, 300))
            fh.write(">%d\n%s\n" % (i, "".join(rng.choice(list("ACGTN"), L))))
    for cls in ("Countgraph", "Nodegraph", "SmallCountgraph"):
        g, o = make_pair(cls, 25, O.get_n_primes_near_x(3, 300007), bigcount=(cls == "Countgraph"))
        from khmer_amd._lib import lib
        lib.kh_graph_set_batch_kmers(g._g, 20000)
        assert g.consume_seqfile(path) == o.consume_fastx(path)
        assert_same(g, o, "ragged " + cls)


@pytest.mark.parametrize("batch", [1 << 27, 100000, 50000])
@pytest.mark.parametrize("path", ["fixed", "variable"])
def test_multibatch_saturated_bigcount(path, batch):
    """Tables saturated over several device batches: bins entering a batch at
    254 - n .. 255 exercise the crossing rule exactly (an insert is full iff
    it sees 255; a bin reaching exactly 255 has no full insert)."""
    import ctypes
    from khmer_amd._lib import lib, check
    sizes = O.get_n_primes_near_x(4, 3001)
    R, L, k = 10000, 150, 21
    o = O.Table(O.BYTE, k, sizes)
    o.set_use_bigcount(True)
    seqs, offs = synth.batch(0, R, L)
    o.consume_batch(seqs, [int(v) for v in offs])
    g = khmer.Countgraph(k, 1, 1, primes=sizes)
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, batch))
    words, koff = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(0, (R * L // 32 + 2) * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(0, (R + 1) * 8, ctypes.byref(koff)))
    try:
        check(lib.kh_synth_packed_device(0, synth.SEED, 0, R, L, k, words, koff))
        if path == "fixed":
            check(lib.kh_consume_packed_fixed_device(g._g, words, R, L))
        else:
            check(lib.kh_consume_packed_device(g._g, words, koff, R, R * (L - k + 1)))
    finally:
        lib.kh_device_free(0, words)
        lib.kh_device_free(0, koff)
    assert_same(g, o, "saturated %s %d" % (path, batch))
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * n.value)()
    vals = (ctypes.c_uint16 * n.value)()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    assert dict(zip(keys, vals)) == o.bigcounts()
    assert len(o.bigcounts()) > 1000
    assert (g.n_unique_kmers(), g.n_occupied()) == (o.n_unique_kmers(), o.n_occupied())


@pytest.mark.parametrize("batch", [1 << 27, 1 << 19])
def test_bigcount_map_growth(batch):
    """Tiny tables saturate at once, so nearly every k-mer of 2.6M is a
    bigcount event with its own hash: the per-pass device map must grow past
    its initial 2^20 slots (and rerun its finalize) and stay exact."""
    import ctypes
    from khmer_amd._lib import lib, check
    sizes = [1009, 1013]
    g, o = make_pair("Countgraph", 21, sizes, bigcount=True)
    check(lib.kh_graph_set_batch_kmers(g._g, batch))
    seqs, offs = synth.batch(0, 20000, 150)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    out = ctypes.c_uint64()
    check(lib.kh_consume_seqs(g._g, seqs, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 20000, 1,
                              ctypes.byref(out)))
    assert out.value == o.consume_batch(seqs, [int(v) for v in offs])
    assert_same(g, o, "bigcount map growth")
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * n.value)()
    vals = (ctypes.c_uint16 * n.value)()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    want = o.bigcounts()
    assert len(want) > (1 << 20)
    assert dict(zip(keys, vals)) == want


@pytest.mark.parametrize("small", ["0", "2048", "100000"])
@pytest.mark.parametrize("cls", ["Countgraph", "SmallCountgraph", "Nodegraph"])
def test_small_pass_threshold(monkeypatch, cls, small):
    """The sequential small-pass kernel and the partition pipeline give the
    same exact results (KH_SMALL_PASS: passes up to that many k-mers go
    sequential; 0 disables it)."""
    monkeypatch.setenv("KH_SMALL_PASS", small)
    sizes = O.get_n_primes_near_x(4, 1e4)
    g, o = make_pair(cls, 12, sizes, bigcount=(cls == "Countgraph"))
    for fname in ("test-abund-read-2.fa", "random-20-a.fa"):
        assert g.consume_seqfile(data(fname)) == o.consume_fastx(data(fname))
    for s in ("A" * 400, "ACGT" * 120):
        assert g.consume(s) == o.consume(s)
    for h in (5, 5, 17, 99991):
        assert g.add(h) == bool(o.add(h))
    assert_same(g, o, "small pass %s" % small)
    if cls == "Countgraph":
        import ctypes
        from khmer_amd._lib import lib, check
        n = ctypes.c_uint64()
        check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
        keys = (ctypes.c_uint64 * max(n.value, 1))()
        vals = (ctypes.c_uint16 * max(n.value, 1))()
        check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
        assert dict(zip(keys[:n.value], vals[:n.value])) == o.bigcounts()


@pytest.mark.parametrize("cls", ["Countgraph", "SmallCountgraph"])
def test_tagging_sparse_complement(tmp_path, cls):
    """consume_seqfile_and_tag (src/oxli/hashgraph.cc:200-320) into sparse
    tables (3 x ~2e7 bins, passes of ~1e6 k-mers): most inserts are is_new
    winners, so the apply runs its complement mode (the coarse-window runs
    carry the losers and k_mark_wf counts them per k-mer), whose per-k-mer new
    flags place the tags.  Counters, tables, the tag set and the .tagset bytes
    equal the oracle's."""
    from khmer_amd import synth
    n, L = 24000, 100
    seqs, _ = synth.genomic_batch(0, n, L, 50_000_000)
    fa = str(tmp_path / "s.fa")
    with open(fa, "wb") as fh:
        for r in range(n):
            fh.write(b">r%d\n%s\n" % (r, seqs[r * L:(r + 1) * L]))
    sizes = O.get_n_primes_near_x(3, 20000003)
    g, o = make_pair(cls, 21, sizes)
    from khmer_amd._lib import lib, check
    check(lib.kh_graph_set_batch_kmers(g._g, 1000000))
    got = g.consume_seqfile_and_tag(fa)
    want = o.consume_fastx(fa, tag=True)
    assert got == want
    assert sorted(g._tag_hashes()) == sorted(o.tags())
    assert len(o.tags()) > 1000
    assert_same(g, o, "sparse tag")
    f1, f2 = str(tmp_path / "g.tagset"), str(tmp_path / "o.tagset")
    g.save_tagset(f1)
    o.save_tagset(f2)
    assert open(f1, "rb").read() == open(f2, "rb").read()


@pytest.mark.parametrize("cls,k,chunk", [("Nodegraph", 21, 0), ("Nodegraph", 31, 20000), ("Countgraph", 25, 7001)])
def test_tagging_genomic_multibatch(tmp_path, monkeypatch, cls, k, chunk):
    """consume_seqfile_and_tag (src/oxli/hashgraph.cc:200-320) on a skewed
    stream (reads of a 30 kbp genome: most k-mers are seen again, so the
    membership test of old k-mers decides where tags fall), in several device
    batches (tags carry from batch to batch) and, with KH_FEED_CHUNK, through
    the chunk-parallel feed: the returned count, the tag set and the
    .tagset bytes equal the oracle's."""
    from khmer_amd import synth
    if chunk:
        monkeypatch.setenv("KH_FEED_CHUNK", str(chunk))
    n, L = 6000, 120
    seqs, _ = synth.genomic_batch(0, n, L, 30000)
    fa = str(tmp_path / "g.fa")
    with open(fa, "wb") as fh:
        for r in range(n):
            fh.write(b">r%d\n%s\n" % (r, seqs[r * L:(r + 1) * L]))
    sizes = O.get_n_primes_near_x(3, 200003)
    g, o = make_pair(cls, k, sizes)
    from khmer_amd._lib import lib, check
    check(lib.kh_graph_set_batch_kmers(g._g, 50000))
    got = g.consume_seqfile_and_tag(fa)
    want = o.consume_fastx(fa, tag=True)
    assert got == want
    assert sorted(g._tag_hashes()) == sorted(o.tags())
    assert len(o.tags()) > 1000
    assert_same(g, o, "tag")
    f1, f2 = str(tmp_path / "g.tagset"), str(tmp_path / "o.tagset")
    g.save_tagset(f1)
    o.save_tagset(f2)
    assert open(f1, "rb").read() == open(f2, "rb").read()
