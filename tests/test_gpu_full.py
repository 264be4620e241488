"""Full-size parity: the HIP path at the production geometry against oracle
golden fixtures (tests/golden/full/*.json, made by
tests/golden/make_full_fixtures.py with the single-threaded oracle).

Covers what the small parity tests cannot reach: the
benchmark's own workload (C2: 50M x 150 bp reads, 4 x 1e9 bytes, three device
passes, exactly bench.py's call sequence including the per-step clear), the
C3 / C4 / C5 table geometries (level-1 fan-out > 1024 buckets, bin ids > 2^32,
32 GB of tables), SmallCounttable k=51 (MurmurHash3) and a skewed genomic
stream whose counts saturate (crossing bins, bigcounts at scale).  Every table
is compared by SHA-256 of its bytes; n_unique_kmers, n_occupied and the
bigcount map (count + digest) must match exactly.

The C5 / C5M configurations are also built through the benchmark's own device
paths (2-bit words for SmallCountgraph, device ASCII + the reverse-complement
stream for SmallCounttable) and queried with get_median_count over their
first million reads, against the oracle's digest of (median, average,
stddev) -- the query at bin ids > 2^32 (VERDICT r2 "Next round" #2).  The
uniform streams give median 1 everywhere; c5_genomic / c5m_genomic (genomic
streams at ~8x k-mer coverage) spread the medians over 1..15 with
saturation at 15, so a wrong count, a broken nibble cap or a wrong
average / stddev at bin ids > 2^32 changes the digest.
"""
import ctypes
import os

import numpy as np
import pytest

from tests import full_digest as FD

pytestmark = pytest.mark.gpu


def _graph(c):
    import khmer_amd
    cls = {(1, 0): khmer_amd.Countgraph, (2, 0): khmer_amd.Nodegraph, (7, 0): khmer_amd.SmallCountgraph,
           (1, 1): khmer_amd.Counttable, (7, 1): khmer_amd.SmallCounttable,
           (2, 1): khmer_amd.Nodetable}[(c["kind"], c["hash"])]
    g = cls(c["k"], c["x"], c["n"])
    if c["bigcount"]:
        g.set_use_bigcount(True)
    return g


def _consume_device(g, c, seed):
    from khmer_amd._lib import lib, check
    import khmer_amd._lib as L
    dev = L.default_device()
    words, koff = ctypes.c_void_p(), ctypes.c_void_p()
    nwords = c["reads"] * c["L"] // 32 + 2
    check(lib.kh_device_malloc(dev, nwords * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(dev, (c["reads"] + 1) * 8, ctypes.byref(koff)))
    try:
        if c["genome"]:
            check(lib.kh_synth_genomic_device(dev, seed, c["genome"], 0, c["reads"], c["L"], c["k"], words, koff))
        else:
            check(lib.kh_synth_packed_device(dev, seed, 0, c["reads"], c["L"], c["k"], words, koff))
        # bench.py's step: clear, then consume the whole stream; twice, so the
        # second step also checks that clear() resets tables and counters
        for _ in range(2):
            check(lib.kh_graph_clear(g._g))
            check(lib.kh_consume_packed_fixed_device(g._g, words, c["reads"], c["L"]))
        check(lib.kh_device_synchronize(dev))
    finally:
        lib.kh_device_free(dev, words)
        lib.kh_device_free(dev, koff)
    return c["reads"] * (c["L"] - c["k"] + 1)


def _consume_host(g, c, seed):
    """Murmur classes hash ASCII: feed host batches through kh_consume_seqs."""
    from khmer_amd import synth
    from khmer_amd._lib import lib, check
    total = 0
    step = 250_000
    for r0 in range(0, c["reads"], step):
        n = min(step, c["reads"] - r0)
        if c["genome"]:
            seqs, offs = synth.genomic_batch(r0, n, c["L"], c["genome"], seed)
        else:
            seqs, offs = synth.batch(r0, n, c["L"], seed)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        out = ctypes.c_uint64()
        check(lib.kh_consume_seqs(g._g, seqs, offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n, 1,
                                  ctypes.byref(out)))
        total += out.value
    return total


def _table_digests(g):
    from khmer_amd._lib import lib, check
    out = []
    for i, n in enumerate(g._raw_sizes()):
        buf = bytearray(n)
        check(lib.kh_graph_copy_table(g._g, i, (ctypes.c_char * n).from_buffer(buf)))
        out.append(FD.sha256_view(memoryview(buf)))
        del buf
    return out


def _bigcounts(g):
    from khmer_amd._lib import lib, check
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    cap = n.value
    keys = (ctypes.c_uint64 * max(cap, 1))()
    vals = (ctypes.c_uint16 * max(cap, 1))()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, cap, ctypes.byref(n)))
    return dict(zip(keys[:n.value], vals[:n.value]))


# the stream-order (single-device) configurations of the suite: the
# group-order ones (exchange / delta interleaves) are the sharded tests', the
# weak-scaling read sets (c2_w*) exist only in group order, and the
# secondary bench lines' workload-size fixtures (c3_50m, c5_50m, c5m_50m,
# c5m_500m, genomic_c2_50m) are checked by those bench lines themselves
# (tools/bench_modes.sh), not here.  A missing fixture is a skip, not a
# silently dropped case.
FULL_SUITE = ["c2_full", "c3_shape", "c4_400k", "c4_50m", "c4_shape", "c5_genomic", "c5_shape", "c5m_genomic",
              "c5m_shape", "genomic_c2"]


@pytest.mark.parametrize("name", FULL_SUITE)
def test_full_geometry(name):
    from khmer_amd._lib import lib, check
    if not os.path.exists(FD.fixture_path(name)):
        pytest.skip("no fixture %s (tests/golden/make_full_fixtures.py %s)" % (name, name))
    fx = FD.load(name)
    c = fx["params"]
    g = _graph(c)
    assert g.hashsizes() == fx["table_sizes"]
    check(lib.kh_graph_set_batch_kmers(g._g, c["batch_kmers"]))
    if c["hash"] == 1:
        consumed = _consume_host(g, c, fx["seed"])
    else:
        consumed = _consume_device(g, c, fx["seed"])
    assert consumed == fx["n_consumed"]
    assert g.n_occupied() == fx["n_occupied"]
    assert g.n_unique_kmers() == fx["n_unique_kmers"]
    bc = _bigcounts(g)
    assert FD.bigcount_digest(bc) == (fx["n_bigcounts"], fx["bigcount_sha256"])
    assert _table_digests(g) == fx["table_sha256"]


def _device_reads(c, seed, ascii_too):
    """The stream's reads in device memory: packed words (and ASCII bytes)."""
    from khmer_amd._lib import lib, check
    import khmer_amd._lib as L
    dev = L.default_device()
    words, koff, asc = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    nwords = c["reads"] * c["L"] // 32 + 2
    check(lib.kh_device_malloc(dev, nwords * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(dev, (c["reads"] + 1) * 8, ctypes.byref(koff)))
    if c["genome"]:
        check(lib.kh_synth_genomic_device(dev, seed, c["genome"], 0, c["reads"], c["L"], min(c["k"], 32), words,
                                          koff))
    else:
        check(lib.kh_synth_packed_device(dev, seed, 0, c["reads"], c["L"], min(c["k"], 32), words, koff))
    if ascii_too:
        check(lib.kh_device_malloc(dev, c["reads"] * c["L"] + 64, ctypes.byref(asc)))
        check(lib.kh_unpack_ascii_device(dev, words, c["reads"] * c["L"], asc))
    return dev, words, koff, asc


# the query fixtures of the suite (c5_50m / c5m_50m: the bench's C5 / C5M
# --query lines check their own digests)
MEDIAN_SUITE = ["c5_genomic", "c5_shape", "c5m_genomic", "c5m_shape"]


@pytest.mark.parametrize("name", MEDIAN_SUITE)
def test_full_device_path_and_median(name):
    from khmer_amd._lib import lib, check
    if not os.path.exists(FD.fixture_path(name)):
        pytest.skip("no fixture %s" % name)
    fx = FD.load(name)
    c = fx["params"]
    assert fx.get("median_reads") == FD.MEDIAN_READS[name]
    g = _graph(c)
    check(lib.kh_graph_set_batch_kmers(g._g, c["batch_kmers"]))
    murmur = c["hash"] == 1
    dev, words, koff, asc = _device_reads(c, fx["seed"], murmur)
    med = ctypes.c_void_p()
    nq = fx["median_reads"]
    try:
        # the bench's consume call (kh_consume_bytes_fixed_device for the
        # Murmur class, kh_consume_packed_fixed_device otherwise)
        if murmur:
            check(lib.kh_consume_bytes_fixed_device(g._g, asc, c["reads"], c["L"]))
        else:
            check(lib.kh_consume_packed_fixed_device(g._g, words, c["reads"], c["L"]))
        check(lib.kh_device_synchronize(dev))
        assert g.n_occupied() == fx["n_occupied"]
        assert g.n_unique_kmers() == fx["n_unique_kmers"]
        assert _table_digests(g) == fx["table_sha256"]
        # the bench's query call over the first nq reads
        check(lib.kh_device_malloc(dev, nq * 10 + 64, ctypes.byref(med)))
        avg = ctypes.c_void_p(med.value + nq * 2)
        sd = ctypes.c_void_p(med.value + nq * 6)
        check(lib.kh_median_counts_fixed_device(g._g, asc if murmur else words, nq, c["L"], med, avg, sd))
        out = (ctypes.c_uint8 * (nq * 10))()
        check(lib.kh_device_copy(dev, out, med, nq * 10))
        raw = bytes(out)
        m = np.frombuffer(raw[:2 * nq], np.uint16)
        a = np.frombuffer(raw[2 * nq:6 * nq], np.float32)
        s = np.frombuffer(raw[6 * nq:], np.float32)
        assert int(m.max()) == fx["median_max"]
        if "median_hist" in fx:   # the genomic streams: medians spread over 1..15 and saturate
            assert np.bincount(m.astype(np.int64), minlength=16)[:16].tolist() == fx["median_hist"]
        assert FD.median_digest(m, a, s) == fx["median_sha256"]
    finally:
        for p in (words, koff, asc, med):
            if p.value:
                lib.kh_device_free(dev, p)
