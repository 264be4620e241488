"""Robustness of the device path (GPU): skewed input that overflows the
fixed-capacity partition, caller buffers without padding, the concurrent
consume_seqfile contract, and lock ordering between two tables.  Every case
is checked against the oracle (tables, counters, bigcounts)."""
import ctypes
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import data

pytestmark = pytest.mark.gpu

khmer = pytest.importorskip("khmer_amd")
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402
from tests.test_gpu_parity import assert_same  # noqa: E402


def _stats(g):
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(g._g, buf, len(buf), ctypes.byref(n)))
    return {line.split("\t")[0] for line in buf.value.decode().splitlines()}


def _write_skewed_fasta(path, n_random, n_n, L=150):
    """n_random uniform reads interleaved with n_n all-'N' reads (cleaned to
    poly-A: one k-mer repeated (L - k + 1) times per read)."""
    rows = synth.read_ascii(0, n_random, L)
    every = max(1, n_random // max(1, n_n))
    with open(path, "w") as fh:
        k = 0
        for i in range(n_random):
            fh.write(">r%d\n%s\n" % (i, rows[i].tobytes().decode()))
            if k < n_n and i % every == 0:
                fh.write(">n%d\n%s\n" % (k, "N" * L))
                k += 1
        while k < n_n:
            fh.write(">n%d\n%s\n" % (k, "N" * L))
            k += 1


@pytest.mark.parametrize("n_n,level", [(770, "region"), (20000, "bucket")])
def test_skewed_pass_overflow_matches_oracle(tmp_path, n_n, level):
    """Poly-A runs concentrate 1e5 (one level-2 region overflows) or 2.6e6
    (its level-1 bucket overflows too) records in one bin per table: the pass
    is redone on the exact path and must still equal the oracle, bigcounts
    included (level 2 must not read an overflowed bucket)."""
    path = str(tmp_path / "skew.fa")
    _write_skewed_fasta(path, 20000, n_n)
    sizes = O.get_n_primes_near_x(4, 1e7)
    g = khmer.Countgraph(21, 1, 1, primes=sizes)
    g.set_use_bigcount(True)
    o = O.Table(O.BYTE, 21, sizes)
    o.set_use_bigcount(True)
    check(lib.kh_graph_set_profiling(g._g, 1))
    assert g.consume_seqfile(path) == o.consume_fastx(path)
    names = _stats(g)
    assert "hist_l2" in names, names   # the exact level 2 ran (an overflow was detected)
    if level == "bucket":
        assert "hist_l1" in names, names
    assert_same(g, o, level)
    assert sorted(o.bigcounts().items()) == sorted(
        (k, v) for k, v in zip(*_bigcounts(g)))
    # the next consume starts on the exact path (cool-down) and stays exact
    assert g.consume_seqfile(path) == o.consume_fastx(path)
    assert_same(g, o, level + " again")


def _bigcounts(g):
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * max(n.value, 1))()
    vals = (ctypes.c_uint16 * max(n.value, 1))()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    return list(keys[:n.value]), list(vals[:n.value])


def test_ascii_device_reads_without_padding():
    """kh_consume_bytes_fixed_device / kh_median_counts_fixed_device on a
    buffer that ends exactly at the last read (the word-window hashing reads
    past it): the library pads a copy; tables and medians equal the oracle."""
    L, n, k = 150, 3000, 51
    rows = synth.read_ascii(0, n, L)
    host = np.ascontiguousarray(rows).tobytes()
    assert len(host) == n * L
    sizes = O.get_n_primes_near_x(4, 100003)
    g = khmer.SmallCounttable(k, 1, 1, primes=sizes)
    o = O.Table(O.NIBBLE, k, sizes, hash=O.MURMUR)
    d = ctypes.c_void_p()
    check(lib.kh_device_malloc(0, n * L, ctypes.byref(d)))
    try:
        check(lib.kh_device_copy(0, d, host, n * L))
        check(lib.kh_consume_bytes_fixed_device(g._g, d, n, L))
        for r in range(n):
            o.consume(host[r * L:(r + 1) * L])
        assert_same(g, o, "bytes")
        med = ctypes.c_void_p()
        check(lib.kh_device_malloc(0, n * 10 + 64, ctypes.byref(med)))
        try:
            avg = ctypes.c_void_p(med.value + n * 2)
            sd = ctypes.c_void_p(med.value + n * 6)
            check(lib.kh_median_counts_fixed_device(g._g, d, n, L, med, avg, sd))
            out = (ctypes.c_uint8 * (n * 10))()
            check(lib.kh_device_copy(0, out, med, n * 10))
            raw = bytes(out)
            m = np.frombuffer(raw[:2 * n], np.uint16)
            a = np.frombuffer(raw[2 * n:6 * n], np.float32)
            s = np.frombuffer(raw[6 * n:], np.float32)
            for r in range(0, n, 97):
                wm, wa, ws = o.median(host[r * L:(r + 1) * L])
                assert (int(m[r]), a[r], s[r]) == (wm, np.float32(wa), np.float32(ws))
        finally:
            lib.kh_device_free(0, med)
    finally:
        lib.kh_device_free(0, d)


def _threaded_consume(g, parser, nthreads, tag=False):
    shares, errs = [], []
    eat = g.consume_seqfile_and_tag if tag else g.consume_seqfile

    def run():
        try:
            shares.append(eat(parser))
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    ts = [threading.Thread(target=run) for _ in range(nthreads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ts)
    assert not errs, errs
    return shares


@pytest.mark.parametrize("fname", ["25k.fq.gz", "random-20-a.fq", "test-abund-read-2.fa"])
def test_concurrent_consume_seqfile_on_one_parser(fname):
    """scripts/load-into-counting.py:143-158: T threads call
    consume_seqfile(rparser) on one table and one parser.  Every read is
    consumed once: the shares sum to the oracle's (reads, k-mers), the tables
    and counters equal the single-threaded oracle's, and the parser reports
    every read."""
    sizes = O.get_n_primes_near_x(4, 1e6)
    g = khmer.Countgraph(21, 1, 1, primes=sizes)
    g.set_use_bigcount(True)
    o = O.Table(O.BYTE, 21, sizes)
    o.set_use_bigcount(True)
    rp = khmer.ReadParser(data(fname))
    shares = _threaded_consume(g, rp, 4)
    want = o.consume_fastx(data(fname))
    assert len(shares) == 4
    assert (sum(s[0] for s in shares), sum(s[1] for s in shares)) == want
    assert rp.num_reads == want[0]
    assert_same(g, o, fname)


def test_concurrent_consume_and_tag_on_one_parser():
    """oxli/functions.py:56-66 with -T 4 (load-graph.py): the tagged graph
    equals the single-threaded oracle (3960 unique k-mers, tests/test_scripts.py:521-552)."""
    sizes = O.get_n_primes_near_x(2, 1e7)
    g = khmer.Nodegraph(20, 1, 1, primes=sizes)
    o = O.Table(O.BIT, 20, sizes)
    rp = khmer.ReadParser(data("random-20-a.fa"))
    shares = _threaded_consume(g, rp, 4, tag=True)
    want = o.consume_fastx(data("random-20-a.fa"), tag=True)
    assert (sum(s[0] for s in shares), sum(s[1] for s in shares)) == want
    assert g.n_unique_kmers() == o.n_unique_kmers() == 3960
    assert sorted(g._tag_hashes()) == sorted(o.tags())


def test_load_into_counting_threads_flag(tmp_path):
    """load-into-counting.py -T 4 gives the same table file as -T 1."""
    from khmer_amd import scripts
    outs = []
    for t in (1, 4):
        out = str(tmp_path / ("t%d.ct" % t))
        assert scripts.load_into_counting(["-x", "1e5", "-N", "2", "-k", "20", "-T", str(t), "-q", out,
                                           data("test-abund-read-2.fa")]) == 0
        with open(out, "rb") as fh:
            outs.append(fh.read())
    assert outs[0] == outs[1]


def test_abundance_distribution_opposite_lock_order():
    """Two threads: a.abundance_distribution(f, b) and
    b.abundance_distribution(f, a) at the same time must both finish (the
    two table locks are taken together, not one after the other)."""
    sizes = O.get_n_primes_near_x(2, 1e5)
    a = khmer.Countgraph(20, 1, 1, primes=sizes)
    b = khmer.Countgraph(20, 1, 1, primes=sizes)
    a.consume_seqfile(data("test-abund-read-2.fa"))
    b.consume_seqfile(data("test-abund-read-2.fa"))
    done = []

    def run(x, y):
        for _ in range(15):
            x.abundance_distribution(data("random-20-a.fa"), y)
        done.append(1)

    ts = [threading.Thread(target=run, args=(a, b)), threading.Thread(target=run, args=(b, a))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert len(done) == 2


def test_large_raw_table_views_are_released(monkeypatch):
    """Above the eager-refresh size, views handed out by get_raw_tables()
    raise after a mutating call instead of returning stale bytes; a new
    get_raw_tables() sees the update."""
    g = khmer.Countgraph(20, 1e5, 2)
    monkeypatch.setattr(g, "_MIRROR_EAGER_BYTES", 1000)
    views = g.get_raw_tables()
    assert sum(bytes(views[0])) == 0
    g.consume("ACGTACGTACGTACGTACGTA")
    with pytest.raises(ValueError):
        bytes(views[0])
    assert sum(bytes(g.get_raw_tables()[0])) == 2
