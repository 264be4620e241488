"""The near-prime partition (one level-1 record per k-mer; khmer_amd/csrc/
kh_nearprime.cuh) against the oracle: every table byte, n_unique_kmers,
n_occupied and the bigcount map, exactly.

Reference semantics: Hashtable::consume_string -> ByteStorage::add
(src/oxli/hashtable.cc:280-294, include/oxli/storage.hh:571-624), tables
sized by get_n_primes_near_x (include/oxli/hashtable.hh:99-123).  The path
is taken for 2-bit fixed-length reads into 2-4 tables whose sizes are close
primes: here k = 19 into 4 x ~1e8 bins (25 level-1 buckets, bins up to 9
regions past a bucket's range) and k = 21 at C2's own 4 x ~1e9 (255 buckets,
15 regions of spill), in several device passes.  KH_NP_JLIM shrinks the k-mer
index span a level-1 block may hold, so nearly every block is closed early
with sentinels; KH_NEAR_PRIME=0 runs the per-table level 1 on the same
stream, and the skewed genomic stream overflows the fixed capacities and
takes the fallback.  KH_NP_L1MAX caps the level-1 buckets, so these tables
take the three-level partition C4's 4 x 8e9 takes (k_scatter_n1b splits
each coarse bucket into up to 16 fine buckets, fine records j << 32 |
q << ob | offset)."""
import ctypes
import os

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6e70   # a stream of its own (synth.batch / genomic_batch take the same seed)


def _bigcounts(g):
    from khmer_amd._lib import lib, check
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * max(n.value, 1))()
    vals = (ctypes.c_uint16 * max(n.value, 1))()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    return dict(zip(keys[:n.value], vals[:n.value]))


def _stream(k, x, n, L, genome, tables):
    from khmer_amd._lib import lib, check, default_device
    from khmer_amd import synth
    from oracle import oracle as O
    import khmer_amd
    dev = default_device()
    words, koff = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(dev, (n * L // 32 + 2) * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(dev, (n + 1) * 8, ctypes.byref(koff)))
    if genome:
        check(lib.kh_synth_genomic_device(dev, SEED, genome, 0, n, L, k, words, koff))
        seqs = synth.genomic_batch(0, n, L, genome, seed=SEED)[0]
    else:
        check(lib.kh_synth_packed_device(dev, SEED, 0, n, L, k, words, koff))
        seqs = synth.batch(0, n, L, seed=SEED)[0]
    sizes = khmer_amd.Countgraph(k, x, tables).hashsizes()
    o = O.Table(O.BYTE, k, sizes)
    o.set_use_bigcount(True)
    o.consume_batch(seqs, [i * L for i in range(n + 1)])
    want = {"tables": [o.table_bytes(i) for i in range(tables)], "n_unique": o.n_unique_kmers(),
            "n_occupied": o.n_occupied(), "bigcounts": o.bigcounts()}
    return dict(words=words, koff=koff, dev=dev, n=n, L=L, k=k, x=x, tables=tables, want=want)


# (k, table size, reads, genome, tables, device batch): the fixed-capacity
# partition (and so this path) needs >= 512 records per region and pass
@pytest.fixture(scope="module", params=[(19, 1e8, 300000, 0, 4, 9000000), (19, 1e8, 200000, 5000, 4, 9000000),
                                        (19, 1e8, 200000, 0, 3, 9000000), (21, 1e9, 500000, 0, 4, 33000000)],
                ids=["k19_uniform", "k19_genomic", "k19_three_tables", "c2_geometry"])
def stream(request):
    k, x, n, genome, tables, batch = request.param
    s = _stream(k, x, n, 150, genome, tables)
    s["batch"] = batch
    yield s
    from khmer_amd._lib import lib
    lib.kh_device_free(s["dev"], s["words"])
    lib.kh_device_free(s["dev"], s["koff"])


def _kernels(g):
    from khmer_amd._lib import lib, check
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(g._g, buf, len(buf), ctypes.byref(n)))
    return {ln.split("\t")[0] for ln in buf.value.decode().splitlines() if ln}


@pytest.mark.parametrize("mode", ["near_prime", "closing_blocks", "per_table", "three_level"])
def test_nearprime_matches_oracle(stream, mode, monkeypatch):
    import khmer_amd
    from khmer_amd._lib import lib, check
    if mode == "closing_blocks":
        monkeypatch.setenv("KH_NP_JLIM", "8191")   # blocks span at most ~2 tiles
    if mode == "per_table":
        monkeypatch.setenv("KH_NEAR_PRIME", "0")
    if mode == "three_level":
        # k = 19, 1e8: 8 coarse buckets of 13 fine ones (63 regions each);
        # C2's geometry: 124 coarse buckets of 16 fine ones (31 regions each)
        monkeypatch.setenv("KH_NP_L1MAX", "8" if stream["k"] == 19 else "128")
    g = khmer_amd.Countgraph(stream["k"], stream["x"], stream["tables"])
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, stream["batch"]))   # several device passes
    check(lib.kh_graph_set_profiling(g._g, 1))
    check(lib.kh_consume_packed_fixed_device(g._g, stream["words"], stream["n"], stream["L"]))
    kernels = _kernels(g)
    genomic = stream["want"]["n_unique"] < stream["n"] * 10
    if mode == "per_table":
        assert "scatter_n1" not in kernels, kernels
    elif not genomic:
        # the near-prime path ran (the skewed genomic stream may overflow the
        # fixed capacities and fall back; its tables must still be exact)
        assert {"scatter_n1", "scatter_n2", "apply_byte"} <= kernels, kernels
        assert ("scatter_n1b" in kernels) == (mode == "three_level"), kernels
    want = stream["want"]
    tabs = g.get_raw_tables()
    for i in range(stream["tables"]):
        got = bytes(tabs[i])
        if got != want["tables"][i]:   # report without pytest's byte-wise diff of 1e8-byte strings
            bad = next(j for j in range(len(got)) if got[j] != want["tables"][i][j])
            pytest.fail("table %d differs first at bin %d (%d vs oracle %d)" % (i, bad, got[bad], want["tables"][i][bad]))
    assert g.n_unique_kmers() == want["n_unique"]
    assert g.n_occupied() == want["n_occupied"]
    assert _bigcounts(g) == want["bigcounts"]
