"""The record-driven apply (k_apply_sparse, khmer_amd/csrc/kh_apply.cuh) and
the per-bin apply (k_apply_count, KH_SPARSE_APPLY=0) against the oracle:
every table byte / nibble, n_unique_kmers, n_occupied and the bigcount map.

Reference semantics: ByteStorage::add / NibbleStorage::add
(include/oxli/storage.hh:571-624, 320-359) via Hashtable::consume_string
(src/oxli/hashtable.cc:280-294).  Sparse regions (here ~1-2K records over
2^14 bins, as C4 / C5's ~6-7K) take the record-driven kernel; the genomic
streams saturate bins (255 / 15), cross 255 inside a pass (bigcount
crossings) and hit bins already full before a pass; the uniform streams'
first passes run in complement mode (losers listed)."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x737061727365


def _bigcounts(g):
    from khmer_amd._lib import lib, check
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * max(n.value, 1))()
    vals = (ctypes.c_uint16 * max(n.value, 1))()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    return dict(zip(keys[:n.value], vals[:n.value]))


# (graph class, oracle kind, k, table size, reads, genome)
STREAMS = [("Countgraph", 1, 21, 2e6, 6000, 0), ("Countgraph", 1, 21, 2e6, 6000, 2000),
           ("SmallCountgraph", 7, 31, 4e6, 8000, 0), ("SmallCountgraph", 7, 31, 4e6, 8000, 1500)]


@pytest.fixture(scope="module", params=STREAMS, ids=["byte_uniform", "byte_genomic", "nibble_uniform",
                                                      "nibble_genomic"])
def stream(request):
    from khmer_amd._lib import lib, check, default_device
    from khmer_amd import synth
    from oracle import oracle as O
    import khmer_amd
    cls, kind, k, x, n, genome = request.param
    L = 150
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
    sizes = getattr(khmer_amd, cls)(k, x, 4).hashsizes()
    o = O.Table(kind, k, sizes)
    o.set_use_bigcount(kind == 1)
    o.consume_batch(seqs, [i * L for i in range(n + 1)])
    want = {"tables": [o.table_bytes(i) for i in range(4)], "n_unique": o.n_unique_kmers(),
            "n_occupied": o.n_occupied(), "bigcounts": o.bigcounts() if kind == 1 else {}}
    yield dict(cls=cls, kind=kind, words=words, n=n, L=L, k=k, x=x, want=want)
    lib.kh_device_free(dev, words)
    lib.kh_device_free(dev, koff)


@pytest.mark.parametrize("sparse", ["1", "0"], ids=["record_driven", "per_bin"])
def test_apply_matches_oracle(stream, sparse, monkeypatch):
    import khmer_amd
    from khmer_amd._lib import lib, check
    monkeypatch.setenv("KH_SPARSE_APPLY", sparse)
    g = getattr(khmer_amd, stream["cls"])(stream["k"], stream["x"], 4)
    if stream["kind"] == 1:
        g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, 200000))   # several device passes: bins full before a pass
    check(lib.kh_consume_packed_fixed_device(g._g, stream["words"], stream["n"], stream["L"]))
    want = stream["want"]
    tabs = g.get_raw_tables()
    for i in range(4):
        got = bytes(tabs[i])
        if got != want["tables"][i]:
            bad = next(j for j in range(len(got)) if got[j] != want["tables"][i][j])
            pytest.fail("table %d differs first at byte %d (%d vs oracle %d)" % (i, bad, got[bad],
                                                                                 want["tables"][i][bad]))
    assert g.n_unique_kmers() == want["n_unique"]
    assert g.n_occupied() == want["n_occupied"]
    if stream["kind"] == 1:
        assert _bigcounts(g) == want["bigcounts"]
