"""Work distribution does not change results: the fixed-capacity level 1 with
one fixed share per workgroup or with dynamically scheduled chunks of 1, 2 or
32 tiles, and apply with a fixed region stride or the region queue
(kh_graph_set_schedule), all give the oracle's tables, n_unique_kmers,
n_occupied and bigcount map.

Reference semantics: Hashtable::consume_string -> ByteStorage::add
(src/oxli/hashtable.cc:280-294, include/oxli/storage.hh:571-624).  The input
is the bench's device path (kh_consume_packed_fixed_device) over the seeded
synthetic stream, in several device passes so that the chunk queue runs with
more chunks than workgroups, ragged last chunks and more than one launch."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x6b686d6572
SCHEDULES = [(0, 0), (1, 1), (2, 0), (3, 1), (32, 1)]


def _bigcounts(g):
    from khmer_amd._lib import lib, check
    n = ctypes.c_uint64()
    check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
    keys = (ctypes.c_uint64 * max(n.value, 1))()
    vals = (ctypes.c_uint16 * max(n.value, 1))()
    check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
    return dict(zip(keys[:n.value], vals[:n.value]))


@pytest.fixture(scope="module", params=[0, 2000], ids=["uniform", "genomic"])
def stream(request):
    """Device reads plus the oracle's results for them (one oracle run per stream)."""
    from khmer_amd._lib import lib, check, default_device
    from khmer_amd import synth
    from oracle import oracle as O
    import khmer_amd
    # 4 x 2e6 bins: ~490 apply regions, more than the apply grid, so the
    # region queue hands out several regions per workgroup
    genome, n, L, k, x = request.param, 6000, 150, 21, 2e6
    dev = default_device()
    words = ctypes.c_void_p()
    koff = ctypes.c_void_p()
    check(lib.kh_device_malloc(dev, (n * L // 32 + 2) * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(dev, (n + 1) * 8, ctypes.byref(koff)))
    if genome:
        check(lib.kh_synth_genomic_device(dev, SEED, genome, 0, n, L, k, words, koff))
        seqs = synth.genomic_batch(0, n, L, genome)[0]
    else:
        check(lib.kh_synth_packed_device(dev, SEED, 0, n, L, k, words, koff))
        seqs = synth.batch(0, n, L)[0]
    sizes = khmer_amd.Countgraph(k, x, 4).hashsizes()
    o = O.Table(O.BYTE, k, sizes)
    o.set_use_bigcount(True)
    o.consume_batch(seqs, [i * L for i in range(n + 1)])
    want = {
        "tables": [o.table_bytes(i) for i in range(4)],
        "n_unique": o.n_unique_kmers(),
        "n_occupied": o.n_occupied(),
        "bigcounts": o.bigcounts(),
    }
    yield dict(words=words, n=n, L=L, k=k, x=x, want=want)
    lib.kh_device_free(dev, words)
    lib.kh_device_free(dev, koff)


@pytest.mark.parametrize("l1_chunk,apply_dyn", SCHEDULES)
def test_schedule_matches_oracle(stream, l1_chunk, apply_dyn):
    import khmer_amd
    from khmer_amd._lib import lib, check
    g = khmer_amd.Countgraph(stream["k"], stream["x"], 4)
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_schedule(g._g, l1_chunk, apply_dyn))
    check(lib.kh_graph_set_batch_kmers(g._g, 150000))   # six device passes
    check(lib.kh_graph_set_profiling(g._g, 1))
    check(lib.kh_consume_packed_fixed_device(g._g, stream["words"], stream["n"], stream["L"]))
    # the fixed-capacity level 1 and level 2 ran (no histogram pass): the
    # schedule under test was the one used
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(g._g, buf, len(buf), ctypes.byref(n)))
    kernels = {ln.split("\t")[0] for ln in buf.value.decode().splitlines() if ln}
    assert {"scatter_l1", "scatter_l2", "apply_byte"} <= kernels and not kernels & {"hist_l1", "hist_l2"}, kernels
    want = stream["want"]
    tabs = g.get_raw_tables()
    for i in range(4):
        assert bytes(tabs[i]) == want["tables"][i], "table %d" % i
    assert g.n_unique_kmers() == want["n_unique"]
    assert g.n_occupied() == want["n_occupied"]
    assert _bigcounts(g) == want["bigcounts"]


def test_schedule_setter_checks_pointer():
    from khmer_amd._lib import lib
    assert lib.kh_graph_set_schedule(None, 1, 1) != 0
