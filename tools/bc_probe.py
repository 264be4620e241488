"""Development probe: bigcounts of the fixed-length device path vs the oracle
on a saturated workload, for several batch sizes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402
from oracle import oracle as O  # noqa: E402

sizes = O.get_n_primes_near_x(4, 3001)
R, L, k = int(sys.argv[1]) if len(sys.argv) > 1 else 10000, 150, 21
o = O.Table(O.BYTE, k, sizes)
o.set_use_bigcount(True)
seqs, offs = synth.batch(0, R, L)
o.consume_batch(seqs, [int(v) for v in offs])
ref = o.bigcounts()
words, koff = ctypes.c_void_p(), ctypes.c_void_p()
check(lib.kh_device_malloc(0, (R * L // 32 + 2) * 8, ctypes.byref(words)))
check(lib.kh_device_malloc(0, (R + 1) * 8, ctypes.byref(koff)))
check(lib.kh_synth_packed_device(0, synth.SEED, 0, R, L, k, words, koff))
for batch in (1 << 27, 100000, 50000):
    for path in ("fixed", "variable"):
        g = khmer_amd.Countgraph(k, 1, 1, primes=sizes)
        g.set_use_bigcount(True)
        check(lib.kh_graph_set_batch_kmers(g._g, batch))
        if path == "fixed":
            check(lib.kh_consume_packed_fixed_device(g._g, words, R, L))
        else:
            check(lib.kh_consume_packed_device(g._g, words, koff, R, R * (L - k + 1)))
        n = ctypes.c_uint64()
        check(lib.kh_graph_get_bigcounts(g._g, None, None, 0, ctypes.byref(n)))
        keys = (ctypes.c_uint64 * max(n.value, 1))()
        vals = (ctypes.c_uint16 * max(n.value, 1))()
        check(lib.kh_graph_get_bigcounts(g._g, keys, vals, n.value, ctypes.byref(n)))
        ours = dict(zip(keys[:n.value], vals[:n.value]))
        extra = {h: v for h, v in ours.items() if ref.get(h) != v}
        missing = {h: v for h, v in ref.items() if h not in ours}
        tabs_ok = all(bytes(g.get_raw_tables()[i]) == o.table_bytes(i) for i in range(4))
        print(batch, path, "ours", len(ours), "ref", len(ref), "diff", len(extra), "missing", len(missing),
              "tables", tabs_ok, "uniq", g.n_unique_kmers(), o.n_unique_kmers(), flush=True)
