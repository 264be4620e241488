"""Timing probe (development only): runs the C2 bench workload for one step
and prints the per-phase cycle counters a debug build accumulates."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
L, k = 150, 21
g = khmer_amd.Countgraph(k, 1e9, 4)
g.set_use_bigcount(True)
check(lib.kh_graph_set_batch_kmers(g._g, 1 << 30))
words, koff = ctypes.c_void_p(), ctypes.c_void_p()
check(lib.kh_device_malloc(0, reads * L // 32 * 8 + 64, ctypes.byref(words)))
check(lib.kh_device_malloc(0, (reads + 1) * 8, ctypes.byref(koff)))
check(lib.kh_synth_packed_device(0, synth.SEED, 0, reads, L, k, words, koff))
dbg = (ctypes.c_uint64 * 64)()
for it in range(2):
    check(lib.kh_graph_clear(g._g))
    lib.kh_debug_read(dbg)
    check(lib.kh_consume_packed_fixed_device(g._g, words, reads, L))
    check(lib.kh_device_synchronize(0))
    lib.kh_debug_read(dbg)
    print("iter", it, "phases:", " ".join("%d:%.3e" % (i, dbg[i]) for i in range(64) if dbg[i]), flush=True)
