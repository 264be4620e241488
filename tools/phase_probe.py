"""Timing probe (development only): runs the C2 bench workload and prints the
per-phase cycle counters a -DKH_PHASES build accumulates (tools/build_variant.sh
phases "-DKH_PHASES"; run with KHMER_AMD_LIB=ab/libphases.so).  Each kernel's
phases are s_memtime stamps summed over workgroups (kh_partition.cuh PH_*)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402

PHASES = {
    "scatter_l1 (exact)": (8, ["tile top", "hash+rank", "scan", "stage", "tails", "write"]),
    "apply": (16, ["init barrier", "records+barrier", "winner scan+barrier", "place+write winners", "pass 1",
                   "init", "prefetch+write-back+count", "scan+reserve"]),
    "scatter_l1f": (24, ["hash+rank", "barrier 1", "starts+scan", "stage", "reserve", "barrier 2", "write-out",
                         "advance+top barrier"]),
    "scatter_l2f": (32, ["wait+rank", "prefetch+barrier", "reserve+flist", "barrier", "flush", "barrier",
                         "stores", "advance+top barrier"]),
}

# usage: phase_probe.py [reads] [table size] [k]
reads = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
x = float(sys.argv[2]) if len(sys.argv) > 2 else 1e9
L, k = 150, int(sys.argv[3]) if len(sys.argv) > 3 else 21
g = khmer_amd.Countgraph(k, x, 4)
g.set_use_bigcount(True)
check(lib.kh_graph_set_batch_kmers(g._g, 3200 << 20))
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
    print("iter", it, flush=True)
    for name, (base, labels) in PHASES.items():
        vals = [dbg[base + i] for i in range(len(labels))]
        tot = sum(vals)
        if not tot:
            continue
        print("  %-20s %s" % (name, "  ".join("%s %.1f%%" % (lab, 100.0 * v / tot) for lab, v in zip(labels, vals))),
              flush=True)
    if dbg[42]:   # scatter_l1f workgroup wall times (100 MHz clock, PH_WG_*)
        print("  scatter_l1f workgroups %d: mean %.2f ms, max %.2f ms (per launch: all resident at once)"
              % (dbg[42], dbg[40] / dbg[42] / 1e5, dbg[41] / 1e5), flush=True)
    if dbg[45]:   # k_apply_count workgroup wall times
        print("  apply workgroups %d: mean %.2f ms, max %.2f ms" % (dbg[45], dbg[43] / dbg[45] / 1e5, dbg[44] / 1e5),
              flush=True)
