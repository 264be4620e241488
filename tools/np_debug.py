"""Development: the near-prime consume against the per-table level 1 on one
device stream (KH_NEAR_PRIME=1 / 0), table by table, with progress on stderr."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd
from khmer_amd._lib import lib, check, default_device

k, x, n, L, batch = int(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3]), 150, int(sys.argv[4])
nt = int(sys.argv[5]) if len(sys.argv) > 5 else 4
dev = default_device()
words, koff = ctypes.c_void_p(), ctypes.c_void_p()
check(lib.kh_device_malloc(dev, (n * L // 32 + 2) * 8, ctypes.byref(words)))
check(lib.kh_device_malloc(dev, (n + 1) * 8, ctypes.byref(koff)))
check(lib.kh_synth_packed_device(dev, 0x6e70, 0, n, L, k, words, koff))


def run(np_on):
    os.environ["KH_NEAR_PRIME"] = "1" if np_on else "0"
    g = khmer_amd.Countgraph(k, x, nt)
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, batch))
    check(lib.kh_graph_set_profiling(g._g, 1))
    t = time.time()
    check(lib.kh_consume_packed_fixed_device(g._g, words, n, L))
    print("np=%d %.3f s n_unique %d n_occ %d" % (np_on, time.time() - t, g.n_unique_kmers(), g.n_occupied()),
          file=sys.stderr, flush=True)
    buf = ctypes.create_string_buffer(1 << 16)
    nn = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(g._g, buf, len(buf), ctypes.byref(nn)))
    print(buf.value.decode(), file=sys.stderr)
    tabs = [np.frombuffer(bytes(t), dtype=np.uint8).copy() for t in g.get_raw_tables()]
    return g, tabs


g1, a = run(True)
g0, b = run(False)
print("sizes", g1.hashsizes(), file=sys.stderr)
for i in range(nt):
    d = np.nonzero(a[i] != b[i])[0]
    print("table %d: %d bins differ; sum np %d per-table %d" % (i, len(d), int(a[i].sum()), int(b[i].sum())),
          file=sys.stderr)
    if len(d):
        print("  first", d[:12].tolist(), "np", a[i][d[:12]].tolist(), "pt", b[i][d[:12]].tolist(), file=sys.stderr)
        reg = d >> 14
        u, c = np.unique(reg, return_counts=True)
        print("  regions", len(u), "first", list(zip(u[:10].tolist(), c[:10].tolist())), file=sys.stderr)
