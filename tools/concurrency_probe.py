"""Development probe: do two independent pipelines on one MI355X overlap?

Two Countgraphs (C2 tables each) consume 25M synthetic reads each, first one
after the other, then at the same time from two host threads (each graph has
its own HIP stream; ctypes releases the GIL).  If the concurrent wall time is
well below the sequential one, kernels of different pipeline stages (level 1,
level 2, apply) fill each other's idle resources -- the case for pipelining a
graph's passes on two streams.
Usage: python tools/concurrency_probe.py [reads_per_graph] [batch_kmers]
"""
import ctypes
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402

reads = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1600 << 20
L, k = 150, 21
gs, bufs = [], []
for i in range(2):
    g = khmer_amd.Countgraph(k, 1e9, 4)
    g.set_use_bigcount(True)
    check(lib.kh_graph_set_batch_kmers(g._g, batch))
    w, ko = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(0, (reads * L // 32 + 2) * 8, ctypes.byref(w)))
    check(lib.kh_device_malloc(0, (reads + 1) * 8, ctypes.byref(ko)))
    check(lib.kh_synth_packed_device(0, synth.SEED, i * reads, reads, L, k, w, ko))
    gs.append(g)
    bufs.append(w)


def run(i):
    check(lib.kh_graph_clear(gs[i]._g))
    check(lib.kh_consume_packed_fixed_device(gs[i]._g, bufs[i], reads, L))
    check(lib.kh_device_synchronize(0))


for i in range(2):   # warm-up
    run(i)
out = {}
for rep in range(2):
    t0 = time.perf_counter()
    run(0)
    run(1)
    t1 = time.perf_counter()
    ts = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    t2 = time.perf_counter()
    out["rep%d" % rep] = {"sequential_ms": (t1 - t0) * 1e3, "concurrent_ms": (t2 - t1) * 1e3}
print(json.dumps({"reads_per_graph": reads, "batch_kmers": batch, **out}), flush=True)
