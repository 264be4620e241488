"""Per-rank cost of the sharded path without RCCL (development).

Runs a G-shard group in loopback mode (all shards in this process on one
device, device copies instead of RCCL broadcasts) over G x R synthetic reads
(weak scaling: R reads per source rank), and prints the wall time per step
divided by G -- the compute time one rank of a real G-GPU group spends, minus
the broadcast -- with the per-kernel breakdown summed over shards / G.
Usage: python tools/loopback_bench.py [world] [reads_per_rank] [steps] [batch_kmers] [exchange] [x]
(exchange = 1: Option A, kh_group_create_mode KH_GROUP_EXCHANGE; x: table size, 1e9 = C2, 8e9 = C4)
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import khmer_amd  # noqa: E402
from khmer_amd import parallel, synth  # noqa: E402
from khmer_amd._lib import lib, check  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reads = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 3200 << 20
exchange = len(sys.argv) > 5 and sys.argv[5] == "1"
x = float(sys.argv[6]) if len(sys.argv) > 6 else 1e9
L, k = 150, 21
sizes = khmer_amd.get_n_primes_near_x(4, x)
g = parallel.ShardedGraph("Countgraph", k, sizes, world, loopback=True, exchange=exchange)
g.set_use_bigcount(True)
g.set_batch_kmers(batch)
bufs = []
for s in range(world):
    w, ko = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(0, (reads * L // 32 + 2) * 8, ctypes.byref(w)))
    check(lib.kh_device_malloc(0, (reads + 1) * 8, ctypes.byref(ko)))
    check(lib.kh_synth_packed_device(0, synth.SEED, s * reads, reads, L, k, w, ko))
    bufs.append(w)


def step():
    g.clear()
    g.consume_packed_fixed_device(bufs, reads, L)
    check(lib.kh_device_synchronize(0))


step()
g.set_profiling(True)
t0 = time.perf_counter()
for _ in range(steps):
    step()
dt = (time.perf_counter() - t0) / steps
tot = {}
for sh in g.shards:
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(sh._g, buf, len(buf), ctypes.byref(n)))
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split("\t")
        tot[name] = tot.get(name, 0.0) + float(ms) / steps / world
u, o = g.counters()
print(json.dumps({"world": world, "exchange": exchange, "reads_per_rank": reads, "ms_per_step_total": dt * 1e3,
                  "ms_per_rank_step": dt * 1e3 / world,
                  "kernels_ms_per_rank_step": {a: round(b, 2) for a, b in sorted(tot.items()) if b > 0.5},
                  "n_unique": u, "n_occupied": o}), flush=True)
