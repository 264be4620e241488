#!/usr/bin/env python3
"""Per-rank cost of a G-rank group at the true pass size, measured on one GPU
(VERDICT r4 "Next round" #4).

A 1-rank RCCL group (the multi-rank code path at world 1: communicator,
collectives, the same kernels) consumes one rank's share of the bench stream
with kernel timing on.  What a rank of a G-rank group does per pass does not
depend on G in delta mode -- it partitions and applies its own chunk twice
(delta tables, then over its prefix), and as owner prefixes W slices of 1/W of
the tables (the table's bytes in all) -- so the world-1 kernel times ARE the
per-rank compute at any G.  Exchange mode's passes shrink with G (a pass takes
batch / G k-mers of every rank), so it runs at batch / G here.  The wire time
is not measured (one GPU): the bytes a rank sends over xGMI per step are
stated, with the time they take at an assumed per-GPU one-way rate.  Delta
mode's pieces travel sparse (bitmap + nonzero bytes, kh_engine.hip
sp_pack): KH_DELTA_PROBE=1 packs the world-1 rank's own delta slices to
measure their sparse size; the estimate keeps the prefixes dense (an upper
bound: a rank's prefix at G > 1 is denser than the world-1 table).

    python tools/rank_model.py --mode delta --world 8 [--config C2|C4] [--reads 50000000]
Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {"C2": ("Countgraph", 21, 1e9), "C4": ("Countgraph", 21, 8e9)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["delta", "exchange"], default="delta")
    ap.add_argument("--world", type=int, default=8, help="the group size being modelled")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C2")
    ap.add_argument("--reads", type=int, default=50_000_000, help="reads per rank")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch-kmers", type=int, default=3200 << 20)
    ap.add_argument("--xgmi-gbs", type=float, default=350.0,
                    help="assumed one-way xGMI rate per GPU for the wire estimate (7 links x ~50 GB/s)")
    a = ap.parse_args()
    os.environ["KH_DELTA_PROBE"] = "1"
    import khmer_amd
    from khmer_amd import parallel, synth
    from khmer_amd._lib import lib, check
    cls, k, x = CONFIGS[a.config]
    L, nt = 150, 4
    sizes = khmer_amd.get_n_primes_near_x(nt, x)
    uid = parallel.ShardedGraph.unique_id()
    g = parallel.ShardedGraph(cls, k, sizes, 1, rank=0, device=0, uid=uid, mode=a.mode)
    g.set_use_bigcount(True)
    batch = a.batch_kmers if a.mode == "delta" else a.batch_kmers // a.world
    g.set_batch_kmers(batch)
    words, koff = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(0, (a.reads * L // 32 + 2) * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(0, (a.reads + 1) * 8, ctypes.byref(koff)))
    check(lib.kh_synth_packed_device(0, synth.SEED, 0, a.reads, L, k, words, koff))

    def step():
        g.clear()
        g.consume_packed_fixed_device([words], a.reads, L)
    step()   # warmup
    check(lib.kh_device_synchronize(0))
    g.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    check(lib.kh_device_synchronize(0))
    dt = (time.perf_counter() - t0) / a.steps
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    check(lib.kh_graph_kernel_stats(g.shards[0]._g, buf, len(buf), ctypes.byref(n)))
    kern = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split("\t")
        kern[name] = round(float(ms) / a.steps, 3)
    kpr = L - k + 1
    kmers = a.reads * kpr
    tbytes = sum(sizes)   # Countgraph: one byte per bin
    W = a.world
    if a.mode == "delta":
        npass = len(parallel.delta_passes(a.reads, L, k, batch))
        wire = 2 * tbytes * (W - 1) / W * npass          # deltas out + prefixes back, per pass
    else:
        npass = len(parallel.exchange_passes(a.reads, L, k, W, a.batch_kmers))
        wire = 8 * nt * kmers * (W - 1) / W                # level-1 records to their owners
    wire_ms = wire / (a.xgmi_gbs * 1e9) * 1e3
    u, occ = g.counters()
    sparse = {}
    if a.mode == "delta":
        dense_b, sent_b = g.wire_stats()   # the probe's own delta slices, every pass of the warmup + timed steps
        if dense_b:
            ratio = sent_b / dense_b
            wire_sp = wire / 2 * ratio + wire / 2   # deltas sparse, prefixes dense
            sparse = {"delta_sparse_ratio": round(ratio, 4), "wire_bytes_sparse_per_rank_step": wire_sp,
                      "wire_ms_sparse_at_assumed_rate": round(wire_sp / (a.xgmi_gbs * 1e9) * 1e3, 1),
                      "rank_step_ms_sparse_unoverlapped": round(dt * 1e3 + wire_sp / (a.xgmi_gbs * 1e9) * 1e3, 1)}
    out = {"mode": a.mode, "world_modelled": W, "config": a.config, "reads_per_rank": a.reads,
           "kmers_per_rank": kmers, "passes_per_step": npass, "batch_kmers": batch,
           "compute_ms_per_rank_step": round(dt * 1e3, 2), "kernels_ms_per_step": kern,
           "wire_bytes_per_rank_step": wire, "wire_bytes_per_kmer": wire / kmers,
           "wire_ms_at_assumed_rate": round(wire_ms, 1), "assumed_xgmi_gbs_one_way": a.xgmi_gbs,
           "rank_step_ms_unoverlapped": round(dt * 1e3 + wire_ms, 1),
           "n_unique": u, "n_occupied": occ, **sparse}
    print(json.dumps(out), flush=True)
    lib.kh_device_free(0, words)
    lib.kh_device_free(0, koff)
    g.close()


if __name__ == "__main__":
    main()
