#!/usr/bin/env python3
"""bench.py -- k-mers hashed/s into a Countgraph on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]): Countgraph k=21,
4 tables of the largest primes < 1e9 (4.0 GB of 8-bit counters, bigcount on as
in load-into-counting.py), 50M synthetic 150 bp reads per GPU (6.5e9 k-mers).
The reads are generated straight into HBM before timing
(kh_synth_packed_device = khmer_amd.synth's seeded stream).  One step = reset
the tables, then consume every read (hash -> partition -> LDS apply ->
finalize), i.e. the whole hot path over the whole batch.

Multi-GPU (one rank per GPU; `--gpus N` starts the N rank processes itself
unless a launcher set WORLD_SIZE): every table is split into G contiguous bin
ranges, one per rank.  Every rank generates its own 50M
reads (weak scaling).  Group mode "auto" (the default) picks delta unless the
tables outweigh the records a rank-pass sends (auto_group_mode: C4 strong
scaling takes exchange).  Delta mode: every rank counts its own
reads into full-size delta tables, the owners turn every rank's deltas of
their slice into per-rank prefixes (table bytes over RCCL/xGMI, grouped
send/recv) and each rank re-applies its reads over its prefix; "exchange"
(Option A): each rank hashes only its own reads into level-1 buckets and
sends every bucket to its owner; "broadcast" (Option B): each rank's reads
are broadcast and every rank hashes every k-mer, keeping its own bins'
updates.  value = all ranks' k-mers / max time.

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM = 8.0e12  # B/s, MI355X spec (MI355X_MICROARCH.md)


def algorithmic_bytes_per_kmer(L, k, n_tables):
    """2-bit input per k-mer + 1 B read + 1 B write per table."""
    return (L / 4.0) / (L - k + 1) + 2.0 * n_tables


# SURVEY.md §8(d) configurations: graph class, k, per-table size.  C2 is the
# BASELINE.json headline (the default); C3 / C5 measure the bit and nibble
# storages on the same pipeline (C5 as its 2-bit SmallCountgraph variant, k=31).
CONFIGS = {
    "C2": ("Countgraph", 21, 1e9),
    "C3": ("Nodegraph", 31, 4e9),
    "C4": ("Countgraph", 21, 8e9),
    "C5": ("SmallCountgraph", 31, 8e9),
    "C5M": ("SmallCounttable", 51, 8e9),
}
DTYPE = {"Countgraph": "u8", "Nodegraph": "u1 (bit)", "SmallCountgraph": "u4 (nibble)",
         "SmallCounttable": "u4 (nibble)"}
ORACLE_KIND = {"Countgraph": "BYTE", "Nodegraph": "BIT", "SmallCountgraph": "NIBBLE", "SmallCounttable": "NIBBLE"}
MURMUR = {"SmallCounttable"}   # Counttable family: MurmurHash3 over ASCII k-mers


def query_bytes_per_kmer(L, k, n_tables):
    """SURVEY.md §8(d) C5 query: 2-bit input + 1 B read per table + the
    per-read outputs (u16 median + 2 x f32) spread over the read's k-mers."""
    kpr = L - k + 1
    return (L / 4.0) / kpr + 1.0 * n_tables + 10.0 / kpr


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=50_000_000, help="reads per GPU")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="C2",
                    help="graph class / k / table size preset (SURVEY.md §8(d))")
    ap.add_argument("-k", type=int, default=None, help="override the preset's k")
    ap.add_argument("--tables", type=int, default=4)
    ap.add_argument("-x", type=float, default=None, help="override the preset's table size")
    ap.add_argument("--batch-kmers", type=int, default=3200 << 20,
                    help="largest device pass (the library cap, MAX_PASS_KMERS); fewer, larger passes "
                         "amortise the per-bin work of every pass")
    ap.add_argument("--no-bigcount", action="store_true")
    ap.add_argument("--genome", type=float, default=0,
                    help="bases of the random genome of the skewed 'genomic' stream (SURVEY.md §8(d): 1e8); "
                         "0 = iid uniform reads")
    ap.add_argument("--strong", action="store_true",
                    help="multi-GPU strong scaling: --reads is the whole job, split over the ranks")
    ap.add_argument("--group-mode", choices=["auto", "delta", "exchange", "broadcast"], default="auto",
                    help="multi-GPU: 'auto' (default: delta unless the tables outweigh the records a rank-pass "
                         "would send, DESIGN.md §6), 'delta' (every rank counts its own reads into full-size delta tables, "
                         "owners turn every rank's deltas of their slice into per-rank prefixes, each rank applies "
                         "its reads over its prefix; only table bytes travel), 'exchange' (Option A: every rank "
                         "hashes only its own reads and sends each level-1 bucket to its owner) or 'broadcast' "
                         "(Option B: reads broadcast, every rank hashes every k-mer and keeps its own bins' "
                         "updates); DESIGN.md §6")
    ap.add_argument("--query", action="store_true",
                    help="time get_median_count over the reads (tables built from them first, untimed)")
    ap.add_argument("--ablate", type=int, default=0,
                    help="timing-only KH_ABLATE bits (results become wrong; never for reported numbers); "
                         "needs a development library built with make EXTRA_HIPFLAGS=-DKH_ABLATE")
    ap.add_argument("--variable-path", action="store_true",
                    help="feed k-mer offsets (variable-length read path) instead of the fixed-length path")
    ap.add_argument("--cpu-reads", type=int, default=1_000_000,
                    help="reads in the oracle CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-unprofiled", dest="unprofiled", action="store_false",
                    help="skip the second, unprofiled run of the K steps (ms_per_step_unprofiled)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    a.graph, k, x = CONFIGS[a.config]
    a.k = k if a.k is None else a.k
    a.x = x if a.x is None else a.x
    a.bigcount = a.graph == "Countgraph" and not a.no_bigcount
    a.genome = int(a.genome)
    a.murmur = a.graph in MURMUR
    if a.group_mode == "auto":
        a.group_mode = auto_group_mode(a)
    a.exchange = a.group_mode == "exchange"
    return a


def auto_group_mode(a):
    """Delta or exchange for this run.  Per rank-pass, delta
    mode sends the table bytes TB twice (deltas to the owners, prefixes back),
    exchange mode every (k-mer, table) record once (8 B x tables per k-mer):
    delta iff TB <= 4 x tables x the k-mers of a rank-pass.  C2 / C4 weak
    scaling (3.25e9 k-mers a rank-pass): delta; C4 strong over 8 ranks (0.8e9
    k-mers a rank, 32 GB of tables): exchange."""
    bytes_per_bin = {"Countgraph": 1.0, "Nodegraph": 0.125, "SmallCountgraph": 0.5, "SmallCounttable": 0.5}[a.graph]
    tb = a.tables * a.x * bytes_per_bin
    reads = (a.reads + a.gpus - 1) // a.gpus if (a.strong and a.gpus > 1) else a.reads
    kpass = min(a.batch_kmers, reads * (a.read_len - a.k + 1))
    return "delta" if tb <= 4.0 * a.tables * kpass else "exchange"


FIXTURE_GRAPH = {(1, 0): "Countgraph", (2, 0): "Nodegraph", (7, 0): "SmallCountgraph", (7, 1): "SmallCounttable"}


def matching_fixture(args, total_reads, order=None):
    """The oracle golden fixture (tests/golden/full/*.json, made by
    tests/golden/make_full_fixtures.py) whose workload is exactly this run's
    whole stream, if any: then the bench line carries a parity check of its
    own (counters and per-table SHA-256 against the single-threaded oracle).
    order = (mode, [world, batch_kmers]) for an exchange- or delta-mode group,
    whose stream is pass-interleaved: a fixture made in that order matches
    exactly; failing that, the rank-order fixture of the same reads
    (order-free outputs only).  Returns (fixture, exact_order)."""
    import glob
    same_reads, interleaved, other_order = None, None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "full", "*.json"))):
        try:
            with open(path) as fh:
                fx = json.load(fh)
            p = fx["params"]
        except (OSError, ValueError, KeyError):
            continue
        if (FIXTURE_GRAPH.get((p["kind"], p["hash"])) == args.graph and p["k"] == args.k and p["n"] == args.tables
                and float(p["x"]) == float(args.x) and p["reads"] == total_reads and p["L"] == args.read_len
                and bool(p["bigcount"]) == bool(args.bigcount) and int(p["genome"]) == int(args.genome)):
            fmode = "exchange" if "exchange" in p else "delta" if "delta" in p else None
            if fmode is None and same_reads is None:
                same_reads = fx
            elif order is not None and fmode == order[0] and p[fmode] == list(order[1]):
                interleaved = fx
            elif fmode is not None and other_order is None:
                other_order = fx
    if order is None and same_reads is not None:
        return same_reads, True
    if order is not None and interleaved is not None:
        return interleaved, True
    # the same reads in another order: the tables and n_occupied still match
    fallback = same_reads if same_reads is not None else other_order
    return (fallback, False) if fallback is not None else (None, False)


def compare_fixture(fx, n_unique, n_occupied, table_sha, stream_order=True):
    """stream_order=False (an exchange-mode run with no fixture in its
    pass-interleaved order): the tables and n_occupied do not depend on the
    order and are compared; n_unique does and is reported beside the
    rank-order fixture's."""
    if not stream_order:
        out = {"fixture": fx["config"], "n_occupied_match": n_occupied == fx["n_occupied"],
               "n_unique": "pass-interleaved stream: no fixture in this order (rank-order fixture %d, run %d)"
                           % (fx["n_unique_kmers"], n_unique)}
        if table_sha is not None:
            out["tables_match"] = list(table_sha) == list(fx["table_sha256"])
        return out
    out = {"fixture": fx["config"], "counters_match": n_unique == fx["n_unique_kmers"] and
           n_occupied == fx["n_occupied"]}
    if table_sha is not None:
        out["tables_match"] = list(table_sha) == list(fx["table_sha256"])
    return out


def kernel_stats(lib, g):
    buf = ctypes.create_string_buffer(1 << 16)
    n = ctypes.c_size_t()
    lib.kh_graph_kernel_stats(g, buf, len(buf), ctypes.byref(n))
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split("\t")
        out[name] = (int(cnt), float(ms))
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """CPU threads this process may use: the affinity set, capped by
    OMP_NUM_THREADS (the GPU box's per-job CPU share; nproc there shows the
    whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args, sizes):
    """The oracle (C restatement of Hashtable::consume_string / consume_seqfile /
    get_median_count, oracle/khmer_oracle.c) on bounded samples of the same
    synthetic stream into same-size tables, on this host's cores:
      * in-memory batch, T = 1 (stream order, the exact semantics)
      * in-memory batch, T = host_threads() (the reference's -T N mode: atomic
        byte updates and shared occupancy counter, src/oxli/hashtable.cc:125-150)
      * end to end from a page-cached FASTQ file, T = 1 (parse + clean + count)
    `value` is the faster of the two in-memory rates.  --query: the oracle's
    get_median_count (src/oxli/hashtable.cc:299-328) per read, T = 1, over
    tables built from the same sample."""
    from oracle import oracle as O
    from khmer_amd import synth
    kind = getattr(O, ORACLE_KIND[args.graph])
    hashfn = O.MURMUR if args.murmur else O.TWOBIT
    n = args.cpu_reads
    chunk = 100_000
    batches = []
    for r0 in range(0, n, chunk):
        if args.genome:
            seqs, offs = synth.genomic_batch(r0, min(chunk, n - r0), args.read_len, args.genome)
        else:
            seqs, offs = synth.batch(r0, min(chunk, n - r0), args.read_len)
        batches.append((seqs, [int(v) for v in offs]))

    def table():
        t = O.Table(kind, args.k, sizes, hashfn)
        t.set_use_bigcount(args.bigcount)
        return t

    def run(threads):
        t = table()
        total, secs = 0, 0.0
        for seqs, offs in batches:
            t0 = time.perf_counter()
            total += t.consume_batch(seqs, offs, threads=threads if threads > 1 else 0)
            secs += time.perf_counter() - t0
        return total, secs, t

    T = host_threads()
    k1, s1, t1 = run(1)
    if args.query:
        nq = min(n, 200_000)
        L = args.read_len
        seqs = batches[0][0] if nq <= chunk else b"".join(b[0] for b in batches)
        t0 = time.perf_counter()
        for r in range(nq):
            t1.median(seqs[r * L:(r + 1) * L])
        dt = time.perf_counter() - t0
        kq = nq * (L - args.k + 1)
        return {
            "value": kq / dt, "unit": "k-mers/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
            "sample": "get_median_count over %d synthetic %d bp reads (%d k-mers) of the benchmark stream, tables "
                      "built from the first %d reads; oracle/khmer_oracle.c, 1 thread" % (nq, L, kq, n),
        }
    del t1
    kT, sT, tT = run(T)
    del tT
    # end to end: FASTQ in the page cache (written, then read once untimed)
    import tempfile
    nfq = min(n, 500_000)
    e2e = None
    if not args.genome:
        with tempfile.TemporaryDirectory() as tmp:
            fq = os.path.join(tmp, "sample.fq")
            synth.write_fastq(fq, nfq, args.read_len)
            with open(fq, "rb") as fh:
                while fh.read(1 << 24):
                    pass
            t = table()
            t0 = time.perf_counter()
            _, kmers = t.consume_fastx(fq)
            e2e = kmers / (time.perf_counter() - t0)
            del t
    r1, rT = k1 / s1, kT / sT
    return {
        "value": max(r1, rT),
        "unit": "k-mers/s",
        "cores": 1 if r1 >= rT else T,
        "kind": "port",
        "cpu_model": cpu_model(),
        "t1_in_memory": r1,
        "tN_in_memory": rT,
        "tN_threads": T,
        "t1_end_to_end_fastq": e2e,
        "sample": "%d synthetic %d bp reads (%d k-mers, the first reads of the benchmark stream) into the same "
                  "%dx%.0e %s; oracle/khmer_oracle.c: value = the faster of 1 thread (stream order) and %d threads "
                  "(the reference's -T N atomic updates; its shared occupancy counter serialises them); "
                  "end-to-end = %d reads parsed from a page-cached FASTQ, 1 thread"
                  % (n, args.read_len, k1, args.tables, args.x, args.graph, T, nfq),
    }


def free_port():
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher: start N rank processes of
    this script (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set as torchrun would), before this process makes any HIP
    call.  Rank 0's JSON line is the output; any failing rank fails the run
    (the others are stopped)."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                sys.stderr.write("bench.py: rank %d exited with %d; stopping the others\n" % (procs.index(p), code))
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 1


def main():
    args = parse()
    if args.ablate:
        os.environ["KH_ABLATE"] = str(args.ablate)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # development only: put every rank on one device (exercising RCCL on a one-GPU box)
    local = int(os.environ.get("KH_BENCH_DEVICE", local))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))

    import khmer_amd
    from khmer_amd import _lib, synth
    from khmer_amd._lib import lib, check
    _lib.set_default_device(local)

    L, k, nt = args.read_len, args.k, args.tables
    if args.strong and world > 1:
        args.reads = (args.reads + world - 1) // world   # per rank
    nreads = args.reads
    nkmers = nreads * (L - k + 1)
    sizes = khmer_amd.get_n_primes_near_x(nt, args.x)

    if world > 1:
        from khmer_amd import parallel
        runner = parallel.ShardedCountgraphBench(args, rank, world, local, sizes)
    else:
        runner = SingleGpuBench(args, local, sizes)

    def progress(what):   # stderr, outside the timed region: long multi-rank runs show life
        if rank == 0:
            sys.stderr.write("bench.py: %s\n" % what)
            sys.stderr.flush()

    runner.setup()
    progress("setup done")
    for _ in range(args.warmup):
        runner.step()
    runner.sync()
    progress("warmup done")
    runner.barrier()
    runner.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step()
    runner.sync()
    t1 = time.perf_counter()
    runner.barrier()
    elapsed = runner.max_over_ranks(t1 - t0)
    progress("timed steps done")
    stats = runner.kernel_stats()
    runner.profile(False)
    # the same K steps again without the per-kernel HIP events: how much the
    # profiling in the timed region costs (reported, never `value`)
    unprof = None
    if args.unprofiled:
        runner.barrier()
        u0 = time.perf_counter()
        for _ in range(args.steps):
            runner.step()
        runner.sync()
        u1 = time.perf_counter()
        runner.barrier()
        unprof = runner.max_over_ranks(u1 - u0) * 1e3 / args.steps
    check_info = runner.check()
    # parity of the timed workload itself, when a golden fixture holds it
    fx, exact_order = matching_fixture(args, nreads * world,
                                       (args.group_mode, [world, args.batch_kmers])
                                       if (args.group_mode != "broadcast" and world > 1) else None)
    if args.query:
        # the tables were built untimed from the same reads; the fixture's
        # get_median_count digest (median, average, stddev of its first
        # reads).  Medians do not depend on the consume order: the
        # stream-order fixture of the same reads holds the digest whatever
        # order the group consumed them in.
        qfx, _ = matching_fixture(args, nreads * world)
        if qfx is not None and qfx.get("median_sha256"):
            q = runner.query_check(qfx)   # collective when sharded
            if rank == 0:
                check_info.update(q)
        elif rank == 0:
            check_info["median_match"] = "no query fixture for this workload"
        fx = None
    if fx is not None:
        progress("hashing the tables for the %s check" % fx["config"])
        sha = runner.table_sha256()   # collective when sharded
        if rank == 0:
            check_info.update(compare_fixture(fx, check_info["n_unique_kmers"], check_info["n_occupied"], sha,
                                              stream_order=exact_order))

    bpk = query_bytes_per_kmer(L, k, nt) if args.query else algorithmic_bytes_per_kmer(L, k, nt)
    total_kmers = nkmers * world * args.steps
    value = total_kmers / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # dominant kernel and its live HIP-event average duration
    dom = max(stats.items(), key=lambda kv: kv[1][1]) if stats else None
    roofline = None
    if dom:
        name, (cnt, ms) = dom
        avg_s = ms / 1e3 / cnt
        kmers_per_launch = nkmers * args.steps / cnt  # per-rank k-mers one launch processes
        achieved = bpk * kmers_per_launch / avg_s
        traffic = None
        try:
            with open(args.traffic_json) as fh:
                tj = json.load(fh)
            if tj.get("config") == runner.config_name():
                traffic = (tj["kernels"].get(name) if "kernels" in tj
                           else tj.get("hbm_bytes_per_launch") if tj.get("kernel") == name else None)
        except (OSError, ValueError):
            pass
        step_s = elapsed / args.steps
        roofline = {
            "bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
            "frac": achieved / PEAK_HBM, "traffic": traffic,
            "kernel": name, "avg_launch_ms": ms / cnt, "launches": cnt,
            "bytes_per_kmer": bpk,
            "pipeline_frac": bpk * nkmers / step_s / PEAK_HBM,
            "kernels_ms_per_step": {n: round(v[1] / args.steps, 3) for n, v in sorted(stats.items())},
        }

    cpu = None
    if rank == 0 and world == 1 and args.cpu_reads > 0:
        cpu = cpu_baseline(args, sizes)

    if rank == 0:
        if args.query:
            metric = "k-mers queried/sec by get_median_count on %s (k=%d, %dx%.0e)" % (args.graph, k, nt, args.x)
        else:
            metric = "k-mers hashed/sec into %s (k=%d, %dx%.0e)" % (args.graph, k, nt, args.x)
        line = {
            "metric": metric,
            "value": value,
            "unit": "k-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "ms_per_step_unprofiled": unprof,
            "higher_is_better": True,
            "scaling": "strong" if (args.strong and world > 1) else "weak",
            "vs_baseline": None,
            "dtype": DTYPE[args.graph],
            "data": ("synthetic genomic stream (reads of a %d-base random genome, both strands, 1%% substitutions, "
                     "generated in HBM)" % args.genome) if args.genome else
                    "synthetic (seeded SplitMix64 reads generated in HBM)",
            "config": {
                "workload": runner.config_name(),
                "k": k, "n_tables": nt, "table_sizes": sizes, "reads_per_gpu": nreads,
                "read_len": L, "kmers_per_gpu_per_step": nkmers, "bigcount": args.bigcount,
                "batch_kmers": args.batch_kmers,
                "parallelism": ("%s%d" % ({"delta": "delta", "exchange": "exchange", "broadcast": "shard"}[args.group_mode],
                                          world)) if world > 1 else "single",
                "path": "get_median_count" if args.query else "consume",
                "hash": "murmur3" if args.murmur else "twobit",
                "genome": args.genome or None,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "check": check_info,
        }
        if world > 1:
            line["rccl"] = runner.rccl_info()
        print(json.dumps(line), flush=True)
    runner.close()


class SingleGpuBench(object):
    def __init__(self, args, device, sizes):
        self.args, self.device, self.sizes = args, device, sizes

    def config_name(self):
        a = self.args
        what = "get_median_count over" if a.query else "consume of"
        return "%s k=%d %dx%.0e, %s %d x %d bp synthetic %sreads, 1xMI355X" % (
            a.graph, a.k, a.tables, a.x, what, a.reads, a.read_len, "genomic " if a.genome else "")

    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        self._ck(self.lib.kh_device_malloc(self.device, nbytes, ctypes.byref(p)))
        self.bufs.append(p)
        return p

    def setup(self):
        import khmer_amd
        from khmer_amd import synth
        from khmer_amd._lib import lib, check
        a = self.args
        self.lib, self._ck, self.bufs = lib, check, []
        self.g = getattr(khmer_amd, a.graph)(a.k, a.x, a.tables)
        if a.bigcount:
            self.g.set_use_bigcount(True)
        check(lib.kh_graph_set_batch_kmers(self.g._g, a.batch_kmers))
        self.nkmers = a.reads * (a.read_len - a.k + 1)
        nwords = a.reads * a.read_len // 32 + 2
        self.words = self._alloc(nwords * 8)
        self.koff = self._alloc((a.reads + 1) * 8)
        ks = min(a.k, 32)   # the packed stream itself does not depend on k
        if a.genome:
            check(lib.kh_synth_genomic_device(self.device, synth.SEED, a.genome, 0, a.reads, a.read_len, ks,
                                              self.words, self.koff))
        else:
            check(lib.kh_synth_packed_device(self.device, synth.SEED, 0, a.reads, a.read_len, ks, self.words,
                                             self.koff))
        self.reads = self.words
        if a.murmur:   # Counttable family: the same bases as ASCII (the packed words are then freed)
            self.reads = self._alloc(a.reads * a.read_len + 64)
            check(lib.kh_unpack_ascii_device(self.device, self.words, a.reads * a.read_len, self.reads))
            check(lib.kh_device_free(self.device, self.words))
            self.bufs.remove(self.words)
            self.words = None
        if a.query:
            self.med = self._alloc(a.reads * 2 + 64)
            self.avg = self._alloc(a.reads * 4 + 64)
            self.sd = self._alloc(a.reads * 4 + 64)
            self._consume()   # the tables being queried (untimed)

    def _consume(self):
        a = self.args
        if a.murmur:
            self._ck(self.lib.kh_consume_bytes_fixed_device(self.g._g, self.reads, a.reads, a.read_len))
        elif a.variable_path:
            self._ck(self.lib.kh_consume_packed_device(self.g._g, self.words, self.koff, a.reads, self.nkmers))
        else:
            self._ck(self.lib.kh_consume_packed_fixed_device(self.g._g, self.words, a.reads, a.read_len))

    def step(self):
        a = self.args
        if a.query:
            self._ck(self.lib.kh_median_counts_fixed_device(self.g._g, self.reads, a.reads, a.read_len, self.med,
                                                            self.avg, self.sd))
            return
        self._ck(self.lib.kh_graph_clear(self.g._g))
        self._consume()

    def sync(self):
        self._ck(self.lib.kh_device_synchronize(self.device))

    def barrier(self):
        pass

    def max_over_ranks(self, t):
        return t

    def profile(self, on):
        self._ck(self.lib.kh_graph_set_profiling(self.g._g, 1 if on else 0))

    def kernel_stats(self):
        return kernel_stats(self.lib, self.g._g)

    def table_sha256(self):
        import hashlib
        out = []
        for i, n in enumerate(self.g._raw_sizes()):
            buf = bytearray(n)
            self._ck(self.lib.kh_graph_copy_table(self.g._g, i, (ctypes.c_char * n).from_buffer(buf)))
            out.append(hashlib.sha256(buf).hexdigest())
            del buf
        return out

    def check(self):
        """Counters of the last consume (the full workload into empty tables);
        --query: also a checksum of the medians."""
        out = {"n_unique_kmers": self.g.n_unique_kmers(), "n_occupied": self.g.n_occupied()}

        if self.args.query:
            from tests import full_digest as FD
            med, avg, sd = self.query_outputs()
            out["median_sha256"] = FD.median_digest(med, avg, sd)   # medians, averages and stddevs
            out["median_max"] = int(med.max()) if len(med) else 0
        return out

    def query_outputs(self):
        """(median u16, average f32, stddev f32) numpy arrays of the last query."""
        import numpy as np
        n = self.args.reads
        med = np.zeros(n, np.uint16)
        avg = np.zeros(n, np.float32)
        sd = np.zeros(n, np.float32)
        self._ck(self.lib.kh_device_synchronize(self.device))
        for arr, dev in ((med, self.med), (avg, self.avg), (sd, self.sd)):
            hip_copy_d2h(self.lib, self.device, arr.ctypes.data_as(ctypes.c_void_p), dev, arr.nbytes)
        return med, avg, sd

    def query_check(self, fx):
        """The fixture's get_median_count digest over its first median_reads
        reads (tests/golden/make_full_fixtures.py: the oracle's float32
        results, bit patterns exactly)."""
        from tests import full_digest as FD
        n = fx["median_reads"]
        med, avg, sd = self.query_outputs()
        return {"fixture": fx["config"], "median_reads": n,
                "median_match": FD.median_digest(med[:n], avg[:n], sd[:n]) == fx["median_sha256"]}

    def close(self):
        for p in self.bufs:
            self.lib.kh_device_free(self.device, p)
        del self.g


def hip_copy_d2h(lib, device, dst, src, nbytes):
    """device -> host copy through the library (no PyTorch on the host side)."""
    from khmer_amd._lib import check
    check(lib.kh_device_copy(device, dst, src, nbytes))


if __name__ == "__main__":
    main()
