"""Digests of full-size tables and counters (shared by the golden-fixture
generator tests/golden/make_full_fixtures.py and the GPU tests that check the
HIP path against those fixtures).  GB-sized tables are compared by SHA-256 of
their bytes, so a fixture stays a few hundred bytes of JSON."""
import hashlib
import json
import os
import struct

FULL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "full")

# Full-size / production-geometry configurations (VERDICT r1 "Next round" #1).
# kind: BYTE/BIT/NIBBLE (file-type codes), hash: 0 two-bit, 1 Murmur.
# genome: 0 = iid uniform stream, G > 0 = genomic stream over a G-base genome.
# batch_kmers: the device pass size the GPU test uses (forces multi-pass runs).
CONFIGS = {
    # the benchmark workload itself (BASELINE configs[1], bench.py default)
    "c2_full": dict(kind=1, hash=0, k=21, n=4, x=1e9, reads=50_000_000, L=150, bigcount=True,
                    genome=0, batch_kmers=2560 << 20),
    # C3 geometry: 4 x 4e9 bits, F1 > 1024 level-1 buckets, bin ids > 2^32
    "c3_shape": dict(kind=2, hash=0, k=31, n=4, x=4e9, reads=4_000_000, L=150, bigcount=False,
                     genome=0, batch_kmers=1 << 27),
    # C4 tables on one GPU: 4 x 8e9 bytes (32 GB)
    "c4_shape": dict(kind=1, hash=0, k=21, n=4, x=8e9, reads=4_000_000, L=150, bigcount=True,
                     genome=0, batch_kmers=1 << 28),
    # C5 geometry (2-bit SmallCountgraph variant): 4 x 8e9 nibbles
    "c5_shape": dict(kind=7, hash=0, k=31, n=4, x=8e9, reads=4_000_000, L=150, bigcount=False,
                     genome=0, batch_kmers=1 << 27),
    # C5 as SURVEY F2 names it: SmallCounttable k=51, MurmurHash3, 4 x 8e9 nibbles
    "c5m_shape": dict(kind=7, hash=1, k=51, n=4, x=8e9, reads=1_000_000, L=150, bigcount=False,
                      genome=0, batch_kmers=1 << 26),
    # skewed ("genomic") stream, 2 Mbp genome at ~750x: saturation + heavy bigcount
    "genomic_c2": dict(kind=1, hash=0, k=21, n=4, x=1e9, reads=10_000_000, L=150, bigcount=True,
                       genome=2_000_000, batch_kmers=1 << 29),
    # BASELINE C4's tables at a read count a multi-rank dry run through the host
    # transport (tools/r4_dry.sh) moves in minutes
    "c4_400k": dict(kind=1, hash=0, k=21, n=4, x=8e9, reads=400_000, L=150, bigcount=True,
                    genome=0, batch_kmers=1 << 28),
    # C5 query geometry with counts that spread over 1..15 and saturate (VERDICT
    # r3 "Next round" #3): 4 x 8e9 nibbles, genomic streams at ~8x k-mer coverage
    "c5_genomic": dict(kind=7, hash=0, k=31, n=4, x=8e9, reads=4_000_000, L=150, bigcount=False,
                       genome=50_000_000, batch_kmers=1 << 27),
    "c5m_genomic": dict(kind=7, hash=1, k=51, n=4, x=8e9, reads=1_000_000, L=150, bigcount=False,
                        genome=10_000_000, batch_kmers=1 << 26),
    # BASELINE C4 (`bench.py --config C4`, 50M reads: one GPU, or strong-scaled
    # over G ranks): 4 x 8e9 bytes; 32 GB of host memory for the oracle
    "c4_50m": dict(kind=1, hash=0, k=21, n=4, x=8e9, reads=50_000_000, L=150, bigcount=True,
                   genome=0, batch_kmers=3200 << 20),
    # the secondary bench lines' own workloads (tools/bench_modes.sh; VERDICT
    # r5 #3): C3, C5 and C5M at 50M reads, C5M at BASELINE configs[4]'s 500M
    # (a read-count prefix pair: one oracle pass with --snapshots), and C2's
    # genomic stream over a 1e8-base genome
    "c3_50m": dict(kind=2, hash=0, k=31, n=4, x=4e9, reads=50_000_000, L=150, bigcount=False,
                   genome=0, batch_kmers=3200 << 20),
    "c5_50m": dict(kind=7, hash=0, k=31, n=4, x=8e9, reads=50_000_000, L=150, bigcount=False,
                   genome=0, batch_kmers=3200 << 20),
    "c5m_50m": dict(kind=7, hash=1, k=51, n=4, x=8e9, reads=50_000_000, L=150, bigcount=False,
                    genome=0, batch_kmers=3200 << 20),
    "c5m_500m": dict(kind=7, hash=1, k=51, n=4, x=8e9, reads=500_000_000, L=150, bigcount=False,
                     genome=0, batch_kmers=3200 << 20),
    "genomic_c2_50m": dict(kind=1, hash=0, k=21, n=4, x=1e9, reads=50_000_000, L=150, bigcount=True,
                           genome=100_000_000, batch_kmers=3200 << 20),
}

# Weak-scaling streams of `bench.py --gpus G` (C2, 50M reads per rank: rank r
# consumes reads [r * 50M, (r + 1) * 50M)): the whole job is reads [0, G * 50M).
# The rank-order fixtures are prefixes of one stream and are made in one oracle
# pass with snapshots (make_full_fixtures.py --snapshots).
WEAK = {"c2_w2": 2, "c2_w4": 4, "c2_w8": 8}
for _name, _g in WEAK.items():
    CONFIGS[_name] = dict(CONFIGS["c2_full"], reads=50_000_000 * _g, batch_kmers=3200 << 20)

# Exchange-mode (Option A) streams: a `world`-rank group consumes reads
# [s * reads / world, (s + 1) * reads / world) on rank s in passes that take
# the next chunk of every rank in rank order (khmer_amd.parallel.exchange_passes
# at `batch_kmers`); n_unique and the bigcount map follow that order.
EXCHANGE = {
    "c2_full_x2": ("c2_full", 2, 1600 << 20),      # tests/test_gpu_shard.py loopback
    "c2_full_x8": ("c2_full", 8, 1600 << 20),
    "c2_full_x2b": ("c2_full", 2, 3200 << 20),     # bench.py --gpus 2 --strong (default batch)
    "genomic_c2_x2": ("genomic_c2", 2, 1 << 29),
    "c4_shape_x2": ("c4_shape", 2, 1 << 28),
    "c4_shape_x8": ("c4_shape", 8, 1 << 28),
    "c4_400k_x2": ("c4_400k", 2, 3200 << 20),     # bench.py --gpus 2 --config C4 --strong --reads 400000
    "c5m_shape_x2": ("c5m_shape", 2, 1 << 26),
    "c5m_shape_x8": ("c5m_shape", 8, 1 << 26),
    "c5m_genomic_x2": ("c5m_genomic", 2, 1 << 26),
    "c5m_genomic_x8": ("c5m_genomic", 8, 1 << 26),
    # bench.py --gpus G (weak scaling, exchange mode, default batch): exact
    # n_unique / bigcounts for the driver's scaling lines
    "c2_w2_x": ("c2_w2", 2, 3200 << 20),
    "c2_w4_x": ("c2_w4", 4, 3200 << 20),
    "c2_w8_x": ("c2_w8", 8, 3200 << 20),
}
for _name, (_base, _world, _batch) in EXCHANGE.items():
    CONFIGS[_name] = dict(CONFIGS[_base], exchange=[_world, _batch])

# Delta-mode (KH_GROUP_DELTA) streams: passes of up to `batch_kmers` k-mers of
# every rank's reads, the rank chunks of a pass in rank order
# (khmer_amd.parallel.delta_passes); n_unique and the bigcount map follow it.
DELTA = {
    # bench.py --gpus G (weak scaling, the default group mode and batch): the
    # driver's scaling lines
    "c2_w2_d": ("c2_w2", 2, 3200 << 20),
    "c2_w4_d": ("c2_w4", 4, 3200 << 20),
    "c2_w8_d": ("c2_w8", 8, 3200 << 20),
    # the bench's multi-rank dry run on one GPU (KH_BENCH_DEVICE, host
    # transport): two ranks' buffers on one device need a smaller batch
    "c2_w2_d800": ("c2_w2", 2, 800 << 20),
    # loopback tests (tests/test_gpu_shard.py): several passes per rank
    "c2_full_d2": ("c2_full", 2, 1600 << 20),
    "genomic_c2_d2": ("genomic_c2", 2, 1 << 28),
    "c4_shape_d2": ("c4_shape", 2, 1 << 28),
}
for _name, (_base, _world, _batch) in DELTA.items():
    CONFIGS[_name] = dict(CONFIGS[_base], delta=[_world, _batch])


def stream_chunks(c, step=1_000_000):
    """[(r0, nreads)] in the order the configuration's stream consumes them:
    the reads in order, or a group mode's pass interleave
    (khmer_amd.parallel.group_stream)."""
    from khmer_amd.parallel import group_stream
    for mode in ("exchange", "delta"):
        if mode in c:
            world, batch = c[mode]
            return group_stream(mode, c["reads"] // world, c["L"], c["k"], world, batch, step=step)
    return [(r0, min(step, c["reads"] - r0)) for r0 in range(0, c["reads"], step)]


def sha256_view(mv, chunk=1 << 28):
    h = hashlib.sha256()
    for a in range(0, len(mv), chunk):
        h.update(mv[a:a + chunk])
    return h.hexdigest()


def bigcount_digest(d):
    keys = sorted(d)
    blob = b"".join(struct.pack("<QH", k, d[k]) for k in keys)
    return len(keys), hashlib.sha256(blob).hexdigest()


def median_digest(med, avg, sd):
    """SHA-256 of get_median_count's outputs over a read range: the u16
    medians, then the f32 averages, then the f32 stddevs (little-endian
    arrays, bit patterns exactly)."""
    import numpy as np
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(med, dtype="<u2").tobytes())
    h.update(np.ascontiguousarray(avg, dtype="<f4").tobytes())
    h.update(np.ascontiguousarray(sd, dtype="<f4").tobytes())
    return h.hexdigest()


# get_median_count digests over the first MEDIAN_READS reads of the stream,
# for the configurations whose query path the bench measures (C5 / C5M)
MEDIAN_READS = {"c5_shape": 1_000_000, "c5m_shape": 1_000_000, "c5_genomic": 1_000_000, "c5m_genomic": 1_000_000,
                "c5_50m": 1_000_000, "c5m_50m": 1_000_000}


def fixture_path(name):
    return os.path.join(FULL, name + ".json")


def load(name):
    with open(fixture_path(name)) as fh:
        return json.load(fh)
