#!/usr/bin/env python3
"""Generate the full-size golden fixtures in tests/golden/full/ with the oracle
(oracle/khmer_oracle.c, single thread, stream order = the reference's
single-threaded semantics).  Each fixture holds the per-table SHA-256, the
counters and the bigcount-map digest of one tests/full_digest.CONFIGS entry.

    python tests/golden/make_full_fixtures.py c2_full c3_shape ...
    python tests/golden/make_full_fixtures.py --snapshots c2_w2 c2_w4 c2_w8
    KH_FIXTURE_THREADS=6 python tests/golden/make_full_fixtures.py c5m_500m

KH_FIXTURE_THREADS > 1: the oracle's or_consume_synth_mt (hashing on worker
threads, one thread per table, flags combined in stream order: the same
tables and counters, tests/test_oracle_mt_cpu.py) -- ~10 M k-mers/s for the
Murmur k=51 stream instead of ~2.3 M.

--snapshots: configurations that differ only in their read count and are
consumed in stream order (no exchange interleave) are prefixes of one stream;
one oracle pass writes each fixture when the stream reaches its read count.

Runs on the CPU (the c2_full run hashes 6.5e9 k-mers: ~7 min, 4 GB of tables;
c4_shape needs 32 GB of host memory)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from khmer_amd import synth  # noqa: E402
from tests import full_digest as FD  # noqa: E402

THREADS = int(os.environ.get("KH_FIXTURE_THREADS", "1"))


def _table(c):
    sizes = O.get_n_primes_near_x(c["n"], c["x"])
    t = O.Table(c["kind"], c["k"], sizes, hash=c["hash"])
    t.set_use_bigcount(c["bigcount"])
    return t, sizes


def _write(name, c, t, sizes, kmers, secs, note=""):
    nbc, bcd = FD.bigcount_digest(t.bigcounts())
    out = {
        "config": name, "params": c, "seed": synth.SEED, "table_sizes": sizes,
        "n_consumed": kmers, "n_unique_kmers": t.n_unique_kmers(), "n_occupied": t.n_occupied(),
        "table_sha256": [FD.sha256_view(t.table_view(i)) for i in range(c["n"])],
        "n_bigcounts": nbc, "bigcount_sha256": bcd,
        "generator": "tests/golden/make_full_fixtures.py (oracle, 1 thread, %.0f s%s)" % (secs, note),
    }
    nmed = FD.MEDIAN_READS.get(name)
    if nmed:
        t0 = time.time()
        med, avg, sd = t.median_synth(synth.SEED, 0, nmed, c["L"], genome=c["genome"])
        out["median_reads"] = nmed
        out["median_sha256"] = FD.median_digest(med, avg, sd)
        out["median_max"] = int(med.max())
        import numpy as np
        out["median_hist"] = np.bincount(med.astype(np.int64), minlength=16)[:16].tolist()
        out["generator"] += ", median digest %.0f s" % (time.time() - t0)
    os.makedirs(FD.FULL, exist_ok=True)
    with open(FD.fixture_path(name), "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")
    print(name, json.dumps({k: out[k] for k in ("n_consumed", "n_unique_kmers", "n_occupied", "n_bigcounts")}),
          "%.0f s" % secs, flush=True)


def make(name):
    c = FD.CONFIGS[name]
    t, sizes = _table(c)
    t0 = time.time()
    kmers = 0
    for r0, nr in FD.stream_chunks(c):
        kmers += t.consume_synth(synth.SEED, r0, nr, c["L"], genome=c["genome"], threads=THREADS)
    _write(name, c, t, sizes, kmers, time.time() - t0, ", %d hash threads" % THREADS if THREADS > 1 else "")


def make_snapshots(names):
    """One stream-order pass over the longest configuration's reads, writing
    every named fixture when the stream reaches its read count."""
    cs = [FD.CONFIGS[n] for n in names]
    base = {k: v for k, v in cs[0].items() if k != "reads"}
    for n, c in zip(names, cs):
        if "exchange" in c or {k: v for k, v in c.items() if k != "reads"} != base:
            raise SystemExit("--snapshots: %s is not a read-count prefix of %s" % (n, names[0]))
    marks = sorted((c["reads"], n) for n, c in zip(names, cs))
    last = marks[-1][0]
    t, sizes = _table(cs[0])
    t0 = time.time()
    kmers, r0, step = 0, 0, 1_000_000
    while marks:
        nr = min(step, marks[0][0] - r0)
        kmers += t.consume_synth(synth.SEED, r0, nr, base["L"], genome=base["genome"], threads=THREADS)
        r0 += nr
        while marks and marks[0][0] == r0:
            _, n = marks.pop(0)
            _write(n, FD.CONFIGS[n], t, sizes, kmers, time.time() - t0,
                   ", snapshot at read %d of a %d-read pass%s" % (r0, last, ", %d hash threads" % THREADS
                                                                  if THREADS > 1 else ""))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--snapshots"]:
        make_snapshots(sys.argv[2:])
    else:
        for name in sys.argv[1:] or sorted(FD.CONFIGS):
            make(name)
