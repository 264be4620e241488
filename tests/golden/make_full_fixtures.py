#!/usr/bin/env python3
"""Generate the full-size golden fixtures in tests/golden/full/ with the oracle
(oracle/khmer_oracle.c, single thread, stream order = the reference's
single-threaded semantics).  Each fixture holds the per-table SHA-256, the
counters and the bigcount-map digest of one tests/full_digest.CONFIGS entry.

    python tests/golden/make_full_fixtures.py c2_full c3_shape ...

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


def make(name):
    c = FD.CONFIGS[name]
    sizes = O.get_n_primes_near_x(c["n"], c["x"])
    t = O.Table(c["kind"], c["k"], sizes, hash=c["hash"])
    t.set_use_bigcount(c["bigcount"])
    t0 = time.time()
    kmers = 0
    for r0, nr in FD.stream_chunks(c):
        kmers += t.consume_synth(synth.SEED, r0, nr, c["L"], genome=c["genome"])
    secs = time.time() - t0
    nbc, bcd = FD.bigcount_digest(t.bigcounts())
    out = {
        "config": name, "params": c, "seed": synth.SEED, "table_sizes": sizes,
        "n_consumed": kmers, "n_unique_kmers": t.n_unique_kmers(), "n_occupied": t.n_occupied(),
        "table_sha256": [FD.sha256_view(t.table_view(i)) for i in range(c["n"])],
        "n_bigcounts": nbc, "bigcount_sha256": bcd,
        "generator": "tests/golden/make_full_fixtures.py (oracle, 1 thread, %.0f s)" % secs,
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


if __name__ == "__main__":
    for name in sys.argv[1:] or sorted(FD.CONFIGS):
        make(name)
