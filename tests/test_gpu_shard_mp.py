"""The one-process-per-rank sharding protocol, multi-process, on one GPU.

RCCL refuses two ranks on one device, so here every rank is its own process
whose group runs the host transport (kh_group_create_hosted): the same
per-rank code path as the RCCL build -- every collective of
group_consume_fixed / group_route_winners / group_merge_full / group_counters
in the same order -- with each collective staged through host memory and the
TCP rendezvous (khmer_amd.rendezvous) instead of xGMI.  Rank s's reads are the
s-th block of the synthetic stream; the oracle consumes the concatenation.
Tables (re-interleaved from every rank's slices), n_unique, n_occupied and
the replicated bigcount maps must equal the oracle's exactly."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

KINDS = {"Countgraph": 1, "Nodegraph": 2, "SmallCountgraph": 7, "Counttable": 1, "SmallCounttable": 7}


def _rank_main():
    """Body of one rank (run as a subprocess by the test)."""
    sys.path.insert(0, ROOT)
    from khmer_amd import parallel, synth, _lib
    from khmer_amd._lib import lib, check
    from khmer_amd.rendezvous import Rendezvous
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    cfg = json.loads(os.environ["KH_MP_CFG"])
    _lib.set_default_device(0)
    rdv = Rendezvous(rank, world, "127.0.0.1", int(os.environ["KH_RDV_PORT"]), timeout=120)
    tp = parallel.HostTransport(rdv)
    g = parallel.ShardedGraph(cfg["cls"], cfg["k"], cfg["sizes"], world, rank, 0, transport=tp, mode=cfg["mode"])
    g.set_batch_kmers(cfg["batch"])
    if cfg["bigcount"]:
        g.set_use_bigcount(True)
    n, L, k = cfg["nreads"], cfg["L"], cfg["k"]
    words, koff = ctypes.c_void_p(), ctypes.c_void_p()
    check(lib.kh_device_malloc(0, (n * L // 32 + 2) * 8, ctypes.byref(words)))
    check(lib.kh_device_malloc(0, (n + 1) * 8, ctypes.byref(koff)))
    ks = min(k, 32)
    if cfg["genome"]:
        check(lib.kh_synth_genomic_device(0, synth.SEED, cfg["genome"], rank * n, n, L, ks, words, koff))
    else:
        check(lib.kh_synth_packed_device(0, synth.SEED, rank * n, n, L, ks, words, koff))
    reads = words
    if g.murmur:   # the Counttable family: ASCII reads
        reads = ctypes.c_void_p()
        check(lib.kh_device_malloc(0, n * L + 64, ctypes.byref(reads)))
        check(lib.kh_unpack_ascii_device(0, words, n * L, reads))
        g.consume_bytes_fixed_device([reads], n, L)
    else:
        g.consume_packed_fixed_device([words], n, L)
    u, occ = g.counters()
    tabs = g.gather_tables(rdv)
    bc = g.shards[0].bigcounts()
    out = {"rank": rank, "n_unique": u, "n_occupied": occ, "bigcounts": [[int(a), int(b)] for a, b in bc],
           "comm": g.comm_info()}
    if cfg.get("query"):   # the sharded get_median_count of this rank's own reads
        import numpy as np
        q = ctypes.c_void_p()
        check(lib.kh_device_malloc(0, n * 10 + 64, ctypes.byref(q)))
        g.median_fixed_device([reads], n, L, [q.value], [q.value + 2 * n], [q.value + 6 * n])
        raw = (ctypes.c_uint8 * (n * 10))()
        check(lib.kh_device_copy(0, raw, q, n * 10))
        lib.kh_device_free(0, q)
        b = bytes(raw)
        out["median"] = np.frombuffer(b[:2 * n], np.uint16).tolist()
        out["avg_sd_hex"] = b[2 * n:].hex()
    if g.murmur:
        lib.kh_device_free(0, reads)
    if rank == 0:
        import hashlib
        out["tables"] = [hashlib.sha256(t).hexdigest() for t in tabs]
    print("RESULT " + json.dumps(out), flush=True)
    lib.kh_device_free(0, words)
    lib.kh_device_free(0, koff)
    g.close()
    rdv.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("cls,world,bigcount,exchange,query",
                         [("Countgraph", 2, True, False, False), ("Countgraph", 3, True, False, False),
                          ("Nodegraph", 2, False, False, False),
                          ("SmallCountgraph", 3, False, False, False),
                          ("Countgraph", 2, True, True, False), ("Countgraph", 3, True, True, False),
                          ("Nodegraph", 2, False, True, False),
                          # the Counttable family and the sharded get_median_count (round 4)
                          ("SmallCounttable", 2, False, False, True), ("SmallCounttable", 3, False, True, True),
                          ("Counttable", 2, True, True, True), ("Countgraph", 3, True, False, True),
                          # delta mode (round 5): table-byte alltoallv both ways
                          ("Countgraph", 2, True, "delta", False), ("Countgraph", 3, True, "delta", True),
                          ("Nodegraph", 2, False, "delta", False), ("SmallCountgraph", 3, False, "delta", False),
                          ("SmallCounttable", 2, False, "delta", True)])
def test_hosted_group_multiprocess(cls, world, bigcount, exchange, query):
    """exchange=True: Option A through the host transport's alltoallv (the
    oracle consumes the pass-interleaved stream, parallel.exchange_passes);
    exchange="delta": delta mode (table-byte alltoallv to the owners and
    back, parallel.delta_passes).
    query=True: every rank's get_median_count of its own reads through the
    host transport's MIN reduce (broadcast) / reduce-scatter (exchange),
    against the oracle's per-read (median, average, stddev) bit patterns."""
    import hashlib
    import numpy as np
    from oracle import oracle as O
    from khmer_amd import parallel, synth
    murmur = cls in parallel.MURMUR_CLASSES
    k = 51 if cls == "SmallCounttable" else 21
    sizes = O.get_n_primes_near_x(4, 100003)
    # bigcount cases read a 6 kbp genome (every k-mer ~400x, past 255 in all
    # tables); the query cases a 40 kbp genome; the others the iid stream
    genome = 6000 if bigcount else 40000 if query else 0
    mode = "delta" if exchange == "delta" else "exchange" if exchange else "broadcast"
    cfg = {"cls": cls, "k": k, "sizes": sizes, "batch": 1 << 20, "bigcount": bigcount, "nreads": 20000, "L": 150,
           "genome": genome, "mode": mode, "query": query}
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), KH_RDV_PORT=str(port), KH_MP_CFG=json.dumps(cfg))
        procs.append(subprocess.Popen([sys.executable, "-c", "import tests.test_gpu_shard_mp as t; t._rank_main()"],
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            so, _ = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, so[-3000:]
        outs.append(json.loads([ln for ln in so.splitlines() if ln.startswith("RESULT ")][-1][7:]))
    o = O.Table(KINDS[cls], k, sizes, hash=O.MURMUR if murmur else O.TWOBIT)
    o.set_use_bigcount(bigcount)
    n = cfg["nreads"]
    order = parallel.group_stream(mode, n, cfg["L"], k, world, cfg["batch"])
    for start, cnt in order:
        if genome:
            seqs, offs = synth.genomic_batch(start, cnt, cfg["L"], genome)
        else:
            seqs, offs = synth.batch(start, cnt, cfg["L"])
        o.consume_batch(seqs, [int(v) for v in offs])
    r0 = [x for x in outs if x["rank"] == 0][0]
    assert r0["tables"] == [hashlib.sha256(o.table_bytes(i)).hexdigest() for i in range(len(sizes))]
    ref_bc = sorted([int(a), int(b)] for a, b in o.bigcounts().items())
    for x in outs:
        assert (x["n_unique"], x["n_occupied"]) == (o.n_unique_kmers(), o.n_occupied())
        assert x["bigcounts"] == ref_bc
        assert x["comm"] == [0, -1]   # no RCCL in a host-transport group
    if bigcount:
        assert ref_bc, "the case should exercise the bigcount merge"
    if query:
        L = cfg["L"]
        got_med = np.concatenate([np.array(x["median"], np.uint16) for x in sorted(outs, key=lambda x: x["rank"])])
        got_f = b"".join(bytes.fromhex(x["avg_sd_hex"]) for x in sorted(outs, key=lambda x: x["rank"]))
        want_med, want_f = [], b""
        for s in range(world):
            seqs = synth.genomic_batch(s * n, n, L, genome)[0]
            m, a, d = np.zeros(n, np.uint16), np.zeros(n, np.float32), np.zeros(n, np.float32)
            for r in range(n):
                m[r], a[r], d[r] = o.median(seqs[r * L:(r + 1) * L])
            want_med.append(m)
            want_f += a.tobytes() + d.tobytes()
        assert np.array_equal(got_med, np.concatenate(want_med))
        assert got_f == want_f
        assert int(got_med.max()) > 2
