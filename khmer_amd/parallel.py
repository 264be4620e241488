"""Multi-GPU sharded Countgraph/Nodegraph.

The reference has no multi-device path; its own hash-space sharding
precedent is k-mer banding (src/oxli/hashtable.cc:192-228,
src/oxli/kmer_hash.cc:262-276), which yields byte-identical tables.  Here a
G-rank group splits every table by bin ownership: rank r holds the contiguous,
8-bin aligned slice [shard_lo(p, G, r), shard_lo(p, G, r + 1)) of each table
(the reference's table layout is recovered by concatenating the slices,
`reinterleave`).  Reads are consumed as one stream in rank order: each source
rank's packed reads are broadcast over RCCL (xGMI), every rank hashes every
k-mer and applies only the updates of the bins it owns (owner-computes), so
the tables are exactly the single-device tables.  n_unique / n_occupied /
bigcounts stay exact (see include/khmer_hip.h, kh_group_*).

Process model: one process per GPU (torchrun or any launcher that sets
RANK / WORLD_SIZE / MASTER_ADDR); a small TCP rendezvous
(khmer_amd.rendezvous, no PyTorch) carries the RCCL unique id, barriers and
the max-over-ranks timing; the data path is the library's own RCCL
communicator.  Two other transports run the same protocol where RCCL cannot:
`loopback=True` holds every shard in one process on one device (device
copies), and `transport=HostTransport(rendezvous)` keeps one shard per
process but routes the collectives through host memory and the rendezvous
(several processes sharing one GPU, as on the one-GPU test box).
"""
import ctypes

from . import _lib
from ._lib import lib, check

KIND = {"Countgraph": _lib.STORAGE_BYTE, "Nodegraph": _lib.STORAGE_BIT, "SmallCountgraph": _lib.STORAGE_NIBBLE,
        # the Counttable family: MurmurHash3 over ASCII k-mers (include/oxli/hashtable.hh:494-627)
        "Counttable": _lib.STORAGE_BYTE, "Nodetable": _lib.STORAGE_BIT, "SmallCounttable": _lib.STORAGE_NIBBLE}
MURMUR_CLASSES = {"Counttable", "Nodetable", "SmallCounttable"}


def shard_lo(p, world, r):
    """First bin of shard r of a p-bin table (kh_internal.h shard_lo)."""
    if r >= world:
        return p
    return (p * r // world) & ~7


def shard_slices(sizes, world):
    """[(lo, size)] per rank per table."""
    return [[(shard_lo(p, world, r), shard_lo(p, world, r + 1) - shard_lo(p, world, r)) for p in sizes]
            for r in range(world)]


def _slice_nbytes(kind, lo, size, p):
    """Bytes a rank slice [lo, lo + size) of a p-bin table contributes to the
    reference layout: whole bytes of its bins, plus the table's spare trailing
    byte (storage.hh) on the slice that ends the table."""
    last = size > 0 and lo + size == p
    if kind == _lib.STORAGE_BIT:
        return size // 8 + (1 if last else 0)
    if kind == _lib.STORAGE_NIBBLE:
        return size // 2 + (1 if last else 0)
    return size


def reinterleave(kind, p, parts, slices=None):
    """Table bytes of a p-bin table from its rank slices (in rank order);
    slices = [(lo, size)] per rank (default: the broadcast-mode shard_lo
    slices).  Non-final Bit/Nibble slices are whole bytes followed by one spare
    byte."""
    world = len(parts)
    if slices is None:
        slices = [(shard_lo(p, world, r), shard_lo(p, world, r + 1) - shard_lo(p, world, r)) for r in range(world)]
    out = bytearray()
    for part, (lo, size) in zip(parts, slices):
        out += bytes(part[:_slice_nbytes(kind, lo, size, p)])
    return bytes(out)


MAX_PASS_KMERS = 3200 << 20   # kh_internal.h


def exchange_passes(nreads, read_len, k, world, batch_kmers):
    """[(r0, nr)]: the passes an exchange-mode group takes from every rank's
    `nreads` reads (kh_engine.hip group_consume_a2a).  Pass p's stream is
    reads [r0, r0 + nr) of rank 0, then of rank 1, ...; n_unique and the
    bigcounts are exact for that order."""
    kpr = read_len - k + 1
    cap = min(int(batch_kmers), MAX_PASS_KMERS) // world
    rpb0 = max(1, (cap - 16 if cap > 16 else 1) // kpr)
    npass = max(1, -(-nreads // rpb0))
    rpb = max(1, -(-nreads // npass))
    return [(r0, min(rpb, nreads - r0)) for r0 in range(0, nreads, rpb)]


def delta_passes(nreads, read_len, k, batch_kmers):
    """[(r0, nr)]: the passes a delta-mode group takes from every rank's
    `nreads` reads (kh_engine.hip group_consume_delta): up to one device pass
    of every rank's own reads, the rank chunks of a pass in rank order."""
    return exchange_passes(nreads, read_len, k, 1, batch_kmers)


def group_stream(mode, nreads, read_len, k, world, batch_kmers, step=None):
    """[(first read, count)] of the whole group's stream in the order a
    `mode` group consumes it, rank r holding reads [r * nreads, (r + 1) *
    nreads): rank order (broadcast), or pass by pass with the rank chunks of a
    pass in rank order (exchange: exchange_passes; delta: delta_passes).
    `step` splits the pieces further (the oracle's batch size)."""
    if mode == "broadcast":
        plan = [(0, nreads)]
    elif mode == "exchange":
        plan = exchange_passes(nreads, read_len, k, world, batch_kmers)
    elif mode == "delta":
        plan = delta_passes(nreads, read_len, k, batch_kmers)
    else:
        raise ValueError("unknown group mode %r" % (mode,))
    out = []
    pieces = [(s * nreads + r0, nr) for r0, nr in plan for s in range(world)]
    for a, n in pieces:
        if step:
            out += [(a + x, min(step, n - x)) for x in range(0, n, step)]
        else:
            out.append((a, n))
    return out


def window_owner_range(fj, world, r):
    """k-mer windows [lo, hi) whose winners rank r unions (kh_engine.hip group_wlo)."""
    return fj * r // world, fj * (r + 1) // world


class _ShardView(object):
    """Non-owning handle of one local shard (kh_group_shard)."""

    def __init__(self, handle):
        self._g = handle

    def __del__(self):
        if self._g:
            lib.kh_graph_destroy(self._g)
            self._g = None

    def bigcounts(self):
        n = ctypes.c_uint64()
        check(lib.kh_graph_get_bigcounts(self._g, None, None, 0, ctypes.byref(n)))
        keys = (ctypes.c_uint64 * max(n.value, 1))()
        vals = (ctypes.c_uint16 * max(n.value, 1))()
        check(lib.kh_graph_get_bigcounts(self._g, keys, vals, n.value, ctypes.byref(n)))
        return list(zip(keys[:n.value], vals[:n.value]))

    def table_bytes(self, i):
        n = ctypes.c_uint64()
        check(lib.kh_graph_table_nbytes(self._g, i, ctypes.byref(n)))
        buf = (ctypes.c_uint8 * max(n.value, 1))()
        check(lib.kh_graph_copy_table(self._g, i, buf))
        return bytes(buf[:n.value])


def _read_mem(addr, n):
    """n bytes at addr as bytes: ctypes.string_at takes a C int size, so
    blocks over 2 GiB are read in pieces."""
    piece = 1 << 30
    if n <= piece:
        return ctypes.string_at(addr, n)
    return b"".join(ctypes.string_at(addr + a, min(piece, n - a)) for a in range(0, n, piece))


_AG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64)
_BC = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int)
_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class _KhTransport(ctypes.Structure):   # include/khmer_hip.h kh_transport
    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", _AG), ("broadcast", _BC), ("alltoallv", _A2A)]


class HostTransport(object):
    """kh_transport over a rendezvous (khmer_amd.rendezvous.Rendezvous or any
    object with allgather / broadcast / alltoallv of byte strings).  A failed
    collective is reported to the library (a failed call on this rank) and
    aborts the rendezvous (if it has abort()), so the peer ranks fail too
    instead of waiting for this one."""

    def __init__(self, rdv):
        self.rdv = rdv
        self.error = None
        world = rdv.world

        import time as _time
        beat = {"t": _time.time(), "n": 0}

        def _beat(fn):
            """A progress line on rank 0's stderr at most every 20 s: a long
            host-transport consume (the bench's multi-rank dry run moves GBs
            per pass through the rendezvous) keeps writing."""
            def call(*a):
                rc = fn(*a)
                beat["n"] += 1
                if rdv.rank == 0 and _time.time() - beat["t"] > 20:
                    import sys
                    beat["t"] = _time.time()
                    sys.stderr.write("host transport: %d collectives done\n" % beat["n"])
                    sys.stderr.flush()
                return rc
            return call

        def failed(e):
            import sys
            self.error = e
            sys.stderr.write("khmer_amd host transport (rank %d): %r\n" % (rdv.rank, e))
            abort = getattr(rdv, "abort", None)
            if abort is not None:
                try:
                    abort()
                except Exception:
                    pass
            return 1

        def allgather(ctx, send, recv, nbytes):
            try:
                parts = rdv.allgather(_read_mem(send, nbytes) if nbytes else b"")
                ctypes.memmove(recv, b"".join(parts), nbytes * world)
                return 0
            except Exception as e:   # reported to the library as a failed collective
                return failed(e)

        def broadcast(ctx, buf, nbytes, root):
            try:
                data = rdv.broadcast(_read_mem(buf, nbytes) if rdv.rank == root else b"", root)
                if rdv.rank != root:
                    ctypes.memmove(buf, data, nbytes)
                return 0
            except Exception as e:
                return failed(e)

        def alltoallv(ctx, send, send_bytes, recv, recv_bytes):
            try:
                blocks, at = [], 0
                for d in range(world):
                    n = send_bytes[d]
                    blocks.append(_read_mem(send + at, n) if n else b"")
                    at += n
                got = rdv.alltoallv(blocks)
                at = 0
                for s in range(world):
                    n = recv_bytes[s]
                    if len(got[s]) != n:
                        raise ValueError("alltoallv: %d bytes from rank %d, expected %d" % (len(got[s]), s, n))
                    if n:
                        ctypes.memmove(recv + at, got[s], n)
                    at += n
                return 0
            except Exception as e:
                return failed(e)

        self._fns = (_AG(_beat(allgather)), _BC(_beat(broadcast)), _A2A(_beat(alltoallv)))
        self.struct = _KhTransport(None, *self._fns)


class ShardedGraph(object):
    """A Countgraph/Nodegraph/SmallCountgraph split over `world` ranks."""

    def __init__(self, cls, k, sizes, world, rank=0, device=0, loopback=False, uid=None, transport=None,
                 exchange=False, mode=None):
        """mode: "broadcast" (Option B, the default), "exchange" (Option A;
        also exchange=True) or "delta" (table deltas, include/khmer_hip.h
        KH_GROUP_DELTA)."""
        self._h = None
        self.shards = []
        self.kind = KIND[cls]
        self.murmur = cls in MURMUR_CLASSES
        hash_kind = _lib.HASH_MURMUR if self.murmur else _lib.HASH_TWOBIT
        self.k, self.sizes, self.world = k, [int(x) for x in sizes], world
        self.loopback = loopback
        self.transport = transport
        nlocal = world if loopback else 1
        devs = (ctypes.c_int * nlocal)(*([device] * nlocal))
        arr = (ctypes.c_uint64 * len(sizes))(*self.sizes)
        h = ctypes.c_void_p()
        self.mode = mode or ("exchange" if exchange else "broadcast")
        mode = _lib.GROUP_MODES[self.mode]
        self.exchange = self.mode != "broadcast"   # bucket-aligned ownership (exchange / delta)
        if transport is not None:
            check(lib.kh_group_create_hosted_mode(self.kind, hash_kind, k, arr, len(sizes), world, rank,
                                                  device, ctypes.byref(transport.struct), mode, ctypes.byref(h)))
        else:
            check(lib.kh_group_create_mode(self.kind, hash_kind, k, arr, len(sizes), world, rank, nlocal,
                                           devs, uid, mode, ctypes.byref(h)))
        self._h = h
        w, nl, r0 = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.kh_group_info(h, ctypes.byref(w), ctypes.byref(nl), ctypes.byref(r0)))
        self.nlocal, self.rank0 = nl.value, r0.value
        self.shards = []
        for l in range(self.nlocal):
            v = ctypes.c_void_p()
            check(lib.kh_group_shard(h, l, ctypes.byref(v)))
            self.shards.append(_ShardView(v))

    def close(self):
        self.shards = []
        if self._h:
            lib.kh_group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        check(lib.kh_group_unique_id(buf, 128))
        return buf.raw

    def comm_info(self):
        """(nranks, device) as RCCL reports them (0, -1 without RCCL)."""
        n, d = ctypes.c_int(), ctypes.c_int()
        check(lib.kh_group_comm_info(self._h, ctypes.byref(n), ctypes.byref(d)))
        return n.value, d.value

    def slice(self, l, table):
        lo, n = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.kh_group_slice(self._h, l, table, ctypes.byref(lo), ctypes.byref(n)))
        return lo.value, n.value

    def rank_slices(self, table):
        """[(lo, size)] of table `table` for every rank, in rank order."""
        out = []
        for r in range(self.world):
            lo, n = ctypes.c_uint64(), ctypes.c_uint64()
            check(lib.kh_group_rank_slice(self._h, r, table, ctypes.byref(lo), ctypes.byref(n)))
            out.append((lo.value, n.value))
        return out

    def set_use_bigcount(self, flag):
        for s in self.shards:
            check(lib.kh_graph_set_use_bigcount(s._g, 1 if flag else 0))

    def set_batch_kmers(self, n):
        for s in self.shards:
            check(lib.kh_graph_set_batch_kmers(s._g, int(n)))

    def set_profiling(self, on):
        for s in self.shards:
            check(lib.kh_graph_set_profiling(s._g, 1 if on else 0))

    def clear(self):
        for s in self.shards:
            check(lib.kh_graph_clear(s._g))

    def consume_packed_fixed_device(self, d_words, nreads, read_len):
        """Collective: d_words = one device pointer per local shard (its own reads)."""
        ptrs = (ctypes.c_void_p * len(d_words))(*[int(p) if not isinstance(p, ctypes.c_void_p) else p.value
                                                   for p in d_words])
        check(lib.kh_group_consume_packed_fixed_device(self._h, ptrs, int(nreads), int(read_len)))

    @staticmethod
    def _ptrs(ps):
        return (ctypes.c_void_p * len(ps))(*[int(p) if not isinstance(p, ctypes.c_void_p) else p.value for p in ps])

    def consume_bytes_fixed_device(self, d_bytes, nreads, read_len):
        """Collective (Counttable family): d_bytes = one device pointer per
        local shard to its own ASCII fixed-length reads."""
        check(lib.kh_group_consume_bytes_fixed_device(self._h, self._ptrs(d_bytes), int(nreads), int(read_len)))

    def median_fixed_device(self, d_reads, nreads, read_len, d_med, d_avg, d_sd):
        """Collective get_median_count (src/oxli/hashtable.cc:299-328) of every
        rank's own fixed-length reads (packed words, or ASCII bytes for the
        Counttable family); outputs into the device arrays d_med / d_avg /
        d_sd (one pointer per local shard, one entry per read)."""
        check(lib.kh_group_median_fixed_device(self._h, self._ptrs(d_reads), int(nreads), int(read_len),
                                               self._ptrs(d_med), self._ptrs(d_avg), self._ptrs(d_sd)))

    def counters(self):
        """(n_unique_kmers, n_occupied) of the whole group (collective)."""
        u, o = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.kh_group_counters(self._h, ctypes.byref(u), ctypes.byref(o)))
        return u.value, o.value

    def wire_stats(self):
        """Delta mode: (dense, sent) bytes of the table pieces exchanged with
        other ranks so far (sparse pieces: bitmap + nonzero bytes)."""
        d, t = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.kh_group_wire_stats(self._h, ctypes.byref(d), ctypes.byref(t)))
        return d.value, t.value

    def local_tables(self):
        """[[slice bytes per table] per local shard]."""
        return [[s.table_bytes(i) for i in range(len(self.sizes))] for s in self.shards]

    def table_sha256(self):
        """SHA-256 of every reference-layout table of a loopback (or 1-rank)
        group, hashed slice by slice in rank order: no table is assembled in
        host memory (C4's 8 GB tables)."""
        import hashlib
        if not (self.loopback or self.world == 1):
            raise ValueError("table_sha256: loopback groups only (ShardedCountgraphBench.table_sha256 otherwise)")
        out = []
        for i, p in enumerate(self.sizes):
            h = hashlib.sha256()
            for r, (lo, size) in enumerate(self.rank_slices(i)):
                sh = self.shards[r]
                n = ctypes.c_uint64()
                check(lib.kh_graph_table_nbytes(sh._g, i, ctypes.byref(n)))
                buf = (ctypes.c_uint8 * max(n.value, 1))()
                check(lib.kh_graph_copy_table(sh._g, i, buf))
                h.update(memoryview(buf).cast("B")[:_slice_nbytes(self.kind, lo, size, p)])
                del buf
            out.append(h.hexdigest())
        return out

    def gather_tables(self, rdv=None):
        """Reference-layout table bytes of the whole group.  Loopback: from the
        local shards; one process per rank: every rank's slices through the
        rendezvous `rdv` (khmer_amd.rendezvous.Rendezvous)."""
        if self.loopback or self.world == 1:
            parts = self.local_tables()
        else:
            mine = self.local_tables()[0]
            parts = [[] for _ in range(self.world)]
            for i in range(len(self.sizes)):
                for r, blob in enumerate(rdv.allgather(mine[i])):
                    parts[r].append(blob)
        return [reinterleave(self.kind, p, [parts[r][i] for r in range(self.world)], self.rank_slices(i))
                for i, p in enumerate(self.sizes)]


class ShardedCountgraphBench(object):
    """bench.py runner for --gpus N > 1 (one process per GPU, torchrun)."""

    def __init__(self, args, rank, world, local, sizes):
        self.args, self.rank, self.world, self.device, self.sizes = args, rank, world, local, sizes

    def config_name(self):
        a = self.args
        return a.graph + " k=%d %dx%.0e sharded over %dxMI355X%s, %s%d x %d bp synthetic %sreads per GPU%s" % (
            a.k, a.tables, a.x, self.world,
            {"exchange": " (exchange: each rank hashes its own reads, buckets sent to owners)",
             "delta": " (delta: each rank counts its own reads, table deltas to owners, prefixes back)"}.get(
                getattr(a, "group_mode", "broadcast"), ""), "get_median_count over " if a.query else "", a.reads, a.read_len,
            "genomic " if a.genome else "",
            " (strong scaling: %d reads in all)" % (a.reads * self.world) if a.strong else "")

    def setup(self):
        from . import synth
        from .rendezvous import Rendezvous
        import os
        a = self.args
        self.rdv = Rendezvous(self.rank, self.world)
        # RCCL (one GPU per rank); "host": the collectives through host memory
        # and the rendezvous -- the dry run of several ranks on one device
        # (KH_BENCH_DEVICE), which RCCL refuses ("Duplicate GPU detected")
        self.transport = os.environ.get("KH_BENCH_TRANSPORT", "host" if "KH_BENCH_DEVICE" in os.environ else "rccl")
        mode = getattr(a, "group_mode", "broadcast")
        if self.transport == "host":
            self.g = ShardedGraph(a.graph, a.k, self.sizes, self.world, self.rank, self.device,
                                  transport=HostTransport(self.rdv), mode=mode)
        else:
            uid = self.rdv.broadcast(ShardedGraph.unique_id() if self.rank == 0 else b"", 0)
            self.g = ShardedGraph(a.graph, a.k, self.sizes, self.world, self.rank, self.device, uid=uid, mode=mode)
        nranks, dev = self.g.comm_info()
        self.comm = [tuple(int(x) for x in p.split(b",")) for p in
                     self.rdv.allgather(b"%d,%d,%d" % (self.rank, nranks, dev))]
        if a.bigcount:
            self.g.set_use_bigcount(True)
        self.g.set_batch_kmers(a.batch_kmers)
        nwords = a.reads * a.read_len // 32 + 2
        self.words, self.koff = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib.kh_device_malloc(self.device, nwords * 8, ctypes.byref(self.words)))
        check(lib.kh_device_malloc(self.device, (a.reads + 1) * 8, ctypes.byref(self.koff)))
        # every rank's own reads: the rank-th block of the synthetic stream
        ks = min(a.k, 32)   # the packed stream itself does not depend on k
        if a.genome:
            check(lib.kh_synth_genomic_device(self.device, synth.SEED, a.genome, self.rank * a.reads, a.reads,
                                              a.read_len, ks, self.words, self.koff))
        else:
            check(lib.kh_synth_packed_device(self.device, synth.SEED, self.rank * a.reads, a.reads, a.read_len, ks,
                                             self.words, self.koff))
        self.reads = self.words
        self.outs = None
        if self.g.murmur:   # the Counttable family hashes ASCII: the same bases unpacked
            self.ascii = ctypes.c_void_p()
            check(lib.kh_device_malloc(self.device, a.reads * a.read_len + 64, ctypes.byref(self.ascii)))
            check(lib.kh_unpack_ascii_device(self.device, self.words, a.reads * a.read_len, self.ascii))
            self.reads = self.ascii
        if a.query:
            self.outs = ctypes.c_void_p()
            check(lib.kh_device_malloc(self.device, a.reads * 10 + 64, ctypes.byref(self.outs)))
            self._consume()   # the tables being queried (untimed)

    def _consume(self):
        a = self.args
        if self.g.murmur:
            self.g.consume_bytes_fixed_device([self.reads], a.reads, a.read_len)
        else:
            self.g.consume_packed_fixed_device([self.words], a.reads, a.read_len)

    def step(self):
        a = self.args
        if a.query:
            o = self.outs.value
            self.g.median_fixed_device([self.reads], a.reads, a.read_len, [o], [o + 2 * a.reads], [o + 6 * a.reads])
            return
        self.g.clear()
        self._consume()

    def query_check(self, fx):
        """The fixture's get_median_count digest over its first median_reads
        reads, from every rank's outputs in rank order (collective)."""
        import numpy as np
        from tests import full_digest as FD
        n = self.args.reads
        raw = (ctypes.c_uint8 * (n * 10))()
        check(lib.kh_device_synchronize(self.device))
        check(lib.kh_device_copy(self.device, raw, self.outs, n * 10))
        parts = self.rdv.allgather(bytes(raw))
        med = np.concatenate([np.frombuffer(p[:2 * n], np.uint16) for p in parts])
        avg = np.concatenate([np.frombuffer(p[2 * n:6 * n], np.float32) for p in parts])
        sd = np.concatenate([np.frombuffer(p[6 * n:], np.float32) for p in parts])
        m = fx["median_reads"]
        return {"fixture": fx["config"], "median_reads": m,
                "median_match": FD.median_digest(med[:m], avg[:m], sd[:m]) == fx["median_sha256"]}

    def sync(self):
        check(lib.kh_device_synchronize(self.device))

    def barrier(self):
        self.rdv.barrier()

    def max_over_ranks(self, t):
        return self.rdv.max(t)

    def rccl_info(self):
        """RCCL's own view: nranks and device of every rank."""
        return {"nranks": sorted({c[1] for c in self.comm}), "devices": [c[2] for c in self.comm]}

    def profile(self, on):
        self.g.set_profiling(on)

    def kernel_stats(self):
        buf = ctypes.create_string_buffer(1 << 16)
        n = ctypes.c_size_t()
        check(lib.kh_graph_kernel_stats(self.g.shards[0]._g, buf, len(buf), ctypes.byref(n)))
        out = {}
        for line in buf.value.decode().splitlines():
            name, cnt, ms = line.split("\t")
            out[name] = (int(cnt), float(ms))
        return out

    def table_sha256(self):
        """SHA-256 of every reference-layout table, computed on rank 0 from
        the rank slices streamed to it in rank order (collective; None on the
        other ranks)."""
        import hashlib
        mine = self.g.local_tables()[0]
        out = []
        for i, p in enumerate(self.sizes):
            h = hashlib.sha256() if self.rank == 0 else None
            slices = self.g.rank_slices(i)
            for r in range(self.world):
                blob = self.rdv.send_to_root(mine[i] if self.rank == r else b"", r)
                if h is not None:
                    lo, size = slices[r]
                    h.update(bytes(blob[:_slice_nbytes(self.g.kind, lo, size, p)]))
            out.append(h.hexdigest() if h is not None else None)
        return out

    def check(self):
        u, o = self.g.counters()
        return {"n_unique_kmers": u, "n_occupied": o}

    def close(self):
        lib.kh_device_free(self.device, self.words)
        lib.kh_device_free(self.device, self.koff)
        if self.g.murmur:
            lib.kh_device_free(self.device, self.ascii)
        if self.outs is not None:
            lib.kh_device_free(self.device, self.outs)
        self.g.close()
        self.rdv.close()

