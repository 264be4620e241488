"""CPU checks of the multi-GPU sharding plan (khmer_amd.parallel), including a
world_size-2 torch.distributed gloo run of the gather/re-interleave path the
one-process-per-GPU build uses to recover reference-layout tables.  No device
calls: each rank cuts its slices out of an oracle table exactly as a shard
stores them (kh_engine.hip graph_create_shard), the ranks all-gather them, and
the re-interleaved bytes must equal the oracle's table."""
import os
import socket

import pytest

from oracle import oracle as O
from tests.conftest import data

torch = pytest.importorskip("torch")
parallel = pytest.importorskip("khmer_amd.parallel")

KINDS = [("Countgraph", O.BYTE), ("Nodegraph", O.BIT), ("SmallCountgraph", O.NIBBLE)]


def shard_bytes(kind, table, p, world, r):
    """What rank r's shard stores for table bytes `table` of a p-bin table."""
    lo = parallel.shard_lo(p, world, r)
    n = parallel.shard_lo(p, world, r + 1) - lo
    last = r == world - 1
    if kind == O.BIT:
        body = table[lo // 8: lo // 8 + n // 8 + (1 if last else 0)]
        return body + (b"" if last else b"\0")
    if kind == O.NIBBLE:
        body = table[lo // 2: lo // 2 + n // 2 + (1 if last else 0)]
        return body + (b"" if last else b"\0")
    return table[lo: lo + n]


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_slices_partition_tables(world):
    for p in (7, 8, 65, 99991, 999999937, 7999999963):
        sl = [parallel.shard_slices([p], world)[r][0] for r in range(world)]
        assert sl[0][0] == 0 and sum(n for _, n in sl) == p
        for r in range(world - 1):
            assert sl[r][0] + sl[r][1] == sl[r + 1][0] and sl[r + 1][0] % 8 == 0


@pytest.mark.parametrize("fj", [1, 2, 7, 1024, 2048])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_window_owners_partition(fj, world):
    rs = [parallel.window_owner_range(fj, world, r) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == fj
    for r in range(world - 1):
        assert rs[r][1] == rs[r + 1][0]


@pytest.mark.parametrize("cls,kind", KINDS)
@pytest.mark.parametrize("world", [2, 3, 8])
def test_reinterleave_recovers_tables(cls, kind, world):
    sizes = O.get_n_primes_near_x(3, 20011) + [13]
    o = O.Table(kind, 12, sizes)
    o.consume_fastx(data("test-abund-read-2.fa"))
    for i, p in enumerate(sizes):
        t = o.table_bytes(i)
        parts = [shard_bytes(kind, t, p, world, r) for r in range(world)]
        assert parallel.reinterleave(kind, p, parts) == t


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, result_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok = True
    for cls, kind in KINDS:
        sizes = O.get_n_primes_near_x(4, 30011)
        o = O.Table(kind, 20, sizes)
        o.consume_fastx(data("random-20-a.fa"))
        # this rank's slices (what its shard would hold after consuming)
        mine = [[shard_bytes(kind, o.table_bytes(i), p, world, rank) for i, p in enumerate(sizes)]]

        def all_gather(obj):
            out = [None] * world
            dist.all_gather_object(out, obj)
            return out

        parts = [x[0] for x in all_gather(mine)]
        tabs = [parallel.reinterleave(kind, p, [parts[r][i] for r in range(world)]) for i, p in enumerate(sizes)]
        ok &= all(tabs[i] == o.table_bytes(i) for i in range(len(sizes)))
        # group counters: partial sums all-reduced (kh_group_counters)
        t = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(t)
        ok &= int(t.item()) == world * (world + 1) // 2
    dist.barrier()
    if rank == 0:
        with open(result_path, "w") as fh:
            fh.write("ok" if ok else "bad")
    dist.destroy_process_group()


def test_gloo_world2_gather(tmp_path):
    import torch.multiprocessing as mp
    res = str(tmp_path / "res.txt")
    mp.spawn(_gloo_worker, args=(2, _free_port(), res), nprocs=2, join=True)
    assert open(res).read() == "ok"


def _bucket_slices(p_list, world, span):
    """Exchange-mode ownership (kh_engine.hip a2a_plan) restated: the
    unsharded tables back to back in span-aligned ranges, F1 buckets split
    into world contiguous ranges."""
    tbase, acc = [], 0
    for p in p_list:
        tbase.append(acc)
        acc += -(-p // span) * span
    f1 = acc // span
    bounds = [f1 * r // world for r in range(world + 1)]
    out = []
    for i, p in enumerate(p_list):
        def bin_of(b):
            x = b * span
            return 0 if x <= tbase[i] else min(p, x - tbase[i])
        out.append([(bin_of(bounds[r]), bin_of(bounds[r + 1]) - bin_of(bounds[r])) for r in range(world)])
    return out


@pytest.mark.parametrize("cls,kind", KINDS)
@pytest.mark.parametrize("world", [2, 3, 5])
def test_reinterleave_bucket_slices(cls, kind, world):
    """Exchange-mode slices (bucket aligned; a rank may hold nothing of a
    table, or its last bins): the generic reinterleave puts the tables back
    together, the table's spare trailing byte taken from the slice that ends
    the table."""
    sizes = O.get_n_primes_near_x(3, 20011) + [13]
    o = O.Table(kind, 12, sizes)
    o.consume_fastx(data("test-abund-read-2.fa"))
    slices = _bucket_slices(sizes, world, 4096)
    for i, p in enumerate(sizes):
        t = o.table_bytes(i)
        parts = []
        for lo, n in slices[i]:
            last = n > 0 and lo + n == p
            if kind == O.BIT:
                parts.append(t[lo // 8: lo // 8 + n // 8 + (1 if last else 0)] + (b"" if last else b"\0"))
            elif kind == O.NIBBLE:
                parts.append(t[lo // 2: lo // 2 + n // 2 + (1 if last else 0)] + (b"" if last else b"\0"))
            else:
                parts.append(t[lo: lo + n])
        assert parallel.reinterleave(kind, p, parts, slices[i]) == t


@pytest.mark.parametrize("nreads,world,batch", [(4000, 2, 1 << 18), (20000, 3, 1 << 20), (7, 8, 10 ** 6),
                                                (50_000_000, 8, 3200 << 20)])
def test_exchange_passes_cover_reads(nreads, world, batch):
    """parallel.exchange_passes (kh_engine.hip group_consume_a2a): the passes
    cover every rank's reads once, in order, and a pass's k-mer index space
    (world x the chunk's k-mers rounded up to 16) stays below the u32 limit
    and the batch size."""
    L, k = 150, 21
    ps = parallel.exchange_passes(nreads, L, k, world, batch)
    assert ps[0][0] == 0 and sum(n for _, n in ps) == nreads
    for (a, n), (b, _) in zip(ps, ps[1:]):
        assert a + n == b
    kpr = L - k + 1
    stride = max((n * kpr + 15) // 16 * 16 for _, n in ps)
    assert world * stride <= min(batch, parallel.MAX_PASS_KMERS) or max(n for _, n in ps) == 1
