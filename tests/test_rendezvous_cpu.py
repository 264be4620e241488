"""The host-side plumbing of the sharded path on CPU (no PyTorch): the TCP
rendezvous (khmer_amd.rendezvous) and the kh_transport callbacks
(khmer_amd.parallel.HostTransport) that carry a host-transport group's
collectives, run by world 2 and 3 separate processes.  The callbacks are
invoked through their C function pointers, exactly as libkhmer_hip.so calls
them (include/khmer_hip.h kh_transport)."""
import ctypes
import multiprocessing as mp
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    try:
        from khmer_amd.rendezvous import Rendezvous
        from khmer_amd.parallel import HostTransport
        rdv = Rendezvous(rank, world, "127.0.0.1", port, timeout=60)
        ok = []
        ok.append(rdv.allgather(b"r%d" % rank) == [b"r%d" % r for r in range(world)])
        for root in range(world):
            ok.append(rdv.broadcast(b"from%d" % rank if rank == root else b"", root) == b"from%d" % root)
        got = rdv.alltoallv([b"%d>%d" % (rank, d) * (d + 1) for d in range(world)])
        ok.append(got == [b"%d>%d" % (s, rank) * (rank + 1) for s in range(world)])
        ok.append(rdv.max(rank * 1.5) == (world - 1) * 1.5)
        rdv.barrier()
        # the transport struct, called through its C function pointers
        t = HostTransport(rdv)
        st = t.struct
        n = 3
        send = (ctypes.c_uint64 * n)(*[rank * 10 + i for i in range(n)])
        recv = (ctypes.c_uint64 * (n * world))()
        ok.append(st.allgather(None, ctypes.addressof(send), ctypes.addressof(recv), 8 * n) == 0)
        ok.append(list(recv) == [r * 10 + i for r in range(world) for i in range(n)])
        buf = (ctypes.c_uint8 * 16)(*([rank + 1] * 16))
        ok.append(st.broadcast(None, ctypes.addressof(buf), 16, world - 1) == 0)
        ok.append(list(buf) == [world] * 16)
        # alltoallv of u32 blocks: rank r sends d+1 words (value 100*r + d) to rank d
        sb = (ctypes.c_uint64 * world)(*[4 * (d + 1) for d in range(world)])
        words = [100 * rank + d for d in range(world) for _ in range(d + 1)]
        sa = (ctypes.c_uint32 * len(words))(*words)
        rb = (ctypes.c_uint64 * world)(*[4 * (rank + 1)] * world)
        ra = (ctypes.c_uint32 * ((rank + 1) * world))()
        ok.append(st.alltoallv(None, ctypes.addressof(sa), sb, ctypes.addressof(ra), rb) == 0)
        ok.append(list(ra) == [100 * s + rank for s in range(world) for _ in range(rank + 1)])
        rdv.close()
        q.put((rank, all(ok), ok))
    except Exception as e:   # reported to the parent
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_and_transport(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res), res


def test_single_rank_is_local():
    from khmer_amd.rendezvous import Rendezvous
    r = Rendezvous(0, 1)
    assert r.allgather(b"x") == [b"x"] and r.broadcast(b"y") == b"y" and r.alltoallv([b"z"]) == [b"z"]
    assert r.max(2.5) == 2.5


def _failing_worker(rank, world, port, q):
    """Rank 1's alltoallv callback fails (wrong receive sizes): it returns 1
    and aborts the rendezvous, and the other ranks' next collective fails
    (returns 1) instead of waiting forever (peers blocked in recv)."""
    try:
        import time
        from khmer_amd.rendezvous import Rendezvous
        from khmer_amd.parallel import HostTransport
        rdv = Rendezvous(rank, world, "127.0.0.1", port, timeout=60, op_timeout=30)
        st = HostTransport(rdv).struct
        sb = (ctypes.c_uint64 * world)(*[4] * world)
        sa = (ctypes.c_uint32 * world)(*range(world))
        rb = (ctypes.c_uint64 * world)(*([8 if rank == 1 else 4] * world))
        ra = (ctypes.c_uint32 * (2 * world))()
        first = st.alltoallv(None, ctypes.addressof(sa), sb, ctypes.addressof(ra), rb)
        t0 = time.time()
        send = (ctypes.c_uint64 * 1)(rank)
        recv = (ctypes.c_uint64 * world)()
        second = st.allgather(None, ctypes.addressof(send), ctypes.addressof(recv), 8) if rank != 1 else 1
        q.put((rank, first, second, time.time() - t0))
    except Exception as e:   # reported to the parent
        q.put((rank, -1, -1, repr(e)))


def test_failed_collective_fails_the_peers():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res[1][1] == 1                                   # rank 1's own failure
    assert all(r[2] == 1 for r in res), res                 # everyone's next collective fails ...
    assert all(r[3] < 25 for r in res if r[0] != 1), res    # ... promptly (not at the op timeout)


def test_send_to_root_single():
    from khmer_amd.rendezvous import Rendezvous
    r = Rendezvous(0, 1)
    assert r.send_to_root(b"abc", 0) == b"abc"
