"""Process-group plumbing without PyTorch: a small TCP rendezvous.

The sharded path (khmer_amd.parallel) needs, on the host,
only a few small exchanges between the ranks: rank 0's RCCL unique id, a
barrier, the max of the per-rank step times, and (host-transport groups) the
collectives of the sharding protocol.  Rank 0 serves; every other rank keeps
one connection to it.  Each operation is collective: every rank calls it in
the same order.  Messages are length-prefixed byte strings (no pickling).

Address: MASTER_ADDR (default 127.0.0.1); port: KH_RDV_PORT, else MASTER_PORT
+ 1 (torchrun's own store listens on MASTER_PORT).

Failure: every socket operation has a finite timeout (`op_timeout`,
KH_RDV_OP_TIMEOUT seconds, default 900), and `abort()` closes this rank's
connections, so a rank whose collective failed makes its peers fail with
ConnectionError instead of waiting forever.
"""
import os
import socket
import struct
import time

_HDR = struct.Struct("<Q")


def _send(sock, data):
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("rendezvous peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


class Rendezvous(object):
    """Star-shaped TCP group of `world` ranks served by rank 0."""

    def __init__(self, rank, world, addr=None, port=None, timeout=600.0, op_timeout=None):
        self.rank, self.world = int(rank), int(world)
        if op_timeout is None:
            op_timeout = float(os.environ.get("KH_RDV_OP_TIMEOUT", "900"))
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("KH_RDV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        self.peers = {}
        self.sock = None
        if self.world == 1:
            return
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < self.world - 1:
                    c, _ = srv.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    c.settimeout(op_timeout)
                    (r,) = struct.unpack("<i", _recv_exact(c, 4))
                    self.peers[r] = c
            finally:
                srv.close()
        else:
            deadline = time.time() + timeout
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=10)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.1)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(op_timeout)
            s.sendall(struct.pack("<i", self.rank))
            self.sock = s

    # ---- collectives (every rank, same order) ----
    def allgather(self, data):
        """[bytes of rank 0, ..., bytes of rank world-1]"""
        data = bytes(data)
        if self.world == 1:
            return [data]
        if self.rank == 0:
            parts = [data] + [None] * (self.world - 1)
            for r in range(1, self.world):
                parts[r] = _recv(self.peers[r])
            blob = b"".join(_HDR.pack(len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self.peers[r], blob)
            return parts
        _send(self.sock, data)
        blob = _recv(self.sock)
        out, at = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(blob, at)
            at += _HDR.size
            out.append(blob[at:at + n])
            at += n
        return out

    def broadcast(self, data, root=0):
        """root's bytes on every rank (routed through rank 0)."""
        if self.world == 1:
            return bytes(data)
        if self.rank == 0:
            payload = bytes(data) if root == 0 else _recv(self.peers[root])
            for r in range(1, self.world):
                if r != root:
                    _send(self.peers[r], payload)
            return payload
        if self.rank == root:
            _send(self.sock, bytes(data))
            return bytes(data)
        return _recv(self.sock)

    def alltoallv(self, blocks):
        """blocks[d] -> rank d; returns [block from rank s for s in ranks]."""
        if self.world == 1:
            return [bytes(blocks[0])]
        if self.rank == 0:
            mats = [[bytes(b) for b in blocks]] + [None] * (self.world - 1)
            for r in range(1, self.world):
                blob = _recv(self.peers[r])
                mats[r] = self._split(blob)
            for r in range(1, self.world):
                _send(self.peers[r], b"".join(_HDR.pack(len(mats[s][r])) + mats[s][r] for s in range(self.world)))
            return [mats[s][0] for s in range(self.world)]
        _send(self.sock, b"".join(_HDR.pack(len(b)) + bytes(b) for b in blocks))
        return self._split(_recv(self.sock))

    def _split(self, blob):
        out, at = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(blob, at)
            at += _HDR.size
            out.append(blob[at:at + n])
            at += n
        return out

    def send_to_root(self, data, src):
        """Rank `src`'s bytes on rank 0 (b"" elsewhere)."""
        if self.world == 1 or src == 0:
            return bytes(data) if self.rank == 0 else b""
        if self.rank == 0:
            return _recv(self.peers[src])
        if self.rank == src:
            _send(self.sock, bytes(data))
        return b""

    def barrier(self):
        self.allgather(b"")

    def max(self, x):
        return max(struct.unpack("<d", p)[0] for p in self.allgather(struct.pack("<d", float(x))))

    def abort(self):
        """Drop this rank's connections after a failed collective: peers
        blocked on it get ConnectionError (or their timeout) and fail too."""
        self.close()

    def close(self):
        for c in self.peers.values():
            c.close()
        self.peers = {}
        if self.sock is not None:
            self.sock.close()
            self.sock = None
