"""Host-side transport between node processes, standard library only (no torch).

In-node multi-GPU runs use one process per GPU.  The processes
need a few host exchanges that are not on the data path: handing rank 0's RCCL
id to every rank once, gathering per-rank result slices of a sharded batch, a
barrier.  The reference's own transport for its ring is plain sockets plus
pickle (DHT_Node.py:27-31, 74-99); this is the same idea as a star through rank
0 over TCP, with length-prefixed raw bytes (nothing is unpickled).

TcpComm also offers the array collectives of shard.RcclComm (allreduce /
broadcast / allgather on numpy buffers), so the frontier searches of shard.py
run unchanged on it (host stand-in engines, CPU tests).
"""
import os
import socket
import struct
import time

import numpy as np

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
            raise ConnectionError("peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


def default_port():
    """SDK_RDZV_PORT, else MASTER_PORT + 1 (torchrun's own store keeps MASTER_PORT)."""
    if os.environ.get("SDK_RDZV_PORT"):
        return int(os.environ["SDK_RDZV_PORT"])
    if os.environ.get("MASTER_PORT"):
        return int(os.environ["MASTER_PORT"]) + 1
    raise ValueError("no rendezvous port: set SDK_RDZV_PORT or MASTER_PORT")


class TcpComm:
    """Star transport: rank 0 listens on (addr, port), ranks 1..world-1 connect.

    `timeout` bounds the rendezvous only (connect / accept / the rank handshake); once
    connected the sockets block without a limit (`data_timeout`, default None): a rank may
    wait as long as a peer's shard takes (hard boards, the per-lane solver)."""

    _OPS = {"sum": np.sum, "min": np.min, "max": np.max}

    def __init__(self, rank, world, addr=None, port=None, timeout=120.0, data_timeout=None):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"bad rank {rank} / world {world}")
        self.rank, self.world = rank, world
        self.peers = {}
        self.sock = None
        if world == 1:
            return
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = default_port() if port is None else int(port)
        deadline = time.time() + timeout
        if rank == 0:
            srv = socket.create_server((addr, port), reuse_port=False)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < world - 1:
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack("<i", _recv_exact(conn, 4))
                    if not 0 < r < world or r in self.peers:
                        conn.close()
                        raise ConnectionError(f"unexpected rank {r} at rendezvous")
                    self.peers[r] = conn
            finally:
                srv.close()
            for conn in self.peers.values():
                conn.settimeout(data_timeout)
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", rank))
            s.settimeout(data_timeout)
            self.sock = s

    # ----------------------------------------------------------- byte level
    def gather_bytes(self, data, root=0):
        """List of every rank's bytes at `root` (rank order), None elsewhere."""
        parts = self._gather0(data)
        if root == 0:
            return parts
        if self.rank == 0:
            _send(self.peers[root], b"".join(_HDR.pack(len(p)) + p for p in parts))
            return None
        if self.rank == root:
            blob = _recv(self.sock)
            out, off = [], 0
            for _ in range(self.world):
                (n,) = _HDR.unpack_from(blob, off)
                out.append(blob[off + 8: off + 8 + n])
                off += 8 + n
            return out
        return None

    def _gather0(self, data):
        if self.world == 1:
            return [bytes(data)]
        if self.rank == 0:
            return [bytes(data)] + [_recv(self.peers[r]) for r in range(1, self.world)]
        _send(self.sock, bytes(data))
        return None

    def broadcast_bytes(self, data, root=0):
        """`root`'s bytes on every rank."""
        if self.world == 1:
            return bytes(data)
        if root != 0:
            if self.rank == root:
                _send(self.sock, bytes(data))
            if self.rank == 0:
                data = _recv(self.peers[root])
        if self.rank == 0:
            data = bytes(data)
            for r in range(1, self.world):
                _send(self.peers[r], data)
            return data
        return _recv(self.sock)

    def allgather_bytes(self, data):
        parts = self._gather0(data)
        blob = b"".join(_HDR.pack(len(p)) + p for p in parts) if self.rank == 0 else None
        blob = self.broadcast_bytes(blob, 0)
        out, off = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(blob, off)
            out.append(blob[off + 8: off + 8 + n])
            off += 8 + n
        return out

    def barrier(self):
        self.allgather_bytes(b"")

    # ------------------------------------------- shard.RcclComm's interface
    def allreduce(self, buf, count, dtype, op):
        dt = np.dtype(dtype)
        parts = self.allgather_bytes(np.ascontiguousarray(buf[:count], dtype=dt).tobytes())
        stack = np.stack([np.frombuffer(p, dtype=dt) for p in parts])
        buf[:count] = self._OPS[op](stack, axis=0).astype(dt)

    def broadcast(self, buf, nbytes, root):
        raw = buf.view(np.uint8)
        raw[:nbytes] = np.frombuffer(self.broadcast_bytes(raw[:nbytes].tobytes(), root), dtype=np.uint8)

    def allgather(self, send, recv, nbytes):
        parts = self.allgather_bytes(send.view(np.uint8)[:nbytes].tobytes())
        recv.view(np.uint8)[:self.world * nbytes] = np.frombuffer(b"".join(parts), dtype=np.uint8)

    def p2p(self, ops):
        """Point-to-point as shard.RcclComm.p2p (host arrays).  A star cannot connect two
        non-root ranks directly, so this is a collective here: every rank calls it (with its own
        ops, possibly none), the messages travel through one allgather, and each rank keeps the
        ones addressed to it."""
        out = b"".join(struct.pack("<iiQ", self.rank, int(peer), int(nbytes)) +
                       np.ascontiguousarray(buf).view(np.uint8).reshape(-1)[:nbytes].tobytes()
                       for kind, peer, buf, nbytes in ops if kind == 0 and nbytes)
        want = {int(peer): (buf, int(nbytes)) for kind, peer, buf, nbytes in ops if kind == 1 and nbytes}
        for blob in self.allgather_bytes(out):
            off = 0
            while off < len(blob):
                src, dst, n = struct.unpack_from("<iiQ", blob, off)
                off += 16
                if dst == self.rank and src in want:
                    buf, nb = want.pop(src)
                    if nb != n:
                        raise ValueError(f"p2p size mismatch from rank {src}: {n} != {nb}")
                    buf.view(np.uint8).reshape(-1)[:n] = np.frombuffer(blob, np.uint8, n, off)
                off += n
        if want:
            raise ConnectionError(f"p2p: nothing arrived from ranks {sorted(want)}")

    def gather(self, local, root=0):
        """Row-concatenation of every rank's array at `root` (None elsewhere)."""
        local = np.ascontiguousarray(local)
        parts = self.gather_bytes(local.tobytes(), root)
        if parts is None:
            return None
        rows = [np.frombuffer(p, dtype=local.dtype).reshape((-1,) + local.shape[1:]) for p in parts]
        return np.concatenate(rows)

    def close(self):
        for s in list(self.peers.values()) + ([self.sock] if self.sock else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers = {}
        self.sock = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
