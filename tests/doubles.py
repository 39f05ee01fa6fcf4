"""Test doubles shared by the CPU multi-process tests (no torch here)."""
import numpy as np

from distributed_sudoku_solver_amd import _lib as L

# the doubles' naive DFS needs far more validations than the GPU engine needs search nodes:
# a node budget b allows b * this many validations
VALIDATIONS_PER_NODE = 10_000


def validation_budget(budget, default):
    """Node budget of a solve_batch call -> the oracle's validation budget."""
    return default if budget is None else (0 if budget == 0 else int(budget) * VALIDATIONS_PER_NODE)


def naive_children(b):
    """Children of a board in the reference's DFS order (lowest empty cell, valid digits
    ascending, utils.py:14-56) -- None if the board is complete."""
    z = np.flatnonzero(b == 0)
    if len(z) == 0:
        return None
    c = int(z[0])
    r, col = divmod(c, 9)
    br, bc = 3 * (r // 3), 3 * (col // 3)
    used = set(b[9 * r: 9 * r + 9].tolist()) | set(b[col::9].tolist()) | {
        int(b[9 * (br + i) + bc + j]) for i in range(3) for j in range(3)}
    out = []
    for d in range(1, 10):
        if d not in used:
            ch = b.copy()
            ch[c] = d
            out.append((ch, d))
    return out


def naive_expand(boards, masks=None, target=64):
    """CPU restatement of sdk_expand_boards without propagation: level 0 always (board i's
    first empty cell restricted to masks[i]), then on while < target boards and something
    branches.  Complete boards stay; boards with no valid digit vanish."""
    fr = [np.asarray(b, dtype=np.uint8).copy() for b in np.asarray(boards).reshape(-1, 81)]
    allowed = [None] * len(fr) if masks is None else [int(m) for m in np.asarray(masks).reshape(-1)]
    level = 0
    while fr and (level == 0 or len(fr) < target):
        nxt, grew = [], False
        for b, m in zip(fr, allowed):
            kids = naive_children(b)
            if kids is None:
                nxt.append(b)
                continue
            grew = True
            nxt += [ch for ch, d in kids if m is None or (m >> d) & 1]
        fr, allowed, level = nxt, [None] * len(nxt), level + 1
        if not grew:
            break
    return np.stack(fr) if fr else np.zeros((0, 81), np.uint8)


class OracleEngine:
    """Test double with the SudokuEngine batch interface, computed by the oracle."""

    def __init__(self):
        from oracle import oracle as O
        self.O = O
        self.calls = []
        self.opts = {}

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        self.calls.append(len(boards))
        out, st, val = self.O.naive_solve_batch(boards, masks, budget=validation_budget(budget, 50_000_000),
                                                threads=2)
        return out, st, (val if want_work else None)

    def expand(self, boards, masks=None, target=64):
        self.calls.append(("expand", len(boards)))
        return naive_expand(boards, masks, target)

    def check_batch(self, boards):
        self.calls.append(len(boards))
        return self.O.check_batch(boards, threads=2)

    # ---- frontier primitives, restated on the CPU (test double of libsudoku_hip's) ----
    def get_option(self, key):
        if key in self.opts:
            return self.opts[key]
        return {L.SDK_OPT_DEVICE_CUS: 1, L.SDK_OPT_WAVES_PER_CU: 2, L.SDK_OPT_NODE_BUDGET: 0}[key]

    def set_option(self, key, value):
        self.opts[key] = int(value)

    def frontier_build(self, board, mask=None, mode=L.SDK_FRONTIER_COUNT, target=0):
        """Naive-DFS order expansion (lowest empty cell, digits ascending, utils.py:14-56)
        without propagation, level by level until >= target boards."""
        self.frontier = self._expand([np.asarray(board, dtype=np.uint8).copy()], target, mask)
        return len(self.frontier), 0

    def frontier_refine(self, first, step, target):
        """This rank's boards first, first+step, ... of the frontier, expanded on until >= target."""
        self.calls.append(("refine", first, step, len(self.frontier)))
        self.frontier = self._expand(list(self.frontier[first::step]), target, None)
        return len(self.frontier), 0

    def frontier_refine_range(self, lo, hi, target):
        """Boards [lo, hi) of the frontier, expanded on until >= target (no leaves dropped here)."""
        self.calls.append(("refine_range", lo, hi, len(self.frontier)))
        self.frontier = self._expand(list(self.frontier[lo:hi]), target, None)
        return len(self.frontier), 0

    def frontier_refine_head(self, lo, mid, hi, target):
        """Boards [lo, mid) expanded on until >= target, then [mid, hi) as they are."""
        self.calls.append(("refine_head", lo, mid, hi, len(self.frontier)))
        rest = list(self.frontier[mid:hi])
        self.frontier = self._expand(list(self.frontier[lo:mid]), target, None) + rest
        return len(self.frontier), 0

    def frontier_records(self, lo, hi):
        recs = np.stack(self.frontier[lo:hi]).reshape(-1) if hi > lo else np.zeros(0, np.uint8)
        return recs, 81 * (hi - lo)

    def record_buffer(self, n):
        return np.zeros(81 * max(1, int(n)), np.uint8)

    def frontier_load(self, buf, n, offset=0):
        self.calls.append(("load", n))
        raw = np.asarray(buf).view(np.uint8).reshape(-1)[81 * offset: 81 * (offset + n)]
        self.frontier = [r.copy() for r in raw.reshape(-1, 81)]

    @staticmethod
    def _expand(fr, target, allowed0):
        while fr and len(fr) < max(target, 1):
            nxt, grew = [], False
            for b in fr:
                z = np.flatnonzero(b == 0)
                if len(z) == 0:
                    nxt.append(b)
                    continue
                grew = True
                c = int(z[0])
                r, col = divmod(c, 9)
                br, bc = 3 * (r // 3), 3 * (col // 3)
                used = set(b[9 * r: 9 * r + 9]) | set(b[col::9]) | {b[9 * (br + i) + bc + j] for i in range(3)
                                                                    for j in range(3)}
                for d in range(1, 10):
                    if allowed0 is not None and not (allowed0 >> d) & 1:
                        continue
                    if d not in used:
                        ch = b.copy()
                        ch[c] = d
                        nxt.append(ch)
            allowed0 = None
            fr = nxt
            if not grew:
                break
        return fr

    def result_buffer(self, count, dtype):
        return np.zeros(count, dtype=dtype)

    def read(self, buf, count, dtype):
        return buf[:count].astype(dtype)

    def frontier_count(self, first, step, end, limit, res):
        idx = list(range(first, min(end, len(self.frontier)), step))
        self.calls.append(("count", idx))
        res[0] = sum(self.O.count(self.frontier[i], limit, 1) for i in idx)
        res[1] = 0

    def frontier_first(self, lo, hi, found, best):
        """The lowest board of [lo, hi) whose naive DFS ends solved or at the node budget
        (SDK_OPT_NODE_BUDGET, in search nodes: VALIDATIONS_PER_NODE validations each)."""
        hi = min(hi, len(self.frontier))
        self.calls.append(("first", lo, hi))
        found[0] = (1 << 63) - 1
        if hi > lo:
            nb = self.get_option(L.SDK_OPT_NODE_BUDGET)
            out, st, _ = self.O.naive_solve_batch(np.stack(self.frontier[lo:hi]),
                                                  budget=validation_budget(nb or None, 50_000_000), threads=2)
            hits = np.flatnonzero(st != 0)
            if len(hits):
                i = int(hits[0])
                found[0] = lo + i
                best[:81] = out[i]
                best[81] = np.int8(st[i]).view(np.uint8)


class _HostBuffer:
    """Host stand-in for engine.DeviceBuffer."""

    def __init__(self, nbytes):
        self.data = np.zeros(int(nbytes), dtype=np.uint8)

    def upload(self, host, offset=0):
        raw = np.ascontiguousarray(host).view(np.uint8).reshape(-1)
        self.data[offset:offset + raw.size] = raw

    def download(self, host):
        raw = host.view(np.uint8).reshape(-1)
        raw[:] = self.data[:raw.size]
        return host

    def free(self):
        self.data = None


class BenchStubEngine(OracleEngine):
    """The device-buffer interface bench.py drives, computed by the oracle on the host:
    lets the CPU tests run bench.py's rank launcher and sharding logic (no GPU here).
    Its "RCCL" is a TcpComm of its own, set up from the id the ranks exchange (an RCCL stub):
    the C5 legs run their real collective pattern through the bench's own transports."""

    _DT = {L.SDK_COMM_U64: np.uint64, L.SDK_COMM_I64: np.int64, L.SDK_COMM_U8: np.uint8}
    _OP = {L.SDK_COMM_SUM: "sum", L.SDK_COMM_MIN: "min", L.SDK_COMM_MAX: "max"}

    def __init__(self, device=0):
        super().__init__()
        self.device = device
        self.opts = {}
        self.launches = 0
        self._comm = None

    def set_option(self, key, value):
        self.opts[key] = int(value)

    def get_option(self, key):
        if key in (L.SDK_OPT_DEVICE_CUS, L.SDK_OPT_WAVES_PER_CU) and key not in self.opts:
            return super().get_option(key)
        return self.opts.get(key, 0)

    # ---- RCCL stub: id = a free TCP port for a second TcpComm between the ranks ----
    @staticmethod
    def comm_unique_id():
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        return port.to_bytes(4, "little") + bytes(L.SDK_COMM_ID_BYTES - 4)

    def comm_init(self, uid, rank, world):
        from distributed_sudoku_solver_amd.hostcomm import TcpComm
        self._comm = TcpComm(rank, world, port=int.from_bytes(uid[:4], "little"))

    def comm_destroy(self):
        if self._comm is not None:
            self._comm.close()
        self._comm = None

    def comm_allreduce(self, buf, count, dtype, op):
        self._comm.allreduce(buf, count, self._DT[dtype], self._OP[op])

    def comm_broadcast(self, buf, nbytes, root):
        self._comm.broadcast(buf, nbytes, root)

    def comm_allgather(self, send, recv, nbytes):
        self._comm.allgather(send, recv, nbytes)

    def comm_p2p(self, ops):
        self._comm.p2p([(k, p, b.data if isinstance(b, _HostBuffer) else b, n) for k, p, b, n in ops])

    def alloc(self, nbytes):
        return _HostBuffer(nbytes)

    def fork(self):
        """A second context on the same device (bench.py pipelines its passes over them)."""
        e = BenchStubEngine(self.device)
        e.opts = dict(self.opts)
        return e

    def solve_batch_dev(self, d_in, d_out, d_st, n, d_mask=None, d_work=None):
        boards = d_in.data[:n * 81].reshape(n, 81)
        out, st, _ = self.O.naive_solve_batch(boards, budget=50_000_000, threads=2)
        d_out.data[:n * 81] = out.reshape(-1)
        d_st.data[:n] = st.view(np.uint8)
        self.launches += 1

    def check_batch_dev(self, d_b, d_v, n):
        d_v.data[:n] = self.O.check_batch(d_b.data[:n * 81].reshape(n, 81), threads=2)
        self.launches += 1

    def synchronize(self):
        pass

    def timer_reset(self):
        self.launches = 0

    def timer_read(self):
        return 1e-3 * max(self.launches, 1), self.launches

    def timer_stop(self):
        pass

    def close(self):
        pass


class StagedDeviceComm:
    """shard.RcclComm's interface over a host transport (hostcomm.TcpComm) for REAL engines on
    one GPU (test only): device buffers and record addresses are staged through host memory.
    RCCL refuses two ranks on one device, so a 1-GPU box runs the multi-rank frontier searches
    (record moves, refinements, the all-gathered found flag) over two contexts this way; only
    the RCCL transport itself is left to the driver's multi-GPU node."""

    def __init__(self, engine, tcp):
        self.engine, self.tcp = engine, tcp
        self.rank, self.world = tcp.rank, tcp.world

    def _down(self, buf, nbytes):
        import ctypes
        host = np.empty(int(nbytes), np.uint8)
        if nbytes:
            src = buf.ptr if hasattr(buf, "ptr") else ctypes.c_void_p(int(buf))
            L.check(self.engine.lib.sdk_memcpy_d2h(self.engine.ctx, ctypes.c_void_p(host.ctypes.data), src,
                                                   host.nbytes), "d2h")
        return host

    def allreduce(self, buf, count, dtype, op):
        host = self._down(buf, count * np.dtype(dtype).itemsize).view(dtype)
        self.tcp.allreduce(host, count, dtype, op)
        buf.upload(host)

    def broadcast(self, buf, nbytes, root):
        host = self._down(buf, nbytes)
        self.tcp.broadcast(host, nbytes, root)
        buf.upload(host)

    def allgather(self, send, recv, nbytes):
        host = self._down(send, nbytes)
        out = np.empty(self.world * nbytes, np.uint8)
        self.tcp.allgather(host, out, nbytes)
        recv.upload(out)

    def p2p(self, ops):
        staged, recvs = [], []
        for kind, peer, buf, nbytes in ops:
            if kind == L.SDK_COMM_SEND:
                staged.append((kind, peer, self._down(buf, nbytes), nbytes))
            else:
                host = np.empty(int(nbytes), np.uint8)
                staged.append((kind, peer, host, nbytes))
                recvs.append((buf, host))
        self.tcp.p2p(staged)
        for buf, host in recvs:
            buf.upload(host)

    def close(self):
        self.tcp.close()
