"""Batch sharding across GPUs -- the in-node replacement for the reference's
network work split (DHT_Node.py:491-510, utils.py:1-9).

Puzzle and check batches are independent units: rank k (one process per GPU)
owns the contiguous slice [k*n/G, (k+1)*n/G), runs it on its own device and the
results are gathered to the root.  There is no collective on the data path;
the only communication is the final gather (gloo on host memory: the results
are already on the host after the per-GPU D2H).

Two front ends:
  * ShardedBatch: one process per GPU (torch.distributed, launched by torchrun);
  * MultiDeviceEngine: one process driving several GPUs from threads (ctypes
    releases the GIL for the duration of each library call).

Whole-tree counts of ONE board split a replicated,
deterministic BFS frontier instead (sharded_count): every rank expands the same
frontier on its GPU, counts its slice, and the only exchange is one all-reduce
of a 64-bit count (plus a min of the status) across ranks.
"""
import threading

import numpy as np


def shard_bounds(n, rank, world):
    """Contiguous slice of n units owned by `rank` of `world` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return (rank * n) // world, ((rank + 1) * n) // world


class ShardedBatch:
    """Solve / check a batch that every rank can see (e.g. generated from a shared
    seed or read from shared storage); results are gathered on `root`."""

    def __init__(self, engine, rank, world, group=None, root=0):
        self.engine = engine
        self.rank = rank
        self.world = world
        self.group = group
        self.root = root

    def _gather(self, local, total_shape, dtype):
        if self.world == 1:
            return local
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(np.ascontiguousarray(local))
        sizes = [shard_bounds(total_shape[0], r, self.world) for r in range(self.world)]
        if self.rank == self.root:
            bufs = [torch.empty((hi - lo,) + tuple(total_shape[1:]), dtype=t.dtype) for lo, hi in sizes]
            # gloo gather needs equal sizes: fall back to point-to-point receives
            for r, (lo, hi) in enumerate(sizes):
                if r == self.root:
                    bufs[r] = t
                else:
                    dist.recv(bufs[r], src=r, group=self.group)
            return np.concatenate([b.numpy() for b in bufs]).astype(dtype, copy=False)
        dist.send(t, dst=self.root, group=self.group)
        return None

    def solve(self, boards, masks=None):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        lo, hi = shard_bounds(n, self.rank, self.world)
        m = None if masks is None else np.asarray(masks, dtype=np.uint16)[lo:hi]
        out, st, _ = self.engine.solve_batch(boards[lo:hi], m)
        return self._gather(out, (n, 81), np.uint8), self._gather(st, (n,), np.int8)

    def check(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        lo, hi = shard_bounds(n, self.rank, self.world)
        v = self.engine.check_batch(boards[lo:hi])
        return self._gather(v, (n,), np.uint8)


class MultiDeviceEngine:
    """Several GPUs from one process: one engine (context + stream) per device,
    one host thread per device, disjoint output slices (no collectives)."""

    def __init__(self, engines):
        self.engines = list(engines)

    @classmethod
    def open(cls, devices):
        from .engine import SudokuEngine
        return cls([SudokuEngine(d) for d in devices])

    def close(self):
        for e in self.engines:
            e.close()

    def _run(self, n, work):
        errors = []

        def body(k):
            try:
                lo, hi = shard_bounds(n, k, len(self.engines))
                if hi > lo:
                    work(self.engines[k], lo, hi)
            except BaseException as exc:  # re-raised on the caller's thread
                errors.append(exc)

        threads = [threading.Thread(target=body, args=(k,)) for k in range(len(self.engines))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]

    def solve_batch(self, boards, masks=None, want_work=False):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        out = np.empty_like(boards)
        st = np.empty(n, dtype=np.int8)
        wk = np.empty(n, dtype=np.uint64) if want_work else None

        def work(eng, lo, hi):
            m = None if masks is None else np.asarray(masks, dtype=np.uint16)[lo:hi]
            o, s, w = eng.solve_batch(boards[lo:hi], m, want_work)
            out[lo:hi], st[lo:hi] = o, s
            if want_work:
                wk[lo:hi] = w

        self._run(n, work)
        return out, st, wk

    def check_batch(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        v = np.empty(n, dtype=np.uint8)

        def work(eng, lo, hi):
            v[lo:hi] = eng.check_batch(boards[lo:hi])

        self._run(n, work)
        return v


def allreduce_gloo(values, op="sum", group=None):
    """Host all-reduce of a few int64 scalars over torch.distributed (any backend
    that takes CPU tensors, e.g. gloo).  Returns a list of ints."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(v) for v in values], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MIN, group=group)
    return [int(x) for x in t.tolist()]


def sharded_count(engine, board, rank, world, limit=0, allreduce=None):
    """Count the completions of `board` with `world` ranks (one GPU each).

    Returns (total, status, frontier_size).  `allreduce(values, op)` combines
    scalars across ranks (default: allreduce_gloo when world > 1)."""
    local, frontier, st = engine.count_solutions_slice(board, rank, world, limit)
    if world > 1:
        red = allreduce or allreduce_gloo
        total = red([local], "sum")[0]
        st = red([st], "min")[0]
    else:
        total = local
    if limit and total > limit:
        total = limit
    if st != -2:
        st = 1 if total > 0 else 0
    return total, st, frontier
