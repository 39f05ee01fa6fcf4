"""Batch sharding across GPUs -- the in-node replacement for the reference's
network work split (DHT_Node.py:491-510, utils.py:1-9).

Puzzle and check batches are independent units: rank k (one process per GPU)
owns the contiguous slice [k*n/G, (k+1)*n/G), runs it on its own device and the
results are gathered to the root.  There is no collective on the data path;
the only communication is the final gather on host memory (the results are
already on the host after the per-GPU D2H).

Two front ends:
  * ShardedBatch: one process per GPU (e.g. launched by torchrun), results
    gathered over a host transport (hostcomm.TcpComm by default);
  * MultiDeviceEngine: one process driving several GPUs from threads (ctypes
    releases the GIL for the duration of each library call).

Searches of ONE board split a replicated,
deterministic breadth-first frontier instead -- the in-node form of the
reference's DFS subtree hand-off (NEEDWORK -> TASK with half of the digit range
and a partial board, DHT_Node.py:491-510, 225-250; utils.py:1-9):
  * sharded_count: every rank expands the same frontier on its GPU, counts the
    boards i = rank, rank+world, ... (interleaved for load balance), and the only
    exchange is one RCCL all-reduce of {count, budget hits} in device memory.
  * sharded_solve: first solution in the reference's DFS order.  The frontier is
    built in lex order and every live board carries a lex key; ranks work on their
    live ranges in rounds (boards above the lowest hit cancelled inside each
    launch, heavy boards refined one level deeper), and before every round an
    RCCL all-gather of the ranks' states carries the found/termination flag (the
    lowest hit key) and drives the same record-moving rebalance as the counts.
    Lower keys always finish before a higher hit is accepted, so the answer is
    identical for every world size.
The collectives go through a `comm` object: RcclComm (device memory, RCCL over
xGMI, the product path), hostcomm.TcpComm (host arrays over standard-library
sockets) or HostComm (host arrays over a torch.distributed group, CPU tests
only).  Nothing on the product path imports torch: one process can drive every
GPU of the node through MultiDeviceEngine.open_clique (ncclCommInitAll), and
one process per GPU rendezvous over hostcomm.TcpComm.
"""
import threading

import numpy as np

from . import _lib as L

INT64_MAX = (1 << 63) - 1


def shard_bounds(n, rank, world):
    """Contiguous slice of n units owned by `rank` of `world` (sizes differ by <= 1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return (rank * n) // world, ((rank + 1) * n) // world


def _host_transport(rank, world, comm=None, group=None):
    """The host transport a multi-process front end uses: `comm` if given, a torch
    group wrapped in HostComm (tests), else the standard-library TcpComm from the
    environment (MASTER_ADDR, SDK_RDZV_PORT / MASTER_PORT + 1)."""
    if comm is not None or world == 1:
        return comm
    if group is not None:
        return HostComm(rank, world, group)
    from .hostcomm import TcpComm
    return TcpComm(rank, world)


class ShardedBatch:
    """Solve / check a batch that every rank can see (e.g. generated from a shared
    seed or read from shared storage); results are gathered on `root`.

    The gather goes through a host transport with `gather(array, root)`:
    hostcomm.TcpComm (standard library, the default) or HostComm (torch group)."""

    def __init__(self, engine, rank, world, comm=None, group=None, root=0):
        self.engine = engine
        self.rank = rank
        self.world = world
        self.root = root
        self._own_comm = comm is None and group is None and world > 1   # made here: closed by close()
        self.comm = _host_transport(rank, world, comm, group)

    def close(self):
        if self._own_comm and self.comm is not None:
            self.comm.close()
        self.comm = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _gather(self, local):
        if self.world == 1:
            return local
        return self.comm.gather(np.ascontiguousarray(local), self.root)

    def solve(self, boards, masks=None):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        lo, hi = shard_bounds(n, self.rank, self.world)
        m = None if masks is None else np.asarray(masks, dtype=np.uint16)[lo:hi]
        out, st, _ = self.engine.solve_batch(boards[lo:hi], m)
        return self._gather(out), self._gather(st)

    def check(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        lo, hi = shard_bounds(n, self.rank, self.world)
        return self._gather(self.engine.check_batch(boards[lo:hi]))


def _run_per_device(items, body):
    """body(k, item) on one host thread per item (ctypes drops the GIL inside every
    library call, so the devices run concurrently); first exception re-raised.  A single
    item runs on the calling thread."""
    if len(items) == 1:
        return [body(0, items[0])]
    errors = []
    results = [None] * len(items)

    def run(k):
        try:
            results[k] = body(k, items[k])
        except BaseException as exc:  # re-raised on the caller's thread
            errors.append(exc)

    threads = [threading.Thread(target=run, args=(k,)) for k in range(len(items))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return results


class MultiDeviceEngine:
    """Several GPUs from one process: one engine (context + stream) per device,
    one host thread per device.  Batches go to disjoint output slices (no
    collectives); with `open_clique` the engines also share one RCCL communicator
    (ncclCommInitAll, sdk_comm_init_all) for the one-board frontier searches --
    the torch-free single-process form of SURVEY §8(e).

    It has the engine surface a node drives (solve_batch with per-call budget and donate,
    expand, fork, get_option), so node.SudokuNode runs on every GPU of the box -- the
    in-node replacement of DHT_Node's network work-splitting (DHT_Node.py:491-510, 225-250):
    each drained TASK batch is sharded over the devices, and a budget-hit board's continued
    search (search.LexSearch) shards every slice's launch and expansion over them."""

    def __init__(self, engines, comms=None):
        self.engines = list(engines)
        if not self.engines:
            raise ValueError("MultiDeviceEngine needs at least one engine")
        self.comms = comms

    @property
    def n_devices(self):
        return len(self.engines)

    def get_option(self, key):
        return self.engines[0].get_option(key)

    def set_option(self, key, value):
        for e in self.engines:
            e.set_option(key, value)

    def fork(self):
        """Second contexts on the same devices (no communicator): a node's search engine.
        Engines that cannot fork (test doubles) are shared: then this engine itself."""
        if not all(hasattr(e, "fork") for e in self.engines):
            return self
        return MultiDeviceEngine([e.fork() for e in self.engines])

    @classmethod
    def open(cls, devices):
        from .engine import SudokuEngine
        return cls([SudokuEngine(d) for d in devices])

    @classmethod
    def open_clique(cls, devices):
        from .engine import SudokuEngine
        engines = SudokuEngine.open_clique(devices)
        n = len(engines)
        return cls(engines, [RcclComm.attach(e, k, n) for k, e in enumerate(engines)])

    def close(self):
        for e in self.engines:
            if hasattr(e, "close"):
                e.close()

    def _parts(self, n):
        """(engine, lo, hi) of every device with a non-empty contiguous share of n units."""
        G = len(self.engines)
        parts = [(e,) + shard_bounds(n, k, G) for k, e in enumerate(self.engines)]
        return [p for p in parts if p[2] > p[1]]

    def _run(self, n, work):
        _run_per_device(self._parts(n), lambda k, p: work(*p))

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        """Contiguous shards, one per device, one launch each (same budget / donate)."""
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        out = np.empty_like(boards)
        st = np.empty(n, dtype=np.int8)
        wk = np.empty(n, dtype=np.uint64) if want_work else None

        def work(eng, lo, hi):
            m = None if masks is None else np.asarray(masks, dtype=np.uint16)[lo:hi]
            o, s, w = eng.solve_batch(boards[lo:hi], m, want_work, budget=budget, donate=donate)
            out[lo:hi], st[lo:hi] = o, s
            if want_work:
                wk[lo:hi] = w

        self._run(n, work)
        return out, st, wk

    def expand(self, boards, masks=None, target=64):
        """Ordered frontier below `boards`, the parents split contiguously over the devices:
        device k expands its parents towards its share of `target`, and the children are
        concatenated in device order -- parents' order kept, so still the ordered partition of
        the parents' completions that search.LexSearch needs."""
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        parts = self._parts(n)
        kids = [None] * len(parts)

        def body(k, p):
            eng, lo, hi = p
            m = None if masks is None else np.asarray(masks, dtype=np.uint16)[lo:hi]
            kids[k] = eng.expand(boards[lo:hi], m, target=max(1, -(-int(target) * (hi - lo) // n)))

        _run_per_device(parts, body)
        return np.concatenate(kids) if kids else np.zeros((0, 81), np.uint8)

    def check_batch(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        v = np.empty(n, dtype=np.uint8)

        def work(eng, lo, hi):
            v[lo:hi] = eng.check_batch(boards[lo:hi])

        self._run(n, work)
        return v

    # ---------------------------------- one-board searches over the clique
    def _clique(self, fn):
        if self.comms is None and len(self.engines) > 1:
            raise ValueError("one-board searches over several GPUs need open_clique (an RCCL communicator)")
        world = len(self.engines)
        comms = self.comms or [None]
        res = _run_per_device(self.engines, lambda k, eng: fn(eng, k, world, comms[k] if world > 1 else None))
        return res[0]

    def count(self, board, limit=0):
        """sharded_count over every device: (total, status, frontier_size)."""
        return self._clique(lambda e, k, w, c: sharded_count(e, board, k, w, limit=limit, comm=c))

    def count_rebalanced(self, board, limit=0, info=None):
        """sharded_count_rebalanced over every device: (total, status, frontier_size)."""
        return self._clique(lambda e, k, w, c: sharded_count_rebalanced(e, board, k, w, limit=limit, comm=c,
                                                                        info=info if k == 0 else None))

    def solve_one(self, board, mask=None):
        """sharded_solve over every device: the reference's answer for one board."""
        return self._clique(lambda e, k, w, c: sharded_solve(e, board, k, w, comm=c, mask=mask))


class RcclComm:
    """RCCL communicator of one engine (one rank per GPU), collectives on device memory.

    Multi-process: rank 0 makes the 128-byte id and a host transport hands it to
    the other ranks once (`transport.broadcast_bytes`; hostcomm.TcpComm by
    default, or a torch group through HostComm in tests).  Single process: the
    engines of SudokuEngine.open_clique already share a communicator (attach)."""

    _DT = {np.dtype(np.uint64): L.SDK_COMM_U64, np.dtype(np.int64): L.SDK_COMM_I64,
           np.dtype(np.uint8): L.SDK_COMM_U8}
    _OP = {"sum": L.SDK_COMM_SUM, "min": L.SDK_COMM_MIN, "max": L.SDK_COMM_MAX}

    def __init__(self, engine, rank, world, group=None, uid=None, transport=None, _attach=False):
        self.engine, self.rank, self.world = engine, rank, world
        if _attach:
            return
        if uid is None:
            own = world > 1 and transport is None and group is None
            t = _host_transport(rank, world, transport, group) if world > 1 else None
            try:
                uid = self.exchange_id(rank, t)
            finally:
                if own and t is not None:
                    t.close()                    # the implicit transport carried the id only
        engine.comm_init(uid, rank, world)

    @classmethod
    def attach(cls, engine, rank, world):
        """Wrap an engine whose context already has a communicator (open_clique)."""
        return cls(engine, rank, world, _attach=True)

    def exchange_id(self, rank, transport):
        """Rank 0's RCCL id (engine.comm_unique_id) on every rank, over the host transport."""
        uid = self.engine.comm_unique_id() if rank == 0 else None
        if transport is None:
            return uid
        return transport.broadcast_bytes(uid, 0)

    def allreduce(self, buf, count, dtype, op):
        self.engine.comm_allreduce(buf, count, self._DT[np.dtype(dtype)], self._OP[op])

    def broadcast(self, buf, nbytes, root):
        self.engine.comm_broadcast(buf, nbytes, root)

    def allgather(self, send, recv, nbytes):
        self.engine.comm_allgather(send, recv, nbytes)

    def p2p(self, ops):
        """Grouped ncclSend / ncclRecv on device memory: ops = [(L.SDK_COMM_SEND | RECV, peer,
        device buffer or address, nbytes)]; a rank without ops need not call."""
        self.engine.comm_p2p(ops)

    def close(self):
        self.engine.comm_destroy()


class HostComm:
    """Same interface over host numpy arrays and a torch.distributed group (gloo):
    the CPU stand-in for RcclComm in multi-process tests (torch is imported only
    here, never on the product path)."""

    _OPS = {"sum": "SUM", "min": "MIN", "max": "MAX"}

    def __init__(self, rank, world, group=None):
        self.rank, self.world, self.group = rank, world, group

    def allreduce(self, buf, count, dtype, op):
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(buf[:count].astype(np.int64))
        dist.all_reduce(t, op=getattr(dist.ReduceOp, self._OPS[op]), group=self.group)
        buf[:count] = t.numpy().astype(buf.dtype)

    def broadcast(self, buf, nbytes, root):
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(buf.view(np.uint8)[:nbytes].copy())
        dist.broadcast(t, src=root, group=self.group)
        buf.view(np.uint8)[:nbytes] = t.numpy()

    def allgather(self, send, recv, nbytes):
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(send.view(np.uint8)[:nbytes].copy())
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        recv.view(np.uint8)[:self.world * nbytes] = torch.cat(parts).numpy()

    def p2p(self, ops):
        """Point-to-point over the group (gloo isend / irecv): ops as RcclComm.p2p, host arrays."""
        import torch
        import torch.distributed as dist
        reqs, recvs = [], []
        for kind, peer, buf, nbytes in ops:
            if not nbytes:
                continue
            if kind == L.SDK_COMM_SEND:
                t = torch.from_numpy(np.ascontiguousarray(buf).view(np.uint8).reshape(-1)[:nbytes].copy())
                reqs.append(dist.isend(t, dst=int(peer), group=self.group))
            else:
                t = torch.empty(int(nbytes), dtype=torch.uint8)
                reqs.append(dist.irecv(t, src=int(peer), group=self.group))
                recvs.append((buf, t))
        for r in reqs:
            r.wait()
        for buf, t in recvs:
            buf.view(np.uint8).reshape(-1)[:t.numel()] = t.numpy()

    def broadcast_bytes(self, data, root=0):
        import torch
        import torch.distributed as dist
        n = torch.tensor([len(data) if self.rank == root else 0], dtype=torch.int64)
        dist.broadcast(n, src=root, group=self.group)
        t = torch.zeros(int(n.item()), dtype=torch.uint8)
        if self.rank == root:
            t[:] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
        dist.broadcast(t, src=root, group=self.group)
        return bytes(t.numpy().tobytes())

    def gather(self, local, root=0):
        """Row-concatenation at `root` (gloo gather needs equal sizes: point-to-point)."""
        import torch
        import torch.distributed as dist
        local = np.ascontiguousarray(local)
        n = torch.tensor([local.shape[0]], dtype=torch.int64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        dist.all_gather(sizes, n, group=self.group)
        row = local.dtype.itemsize * int(np.prod(local.shape[1:], dtype=np.int64))
        if self.rank != root:
            if local.shape[0]:
                dist.send(torch.from_numpy(local.view(np.uint8).reshape(-1).copy()), dst=root, group=self.group)
            return None
        parts = []
        for r in range(self.world):
            k = int(sizes[r].item())
            if r == root:
                parts.append(local)
            elif k:
                buf = torch.empty(k * row, dtype=torch.uint8)
                dist.recv(buf, src=r, group=self.group)
                parts.append(buf.numpy().view(local.dtype).reshape((k,) + local.shape[1:]))
        return np.concatenate(parts)

    def close(self):
        pass


def default_target(engine, world):
    """Frontier size: 8 boards per resident solver wave per GPU."""
    return engine.get_option(L.SDK_OPT_DEVICE_CUS) * engine.get_option(L.SDK_OPT_WAVES_PER_CU) * 8 * world


def count_target(engine, world):
    """Frontier size of an exhaustive count: 64 boards per resident solver wave per GPU (512k on
    an MI355X).  A count launch ends with its heaviest subtrees, so finer subtrees shorten it,
    and the frontier build is cheap (1M boards in 1.7 ms): 14-clue C5 board 46.9 ms at 65k boards,
    24.3 ms at 512k, 22.8 ms at 1M; 15-clue 7.1 / 6.0 / 6.2 ms (profiles/r03/c5_target.log)."""
    return default_target(engine, world) * 8


def sharded_count(engine, board, rank, world, limit=0, comm=None, target=None, refine=True):
    """Count the completions of `board` with `world` ranks (one GPU each).

    world == 1 (or refine=False): one frontier of `target` boards, rank k counting boards
    k, k + world, ...  world > 1: a two-stage split -- every rank expands the same SMALL
    frontier (1024 boards per rank), takes its interleaved share and grows that on its own
    GPU to one GPU's frontier (engine.frontier_refine), so the replicated part does not grow
    with the world size.  Completions met while expanding are counted once: those of the
    replicated stage by rank 0, those of a refinement by its rank.

    Returns (total, status, frontier_size); status 1 = >= 1 completion, 0 = none,
    -2 = some subtree hit the node budget (total is then a lower bound)."""
    if world > 1 and comm is None:
        raise ValueError("world > 1 needs a comm (RcclComm or HostComm)")
    two_stage = world > 1 and refine and hasattr(engine, "frontier_refine")
    if two_stage:
        size, leaves0 = engine.frontier_build(board, mode=L.SDK_FRONTIER_COUNT, target=1024 * world)
        mine, leaves1 = engine.frontier_refine(rank, world, count_target(engine, 1) if target is None else target)
        first, step, end = 0, 1, mine
        own_leaves = leaves1 + (leaves0 if rank == 0 else 0)
    else:
        size, leaves = engine.frontier_build(board, mode=L.SDK_FRONTIER_COUNT,
                                             target=count_target(engine, world) if target is None else target)
        first, step, end = rank, world, size
        own_leaves = None
    res = engine.result_buffer(2, np.uint64)
    try:
        engine.frontier_count(first, step, end, limit, res)
        if two_stage:   # this rank's leaves ride in the same all-reduce
            _add_to_result(engine, res, own_leaves)
        if comm is not None:
            comm.allreduce(res, 2, np.uint64, "sum")
        count, hits = (int(x) for x in engine.read(res, 2, np.uint64))
    finally:
        if hasattr(res, "free"):
            res.free()
    total = count + (0 if two_stage else leaves)                   # single stage: leaves are on every rank
    if limit and total > limit:
        total = limit
    st = -2 if hits else (1 if total > 0 else 0)
    return total, st, size


def _add_to_result(engine, res, k):
    """res[0] += k (the 2 x u64 result buffer is a device buffer, or a host array for doubles)."""
    if not k:
        return
    vals = np.asarray(engine.read(res, 2, np.uint64), dtype=np.uint64).copy()
    vals[0] += np.uint64(k)
    if hasattr(res, "upload"):
        res.upload(vals)
    else:
        res[:2] = vals


KEY_SPACE = 1 << 62       # lex keys of a first-solution search (sharded_solve)
ROUND_BUDGET = 512        # search nodes per frontier board and round of sharded_solve (refined after)


def _key_trim(hi, key_lo, key_step, g):
    """Live boards [., hi) of a rank whose board t has lex key key_lo + t * key_step: those with
    a key above g (a completion or budget hit already met at key g) cannot hold the answer."""
    if g >= INT64_MAX or key_step <= 0:
        return hi
    return min(hi, max(0, (g - key_lo) // key_step + 1))


def _renormalize_keys(S, g):
    """Monotone re-keying of the gathered state S (rows lo, hi, local, key_lo, key_step, best,
    heavy; trimmed at g) in place, computed identically on every rank.  The ranks' live ranges
    occupy disjoint key intervals, so ordered by the key of their first board they are laid end
    to end with one common step; the lowest hit g maps above every live key and the other hits
    (all above g, so never the answer) are dropped.  The step leaves room for key_lo = base -
    lo * step to stay within int64 (lo is an index into a frontier of at most 2^25 boards)."""
    live = sorted((k for k in range(len(S)) if S[k][1] > S[k][0]), key=lambda k: S[k][3] + S[k][0] * S[k][4])
    total = sum(S[k][1] - S[k][0] for k in live)
    step = max(1, KEY_SPACE // (total + max((S[k][0] for k in live), default=0) + 1))
    base = 0
    for k in live:
        S[k][3], S[k][4] = base - S[k][0] * step, step
        base += (S[k][1] - S[k][0]) * step
    for s in S:
        if s[1] <= s[0]:
            s[3], s[4] = 0, step
        s[5] = KEY_SPACE + 1 if (g != INT64_MAX and s[5] == g) else INT64_MAX


def sharded_solve(engine, board, rank, world, comm=None, mask=None, target=None, chunk=None, info=None,
                  ranges=None, round_budget=None):
    """First completion of `board` in the reference's DFS order, split over `world` ranks.

    Returns (out uint8[81], status) with solve_sudoku's contract: the lex-first
    completion and 1, or the input and 0 (no completion) / -2 (node budget hit in
    a subtree that precedes every completion found; only with a context node budget).

    The lex frontier is built on every rank (replicated, no exchange); frontier board t's
    completions all precede board t+1's.  Every live board carries a lex KEY (board t of a
    rank's frontier: key_lo + t * key_step; the replicated frontier spans [0, KEY_SPACE)), so
    boards on different ranks compare in the reference's DFS order.  Each rank starts on a
    contiguous block (or `ranges`) and works in rounds:
      * its live boards [lo, min(hi, lo + chunk)) are solved in one launch with a per-board node
        budget; boards above the lowest hit (completion or budget hit) stop inside the launch
        (sdk_frontier_first);
      * a completion at t makes key(t) the rank's best and ends its range (everything after it
        is lex-greater); a budget hit at t keeps [t, hi) live, and board t is split into its
        lex-ordered sub-boards at the start of the next round (engine.frontier_refine_head:
        the rest of the range stays as it is, keys re-spread monotonically over the same key
        interval) -- the device form of the reference handing a partial board on
        (DHT_Node.py:491-510), here to the rank itself and, through the rebalance below, to
        others;
      * before every round the ranks all-gather (lo, hi, local, key_lo, key_step, best_key, heavy)
        (RCCL ncclAllGather of 7 x int64 per rank): the minimum best_key is the found flag --
        every rank drops its boards keyed above it, and all ranks re-key the live boards over the
        whole key space with one monotone map (_renormalize_keys: refinements never exhaust the
        keys) -- and rebalance_plan gives dry ranks the
        upper half of the largest live range, as board RECORDS (grouped ncclSend/ncclRecv) when
        either side no longer holds the replicated frontier.  A rank whose remainder is one board
        (or heavy: it hit the budget) refines it while another is dry, so one heavy subtree does
        not stay on one GPU.
    The search ends when no rank holds a board keyed below the minimum; the owner of that key
    broadcasts its board.  With a context node budget (SDK_OPT_NODE_BUDGET > 0) budget hits are
    final (status -2) instead of being refined.  `info` (dict) gets rounds, steals, moved
    records and refinements."""
    if world > 1 and comm is None:
        raise ValueError("world > 1 needs a comm (RcclComm or HostComm)")
    board = np.ascontiguousarray(board, dtype=np.uint8).reshape(81)
    size, _ = engine.frontier_build(board, mask=mask, mode=L.SDK_FRONTIER_FIRST,
                                    target=default_target(engine, world) if target is None else target)
    if size == 0:
        return board.copy(), 0
    user_budget = int(engine.get_option(L.SDK_OPT_NODE_BUDGET) or 0)
    rbudget = user_budget or int(round_budget or ROUND_BUDGET)
    if chunk is None:    # the whole live range per round: the launch cancels what lies above a hit
        chunk = 1 << 62
    split = 2
    key_lo, key_step = 0, KEY_SPACE // size
    lo, hi = shard_bounds(size, rank, world) if ranges is None else (int(ranges[rank][0]), int(ranges[rank][1]))
    lo, hi = min(lo, size), min(hi, size)
    local = heavy = 0
    my_best = INT64_MAX                                   # key of this rank's lowest hit
    found = engine.result_buffer(1, np.int64)
    best = engine.result_buffer(82, np.uint8)
    keep = engine.result_buffer(82, np.uint8)            # the board behind my_best
    mine = engine.result_buffer(7, np.int64)
    allr = engine.result_buffer(7 * world, np.int64)
    inbox = None
    rounds = steals = moved = refined = 0
    g = INT64_MAX
    owner = rank
    engine.set_option(L.SDK_OPT_NODE_BUDGET, rbudget)
    try:
        while True:
            if comm is not None:
                _store(mine, [lo, hi, local, key_lo, key_step, my_best, heavy], np.int64)
                comm.allgather(mine, allr, 56)
                S = engine.read(allr, 7 * world, np.int64).reshape(world, 7).tolist()
            else:
                S = [[lo, hi, local, key_lo, key_step, my_best, heavy]]
            g = min(s[5] for s in S)                      # found / termination flag
            owner = min(range(len(S)), key=lambda k: (S[k][5], k))
            for s in S:                                   # boards keyed above the lowest hit are done
                s[1] = _key_trim(s[1], s[3], s[4], g)
                if s[1] <= s[0]:
                    s[6] = 0
            if all(s[1] <= s[0] for s in S):
                break
            # re-spread the live keys over the whole key space (same map on every rank): repeated
            # refinements only divide a rank's own interval, so without this a long search runs
            # out of integer keys
            _renormalize_keys(S, g)
            key_lo, key_step, my_best = S[rank if comm is not None else 0][3:6]
            skip = False
            if comm is not None:
                newS, moves, refines = rebalance_plan([s[:3] + [s[6]] for s in S], min_split=split)
                steals += sum(1 for a, b in zip(S, newS) if a[1] <= a[0] and b[1] > b[0])
                ops, got = [], None
                for donor, recv, mid, end, by_records in moves:
                    if rank == recv:                      # the keys of what this rank takes over
                        d = S[donor]
                        key_lo, key_step = (d[3] + mid * d[4], d[4]) if by_records else (d[3], d[4])
                    if not by_records:
                        continue
                    moved += end - mid
                    if rank == donor:
                        ops.append((L.SDK_COMM_SEND, recv) + engine.frontier_records(mid, end))
                    elif rank == recv:
                        inbox = _grow_records(engine, inbox, end - mid)
                        ops.append((L.SDK_COMM_RECV, donor, inbox, 81 * (end - mid)))
                        got = end - mid
                if any(m[4] for m in moves):
                    comm.p2p(ops)                         # every rank: a collective on host transports
                if got is not None:
                    engine.frontier_load(inbox, got)      # received records: board t has key key_lo + t * step
                lo, hi, local = (int(v) for v in newS[rank])
                heavy = S[rank][6]
                if rank in refines and not user_budget:
                    heavy, skip = 1, True                 # refine now; the next round can split it
            else:
                lo, hi, heavy = S[0][0], S[0][1], S[0][6]
            if heavy and hi > lo and not user_budget:
                # the heavy board (the first live one) split into its lex-ordered sub-boards, the
                # rest of the range kept as it is; the rank's keys are re-spread over its same
                # interval [key(lo), key(hi)) -- monotone, so the order across ranks holds
                k0, k1 = key_lo + lo * key_step, key_lo + hi * key_step
                n, _ = engine.frontier_refine_head(lo, lo + 1, hi, refine_target(world, split))
                refined += 1
                if n and (k1 - k0) // n < 1:
                    raise RuntimeError("sharded_solve: lex keys exhausted (a range refined ~40 times)")
                lo, hi, local = 0, n, 1
                key_lo, key_step = k0, ((k1 - k0) // n if n else 1)
                heavy = 0
            end = min(hi, lo + chunk)
            if end > lo and not skip:
                engine.frontier_first(lo, end, found, best)
                f = int(engine.read(found, 1, np.int64)[0])
                if f == INT64_MAX:
                    lo = end                              # every board refuted
                else:
                    b = engine.read(best, 82, np.uint8)
                    st = int(b[81].view(np.int8))
                    if st == -2 and not user_budget:
                        lo, heavy = f, 1                  # boards below f refuted; f and on stay live
                    else:
                        k = key_lo + f * key_step
                        if k < my_best:
                            my_best = k
                            _store(keep, b, np.uint8)
                        lo = hi                           # the rest of the range is lex-greater
            rounds += 1
        status = 0
        out = board.copy()
        if g != INT64_MAX:
            if comm is not None:
                comm.broadcast(keep, 82, owner)           # the owner of the lowest key has its board
            b = engine.read(keep, 82, np.uint8)
            status = int(b[81].view(np.int8))
            if status == 1:
                out = b[:81].copy()
    finally:
        engine.set_option(L.SDK_OPT_NODE_BUDGET, user_budget)
        for h in (found, best, keep, mine, allr, inbox):
            if hasattr(h, "free"):
                h.free()
    if info is not None:
        info.update(rounds=rounds, steals=steals, moved_records=moved, refines=refined, frontier=size)
    return out, status


def _store(buf, values, dtype):
    arr = np.asarray(values, dtype=dtype)
    if hasattr(buf, "upload"):
        buf.upload(arr)
    else:
        buf[:len(arr)] = arr


def rebalance_ranges(ranges, min_split=2):
    """One rebalancing step over the all-gathered live ranges [lo, hi) of the ranks.

    In rank order, every rank whose range is empty takes the upper half of the currently largest
    remaining range (ties -> lowest rank); ranges shorter than `min_split` are not split.  A pure
    function of the gathered values, so every rank computes the same assignment and only the
    2 x int64 per rank travel (the frontier itself is replicated)."""
    R = [[int(a), int(b)] for a, b in ranges]
    for r in range(len(R)):
        if R[r][1] > R[r][0]:
            continue
        donor = max(range(len(R)), key=lambda k: (R[k][1] - R[k][0], -k))
        rem = R[donor][1] - R[donor][0]
        if rem < max(2, min_split):
            continue
        mid = R[donor][0] + rem // 2
        R[r] = [mid, R[donor][1]]
        R[donor][1] = mid
    return R


def rebalance_plan(states, min_split=2):
    """One rebalancing step over the all-gathered rank states (lo, hi, local[, heavy]): `local` =
    the rank's frontier is no longer the replicated one (it received or refined records);
    `heavy` (optional) = its first live board is known to be too heavy to finish in a round (a
    first-solution search: it hit the round's node budget).

    Returns (new_states, moves, refines), a pure function of the gathered values (every rank
    computes the same):
      * in rank order, a rank with an empty range takes the upper half [mid, hi) of the largest
        remaining range (ties -> lowest rank; not below `min_split` boards; a rank that takes
        records this step gives none).  moves = [(donor, receiver, mid, hi, by_records)]:
        by_records when either frontier is not the replicated one -- the donor then sends the
        board records (81 B each) of [mid, hi) and the receiver's frontier becomes them;
        otherwise only the range travels;
      * if a rank is still empty after that, every rank whose remaining boards are too few to
        split refines them into their second-level children (refines = [rank]) -- when that
        remainder is ONE board or the rank is heavy (a few lighter boards it finishes in the
        round anyway): the next step splits those records -- the device form of the reference
        handing on a partial board mid-search (DHT_Node.py:502-509), here for a subtree too heavy
        to leave on one GPU."""
    S = [[int(x[0]), int(x[1]), int(x[2])] for x in states]
    heavy = [bool(x[3]) if len(x) > 3 else False for x in states]
    moves, takers = [], set()
    split = max(2, min_split)
    for r in range(len(S)):
        if S[r][1] > S[r][0]:
            continue
        cands = [k for k in range(len(S)) if k not in takers and k != r]
        if not cands:
            continue
        donor = max(cands, key=lambda k: (S[k][1] - S[k][0], -k))
        rem = S[donor][1] - S[donor][0]
        if rem < split:
            continue
        mid = S[donor][0] + rem // 2
        end = S[donor][1]
        by_records = bool(S[donor][2] or S[r][2])
        moves.append((donor, r, mid, end, by_records))
        S[r] = [0, end - mid, 1] if by_records else [mid, end, S[r][2]]
        S[donor][1] = mid
        takers.add(r)
    refines = []
    if any(b <= a for a, b, _ in S):
        refines = [k for k in range(len(S)) if 0 < S[k][1] - S[k][0] < split and k not in takers
                   and (S[k][1] - S[k][0] == 1 or heavy[k])]
    return S, moves, refines


def refine_target(world, min_split):
    """Boards a rank's refined subtree should come to: enough to give every rank a split."""
    return max(4 * world, 2 * max(2, min_split))


def sharded_count_rebalanced(engine, board, rank, world, limit=0, comm=None, target=None, chunk=None, info=None,
                             ranges=None, move_records=True):
    """sharded_count with dynamic rebalancing.

    Each rank starts on a contiguous block of the replicated frontier (or on `ranges`, one
    (lo, hi) per rank, the same on every rank) and counts it `chunk` boards per round.  Before
    every round the ranks all-gather their state (lo, hi, local: RCCL ncclAllGather of 3 x int64
    per rank on device memory, or gloo / TcpComm in the CPU tests) and rebalance_plan moves work
    to ranks that ran dry: the upper half of the largest live range -- as an index range while
    both frontiers are the replicated one, else as board records sent with grouped
    ncclSend/ncclRecv (comm.p2p) straight from the donor's frontier into the receiver's.  A
    rank left with too few boards to split while another is dry refines them into their
    second-level children first (engine.frontier_refine_range) and skips that round's count, so
    the next round can hand half of them on: one heavy subtree does not stay on one GPU.
    Counts (with the completions each rank met while refining) are combined by one
    all-reduce(sum) at the end.  move_records=False keeps round 3's index-only rebalancing.
    Returns (total, status, frontier_size) like sharded_count; `info` (dict) gets rounds,
    steals, moved records and refinements."""
    if world > 1 and comm is None:
        raise ValueError("world > 1 needs a comm (RcclComm or HostComm)")
    size, leaves = engine.frontier_build(board, mode=L.SDK_FRONTIER_COUNT,
                                         target=count_target(engine, world) if target is None else target)
    if chunk is None:   # one launch when there is no one to rebalance with; else 2 boards per resident wave
        chunk = max(1, size) if comm is None else max(1, default_target(engine, 1) // 4)
    min_split = max(2, chunk // 2)
    lo, hi = shard_bounds(size, rank, world) if ranges is None else (int(ranges[rank][0]), int(ranges[rank][1]))
    lo, hi = min(lo, size), min(hi, size)
    local = 0
    res = engine.result_buffer(2, np.uint64)
    mine = engine.result_buffer(3, np.int64)
    allr = engine.result_buffer(3 * world, np.int64)
    tot = engine.result_buffer(2, np.uint64)
    inbox = None                                         # receive buffer of moved records (grown as needed)
    count = hits = rounds = steals = moved = refined = 0
    own_leaves = 0
    try:
        while True:
            skip = False
            if comm is not None:
                _store(mine, [lo, hi, local], np.int64)
                comm.allgather(mine, allr, 24)
                S = engine.read(allr, 3 * world, np.int64).reshape(world, 3)
                if all(b <= a for a, b, _ in S):
                    break
                if move_records:
                    newS, moves, refines = rebalance_plan(S, min_split=min_split)
                else:
                    newR = rebalance_ranges(S[:, :2], min_split=min_split)
                    newS = [[a, b, 0] for a, b in newR]
                    moves, refines = [], []
                steals += sum(1 for a, b in zip(S.tolist(), newS) if a[:2] != b[:2] and a[1] <= a[0])
                ops, got = [], None
                for donor, recv, mid, end, by_records in moves:
                    if not by_records:
                        continue
                    moved += end - mid
                    if rank == donor:
                        ops.append((L.SDK_COMM_SEND, recv) + engine.frontier_records(mid, end))
                    elif rank == recv:
                        inbox = _grow_records(engine, inbox, end - mid)
                        ops.append((L.SDK_COMM_RECV, donor, inbox, 81 * (end - mid)))
                        got = end - mid
                if any(m[4] for m in moves):
                    comm.p2p(ops)                         # every rank: a collective on host transports
                if got is not None:
                    engine.frontier_load(inbox, got)
                lo, hi, local = (int(v) for v in newS[rank])
                if rank in refines:
                    n_kids, lv = engine.frontier_refine_range(lo, hi, refine_target(world, min_split))
                    own_leaves += lv
                    lo, hi, local = 0, n_kids, 1
                    refined += 1
                    skip = True
            end = min(hi, lo + chunk)
            if end > lo and not skip:
                engine.frontier_count(lo, 1, end, limit, res)
                c, h = (int(x) for x in engine.read(res, 2, np.uint64))
                count += c
                hits += h
                lo = end
                if limit and count + own_leaves >= limit:
                    lo = hi                                    # this rank alone reached the limit
            rounds += 1
            if comm is None and lo >= hi:                     # single rank, nothing to exchange
                break
        _store(tot, [count + own_leaves, hits], np.uint64)
        if comm is not None:
            comm.allreduce(tot, 2, np.uint64, "sum")
        count, hits = (int(x) for x in engine.read(tot, 2, np.uint64))
    finally:
        for h in (res, mine, allr, tot, inbox):
            if hasattr(h, "free"):
                h.free()
    if info is not None:
        info.update(rounds=rounds, steals=steals, chunk=chunk, moved_records=moved, refines=refined)
    total = count + leaves
    if limit and total > limit:
        total = limit
    st = -2 if hits else (1 if total > 0 else 0)
    return total, st, size


def _grow_records(engine, buf, n):
    """A receive buffer for n board records (the engine's: a DeviceBuffer, or a host array)."""
    need = 81 * max(1, int(n))
    have = (buf.nbytes if hasattr(buf, "nbytes") else 0) if buf is not None else 0
    if buf is not None and have >= need:
        return buf
    if buf is not None and hasattr(buf, "free"):
        buf.free()
    return engine.record_buffer(max(need, 2 * have) // 81)
