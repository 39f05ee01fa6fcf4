"""SudokuEngine: numpy-level batch API over libsudoku_hip.so.

This is the host side of the drop-in boundary.  Every method
ends in a HIP kernel launched by the C library; nothing here computes a
solution or a verdict.
"""
import ctypes
import numbers
import threading

import numpy as np

from . import _lib as L

ALL_DIGITS_MASK = 0x3FE  # bits 1..9: range(1, 10)
INERT_VALUE = 10         # any given that is never equal to a digit 1..9


# ----------------------------------------------------------------- encoding
def _as_int(v):
    """The reference compares cells with `==` (utils.py:22,36,44,53): 5.0 == 5, True == 1."""
    if isinstance(v, numbers.Integral):
        return int(v)
    if isinstance(v, numbers.Real) and float(v).is_integer():
        return int(v)
    return None


def encode_solve_grid(grid):
    """9x9 (or flat 81) Python grid -> uint8[81] for the solver.

    0 -> empty; a value equal to a digit 1..9 -> that digit; anything else is a
    given that never equals a guess 1..9 (the reference never rejects it) and
    is encoded as the inert value 10."""
    flat = [v for row in grid for v in row] if len(grid) == 9 else list(grid)
    if len(flat) != 81:
        raise ValueError("a Sudoku grid has 81 cells")
    out = np.empty(81, dtype=np.uint8)
    for i, v in enumerate(flat):
        iv = _as_int(v)
        if iv == 0:
            out[i] = 0
        elif iv is not None and 1 <= iv <= 9:
            out[i] = iv
        else:
            out[i] = INERT_VALUE
    return out


CHECK_I64_LIMIT = 1 << 59   # sdk_check_batch_i64: |v| below this keeps a unit's sum exact


def encode_check_grid(grid):
    """9x9 grid -> uint8[81] (every value an integer 0..255) or int64[81] (any integer with
    |v| < 2^59) for the checker: the literal `sum == 45 and len(set) == 9` rule needs the exact
    values (5.0 counts as 5, like the reference's `==`).  Non-integral numbers raise ValueError."""
    flat = [v for row in grid for v in row] if len(grid) == 9 else list(grid)
    if len(flat) != 81:
        raise ValueError("a Sudoku grid has 81 cells")
    vals = []
    for i, v in enumerate(flat):
        iv = _as_int(v)
        if iv is None or not -CHECK_I64_LIMIT < iv < CHECK_I64_LIMIT:
            raise ValueError(f"cell {i} = {v!r}: the HIP checker takes integers with |v| < 2^59")
        vals.append(iv)
    if all(0 <= v <= 255 for v in vals):
        return np.array(vals, dtype=np.uint8)
    return np.array(vals, dtype=np.int64)


def range_to_mask(arr):
    """TASK digit range (a `range` from split_array_in_middle, utils.py:1-9) -> first-cell mask.

    bit d = digit d may be guessed at the lowest empty cell.  Guess 0 is never
    valid in the reference (the empty cell itself holds 0, utils.py:36), so it
    is dropped.  Order matters to the reference (`for guess in arr`), so only
    ascending digit sequences in 0..9 are representable."""
    vals = [_as_int(v) for v in arr]
    if any(v is None or v < 0 or v > 9 for v in vals):
        raise ValueError(f"digit range {arr!r} has values outside 0..9")
    if any(b <= a for a, b in zip(vals, vals[1:])):
        raise ValueError(f"digit range {arr!r} is not strictly ascending")
    m = 0
    for v in vals:
        if v >= 1:
            m |= 1 << v
    return m


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


# ------------------------------------------------------------------- device
class DeviceBuffer:
    """A device allocation owned by an engine context (for resident-input benchmarks)."""

    def __init__(self, engine, nbytes):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        L.check(engine.lib.sdk_dev_alloc(engine.ctx, self.nbytes, ctypes.byref(p)), "sdk_dev_alloc")
        self.ptr = p

    def upload(self, host, offset=0):
        """Copy `host` to this buffer at byte `offset`."""
        host = np.ascontiguousarray(host)
        if offset < 0 or offset + host.nbytes > self.nbytes:
            raise ValueError("upload out of bounds")
        dst = ctypes.c_void_p(self.ptr.value + int(offset))
        L.check(self.engine.lib.sdk_memcpy_h2d(self.engine.ctx, dst, _ptr(host), host.nbytes), "h2d")

    def download(self, host):
        assert host.flags.c_contiguous and host.nbytes <= self.nbytes
        L.check(self.engine.lib.sdk_memcpy_d2h(self.engine.ctx, _ptr(host), self.ptr, host.nbytes), "d2h")
        return host

    def free(self):
        if self.ptr is not None and self.engine.ctx is not None:
            L.check(self.engine.lib.sdk_dev_free(self.engine.ctx, self.ptr), "sdk_dev_free")
        self.ptr = None


class SudokuEngine:
    """One HIP device + stream.  Thread-safe (the C library serialises per context)."""

    def __init__(self, device=0, order=None, node_budget=None, waves_per_cu=None):
        self._tls = threading.local()
        self.lib = L.load()
        ctx = ctypes.c_void_p()
        L.check(self.lib.sdk_create(int(device), ctypes.byref(ctx)), f"sdk_create(device={device})")
        self.ctx = ctx
        self.device = device
        if order is not None:
            self.set_option(L.SDK_OPT_ORDER, order)
        if node_budget is not None:
            self.set_option(L.SDK_OPT_NODE_BUDGET, node_budget)
        if waves_per_cu is not None:
            self.set_option(L.SDK_OPT_WAVES_PER_CU, waves_per_cu)

    @classmethod
    def open_clique(cls, devices):
        """One engine per device of `devices`, joined by ONE RCCL communicator made
        in this process (sdk_comm_init_all = ncclCommInitAll); engine k is rank k.
        Collectives must then be issued from one host thread per engine."""
        lib = L.load()
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        ctxs = (ctypes.c_void_p * len(devices))()
        L.check(lib.sdk_comm_init_all(devs, len(devices), ctxs), f"sdk_comm_init_all({list(devices)})")
        engines = []
        for k, d in enumerate(devices):
            e = cls.__new__(cls)
            e.lib, e.ctx, e.device = lib, ctypes.c_void_p(ctxs[k]), int(d)
            e._tls = threading.local()
            engines.append(e)
        return engines

    # options a forked engine takes over (everything a caller sets that shapes a solve)
    _FORK_OPTIONS = (L.SDK_OPT_ORDER, L.SDK_OPT_NODE_BUDGET, L.SDK_OPT_WAVES_PER_CU, L.SDK_OPT_WORK_COUNTER,
                     L.SDK_OPT_SOLVER, L.SDK_OPT_WAVES_PER_CU2, L.SDK_OPT_SOLVE_CHUNK, L.SDK_OPT_LOCKED,
                     L.SDK_OPT_XCD_HEADS, L.SDK_OPT_DONATE, L.SDK_OPT_DONATE_MODE, L.SDK_OPT_DONATE_MAX,
                     L.SDK_OPT_DONATE_HELPERS, L.SDK_OPT_DONATE_RESUME, L.SDK_OPT_PROP32, L.SDK_OPT_PROP32_LC,
                     L.SDK_OPT_PROP32_MIN, L.SDK_OPT_PROP32_HANDOVER, L.SDK_OPT_PROP32_TAIL)

    def fork(self):
        """A second engine on the same device with its own context and stream (same options):
        its launches never queue behind this one's, and the GPU runs both at once.  A node
        gives its new batches and its long searches one each (node.py)."""
        e = SudokuEngine(self.device)
        for k in self._FORK_OPTIONS:
            e.set_option(k, self.get_option(k))
        return e

    # -------------------------------------------------------------- plumbing
    def close(self):
        if getattr(self, "ctx", None) is not None:
            self.lib.sdk_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_option(self, key, value):
        L.check(self.lib.sdk_set_option(self.ctx, key, int(value)), "sdk_set_option")

    def get_option(self, key):
        v = ctypes.c_int64()
        L.check(self.lib.sdk_get_option(self.ctx, key, ctypes.byref(v)), "sdk_get_option")
        return v.value

    def synchronize(self):
        L.check(self.lib.sdk_synchronize(self.ctx), "sdk_synchronize")

    def timer_reset(self):
        """Start (or restart) kernel timing: turns SDK_OPT_TIMING on and drops old events."""
        self.set_option(L.SDK_OPT_TIMING, 1)
        L.check(self.lib.sdk_timer_reset(self.ctx), "sdk_timer_reset")

    def timer_stop(self):
        """Stop recording kernel events (the pairs already made are kept for reuse)."""
        self.set_option(L.SDK_OPT_TIMING, 0)

    def timer_read(self):
        ms = ctypes.c_double()
        n = ctypes.c_int64()
        L.check(self.lib.sdk_timer_read(self.ctx, ctypes.byref(ms), ctypes.byref(n)), "sdk_timer_read")
        return ms.value, n.value

    def alloc(self, nbytes):
        return DeviceBuffer(self, nbytes)

    # ----------------------------------------------------------- host batch
    def check_batch(self, boards):
        """uint8[n,81] (or int64[n,81]: sdk_check_batch_i64) -> uint8[n] verdict bits
        (SDK_CHECK_OK | SDK_CHECK_RAW_NAMEERROR)."""
        wide = np.asarray(boards).dtype == np.int64
        boards = np.ascontiguousarray(boards, dtype=np.int64 if wide else np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        verdict = np.empty(n, dtype=np.uint8)
        fn = self.lib.sdk_check_batch_i64 if wide else self.lib.sdk_check_batch
        L.check(fn(self.ctx, _ptr(boards), _ptr(verdict), n), "sdk_check_batch_i64" if wide else "sdk_check_batch")
        return verdict

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        """uint8[n,81] (+ optional uint16[n] first-cell masks) -> (out uint8[n,81], status int8[n], work).

        budget: search nodes per board for this call (0 = unlimited), None = the context's
        SDK_OPT_NODE_BUDGET.  A board that runs out is SDK_BUDGET_HIT.
        donate: SDK_OPT_DONATE for this call only (0 = one launch, one slot per board: what a
        bounded slice of search.LexSearch or a node's batch wants), None = the context's.
        Both are arguments of the one sdk_solve_batch_ex call: the shared context options are
        never touched, so threads sharing an engine cannot see each other's settings."""
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        if masks is not None:
            masks = np.ascontiguousarray(masks, dtype=np.uint16).reshape(n)
        out = np.empty_like(boards)
        status = np.empty(n, dtype=np.int8)
        work = np.empty(n, dtype=np.uint64) if want_work else None
        if budget is not None and not 0 <= int(budget) < (1 << 63):
            raise ValueError("budget must be 0 (unlimited) or a positive node count")
        if donate is not None and not 0 <= int(donate) <= (1 << 30):
            raise ValueError("donate must be 0, 1 or a split budget >= 2")
        if not hasattr(self.lib, "sdk_solve_batch_ex"):
            # an older library named by SDK_LIB_PATH (dev A/B builds): per-call donate by the option
            return self._solve_batch_old(boards, masks, out, status, work, budget, donate)
        L.check(self.lib.sdk_solve_batch_ex(self.ctx, _ptr(boards), _ptr(masks), _ptr(out), _ptr(status), _ptr(work),
                                            n, L.SDK_BUDGET_CONTEXT if budget is None else int(budget),
                                            L.SDK_DONATE_CONTEXT if donate is None else int(donate)),
                "sdk_solve_batch_ex")
        return out, status, work

    def _solve_batch_old(self, boards, masks, out, status, work, budget, donate):
        old = self.get_option(L.SDK_OPT_DONATE)
        if donate is not None:
            self.set_option(L.SDK_OPT_DONATE, int(donate))
        try:
            L.check(self.lib.sdk_solve_batch_budget(self.ctx, _ptr(boards), _ptr(masks), _ptr(out), _ptr(status),
                                                    _ptr(work), len(boards),
                                                    L.SDK_BUDGET_CONTEXT if budget is None else int(budget)),
                    "sdk_solve_batch_budget")
        finally:
            self.set_option(L.SDK_OPT_DONATE, old)
        return out, status, work

    def expand(self, boards, masks=None, target=64):
        """Lex-ordered frontier below `boards` (sdk_expand_boards): uint8[k,81], children in the
        reference's DFS order, parents' order kept; at least one level, >= target boards unless
        nothing branches.  Contradicted subtrees vanish, solved boards stay."""
        boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
        n = boards.shape[0]
        if masks is not None:
            masks = np.ascontiguousarray(masks, dtype=np.uint16).reshape(n)
        cap = 9 * max(n, int(target), 1)
        # a per-thread staging buffer, grown as needed: a fresh 9 x target board array per call
        # is megabytes of new pages for every slice of a continued search (search.LexSearch)
        tl = self._tls
        out = getattr(tl, "expand_buf", None)
        if out is None or out.shape[0] < cap:
            out = tl.expand_buf = np.empty((cap, 81), dtype=np.uint8)
        k = ctypes.c_uint64()
        L.check(self.lib.sdk_expand_boards(self.ctx, _ptr(boards), _ptr(masks), n, int(target), _ptr(out), cap,
                                           ctypes.byref(k)), "sdk_expand_boards")
        return out[:k.value].copy()

    def count_solutions(self, board, limit=0):
        board = np.ascontiguousarray(board, dtype=np.uint8).reshape(81)
        cnt = ctypes.c_uint64()
        st = ctypes.c_int8()
        L.check(self.lib.sdk_count_solutions(self.ctx, _ptr(board), int(limit), ctypes.byref(cnt), ctypes.byref(st)),
                "sdk_count_solutions")
        return cnt.value, st.value

    def count_solutions_slice(self, board, rank, world, limit=0):
        """This rank's share of a frontier-split count: (local_count, frontier_size, status)."""
        board = np.ascontiguousarray(board, dtype=np.uint8).reshape(81)
        cnt = ctypes.c_uint64()
        fr = ctypes.c_uint64()
        st = ctypes.c_int8()
        L.check(self.lib.sdk_count_solutions_slice(self.ctx, _ptr(board), int(limit), int(rank), int(world),
                                                   ctypes.byref(cnt), ctypes.byref(fr), ctypes.byref(st)),
                "sdk_count_solutions_slice")
        return cnt.value, fr.value, st.value

    # frontier records (rebalanced counts move them between ranks)
    def frontier_boards(self):
        """(device address, size) of the current frontier's uint8[size][81] records."""
        p = ctypes.c_void_p()
        size = ctypes.c_uint64()
        L.check(self.lib.sdk_frontier_boards_dev(self.ctx, ctypes.byref(p), ctypes.byref(size)),
                "sdk_frontier_boards_dev")
        return p.value, size.value

    def frontier_records(self, lo, hi):
        """(device address, bytes) of records [lo, hi) of the current frontier: what a rank sends
        to another (comm p2p) when it hands on part of its live subtrees."""
        p, size = self.frontier_boards()
        if not 0 <= lo <= hi <= size:
            raise ValueError(f"records [{lo}, {hi}) outside the frontier of {size}")
        return p + 81 * int(lo), 81 * (int(hi) - int(lo))

    def record_buffer(self, n):
        """A device buffer for n board records (a receive buffer of moved records)."""
        return self.alloc(81 * max(1, int(n)))

    def frontier_load(self, d_boards, n, offset=0):
        """The n records at device buffer `d_boards` (+ offset boards) become the current
        frontier (in the mode of the frontier built last)."""
        ptr = (d_boards.ptr.value if hasattr(d_boards, "ptr") else int(d_boards)) + 81 * int(offset)
        L.check(self.lib.sdk_frontier_load_dev(self.ctx, ctypes.c_void_p(ptr), int(n)), "sdk_frontier_load_dev")

    def frontier_refine_range(self, lo, hi, target):
        """Keep frontier boards [lo, hi) and expand them until they number `target`: (size, leaves)."""
        size = ctypes.c_uint64()
        leaves = ctypes.c_uint64()
        L.check(self.lib.sdk_frontier_refine_range(self.ctx, int(lo), int(hi), int(target), ctypes.byref(size),
                                                   ctypes.byref(leaves)), "sdk_frontier_refine_range")
        return size.value, leaves.value

    def frontier_refine_head(self, lo, mid, hi, target):
        """Frontier boards [lo, mid) refined towards `target`, then [mid, hi) unchanged: (size, leaves)."""
        size = ctypes.c_uint64()
        leaves = ctypes.c_uint64()
        L.check(self.lib.sdk_frontier_refine_head(self.ctx, int(lo), int(mid), int(hi), int(target),
                                                  ctypes.byref(size), ctypes.byref(leaves)),
                "sdk_frontier_refine_head")
        return size.value, leaves.value

    # ------------------------------------------- one-board multi-GPU searches
    def frontier_build(self, board, mask=None, mode=L.SDK_FRONTIER_COUNT, target=0):
        """Build the deterministic frontier of `board` on this GPU: (size, leaves)."""
        board = np.ascontiguousarray(board, dtype=np.uint8).reshape(81)
        m = None if mask is None else np.array([int(mask)], dtype=np.uint16)
        size = ctypes.c_uint64()
        leaves = ctypes.c_uint64()
        L.check(self.lib.sdk_frontier_build(self.ctx, _ptr(board), _ptr(m), int(mode), int(target),
                                            ctypes.byref(size), ctypes.byref(leaves)), "sdk_frontier_build")
        return size.value, leaves.value

    def frontier_refine(self, first, step, target):
        """Keep frontier boards first, first+step, ... and expand them on this GPU until they
        number `target` (the rank-local second stage of a split): (size, leaves met)."""
        size = ctypes.c_uint64()
        leaves = ctypes.c_uint64()
        L.check(self.lib.sdk_frontier_refine(self.ctx, int(first), int(step), int(target), ctypes.byref(size),
                                             ctypes.byref(leaves)), "sdk_frontier_refine")
        return size.value, leaves.value

    def frontier_count(self, first, step, end, limit, d_result):
        """Completions below frontier boards first, first+step, ... < end -> d_result {count, budget hits}."""
        L.check(self.lib.sdk_frontier_count_dev(self.ctx, int(first), int(step), int(end), int(limit), d_result.ptr),
                "sdk_frontier_count_dev")

    def frontier_first(self, lo, hi, d_found, d_best):
        """Lex-ordered scan step: lowest hit index in [lo, hi) -> d_found, its board + status -> d_best."""
        L.check(self.lib.sdk_frontier_first_dev(self.ctx, int(lo), int(hi), d_found.ptr, d_best.ptr),
                "sdk_frontier_first_dev")

    def result_buffer(self, count, dtype):
        """A small device buffer for per-rank results (a handle for the comm layer)."""
        buf = self.alloc(count * np.dtype(dtype).itemsize)
        buf.upload(np.zeros(count, dtype=dtype))
        return buf

    def read(self, buf, count, dtype):
        out = np.empty(count, dtype=dtype)
        return buf.download(out)

    # ----------------------------------------------------------------- RCCL
    @staticmethod
    def comm_unique_id():
        lib = L.load()
        buf = (ctypes.c_uint8 * L.SDK_COMM_ID_BYTES)()
        L.check(lib.sdk_comm_unique_id(buf), "sdk_comm_unique_id")
        return bytes(buf)

    def comm_init(self, uid, rank, world):
        buf = (ctypes.c_uint8 * L.SDK_COMM_ID_BYTES).from_buffer_copy(uid)
        L.check(self.lib.sdk_comm_init(self.ctx, buf, int(rank), int(world)), "sdk_comm_init")

    def comm_destroy(self):
        L.check(self.lib.sdk_comm_destroy(self.ctx), "sdk_comm_destroy")

    def comm_allreduce(self, d_buf, count, dtype, op):
        L.check(self.lib.sdk_comm_allreduce_dev(self.ctx, d_buf.ptr, int(count), int(dtype), int(op)),
                "sdk_comm_allreduce_dev")

    def comm_broadcast(self, d_buf, nbytes, root):
        L.check(self.lib.sdk_comm_broadcast_dev(self.ctx, d_buf.ptr, int(nbytes), int(root)), "sdk_comm_broadcast_dev")

    def comm_p2p(self, ops):
        """One grouped ncclSend/ncclRecv: ops = [(L.SDK_COMM_SEND | L.SDK_COMM_RECV, peer,
        device address or DeviceBuffer, nbytes), ...]."""
        k = len(ops)
        if k == 0:
            return
        kinds = (ctypes.c_int * k)(*[int(o[0]) for o in ops])
        peers = (ctypes.c_int * k)(*[int(o[1]) for o in ops])
        bufs = (ctypes.c_void_p * k)(*[(o[2].ptr.value if hasattr(o[2], "ptr") else int(o[2])) for o in ops])
        sizes = (ctypes.c_size_t * k)(*[int(o[3]) for o in ops])
        L.check(self.lib.sdk_comm_p2p_dev(self.ctx, k, kinds, peers, bufs, sizes), "sdk_comm_p2p_dev")

    def comm_allgather(self, d_send, d_recv, nbytes):
        L.check(self.lib.sdk_comm_allgather_dev(self.ctx, d_send.ptr, d_recv.ptr, int(nbytes)),
                "sdk_comm_allgather_dev")

    # --------------------------------------------------------- device batch
    def check_batch_dev(self, d_boards, d_verdict, n):
        L.check(self.lib.sdk_check_batch_dev(self.ctx, d_boards.ptr, d_verdict.ptr, int(n)), "sdk_check_batch_dev")

    def solve_batch_dev(self, d_in, d_out, d_status, n, d_mask=None, d_work=None):
        L.check(self.lib.sdk_solve_batch_dev(self.ctx, d_in.ptr, d_mask.ptr if d_mask else None, d_out.ptr,
                                             d_status.ptr, d_work.ptr if d_work else None, int(n)),
                "sdk_solve_batch_dev")
