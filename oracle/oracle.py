"""oracle.py -- Python handle on the CPU restatement of the reference hot path.

*** TEST INFRASTRUCTURE ONLY ***  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  The product
(distributed_sudoku_solver_amd + libsudoku_hip.so) never imports it.

Two restatements, cross-checked against each other and against the golden
vectors the reference produced (tests/golden/make_golden.py):

* ``liboracle.so`` (sudoku_oracle.c): naive DFS with the reference's exact
  ``validations`` count, the literal Sudoku.check(), a solution counter.
* ``py_naive_solve`` / ``py_check``: pure-Python loops that follow
  DHT_Node.py:474-538 / utils.py:14-56 / sudoku.py:43-94 line by line (small
  cases only).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
ALL_DIGITS = 0x3FE

_lib = None


def build(force=False):
    """Compile liboracle.so with gcc (no reference sources are involved)."""
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "sudoku_oracle.c"))
    ):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_naive_solve.argtypes = [u8p, ctypes.c_uint16, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.orc_naive_solve.restype = ctypes.c_int
        L.orc_check.argtypes = [u8p]
        L.orc_check.restype = ctypes.c_uint8
        L.orc_count.argtypes = [u8p, ctypes.c_int64, ctypes.c_int]
        L.orc_count.restype = ctypes.c_int64
        L.orc_naive_solve_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int]
        L.orc_naive_solve_batch.restype = ctypes.c_int
        L.orc_check_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.orc_check_batch.restype = ctypes.c_int
        _lib = L
    return _lib


def _u8(cells):
    a = np.ascontiguousarray(np.asarray(cells, dtype=np.uint8).reshape(81))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def range_mask(lo, hi):
    """TASK `range(lo, hi)` -> first-cell digit mask, bit d = digit d."""
    m = 0
    for d in range(max(lo, 1), min(hi, 10)):
        m |= 1 << d
    return m


def naive_solve(cells, mask=ALL_DIGITS, budget=0):
    """C restatement. Returns (status, board, validations); status 1/0/-2."""
    a, p = _u8(cells)
    v = ctypes.c_uint64(0)
    st = lib().orc_naive_solve(p, mask, budget, ctypes.byref(v))
    return st, a.tolist(), v.value


def check(cells):
    """Literal Sudoku.check(): returns verdict byte (bit0 intended ok, bit1 raw NameError)."""
    a, p = _u8(cells)
    return int(lib().orc_check(p))


def count(cells, limit=0, order=1):
    a, p = _u8(cells)
    return int(lib().orc_count(p, limit, order))


def naive_solve_batch(boards, masks=None, budget=0, threads=1):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    n = boards.shape[0]
    out = np.empty_like(boards)
    status = np.empty(n, dtype=np.int8)
    val = np.empty(n, dtype=np.uint64)
    mp = None
    if masks is not None:
        masks = np.ascontiguousarray(masks, dtype=np.uint16)
        mp = masks.ctypes.data
    lib().orc_naive_solve_batch(boards.ctypes.data, mp, out.ctypes.data, status.ctypes.data, val.ctypes.data,
                                n, budget, threads)
    return out, status, val


def check_batch(boards, threads=1):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    out = np.empty(boards.shape[0], dtype=np.uint8)
    lib().orc_check_batch(boards.ctypes.data, out.ctypes.data, boards.shape[0], threads)
    return out


# --------------------------------------------------------------- pure Python
class _Budget(Exception):
    pass


def py_naive_solve(cells, lo=1, hi=10, budget=0):
    """Line-by-line Python restatement of DHTNode.solve_sudoku (DHT_Node.py:474-538),
    with find_next_empty (utils.py:14-25) and is_valid (utils.py:27-56) inlined.
    Returns (ok, board, validations); ok is None when `budget` (> 0) validations
    were spent first (the per-puzzle timeout of the cpu_baseline leg).  Small cases only."""
    grid = [list(cells[9 * r: 9 * r + 9]) for r in range(9)]
    counter = [0]

    def find_next_empty():
        for r in range(9):
            for c in range(9):
                if grid[r][c] == 0:
                    return r, c
        return None, None

    def is_valid(guess, row, col):
        if guess in grid[row]:
            return False
        if guess in [grid[i][col] for i in range(9)]:
            return False
        rs, cs = (row // 3) * 3, (col // 3) * 3
        for r in range(rs, rs + 3):
            for c in range(cs, cs + 3):
                if grid[r][c] == guess:
                    return False
        return True

    def solve(arr):
        counter[0] += 1                      # DHT_Node.py:513
        if budget and counter[0] > budget:
            raise _Budget()
        row, col = find_next_empty()
        if row is None:
            return True
        for guess in arr:
            if is_valid(guess, row, col):
                counter[0] += 1              # DHT_Node.py:528
                grid[row][col] = guess
                if solve(range(1, 10)):      # DHT_Node.py:531 (default range)
                    return True
            grid[row][col] = 0               # DHT_Node.py:535
        return False

    try:
        ok = solve(range(lo, hi))
    except _Budget:
        return None, list(cells), counter[0]
    return ok, [v for row in grid for v in row], counter[0]


def py_check(cells):
    """Literal restatement of Sudoku.check (sudoku.py:43-94). Returns (raw, intended)
    with raw in {"False", "NameError"} ("True" is unreachable, see sudoku.py:68)."""
    g = [list(cells[9 * r: 9 * r + 9]) for r in range(9)]

    def ok(vals):
        return sum(vals) == 45 and len(set(vals)) == 9

    rows = all(ok(g[r]) for r in range(9))
    cols = rows and all(ok([g[r][c] for r in range(9)]) for c in range(9))
    boxes = cols and all(ok([g[3 * bi + k][3 * bj + l] for k in range(3) for l in range(3)])
                         for bi in range(3) for bj in range(3))
    box00_sum = sum(g[k][l] for k in range(3) for l in range(3))
    raw = "NameError" if (rows and cols and box00_sum == 45) else "False"
    return raw, bool(boxes)


def py_solve_timed(boards, seconds, budget=0):
    """Baseline worker (bench.py cpu_baseline leg): the Python restatement above on
    `boards` (list of 81-int lists) one after another until `seconds` have passed,
    each puzzle capped at `budget` validations (0 = none).
    Returns (done, solved, wall_s, timeouts)."""
    import time
    t0 = time.perf_counter()
    done = solved = timeouts = 0
    for cells in boards:
        if time.perf_counter() - t0 >= seconds:
            break
        ok, _, _ = py_naive_solve(cells, budget=budget)
        done += 1
        solved += int(bool(ok))
        timeouts += int(ok is None)
    return done, solved, time.perf_counter() - t0, timeouts


def py_check_timed(boards):
    """Baseline worker (bench.py checker cpu_baseline): py_check over `boards` (81-int lists).
    Returns (boards checked, intended-valid count, wall seconds)."""
    import time
    t0 = time.perf_counter()
    ok = 0
    for cells in boards:
        ok += int(py_check(cells)[1])
    return len(boards), ok, time.perf_counter() - t0
