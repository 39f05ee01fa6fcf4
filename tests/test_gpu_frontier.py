"""expand4_kernel (four boards per wave, solve4's round) builds the same frontier, byte for byte,
as expand_kernel (one board per wave): first-solution frontiers compared board by board, count
frontiers by size, leaves and the counts below them (the oracle's counter)."""
import ctypes

import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth, _lib as L
from distributed_sudoku_solver_amd.engine import range_to_mask
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _random_puzzles(n, seed, lo_clues, hi_clues):
    rng = np.random.default_rng(seed)
    _, sol = synth.make_17clue(n, seed=seed)
    keep = rng.random((n, 81)) < rng.uniform(lo_clues, hi_clues, (n, 1)) / 81.0
    return np.where(keep, sol, 0).astype(np.uint8)


def _with_solver(engine, solver, fn):
    engine.set_option(L.SDK_OPT_SOLVER, solver)
    try:
        return fn()
    finally:
        engine.set_option(L.SDK_OPT_SOLVER, L.SDK_SOLVER_QUAD)


@pytest.mark.parametrize("target", [1, 64, 5000, 200_000])
def test_first_mode_frontier_identical(engine, solve_cases, target):
    s1 = synth.SEEDS17["S1"]
    seeds = [synth.parse(s1[:-9] + "000800000"), synth.parse(s1[:-9] + "0" * 9),
             synth.parse(synth.WIKI)] + [np.array(c["puzzle"], np.uint8) for c in solve_cases[:20]]
    seeds += list(_random_puzzles(20, 91, 10, 24))
    dead = synth.parse(synth.WIKI).copy()
    dead[2] = 5
    seeds.append(dead)
    for k, b in enumerate(seeds):
        mask = np.array([range_to_mask(range(1 + k % 5, 10))], np.uint16)
        quad = engine.expand(b[None], mask, target=target)
        half = _with_solver(engine, L.SDK_SOLVER_HALFWAVE, lambda: engine.expand(b[None], mask, target=target))
        assert quad.shape == half.shape and (quad == half).all(), (k, target)
    # several seeds at once, each with its own first-cell range
    b = np.array([c["puzzle"] for c in solve_cases[:40]], np.uint8)
    m = np.array([range_to_mask(range(*c["range"])) for c in solve_cases[:40]], np.uint16)
    quad = engine.expand(b, m, target=target)
    half = _with_solver(engine, L.SDK_SOLVER_HALFWAVE, lambda: engine.expand(b, m, target=target))
    assert quad.shape == half.shape and (quad == half).all()


def test_count_mode_frontier_identical(engine):
    s1 = synth.SEEDS17["S1"]
    b15 = s1[:-9] + "0" * 9
    boards = [synth.parse(s1[:-9] + "000800000"), synth.parse(b15), synth.parse(b15[:63] + "000100000" + "0" * 9)]
    boards += list(_random_puzzles(10, 93, 22, 30))
    for b in boards:
        for target in (10, 1000, 300_000):
            q = engine.frontier_build(b, mode=L.SDK_FRONTIER_COUNT, target=target)
            h = _with_solver(engine, L.SDK_SOLVER_HALFWAVE,
                             lambda: engine.frontier_build(b, mode=L.SDK_FRONTIER_COUNT, target=target))
            assert q == h, (target, q, h)
    for b in boards[3:]:
        assert engine.count_solutions(b)[0] == O.count(b, 0, 1)
    assert engine.count_solutions(boards[1]) == (3481026, 1)


def _count(e, lo, hi):
    res = e.result_buffer(2, np.uint64)
    try:
        e.frontier_count(lo, 1, hi, 0, res)
        c, h = (int(x) for x in e.read(res, 2, np.uint64))
    finally:
        res.free()
    assert h == 0
    return c


def test_frontier_records_move_and_refine(engine):
    """The device primitives of the record-moving rebalance (shard.sharded_count_rebalanced):
    records [mid, size) of one context's frontier, loaded into another context's frontier
    straight from device memory (what ncclSend/ncclRecv move between ranks), count what they
    counted in place; a range refined into second-level records keeps its count (15-clue C5
    board, 3,481,026 completions in all)."""
    s1 = synth.SEEDS17["S1"]
    b15 = synth.parse(s1[:-9] + "0" * 9)
    a, b = engine.fork(), engine.fork()
    try:
        size, leaves = a.frontier_build(b15, mode=L.SDK_FRONTIER_COUNT, target=4096)
        assert size >= 4096
        mid = size // 3
        whole = _count(a, 0, size)
        assert whole + leaves == 3481026
        ptr, nbytes = a.frontier_records(mid, size)
        assert nbytes == 81 * (size - mid)
        b.frontier_load(ptr, size - mid)
        assert b.frontier_boards()[1] == size - mid
        assert _count(a, 0, mid) + _count(b, 0, size - mid) == whole
        # one board's subtree, refined into its second-level records: same count
        one = _count(a, 7, 8)
        k, lv = a.frontier_refine_range(7, 8, 64)
        assert k >= 2 and _count(a, 0, k) + lv == one
        # records from a DeviceBuffer (a receive buffer), and a range of the context's own frontier
        buf = b.record_buffer(5)
        ptr, nbytes = b.frontier_records(0, 5)
        host = np.empty(nbytes, np.uint8)
        L.check(b.lib.sdk_memcpy_d2h(b.ctx, host.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), nbytes))
        buf.upload(host)
        first5 = sum(_count(b, i, i + 1) for i in range(5))
        a.frontier_load(buf, 5)
        assert _count(a, 0, 5) == first5
        p, n = b.frontier_boards()
        b.frontier_load(p + 81 * 2, 3)                   # overlapping: staged through the second buffer
        assert _count(b, 0, 3) == sum(_count(a, i, i + 1) for i in range(2, 5))
        buf.free()
    finally:
        a.close()
        b.close()
