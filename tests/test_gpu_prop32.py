"""The QUAD solver's bit-sliced propagation pass (prop32_kernel.h) against the reference fixtures, the
oracle and the search-only path: identical boards and statuses, whatever the pass decides itself and
whatever it hands to the search."""
import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth, _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ORDERS = [L.SDK_ORDER_LEX, L.SDK_ORDER_MRV_UNIQUE]
ORDER_IDS = ["lex", "mrv_unique"]


@pytest.fixture(params=ORDERS, ids=ORDER_IDS)
def p32_engine(request, engine):
    engine.set_option(L.SDK_OPT_SOLVER, L.SDK_SOLVER_QUAD)
    engine.set_option(L.SDK_OPT_ORDER, request.param)
    engine.set_option(L.SDK_OPT_PROP32, 1)
    yield engine
    engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX)
    engine.set_option(L.SDK_OPT_PROP32, 1)
    engine.set_option(L.SDK_OPT_PROP32_HANDOVER, 1)
    engine.set_option(L.SDK_OPT_PROP32_TAIL, 0)
    engine.set_option(L.SDK_OPT_NODE_BUDGET, 0)


def edge_boards(n, seed=5):
    """Out-of-domain and duplicated givens, contradictions, complete grids (valid and not), the empty
    board and easy boards -- on 37-clue boards, so the search stays short on the broken ones."""
    rng = np.random.default_rng(seed)
    base, _ = synth.make_30clue(n, seed=seed, extra=20)
    sol, _ = synth.make_30clue(n, seed=seed + 1, extra=64)
    out = base.copy()
    for i, k in enumerate(rng.integers(0, 8, n)):
        if k == 1:
            out[i, rng.integers(0, 81)] = rng.integers(10, 256)
        elif k == 2:
            r = rng.integers(0, 9)
            row = out[i, 9 * r:9 * r + 9]
            nz, z = np.flatnonzero(row), np.flatnonzero(row == 0)
            if len(nz) and len(z):
                out[i, 9 * r + z[0]] = row[nz[0]]
        elif k == 3:
            out[i] = sol[i]
        elif k == 4:
            out[i] = sol[i]
            c = rng.integers(0, 81)
            out[i, c] = out[i, c] % 9 + 1
        elif k == 5:
            out[i] = 0
        elif k == 6:
            out[i] = sol[i]
            out[i, rng.choice(81, 40, replace=False)] = 0
            nz = np.flatnonzero(out[i])
            c = nz[rng.integers(0, len(nz))]
            out[i, c] = out[i, c] % 9 + 1
    return out


def _both(engine, boards, **opts):
    """(out, status) with the pass on and off, same other options."""
    res = []
    for p in (1, 0):
        engine.set_option(L.SDK_OPT_PROP32, p)
        for k, v in opts.items():
            engine.set_option(getattr(L, k), v)
        out, st, _ = engine.solve_batch(boards)
        res.append((out, st))
    engine.set_option(L.SDK_OPT_PROP32, 1)
    return res


def test_prop32_golden_cases_tiled(p32_engine, solve_cases):
    """The reference's own solve fixtures (full digit range), tiled past the pass's minimum batch and
    a ragged last group: every copy as the fixture says."""
    cases = [c for c in solve_cases if tuple(c["range"]) == (1, 10)]
    puz = np.array([c["puzzle"] for c in cases], dtype=np.uint8)
    reps = (4096 + 37) // len(cases) + 1
    boards = np.tile(puz, (reps, 1))[:4096 + 37]
    out, st, _ = p32_engine.solve_batch(boards)
    for i in range(len(boards)):
        c = cases[i % len(cases)]
        assert (st[i] == 1) == c["ok"], (i, c["name"])
        assert out[i].tolist() == (c["board"] if c["ok"] else c["puzzle"]), (i, c["name"])


@pytest.mark.parametrize("kind", ["17clue", "30clue", "minimal"])
def test_prop32_matches_known_solutions(p32_engine, kind):
    """Unique-solution workloads with their solutions known by construction (the naive-DFS oracle
    takes minutes on 17-clue boards; its parity with these generators is pinned in test_gpu_solve)."""
    n = 8192 + 63
    if kind == "17clue":
        boards, sol = synth.make_17clue(n, seed=3)
    elif kind == "30clue":
        boards, sol = synth.make_30clue(n, seed=4)
    else:
        boards, sol = synth.make_minimal_sym(n, seed=5, threads=8)
    out, st, _ = p32_engine.solve_batch(boards)
    assert (st == 1).all()
    assert np.array_equal(out, sol)


@pytest.mark.parametrize("handover", [1, 0])
def test_prop32_edge_batch_same_as_search_only(p32_engine, handover):
    """Inert and duplicated givens, refutations at the root, complete grids and boards with many
    completions: the pass on (handing the rest over with or without their propagated grids) gives what
    the search alone gives, byte for byte, and the oracle agrees."""
    boards = edge_boards(4096 + 37)
    (o1, s1), (o0, s0) = _both(p32_engine, boards, SDK_OPT_PROP32_HANDOVER=handover)
    assert np.array_equal(s1, s0)
    assert np.array_equal(o1, o0)
    ref_out, ref_st, _ = O.naive_solve_batch(boards, threads=8)
    assert np.array_equal(s1 == 1, ref_st == 1)
    assert np.array_equal(o1, ref_out)


def test_prop32_tail_handoff_same_answers(p32_engine):
    boards = np.concatenate([edge_boards(2048, seed=7), synth.make_minimal_sym(4096, seed=9, threads=8)[0]])
    (o1, s1), (o0, s0) = _both(p32_engine, boards, SDK_OPT_PROP32_TAIL=4 | (8 << 8))
    assert np.array_equal(s1, s0) and np.array_equal(o1, o0)


def test_prop32_with_node_budget(p32_engine):
    """A node budget applies to the search from each board's input: the pass then hands over inputs,
    not propagated grids.  solve4's node count for a board is not a pure function of the board -- a
    branch is refuted a round earlier or later depending on whether every board of its wave is exact
    and past its first round (solve4_kernel.h unit4x / unit4f), i.e. on the boards it shares a wave
    with -- so a board near the budget can be a budget hit in one batch and solved in another, with or
    without the pass.  Asserted: the same answers wherever both solve, budget hits only where the
    other side solves or also hits, their input back, and few such boards."""
    boards, sol = synth.make_minimal_sym(8192, seed=13, threads=8)
    (o1, s1), (o0, s0) = _both(p32_engine, boards, SDK_OPT_NODE_BUDGET=24)
    assert (s0 == L.SDK_BUDGET_HIT).any()
    assert set(np.unique(s1).tolist()) <= {1, L.SDK_BUDGET_HIT} and set(np.unique(s0).tolist()) <= {1, L.SDK_BUDGET_HIT}
    for o, st in ((o1, s1), (o0, s0)):
        assert np.array_equal(o[st == 1], sol[st == 1])
        assert np.array_equal(o[st != 1], boards[st != 1])
    assert np.count_nonzero(s1 != s0) <= len(boards) // 200


def test_prop32_decides_every_c4_board(engine):
    """The headline workload: the pass decides every board (nothing handed to the search)."""
    engine.set_option(L.SDK_OPT_PROP32, 1)
    boards, sol = synth.make_17clue(65536, seed=20250614)
    engine.timer_reset()
    out, st, _ = engine.solve_batch(boards)
    _, spans = engine.timer_read()
    engine.timer_stop()
    assert spans == 2                     # the pass ran (its span and its fallback's)
    assert engine.get_option(L.SDK_OPT_PROP32_UNDECIDED) == 0
    assert (st == 1).all() and np.array_equal(out, sol)


def test_prop32_below_minimum_batch_not_used(engine):
    engine.set_option(L.SDK_OPT_PROP32, 1)
    boards, sol = synth.make_17clue(engine.get_option(L.SDK_OPT_PROP32_MIN) - 1, seed=2)
    engine.timer_reset()
    out, st, _ = engine.solve_batch(boards)
    _, spans = engine.timer_read()
    engine.timer_stop()
    assert spans == 1                     # the search alone
    assert np.array_equal(out, sol)


def test_prop32_options_validated(engine):
    for key, bad in ((L.SDK_OPT_PROP32, 2), (L.SDK_OPT_PROP32_LC, 0), (L.SDK_OPT_PROP32_MIN, 0),
                     (L.SDK_OPT_PROP32_HANDOVER, 3), (L.SDK_OPT_PROP32_TAIL, 65)):
        with pytest.raises(Exception):
            engine.set_option(key, bad)
    assert engine.get_option(L.SDK_OPT_PROP32) == 1


def test_prop32_fallback_split_phase_within_node_budget(engine):
    """a prop32 fallback batch with more than 2^19 undecided boards splits at 256 nodes
    only where the caller's node budget is above that; with a budget B <= 256 the split phase stays
    at 128, so no board is finished there past B nodes.  The split phase is one slot per board,
    so the count of boards it passes on is the witness: about the same under B = 129 and 200 (split
    128), several times more than under B = 0 or 300 (split 256; measured 1,661-1,665 against
    191-194).  (Not exactly equal: solve4's node count for a board depends on the boards it shares a
    wave with, see test_prop32_with_node_budget.)  Decided boards equal their known solutions;
    budget hits come back as their input."""
    engine.set_option(L.SDK_OPT_PROP32, 1)
    boards, sol = synth.make_hard_sym(1 << 20, threads=8)
    passed = {}
    for b in (0, 300, 129, 200):
        out, st, _ = engine.solve_batch(boards, budget=b)
        assert engine.get_option(L.SDK_OPT_PROP32_UNDECIDED) > (1 << 19)
        assert set(np.unique(st).tolist()) <= {1, L.SDK_BUDGET_HIT}, b
        assert np.array_equal(out[st == 1], sol[st == 1]), b
        assert np.array_equal(out[st != 1], boards[st != 1]), b
        if b == 0:
            assert (st == 1).all()
        passed[b] = engine.get_option(L.SDK_OPT_SPLIT_BOARDS)
    assert abs(passed[129] - passed[200]) <= 0.02 * passed[200], passed
    assert abs(passed[0] - passed[300]) <= 0.05 * passed[300] + 2, passed
    assert passed[200] > 4 * passed[300], passed


def test_prop32_not_used_without_locked_candidates_under_budget(engine):
    """prop32 always runs locked-candidates passes, so with SDK_OPT_LOCKED 0 and a node
    budget the search alone runs (one span); without a budget the pass still runs (two spans)."""
    engine.set_option(L.SDK_OPT_PROP32, 1)
    engine.set_option(L.SDK_OPT_LOCKED, 0)
    try:
        boards, sol = synth.make_17clue(8192, seed=4)
        for budget, spans_want in ((1000, 1), (0, 2)):
            engine.timer_reset()
            out, st, _ = engine.solve_batch(boards, budget=budget)
            _, spans = engine.timer_read()
            engine.timer_stop()
            assert spans == spans_want, budget
            assert np.array_equal(out[st == 1], sol[st == 1])
    finally:
        engine.set_option(L.SDK_OPT_LOCKED, 1)


@pytest.mark.parametrize("lc", [4, 5 | (3 << 8), 1, 7 | (1 << 8), 64])
def test_prop32_lc_schedules_same_answers(engine, lc):
    """Round 6: the locked-candidates schedule (SDK_OPT_PROP32_LC = period | first step << 8) only
    changes when the pass runs, never an answer: every schedule gives the search-only boards and
    statuses on the edge batch and minimal puzzles."""
    boards = np.concatenate([edge_boards(2048, seed=17), synth.make_minimal_sym(4096, seed=19, threads=8)[0]])
    try:
        (o1, s1), (o0, s0) = _both(engine, boards, SDK_OPT_PROP32_LC=lc)
    finally:
        engine.set_option(L.SDK_OPT_PROP32_LC, 5 | (3 << 8))
    assert np.array_equal(s1, s0) and np.array_equal(o1, o0)


def test_prop32_lc_option_encoding(engine):
    assert engine.get_option(L.SDK_OPT_PROP32_LC) == 5 | (3 << 8)          # the default schedule
    for bad in (0, 65, 5 | (65 << 8), 3 << 8):
        with pytest.raises(Exception):
            engine.set_option(L.SDK_OPT_PROP32_LC, bad)
    assert engine.get_option(L.SDK_OPT_PROP32_LC) == 5 | (3 << 8)


def test_prop32_clock_twin_same_answers_and_plausible_clock(engine):
    """The stamped twin of the pass (sdk_debug_clock_arm, the bench's live clock for roofline.valu)
    gives the same boards and statuses as the pass itself, and its stamps a clock inside the card's
    range (MI355X: at most 2.4 GHz)."""
    import ctypes
    lib = engine.lib
    engine.set_option(L.SDK_OPT_PROP32, 1)
    boards = np.concatenate([edge_boards(2048, seed=23), synth.make_17clue(8192, seed=29)[0]])
    out0, st0, _ = engine.solve_batch(boards)
    assert lib.sdk_debug_clock_arm(engine.ctx, 1) == 0
    try:
        out1, st1, _ = engine.solve_batch(boards)
        out4 = (ctypes.c_double * 4)()
        wgs = ctypes.c_int64()
        assert lib.sdk_debug_clock_read(engine.ctx, out4, ctypes.byref(wgs)) == 0
    finally:
        lib.sdk_debug_clock_arm(engine.ctx, 0)
    assert np.array_equal(st0, st1) and np.array_equal(out0, out1)
    assert wgs.value > 0
    assert 0.5 < out4[1] <= out4[0] <= out4[2] < 2.6, list(out4)
