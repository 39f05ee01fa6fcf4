"""Two-phase solve with subtree donation (SDK_OPT_DONATE, solve4_kernel<true>): boards that
need more than the split budget are solved again by the donation kernel, where idle waves
take their shallowest untried branches.  Whatever is donated, every board, status and
lex-first answer must be the one a single slot finds (and the reference's: the oracle's
naive DFS, DHT_Node.py:474-538)."""
import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth, _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _random_puzzles(n, seed, lo_clues, hi_clues):
    rng = np.random.default_rng(seed)
    _, sol = synth.make_17clue(n, seed=seed)
    keep = rng.random((n, 81)) < rng.uniform(lo_clues, hi_clues, (n, 1)) / 81.0
    return np.where(keep, sol, 0).astype(np.uint8)


def _masks(n, seed):
    rng = np.random.default_rng(seed)
    lo = rng.integers(1, 10, n)
    hi = np.minimum(10, lo + rng.integers(1, 10, n))
    return np.array([O.range_mask(a, b) for a, b in zip(lo, hi)], dtype=np.uint16)


SPLIT = 16    # a small split budget: most searching boards go through the donation phase


def _solve(engine, boards, masks=None, donate=SPLIT, budget=None, mode=1):
    engine.set_option(L.SDK_OPT_DONATE, donate)
    engine.set_option(L.SDK_OPT_DONATE_MODE, mode)
    engine.set_option(L.SDK_OPT_DONATE_MAX, 0)      # phased whatever the batch size
    try:
        out, st, work = engine.solve_batch(boards, masks, want_work=True, budget=budget)
        donated = engine.get_option(L.SDK_OPT_DONATED) if donate else 0
        split = engine.get_option(L.SDK_OPT_SPLIT_BOARDS)
    finally:
        engine.set_option(L.SDK_OPT_DONATE, 1)
        engine.set_option(L.SDK_OPT_DONATE_MODE, 1)
        engine.set_option(L.SDK_OPT_DONATE_MAX, 1 << 19)
    if not donate:
        assert split == 0
    return out, st, work, donated


_HARD = {}


def _heavy_minimal(engine, n_scan, keep, seed):
    """The `keep` puzzles of a slice of the committed hard set (distinct minimal unique puzzles
    that need >= 20 nodes of a singles DFS) that take solve4 the most search nodes."""
    if "p" not in _HARD:
        _HARD["p"], _HARD["s"], _ = synth.load_hard(threads=16)
    lo = seed % (len(_HARD["p"]) - n_scan)
    p, s = _HARD["p"][lo:lo + n_scan], _HARD["s"][lo:lo + n_scan]
    _, st, work, _ = _solve(engine, p, donate=0)
    assert (st == 1).all()
    idx = np.argsort(-work.astype(np.int64), kind="stable")[:keep]
    return p[idx], s[idx], work[idx]


def test_donation_option_roundtrip(engine):
    assert engine.get_option(L.SDK_OPT_DONATE) == 1
    for v in (0, 2, 300):
        engine.set_option(L.SDK_OPT_DONATE, v)
        assert engine.get_option(L.SDK_OPT_DONATE) == v
    engine.set_option(L.SDK_OPT_DONATE, 1)
    with pytest.raises(L.SudokuHipError):
        engine.set_option(L.SDK_OPT_DONATE, -1)
    assert engine.get_option(L.SDK_OPT_DONATE_MODE) == 1
    with pytest.raises(L.SudokuHipError):
        engine.set_option(L.SDK_OPT_DONATE_MODE, 2)
    for ro in (L.SDK_OPT_DONATED, L.SDK_OPT_SPLIT_BOARDS, L.SDK_OPT_LEX_BOARDS):
        with pytest.raises(L.SudokuHipError):
            engine.set_option(ro, 1)
    assert engine.get_option(L.SDK_OPT_DONATE_MAX) == 1 << 19
    with pytest.raises(L.SudokuHipError):
        engine.set_option(L.SDK_OPT_DONATE_MAX, -1)


def test_batch_over_donate_max_is_one_launch(engine):
    """A batch above SDK_OPT_DONATE_MAX is one launch (its heavy boards never split), with the
    same answers; at or below it the heavy boards go to the donation phase."""
    p, s, _ = _heavy_minimal(engine, 20000, 64, seed=5)
    engine.set_option(L.SDK_OPT_DONATE_MAX, len(p) - 1)
    try:
        out, st, _ = engine.solve_batch(p, want_work=True)
        assert engine.get_option(L.SDK_OPT_SPLIT_BOARDS) == 0
        assert engine.get_option(L.SDK_OPT_DONATED) == 0
        assert (st == 1).all() and (out == s).all()
        engine.set_option(L.SDK_OPT_DONATE_MAX, len(p))
        engine.set_option(L.SDK_OPT_DONATE, SPLIT)
        out, st, _ = engine.solve_batch(p, want_work=True)
        assert engine.get_option(L.SDK_OPT_SPLIT_BOARDS) > 0
        assert (st == 1).all() and (out == s).all()
    finally:
        engine.set_option(L.SDK_OPT_DONATE_MAX, 1 << 19)
        engine.set_option(L.SDK_OPT_DONATE, 1)


def test_easy_batch_takes_one_launch(engine):
    """Boards within the split budget never reach the donation phase (the C4 launch alone)."""
    p, s = synth.make_17clue(100_000, seed=9)
    out, st, _, donated = _solve(engine, p, donate=1)
    assert engine.get_option(L.SDK_OPT_SPLIT_BOARDS) == 0 and donated == 0
    assert (st == 1).all() and (out == s).all()


MODES = pytest.mark.parametrize("mode", [1, 0], ids=["exhaustive", "lex"])


@MODES
def test_heavy_unique_boards_donate_and_match(engine, mode):
    """A few heavy minimal puzzles alone on the chip: the whole grid is idle, so they donate;
    every board is still its generating grid, and the summed work covers the single-slot work."""
    p, s, w0 = _heavy_minimal(engine, 20000, 64, seed=3)
    assert w0.min() > 4 * SPLIT
    out, st, work, donated = _solve(engine, p, mode=mode)
    assert engine.get_option(L.SDK_OPT_SPLIT_BOARDS) == len(p) and donated > 0
    assert (st == 1).all() and (out == s).all()
    if mode == 0:
        assert (work >= w0).mean() > 0.5  # LEX: both phases and every part are counted
    out0, st0, _, _ = _solve(engine, p, donate=0)
    assert (out0 == out).all() and (st0 == st).all()


@MODES
@pytest.mark.parametrize("n", [1, 4, 37, 2000])
def test_multi_solution_lex_first_with_donation(engine, n, mode):
    """Sparse boards (many completions) with random first-cell ranges: the donated parts find
    completions in any order; the answer must still be the lex-first one (oracle)."""
    puz = _random_puzzles(n, 300 + n, 14, 24)
    masks = _masks(n, 301 + n)
    out, st, _, _ = _solve(engine, puz, masks, budget=0, mode=mode)
    if mode == 1 and n >= 37:
        assert engine.get_option(L.SDK_OPT_LEX_BOARDS) > 0     # several completions: the LEX re-solve ran
    out0, st0, _, _ = _solve(engine, puz, masks, donate=0, budget=0)
    assert (st == st0).all() and (out == out0).all()
    ref_out, ref_st, _ = O.naive_solve_batch(puz, masks, budget=20_000_000, threads=16)
    done = ref_st != -2
    assert done.mean() > 0.8
    assert (st[done] == ref_st[done]).all() and (out[done] == ref_out[done]).all()


@MODES
def test_unsolvable_and_budget_hit_with_donation(engine, mode):
    """'55' + 79 zeros (no completion, propagation cannot refute it) with a node budget: the
    donated parts hit the budget, so the board is SDK_BUDGET_HIT (undecided), never NO_SOLUTION
    and never a completion; refutable boards in the same launch stay exact."""
    c55 = np.zeros((1, 81), np.uint8)
    c55[0, :2] = 5
    p, s, _ = _heavy_minimal(engine, 4000, 8, seed=7)
    dup = s[:4].copy()
    dup[:, 0] = dup[:, 1]                                          # a given-vs-given conflict
    boards = np.concatenate([c55, p, np.where(np.arange(81) < 30, dup, 0).astype(np.uint8)])
    out, st, _, donated = _solve(engine, boards, budget=5000, mode=mode)
    assert donated > 0
    assert st[0] == L.SDK_BUDGET_HIT and (out[0] == c55[0]).all()
    assert (st[1:9] == 1).all() and (out[1:9] == s).all()
    assert (st[9:] != L.SDK_BUDGET_HIT).all()
    ref_out, ref_st, _ = O.naive_solve_batch(boards[9:], budget=20_000_000, threads=4)
    ok = ref_st != -2                         # the naive DFS may run out on a given-vs-given conflict
    assert (st[9:][ok] == ref_st[ok]).all() and (out[9:][ok] == ref_out[ok]).all()
    o0, s0, _, _ = _solve(engine, boards[9:], donate=0, budget=5000)
    assert (s0 == st[9:]).all() and (o0 == out[9:]).all()


def _corrupt(p, seed):
    """Change one clue of each puzzle to a digit its row, column and box do not hold: the units
    stay exact (no duplicated given) and the board almost always loses every completion, which
    propagation alone rarely proves -- unsolvable boards that search and donate."""
    rng = np.random.default_rng(seed)
    out = p.copy()
    for b in out:
        for i in rng.permutation(np.flatnonzero(b)):
            r, c = divmod(int(i), 9)
            br, bc = 3 * (r // 3), 3 * (c // 3)
            used = set(b[9 * r: 9 * r + 9]) | set(b[c::9]) | {b[9 * (br + k) + bc + j] for k in range(3) for j in range(3)}
            free = [d for d in range(1, 10) if d not in used]
            if free:
                b[i] = rng.choice(free)
                break
    return out


@MODES
def test_donation_under_small_budget_is_never_wrong(engine, mode):
    """With a tight per-part budget some boards end undecided; every decided board equals the
    single-slot unbudgeted answer (a budget hit never turns into a wrong completion), on
    multi-solution, unique and exact unsolvable boards."""
    heavy = _heavy_minimal(engine, 8000, 200, 99)[0]
    puz = np.concatenate([_random_puzzles(500, 77, 16, 26), heavy, _corrupt(heavy, 5)])
    masks = _masks(len(puz), 78)
    ref, rst, _, _ = _solve(engine, puz, masks, donate=0, budget=0)
    for budget in (65, 200, 1000):             # all above SPLIT: the donation phase runs
        out, st, _, _ = _solve(engine, puz, masks, budget=budget, mode=mode)
        dec = st != L.SDK_BUDGET_HIT
        assert dec.mean() > 0.3, budget
        assert (st[dec] == rst[dec]).all() and (out[dec] == ref[dec]).all(), budget
        assert (out[~dec] == puz[~dec]).all()


@MODES
def test_large_batch_with_hard_tail(engine, mode):
    """1M easy boards plus heavy minimal puzzles: the heavy ones are solved by donation at the
    end of the launch; everything equals its known answer."""
    p17, s17 = synth.make_17clue(1_000_000, seed=123)
    ph, sh, _ = _heavy_minimal(engine, 20000, 256, seed=11)
    boards = np.concatenate([p17, ph])
    out, st, _, _ = _solve(engine, boards, mode=mode)
    assert (st == 1).all()
    assert (out[:len(p17)] == s17).all() and (out[len(p17):] == sh).all()


def test_bounded_wait_reports_an_error(engine):
    """Every wait on another wave inside a donation launch is bounded (solve4_kernel.h
    kDnWaitTicks).  SDK_OPT_DN_FAULT (test only) makes idle waves skip writing their
    registration entry, so a donor's wait for it runs out: the launch still ends, the solve
    fails with SDK_EHIP naming the wait, and the next solve on the context is exact again."""
    fork = engine.fork()
    try:
        p, s, _ = _heavy_minimal(fork, 20000, 64, seed=3)
        fork.set_option(L.SDK_OPT_DN_FAULT, 1)
        assert fork.get_option(L.SDK_OPT_DN_FAULT) == 1
        with pytest.raises(L.SudokuHipError, match="bounded wait"):
            _solve(fork, p)
        fork.set_option(L.SDK_OPT_DN_FAULT, 0)
        out, st, _, donated = _solve(fork, p)
        assert donated > 0 and (st == 1).all() and (out == s).all()
    finally:
        fork.close()


def test_donation_beside_another_context_on_the_gpu(engine):
    """a donation launch must end whether or not its whole grid is resident at
    once.  Two contexts on one GPU run phased solves of the heavy boards at the same time (each
    launch's grid is the full resident grid, so neither fits beside the other); both finish
    promptly and exactly.  Round 3's kernel, which waited for the whole grid to be counted idle,
    took seconds here (profiles/r03/bench_2rank_shared_gpu.json: 4,155 ms for a 2 ms solve)."""
    import threading
    import time
    p, s, _ = _heavy_minimal(engine, 20000, 1000, seed=21)
    engines = [engine.fork(), engine.fork()]
    res, errs = {}, []

    def run(k):
        try:
            t0 = time.perf_counter()
            for _ in range(5):
                out, st, _, _ = _solve(engines[k], p)
                assert (st == 1).all() and (out == s).all()
            res[k] = time.perf_counter() - t0
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)

    try:
        ths = [threading.Thread(target=run, args=(k,)) for k in range(2)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(120)
        assert not errs, errs
        assert len(res) == 2 and max(res.values()) < 3.0, res
    finally:
        for e in engines:
            e.close()


def test_per_call_donate_leaves_the_context_option(engine):
    """solve_batch(donate=...) is one sdk_solve_batch_ex argument; the context's
    SDK_OPT_DONATE is never rewritten (threads sharing an engine cannot see each other's)."""
    p, s, _ = _heavy_minimal(engine, 20000, 64, seed=3)
    engine.set_option(L.SDK_OPT_DONATE_MAX, 0)
    try:
        assert engine.get_option(L.SDK_OPT_DONATE) == 1
        out, st, _ = engine.solve_batch(p, donate=SPLIT)
        assert engine.get_option(L.SDK_OPT_DONATE) == 1 and engine.get_option(L.SDK_OPT_SPLIT_BOARDS) == len(p)
        assert (st == 1).all() and (out == s).all()
        out, st, _ = engine.solve_batch(p, donate=0)
        assert engine.get_option(L.SDK_OPT_SPLIT_BOARDS) == 0 and (out == s).all()
    finally:
        engine.set_option(L.SDK_OPT_DONATE_MAX, 1 << 19)


def test_phased_solve_in_mrv_unique_order(engine):
    """The phased solve also runs under SDK_ORDER_MRV_UNIQUE (split phase counting to two
    completions, LEX re-search of multi-solution boards in the slot): heavy unique boards,
    sparse multi-solution boards with ranges and exact-unsolvable boards give the one-slot LEX
    answers (the reference's)."""
    heavy, hs, _ = _heavy_minimal(engine, 8000, 100, 41)
    puz = np.concatenate([heavy, _random_puzzles(300, 43, 14, 24), _corrupt(heavy[:50], 7)])
    masks = _masks(len(puz), 44)
    ref, rst, _, _ = _solve(engine, puz, masks, donate=0, budget=0)
    engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_MRV_UNIQUE)
    try:
        out, st, _, donated = _solve(engine, puz, masks, budget=0)
        split = engine.get_option(L.SDK_OPT_SPLIT_BOARDS)
    finally:
        engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX)
    assert split > 0 and donated > 0
    assert (st == rst).all() and (out == ref).all()
    solved = st[:len(heavy)] == 1   # a unique puzzle whose answer lies outside its range has none
    assert solved.any() and (out[:len(heavy)][solved] == hs[solved]).all()


@pytest.mark.parametrize("mode", [1, 0])
@pytest.mark.parametrize("order", ["lex", "mrv_unique"])
def test_resumed_split_boards_match_restarted(engine, mode, order):
    """SDK_OPT_DONATE_RESUME: the boards the split phase stops go on in the donation launch from
    their saved stacks (the open subtrees of every level as items).  Heavy unique boards, sparse
    multi-solution boards under first-cell ranges, exact-unsolvable and conflicting boards give
    the same boards and statuses as restarting them and as one slot per board (LEX: the
    reference's answer); MRV stacks are resumed only into the exhaustive donation order."""
    heavy, hs, _ = _heavy_minimal(engine, 8000, 150, 77)
    puz = np.concatenate([heavy, _random_puzzles(300, 78, 14, 24), _corrupt(heavy[:40], 9)])
    masks = _masks(len(puz), 79)
    ref, rst, _, _ = _solve(engine, puz, masks, donate=0, budget=0)
    ordv = L.SDK_ORDER_LEX if order == "lex" else L.SDK_ORDER_MRV_UNIQUE
    engine.set_option(L.SDK_OPT_ORDER, ordv)
    try:
        res = {}
        for resume in (1, 0):
            engine.set_option(L.SDK_OPT_DONATE_RESUME, resume)
            out, st, _, _ = _solve(engine, puz, masks, budget=0, mode=mode)
            res[resume] = (out, st, engine.get_option(L.SDK_OPT_RESUMED),
                           engine.get_option(L.SDK_OPT_SPLIT_BOARDS))
    finally:
        engine.set_option(L.SDK_OPT_DONATE_RESUME, 1)
        engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX)
    for resume, (out, st, resumed, split) in res.items():
        assert (st == rst).all() and (out == ref).all(), f"resume={resume}"
        assert split > 0
    assert res[0][2] == 0
    if order == "mrv_unique" and mode == 1:   # MRV stacks into the exhaustive launch only
        assert res[1][2] > 0
    else:
        assert res[1][2] == 0


def test_resumed_boards_under_a_budget_and_heaviest(engine):
    """Resumed boards under a caller's node budget (parts that hit it make the board
    SDK_BUDGET_HIT unless a completion below it is known, as for a restarted board: never a
    wrong answer), and the heaviest boards of the hard set resumed at the default split."""
    heavy, hs, _ = _heavy_minimal(engine, 20000, 1000, 21)
    engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_MRV_UNIQUE)
    try:
        runs = []
        for budget in (0, 300, 2000):
            out, st, _, _ = _solve(engine, heavy, donate=1, budget=budget)
            runs.append((budget, out, st, engine.get_option(L.SDK_OPT_RESUMED)))
    finally:
        engine.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX)
    for budget, out, st, resumed in runs:
        ok = st == 1
        assert (out[ok] == hs[ok]).all()
        assert ((st == 1) | (st == -2)).all()
        assert (out[~ok] == heavy[~ok]).all()
        if budget == 0:
            assert ok.all() and resumed > 0
