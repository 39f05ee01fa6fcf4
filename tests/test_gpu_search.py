"""Bounded, resumable lex-first search on the HIP engine (search.LexSearch, sdk_solve_batch_budget,
sdk_expand_boards): whatever the per-launch node budget, the answers are the reference's
(golden vectors, the oracle's naive DFS = DHT_Node.py:474-538), and an unrefutable board ends
as SDK_BUDGET_HIT without holding back anything else."""
import time

import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth, _lib as L
from distributed_sudoku_solver_amd.engine import range_to_mask
from distributed_sudoku_solver_amd.search import LexSearch, solve_bounded
from oracle import oracle as O

from test_gpu_solve import _random_puzzles

pytestmark = pytest.mark.gpu

CONFLICT55 = "55" + "0" * 79


def test_per_call_budget_does_not_touch_the_context(engine):
    p, s = synth.make_minimal(4096, threads=16)
    out, st, nodes = engine.solve_batch(p, want_work=True, budget=1)
    branching = nodes > 1
    assert (st[~branching] == 1).all() and (out[~branching] == s[~branching]).all()
    assert engine.get_option(L.SDK_OPT_NODE_BUDGET) == 0
    out2, st2, nodes2 = engine.solve_batch(p, want_work=True, budget=0)       # 0 = unlimited
    assert (st2 == 1).all() and (out2 == s).all()
    hit = st == L.SDK_BUDGET_HIT
    assert hit.any() and (nodes2[hit] > 1).all() and (out[hit] == p[hit]).all()   # input kept on a hit


def test_expand_boards_is_an_ordered_partition(engine):
    """The children's completions, in order, are the parents' completions in order: solving every
    frontier board gives strictly increasing lex-first completions, the first of which is the
    parent's answer, and the per-board solution counts add up to the parent's (oracle counter)."""
    b16 = synth.parse(synth.SEEDS17["S1"][:-9] + "000800000")      # 7,309 completions
    n_all = O.count(b16)
    assert n_all == 7309
    kids = engine.expand(b16[None], target=200)
    assert len(kids) >= 200
    assert sum(O.count(k) for k in kids) == n_all
    out, st, _ = engine.solve_batch(kids)
    sols = ["".join(map(str, o)) for o, s in zip(out, st) if s == 1]
    assert sols == sorted(sols) and len(set(sols)) == len(sols)
    ref_st, ref_b, _ = O.naive_solve(b16)
    assert ref_st == 1 and sols[0] == "".join(map(str, ref_b))


def test_expand_boards_per_board_masks(engine, solve_cases):
    """Several seeds at once, each with its own first-cell range: the concatenated frontier's
    first solved board is each case's golden answer in turn."""
    cs = [c for c in solve_cases if c["ok"]][:40]
    for c in cs:
        b = np.array(c["puzzle"], np.uint8)
        kids = engine.expand(b[None], np.array([range_to_mask(range(*c["range"]))], np.uint16), target=16)
        out, st, _ = engine.solve_batch(kids)
        first = int(np.flatnonzero(st == 1)[0])
        assert out[first].tolist() == c["board"], c["name"]
    seeds = np.array([c["puzzle"] for c in cs], np.uint8)
    masks = np.array([range_to_mask(range(*c["range"])) for c in cs], np.uint16)
    kids = engine.expand(seeds, masks, target=1)            # one level: seeds' subtrees in seed order
    assert len(kids) >= len(cs)


@pytest.mark.parametrize("width,max_budget", [(1, 1), (64, 1), (16384, 64)])
def test_lex_search_golden_every_launch_hits(engine, solve_cases, width, max_budget):
    """Budget 1: every board that needs a second search node goes through expansions (and, at
    width 16384, through the budget escalation)."""
    for c in solve_cases:
        b = np.array(c["puzzle"], np.uint8)
        s = LexSearch(engine, b, range_to_mask(range(*c["range"])), budget=1, width=width, max_budget=max_budget)
        st, out = s.run(time.monotonic() + 30)
        assert st == (L.SDK_SOLVED if c["ok"] else L.SDK_UNSOLVABLE), c["name"]
        assert out.tolist() == (c["board"] if c["ok"] else c["puzzle"]), c["name"]


def test_solve_bounded_random_and_conflicting_vs_oracle(engine):
    """Sparse multi-solution boards with random ranges, planted given-vs-given duplicates and
    inert givens, budget 2 per launch: statuses and boards equal the oracle's naive DFS."""
    rng = np.random.default_rng(5)
    puz = np.concatenate([_random_puzzles(300, 41, 8, 30), _random_puzzles(300, 42, 20, 45)])
    for i in range(300, 600):
        nz = np.flatnonzero(puz[i])
        if i % 2 == 0 and len(nz) >= 2:
            a, b = rng.choice(nz, 2, replace=False)
            puz[i, b] = puz[i, a]
        else:
            puz[i, rng.choice(81, 2, replace=False)] = rng.integers(10, 256, 2)
    lo = rng.integers(1, 10, len(puz))
    hi = np.minimum(10, lo + rng.integers(1, 10, len(puz)))
    masks = np.array([O.range_mask(a, b) for a, b in zip(lo, hi)], dtype=np.uint16)
    out, st, _ = solve_bounded(engine, puz, masks, budget=2, time_limit=2.0, width=4096, max_pending=200_000)
    ref_out, ref_st, _ = O.naive_solve_batch(puz, masks, budget=20_000_000, threads=16)
    done = (ref_st != -2) & (st != L.SDK_BUDGET_HIT)
    assert done.mean() > 0.8
    assert (st[done] == ref_st[done]).all() and (out[done] == ref_out[done]).all()
    # nothing the oracle decided came back "no solution" where it has one, or vice versa
    assert not ((st == L.SDK_UNSOLVABLE) & (ref_st == 1)).any()


def test_minimal_puzzles_through_budget_hits(engine):
    p, s = synth.make_minimal(3000, seed=77, threads=16)
    out, st, work = solve_bounded(engine, p, budget=1, width=256)
    assert (st == 1).all() and (out == s).all()


def test_conflict55_exhausts_quickly(engine):
    """'55' + 79 zeros has no completion and propagation cannot refute it (the reference
    never finishes).  Bounded: it ends as SDK_BUDGET_HIT (exhausted), input unchanged, in well
    under a second, and the batch it was launched with is answered in one bounded launch."""
    from distributed_sudoku_solver_amd.search import SLICE_TARGET_S
    b = synth.parse(CONFLICT55)
    t0 = time.perf_counter()
    s = LexSearch.for_node(engine, b)                   # the node's bounded slices
    slices = []
    while not s.done and time.perf_counter() - t0 < 3.0:
        t1 = time.perf_counter()
        s.step()
        slices.append(time.perf_counter() - t1)
    st, out = s.run(time.monotonic())                   # deadline passed: exhausted
    assert st == L.SDK_BUDGET_HIT and (out == b).all()
    assert time.perf_counter() - t0 < 4.0
    srt = sorted(slices[1:])                            # the first slice sizes the buffers
    assert len(srt) > 20 and srt[len(srt) // 2] <= SLICE_TARGET_S and srt[int(0.9 * len(srt))] <= 1.5 * SLICE_TARGET_S, \
        (["%.2f" % (1e3 * t) for t in slices], s.budget)
    batch = np.stack([b, synth.parse(synth.WIKI)])
    t0 = time.perf_counter()
    out, st, _ = engine.solve_batch(batch, want_work=True, budget=2048)
    one = time.perf_counter() - t0
    assert st.tolist() == [L.SDK_BUDGET_HIT, L.SDK_SOLVED]
    assert "".join(map(str, out[1])) == synth.WIKI_SOLUTION
    assert one < 0.05, one


def test_dropin_solve_grid_is_bounded(engine):
    from distributed_sudoku_solver_amd.solver import SearchExhausted, solve_grid
    grid = [list(map(int, CONFLICT55[9 * r: 9 * r + 9])) for r in range(9)]
    with pytest.raises(SearchExhausted):
        solve_grid(grid, engine=engine, time_limit=2.0)
    assert [v for row in grid for v in row] == [int(c) for c in CONFLICT55]
    grid = [list(map(int, synth.SEEDS17["S2"][9 * r: 9 * r + 9])) for r in range(9)]
    ok, _ = solve_grid(grid, engine=engine, budget=1)
    assert ok and "".join(str(v) for row in grid for v in row) == synth.SEED_SOLUTIONS["S2"]


def test_node_slices_are_bounded(engine):
    """a node's continued search (LexSearch.for_node, on its own context) keeps
    every slice -- launch, expansion and host copies together -- within 1.5 x the slice target,
    on '55'+79 zeros (unrefutable: every sub-board hits the budget, the worst case)."""
    from distributed_sudoku_solver_amd.search import LAUNCH_SHARE, SLICE_TARGET_S
    fork = engine.fork()
    try:
        b = synth.parse(CONFLICT55)
        s = LexSearch.for_node(fork, b)
        s.step()                                        # warm: the first slice sizes the buffers
        times = []
        for _ in range(40):
            s.step()
            times.append(s.last_slice_s)
            # the design bound, before the next launch runs: its budget x the measured wall time
            # per node of a launch's critical path stays within LAUNCH_SHARE of the target
            assert s.budget == 1 or s.budget * s.t_node <= LAUNCH_SHARE * SLICE_TARGET_S * 1.001, (s.budget, s.t_node)
        assert not s.done
        # measured: the slices themselves, every one.  The slow slices of round 4 (12-27 ms, kernel
        # 0.2-2 ms) were HIP's pageable-memory path in the calling thread; the host-pointer calls
        # now stage through pinned memory (sudoku_hip.hip, HostBuf) and the worst of 199 slices
        # after the first was 5.6 ms (profiles/r05/slice_probe_timing_r05d.log)
        assert max(times) <= 1.5 * SLICE_TARGET_S, (["%.2f" % (1e3 * t) for t in times], s.budget, s.width)
        assert s.budget > 1                            # the bound leaves room to search
    finally:
        fork.close()
