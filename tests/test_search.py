"""search.LexSearch (the bounded, resumable lex-first search every product solve goes through)
on the oracle double: whatever the node budget, the answer is the reference's (golden vectors
made by importing the reference, DHT_Node.py:474-538), and a board no budget finishes ends as
SDK_BUDGET_HIT, never as "no solution".  tests/test_gpu_search.py runs the same on the GPU."""
import time

import numpy as np
import pytest

from distributed_sudoku_solver_amd import _lib as L, synth
from distributed_sudoku_solver_amd.engine import range_to_mask
from distributed_sudoku_solver_amd.search import LexSearch, solve_bounded

from doubles import OracleEngine, naive_expand

CONFLICT55 = "55" + "0" * 79        # provably unsolvable, the reference never finishes


def _case_board(c):
    return np.array(c["puzzle"], dtype=np.uint8), range_to_mask(range(*c["range"]))


@pytest.mark.parametrize("width", [1, 7, 256])
def test_lex_search_matches_golden_at_any_width(solve_cases, width):
    eng = OracleEngine()
    for c in solve_cases:
        if c["validations"] > 200_000:
            continue
        b, m = _case_board(c)
        s = LexSearch(eng, b, m, budget=1, width=width)      # 1 node = 10k validations on the double
        st, out = s.run()
        assert st == (L.SDK_SOLVED if c["ok"] else L.SDK_UNSOLVABLE), c["name"]
        assert out.tolist() == (c["board"] if c["ok"] else c["puzzle"]), c["name"]


def test_lex_search_continues_budget_hits(solve_cases):
    """The cases that need more than one budget go through expansions and still match."""
    eng = OracleEngine()
    hard = [c for c in solve_cases if 10_000 < c["validations"]]
    assert len(hard) >= 5
    for c in hard:
        b, m = _case_board(c)
        s = LexSearch(eng, b, m, budget=1, width=64)
        st, out = s.run()
        assert s.expansions >= 1, c["name"]
        assert st == (L.SDK_SOLVED if c["ok"] else L.SDK_UNSOLVABLE), c["name"]
        assert out.tolist() == (c["board"] if c["ok"] else c["puzzle"]), c["name"]


def test_exhausted_is_not_unsolvable():
    eng = OracleEngine()
    s = LexSearch(eng, synth.parse(CONFLICT55), budget=1, width=32, max_pending=200, max_budget=1)
    st, out = s.run(time.monotonic() + 60)
    assert s.pending == 0 and s.expansions > 1
    assert st == L.SDK_BUDGET_HIT and out.tolist() == synth.parse(CONFLICT55).tolist()
    s = LexSearch(eng, synth.parse(CONFLICT55), budget=1, width=32)
    st, _ = s.run(deadline=time.monotonic() + 0.5)
    assert st == L.SDK_BUDGET_HIT


def test_solve_bounded_mixes_easy_and_hard(solve_cases):
    eng = OracleEngine()
    cs = [c for c in solve_cases if c["validations"] < 200_000]
    boards = np.array([c["puzzle"] for c in cs], dtype=np.uint8)
    masks = np.array([range_to_mask(range(*c["range"])) for c in cs], dtype=np.uint16)
    out, st, work = solve_bounded(eng, boards, masks, budget=1, width=16)
    for c, o, s in zip(cs, out, st):
        assert s == (1 if c["ok"] else 0), c["name"]
        assert o.tolist() == (c["board"] if c["ok"] else c["puzzle"]), c["name"]


def test_naive_expand_keeps_lex_order():
    """The double's expansion: children in DFS order, so the concatenated completions stay sorted."""
    b = synth.parse("000100000000320000000009000000000070000000000000900000000000900000000003000000000")
    kids = naive_expand(b[None], np.array([range_to_mask(range(1, 5))]), target=50)
    assert len(kids) >= 50
    keys = ["".join(map(str, k)) for k in kids]
    assert keys == sorted(keys)
    assert all(k[0] in (1, 2, 3, 4) for k in kids)       # cell 0 is the first empty cell: digits 1..4 only


def test_lex_search_over_multi_device_engine(solve_cases):
    """The node's continued search on every GPU of the box: LexSearch.for_node over a 3-device
    MultiDeviceEngine (oracle doubles) shards each slice's launch and expansion over the devices
    and still returns the golden answers; the slice is as wide as 3 single-device slices."""
    from distributed_sudoku_solver_amd.shard import MultiDeviceEngine
    devs = [OracleEngine() for _ in range(3)]
    mde = MultiDeviceEngine(devs)
    hard = [c for c in solve_cases if 10_000 < c["validations"] < 2_000_000]
    assert len(hard) >= 5
    for c in hard:
        b, m = _case_board(c)
        s = LexSearch.for_node(mde, b, m, budget=1, width=8, slice_target_s=10.0)
        assert s.width == 24
        st, out = s.run(time.monotonic() + 60)
        assert st == (L.SDK_SOLVED if c["ok"] else L.SDK_UNSOLVABLE), c["name"]
        assert out.tolist() == (c["board"] if c["ok"] else c["puzzle"]), c["name"]
    assert all(sum(1 for x in d.calls if isinstance(x, int)) > 0 for d in devs)   # every device launched


def test_for_node_bounds_the_budget_by_measured_node_time():
    """LexSearch.for_node starts at the smallest budget and never lets budget x (measured wall time
    per node of a launch's longest board) exceed half the slice target."""
    from distributed_sudoku_solver_amd import search as S

    class Slow(OracleEngine):
        # every launch takes 1 ms per node of its longest board (a synthetic clock)
        def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
            out, st, _ = super().solve_batch(boards, masks, True, budget, donate)
            time.sleep(1e-3 * (int(budget) if budget else 1))
            return out, st, np.full(len(boards), int(budget) if budget else 1, np.uint64)   # nodes used

    eng = Slow()
    s = LexSearch.for_node(eng, synth.parse(CONFLICT55), None, budget=64, width=4, slice_target_s=0.02)
    assert s.budget == 8                                    # node budget / 8
    seen = []
    for _ in range(8):
        s.step()
        seen.append(s.budget)
        assert s.budget * 1e-3 <= S.LAUNCH_SHARE * 0.02 * 1.05, seen        # 10 nodes of 1 ms: half the target
    assert s.t_node is not None and s.t_node >= 1e-3
