"""Host-side boundary logic: grid encoding, TASK range -> mask, synthetic workloads."""
import numpy as np
import pytest

from distributed_sudoku_solver_amd import engine as E, synth
from distributed_sudoku_solver_amd.utils import split_array_in_middle
from oracle import oracle as O


def test_encode_solve_grid_follows_reference_equality():
    g = [[0] * 9 for _ in range(9)]
    g[0][0], g[0][1], g[0][2], g[0][3], g[0][4] = 5, 5.0, True, 10, 2.5
    g[1][0], g[1][1] = -3, 0.0
    b = E.encode_solve_grid(g)
    assert b[:5].tolist() == [5, 5, 1, 10, 10]
    assert b[9] == 10 and b[10] == 0


def test_encode_check_grid_domain():
    g = [[1] * 9 for _ in range(9)]
    g[0][0] = 255
    b = E.encode_check_grid(g)
    assert b.dtype == np.uint8 and b[0] == 255
    g[0][0] = 256                                  # any Python int: the int64 checker path
    b = E.encode_check_grid(g)
    assert b.dtype == np.int64 and b[0] == 256
    g[0][0] = -7.0                                 # 5.0 == 5 in the reference
    assert E.encode_check_grid(g)[0] == -7
    for bad in (4.5, 1 << 59, -(1 << 59), "5", None):
        g[0][0] = bad
        with pytest.raises(ValueError):
            E.encode_check_grid(g)


def test_range_to_mask_matches_split_semantics():
    assert E.range_to_mask(range(1, 10)) == 0x3FE
    a, b = split_array_in_middle(range(1, 10))
    assert (E.range_to_mask(a), E.range_to_mask(b)) == (0b11110, 0b1111100000)
    assert E.range_to_mask(a) | E.range_to_mask(b) == 0x3FE
    assert E.range_to_mask(range(5, 5)) == 0
    assert E.range_to_mask(range(0, 3)) == 0b110
    assert E.range_to_mask([2, 4, 7]) == (1 << 2) | (1 << 4) | (1 << 7)
    for bad in ([3, 1], range(1, 11), [-1]):
        with pytest.raises(ValueError):
            E.range_to_mask(bad)
    for lo in range(1, 10):
        for hi in range(lo, 11):
            assert E.range_to_mask(range(lo, hi)) == O.range_mask(lo, hi)


def test_split_array_in_middle():
    assert split_array_in_middle(range(1, 10)) == (range(1, 5), range(5, 10))
    assert split_array_in_middle(range(9, 10)) == (range(9, 9), range(9, 10))


def test_synth_17clue_is_unique_and_consistent():
    p, s = synth.make_17clue(2000, seed=7)
    assert ((p > 0).sum(1) == 17).all()
    assert ((p == 0) | (p == s)).all()
    assert (O.check_batch(s, 4) == 3).all()
    for i in range(0, 2000, 400):
        assert O.count(p[i], 2, 1) == 1
    # deterministic for a seed
    p2, _ = synth.make_17clue(2000, seed=7)
    assert (p == p2).all()


def test_synth_30clue_and_check_boards():
    p, s = synth.make_30clue(2000, seed=9)
    assert ((p > 0).sum(1) == 30).all() and ((p == 0) | (p == s)).all()
    b, exp = synth.make_check_boards(20000, seed=11)
    assert (O.check_batch(b, 4) == exp).all()
    assert 0.45 < (exp == 3).mean() < 0.55


def test_renormalize_keys_monotone_and_in_range():
    """shard._renormalize_keys: the live boards of all ranks keep their lex order,
    land in [0, KEY_SPACE), key_lo stays in int64, the lowest hit maps above every live key."""
    from distributed_sudoku_solver_amd.shard import KEY_SPACE, INT64_MAX, _renormalize_keys
    rng = np.random.default_rng(3)
    for _ in range(300):
        w = int(rng.integers(1, 9))
        S, base = [], 0
        for k in rng.permutation(w):            # disjoint key intervals in a random rank order
            lo = int(rng.integers(0, 1 << 25))
            n = int(rng.integers(0, 40))
            step = int(rng.integers(1, 1 << 20))
            S.append([k, lo, lo + n, 0, base - lo * step, step, INT64_MAX, 0])
            base += n * step + int(rng.integers(0, 1 << 30))
        S = [s[1:] for s in sorted(S)]
        g = INT64_MAX if rng.integers(0, 2) else base
        if g != INT64_MAX:
            S[0][5] = g
        before = sorted((s[3] + t * s[4], r, t) for r, s in enumerate(S) for t in range(s[0], s[1]))
        _renormalize_keys(S, g)
        after = sorted((s[3] + t * s[4], r, t) for r, s in enumerate(S) for t in range(s[0], s[1]))
        assert [x[1:] for x in before] == [x[1:] for x in after]
        assert all(0 <= x[0] < KEY_SPACE for x in after)
        assert all(-(1 << 63) <= s[3] < (1 << 63) and s[4] >= 1 for s in S)
        assert [s[5] for s in S] == [KEY_SPACE + 1 if (g != INT64_MAX and r == 0) else INT64_MAX
                                     for r in range(len(S))]


def test_sharded_solve_thousands_of_refinements():
    """a long first-solution search (S1 under a 1-node round budget, one board per
    refinement head: ~3,200 refinements) no longer runs out of lex keys; answer = the seed's."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from doubles import OracleEngine
    from distributed_sudoku_solver_amd.shard import sharded_solve
    info = {}
    out, st = sharded_solve(OracleEngine(), synth.parse(synth.SEEDS17["S1"]), 0, 1, target=1, round_budget=1,
                            info=info)
    assert st == 1 and "".join(map(str, out)) == synth.SEED_SOLUTIONS["S1"]
    assert info["refines"] > 1000, info
