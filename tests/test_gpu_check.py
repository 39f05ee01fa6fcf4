"""HIP checker vs the oracle (bit-exact verdict bytes) and vs the reference's fixtures."""
import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth, _lib as L
from distributed_sudoku_solver_amd.sudoku import Sudoku
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def test_golden_check_cases(engine, check_cases):
    boards = np.array([c["board"] for c in check_cases], dtype=np.uint8)
    v = engine.check_batch(boards)
    for c, x in zip(check_cases, v):
        assert bool(x & L.SDK_CHECK_OK) == c["intended"], c["name"]
        assert ("NameError" if x & L.SDK_CHECK_RAW_NAMEERROR else "False") == c["raw"], c["name"]


def test_sudoku_class_dropin(engine, check_cases):
    for c in check_cases[:20]:
        grid = [c["board"][9 * r: 9 * r + 9] for r in range(9)]
        s = Sudoku(grid, engine=engine)
        assert s.check() == c["intended"]
        if c["raw"] == "NameError":
            with pytest.raises(NameError):
                s.check(raw=True)
        else:
            assert s.check(raw=True) is False


@pytest.mark.parametrize("n", [1, 2, 3, 4, 255, 256, 257, 511, 1000, 4099])
def test_ragged_sizes(engine, n):
    b, exp = synth.make_check_boards(n, seed=n)
    assert (engine.check_batch(b) == exp).all()


def test_random_values_vs_oracle(engine):
    rng = np.random.default_rng(5)
    parts = [rng.integers(0, 10, (20000, 81)), rng.integers(0, 256, (5000, 81)), rng.integers(0, 20, (20000, 81))]
    b = np.concatenate(parts).astype(np.uint8)
    # literal-rule boards: valid grids relabelled to {0..7,17}, {0,2..8,10}, etc.
    sols, _ = synth.make_check_boards(3000, seed=3)
    for mp in ({1: 0, 9: 10}, {1: 0, 2: 1, 3: 2, 4: 3, 5: 4, 6: 5, 7: 6, 8: 7, 9: 17},
               {1: 0, 2: 1, 3: 2, 4: 3, 5: 4, 6: 5, 7: 6, 8: 8, 9: 16}, {9: 18}, {1: 0, 9: 255}):
        lut = np.arange(256, dtype=np.uint8)
        for k, v in mp.items():
            lut[k] = v
        b = np.concatenate([b, lut[sols]])
    assert (engine.check_batch(b) == O.check_batch(b, threads=8)).all()


def test_one_million_synthetic(engine):
    b, exp = synth.make_check_boards(1 << 20, seed=1234)
    v = engine.check_batch(b)
    assert (v == exp).all()


def test_empty_batch(engine):
    assert engine.check_batch(np.zeros((0, 81), np.uint8)).shape == (0,)


VARIANTS = [L.SDK_CHECK_REG1, L.SDK_CHECK_REG2, L.SDK_CHECK_GLDS2, L.SDK_CHECK_GLDS3, L.SDK_CHECK_GLDS4,
            L.SDK_CHECK_WAVE1, L.SDK_CHECK_WAVE2]


@pytest.mark.parametrize("variant", VARIANTS)
def test_pipeline_variants_bit_exact(engine, variant):
    """Every tile pipeline (register ring, LDS-DMA ring) gives the oracle's verdict bytes, at sizes that
    hit every prologue/steady-state/tail combination of the grid (CUs x blocks/CU workgroups)."""
    cus = engine.get_option(L.SDK_OPT_DEVICE_CUS)
    rng = np.random.default_rng(11 + variant)
    pool, pool_exp = synth.make_check_boards(1 << 18, seed=77)
    odd = rng.integers(0, 20, (4096, 81)).astype(np.uint8)
    odd_exp = O.check_batch(odd, threads=8)
    try:
        engine.set_option(L.SDK_OPT_CHECK_VARIANT, variant)
        for bpc in (1, 2, 3, 4):
            engine.set_option(L.SDK_OPT_CHECK_BLOCKS_PER_CU, bpc)
            g = cus * bpc
            for n in (1, 255, 256, 257, 256 * g - 1, 256 * g, 256 * g * 2 + 17, 256 * g * 3 + 256, 256 * g * 4 + 100):
                idx = rng.integers(0, len(pool), n)
                b, exp = pool[idx], pool_exp[idx]
                if n > 8192:   # splice exact-path boards (values >= 10) into the middle and the tail
                    b = b.copy(); exp = exp.copy()
                    b[n // 2: n // 2 + 4096] = odd; exp[n // 2: n // 2 + 4096] = odd_exp
                    b[-100:] = odd[:100]; exp[-100:] = odd_exp[:100]
                v = engine.check_batch(b)
                bad = np.flatnonzero(v != exp)
                assert bad.size == 0, (variant, bpc, n, bad[:10])
    finally:
        engine.set_option(L.SDK_OPT_CHECK_VARIANT, L.SDK_CHECK_REG1)
        engine.set_option(L.SDK_OPT_CHECK_BLOCKS_PER_CU, 3)


def test_int64_boards_vs_python_restatement(engine):
    """Out-of-domain ints (the reference's check() takes any Python int): the int64 kernel
    follows the literal rule, e.g. [0, 2, ..., 8, 10] passes a row (sum 45, 9 distinct)."""
    from distributed_sudoku_solver_amd.sudoku import Sudoku
    rng = np.random.default_rng(5)
    sols, _ = synth.make_check_boards(400, seed=17)
    boards = sols.astype(np.int64)
    for i in range(len(boards)):
        b = boards[i]
        k = i % 4
        if k == 0:                                    # swap digits 1 -> 0 and 9 -> 10 (sums stay 45)
            b[b == 1] = 0
            b[b == 9] = 10
        elif k == 1:
            b[rng.integers(0, 81)] = int(rng.integers(-(1 << 40), 1 << 40))
        elif k == 2:                                  # shift one digit by +-d and a partner by -+d
            b[b == 3] = 1000
            b[b == 4] = -993
        else:
            b[rng.integers(0, 81, 3)] = rng.integers(-300, 300, 3)
    v = engine.check_batch(boards)
    for b, x in zip(boards, v):
        raw, intended = O.py_check([int(t) for t in b])
        assert bool(x & 1) == intended and bool(x & 2) == (raw == "NameError"), b.tolist()
    assert (v & 1).any() and (v & 2).any()
    g = [[int(t) for t in boards[0][9 * r: 9 * r + 9]] for r in range(9)]
    assert Sudoku(g, engine=engine).check() == bool(v[0] & 1)


def test_host_pointer_large_check(engine):
    """A 3M-board host-pointer check batch: verdicts equal the expected ones."""
    b, exp = synth.make_check_boards(3_000_000, seed=78)
    v = engine.check_batch(b)
    assert (v == exp).all()
