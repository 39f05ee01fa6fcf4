"""Seeded synthetic workloads of SURVEY §8(d) (configs C2/C3/C4), vectorised in numpy.

Every generated puzzle comes with its expected answer, so full-size runs are
checked by construction (size-independent parity):
  * 17-clue hard puzzles: seeds S1-S5 (17 givens, exactly one completion each,
    SURVEY App. A) under random Sudoku symmetries; symmetries preserve the
    number of completions, so the expected answer is the transformed solution.
  * ~30-clue unique puzzles: a seed's givens plus 13 more cells of its
    solution (a superset of a unique puzzle's givens stays unique), transformed.
  * check boards: 50 % valid (transformed solutions, verdict 3 = ok and the raw
    reference call raises NameError), 50 % with one corruption (verdict 0):
    two cells of a row swapped, or one value changed to another digit.
Seeds and their solutions are data produced by the reference itself
(tests/golden/make_golden.py re-derives S4/S5; SURVEY App. A lists all five).
"""
import numpy as np

SEEDS17 = {
    "S1": "000000010400000000020000000000050407008000300001090000300400200050100000000806000",
    "S2": "000000010400000000020000000000050604008000300001090000300400200050100000000807000",
    "S3": "000000012000035000000600070700000300000400800100000000000120000080000040050000600",
    "S4": "000000012003600000000007000410020000000500300700000600280000040000300500000000000",
    "S5": "000000012008030000000000040120500000000004700060000000507000300000620000000100000",
}
SEED_SOLUTIONS = {
    "S1": "693784512487512936125963874932651487568247391741398625319475268856129743274836159",
    "S2": "793684512486512937125973846932751684578246391641398725319465278857129463264837159",
    "S3": "673894512912735486845612973798261354526473891134589267469128735287356149351947628",
    "S4": "679835412123694758548217936416723895892561374735489621287956143961342587354178269",
    "S5": "346795812258431697971862543129576438835214769764389251517948326493627185682153974",
}
WIKI = "530070000600195000098000060800060003400803001700020006060000280000419005000080079"
WIKI_SOLUTION = "534678912672195348198342567859761423426853791713924856961537284287419635345286179"

DEFAULT_SEED = 20250614


def parse(s):
    return np.frombuffer(s.encode(), dtype=np.uint8) - ord("0")


def seed_arrays():
    names = sorted(SEEDS17)
    puz = np.stack([parse(SEEDS17[k]) for k in names])
    sol = np.stack([parse(SEED_SOLUTIONS[k]) for k in names])
    return puz, sol


def _line_perms(rng, n):
    """n random row (or column) permutations that keep bands: band perm x in-band perms."""
    bands = np.argsort(rng.random((n, 3)), axis=1)            # [n,3]
    inner = np.argsort(rng.random((n, 3, 3)), axis=2)         # [n,3,3]
    return (3 * bands[:, :, None] + inner).reshape(n, 9)      # [n,9]


def random_symmetries(rng, n):
    """Per puzzle: gather index [n,81] (new cell -> old cell) and digit relabel [n,10]."""
    rp = _line_perms(rng, n)
    cp = _line_perms(rng, n)
    tr = rng.random(n) < 0.5
    r = np.arange(9)[None, :, None]
    c = np.arange(9)[None, None, :]
    rr = np.where(tr[:, None, None], c, r)
    cc = np.where(tr[:, None, None], r, c)
    # src_r[p, i, j] = rp[p, rr[p, i, j]]
    src_r = rp[np.arange(n)[:, None, None], np.broadcast_to(rr, (n, 9, 9))]
    src_c = cp[np.arange(n)[:, None, None], np.broadcast_to(cc, (n, 9, 9))]
    gather = (9 * src_r + src_c).reshape(n, 81).astype(np.int16)
    relabel = np.zeros((n, 10), dtype=np.uint8)
    relabel[:, 1:] = (np.argsort(rng.random((n, 9)), axis=1) + 1).astype(np.uint8)
    return gather, relabel


def apply_symmetries(boards, gather, relabel):
    """boards [n,81] uint8 (values 0..9) -> transformed boards."""
    n = boards.shape[0]
    moved = np.take_along_axis(boards, gather.astype(np.int64), axis=1)
    return np.take_along_axis(relabel, moved.astype(np.int64), axis=1).astype(np.uint8)


def _chunked(n, chunk, fn):
    outs = []
    for s in range(0, n, chunk):
        outs.append(fn(s, min(chunk, n - s)))
    return [np.concatenate(parts) for parts in zip(*outs)]


def make_17clue(n, seed=DEFAULT_SEED, chunk=1 << 20):
    """C4 workload: n transformed 17-clue puzzles and their unique solutions."""
    puz, sol = seed_arrays()
    rng = np.random.default_rng(seed)

    def part(s, m):
        k = rng.integers(0, len(puz), m)
        g, rl = random_symmetries(rng, m)
        return apply_symmetries(puz[k], g, rl), apply_symmetries(sol[k], g, rl)

    return _chunked(n, chunk, part)


def make_30clue(n, seed=DEFAULT_SEED + 1, extra=13, chunk=1 << 20):
    """C2 workload: 17 seed givens + `extra` solution cells (unique), transformed."""
    puz, sol = seed_arrays()
    rng = np.random.default_rng(seed)

    def part(s, m):
        k = rng.integers(0, len(puz), m)
        p = puz[k].copy()
        sl = sol[k]
        # choose `extra` currently-empty cells per puzzle: random keys, givens pushed last
        keys = rng.random((m, 81)) + (p > 0) * 2.0
        pick = np.argsort(keys, axis=1)[:, :extra]
        rows = np.arange(m)[:, None]
        p[rows, pick] = sl[rows, pick]
        g, rl = random_symmetries(rng, m)
        return apply_symmetries(p, g, rl), apply_symmetries(sl, g, rl)

    return _chunked(n, chunk, part)


def make_check_boards(n, seed=DEFAULT_SEED + 2, chunk=1 << 20):
    """C3 workload: boards [n,81] and expected verdict bytes [n] (3 valid, 0 corrupted)."""
    _, sol = seed_arrays()
    sol = np.concatenate([sol, parse(WIKI_SOLUTION)[None]])
    rng = np.random.default_rng(seed)

    def part(s, m):
        k = rng.integers(0, len(sol), m)
        g, rl = random_symmetries(rng, m)
        b = apply_symmetries(sol[k], g, rl)
        bad = rng.random(m) < 0.5
        kind = rng.integers(0, 2, m)
        rows = np.arange(m)
        # swap two distinct cells of one row
        r = rng.integers(0, 9, m)
        a = rng.integers(0, 9, m)
        d = (a + rng.integers(1, 9, m)) % 9
        sw = bad & (kind == 0)
        ia, id_ = 9 * r[sw] + a[sw], 9 * r[sw] + d[sw]
        tmp = b[rows[sw], ia].copy()
        b[rows[sw], ia] = b[rows[sw], id_]
        b[rows[sw], id_] = tmp
        # change one value to a different digit
        ch = bad & (kind == 1)
        cell = rng.integers(0, 81, m)
        delta = rng.integers(1, 9, m)
        old = b[rows[ch], cell[ch]].astype(np.int64)
        b[rows[ch], cell[ch]] = ((old - 1 + delta[ch]) % 9 + 1).astype(np.uint8)
        verdict = np.where(bad, 0, 3).astype(np.uint8)
        return b, verdict

    return _chunked(n, chunk, part)
