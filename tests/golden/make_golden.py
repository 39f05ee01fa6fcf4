#!/usr/bin/env python3
"""Generate the golden vectors that pin the oracle (and, through it, the HIP engine).

Run ONCE in the build container, where the read-only reference lives at
/root/reference. The reference itself never travels: only the JSON data this
script writes (inputs + the reference's outputs) is committed under tests/golden/.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

Recipes:
  * solve:  DHT_Node.DHTNode.__new__ (no sockets/threads), task={'uuid':0},
            neighbor=None, handicap=0, non_blocking_receive stubbed.  The
            reference's solve_sudoku (DHT_Node.py:474-538) mutates the grid and
            bumps .validations (DHT_Node.py:513,528).  main.DHTNode.solve_sudoku
            (main.py:301-354) is run on the same inputs to pin the twin.
  * check:  Sudoku._limit_calls disabled (sudoku.py:10-17).  "raw" is what
            Sudoku(g).check() does (True / False / NameError, bug at sudoku.py:68);
            "intended" injects module globals i, j before each check_square so
            the box test sees its own box.
"""
import argparse
import json
import os
import random
import signal
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))

WIKI = "530070000600195000098000060800060003400803001700020006060000280000419005000080079"
DEMO8 = "000100000000320000000009000000000070000000000000900000000000900000000003000000000"
SEEDS17 = {
    "S1": "000000010400000000020000000000050407008000300001090000300400200050100000000806000",
    "S2": "000000010400000000020000000000050604008000300001090000300400200050100000000807000",
    "S3": "000000012000035000000600070700000300000400800100000000000120000080000040050000600",
    "S4": "000000012003600000000007000410020000000500300700000600280000040000300500000000000",
    "S5": "000000012008030000000000040120500000000004700060000000507000300000620000000100000",
}


class Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise Timeout()


def to_grid(cells):
    return [list(cells[9 * r: 9 * r + 9]) for r in range(9)]


def from_str(s):
    return [int(ch) for ch in s]


def flat(grid):
    return [v for row in grid for v in row]


def make_node(mod):
    n = mod.DHTNode.__new__(mod.DHTNode)
    n.task = {"uuid": 0}
    n.neighbor = None
    n.neighborfree = False
    n.validations = 0
    n.handicap = 0
    n.non_blocking_receive = lambda: (None, None)
    return n


def run_solve(DHT_Node, main, cells, lo, hi, timeout_s):
    """Run both reference solvers; return the fixture dict or None on timeout."""
    out = {}
    for tag, mod in (("dht", DHT_Node), ("main", main)):
        node = make_node(mod)
        grid = to_grid(cells)
        signal.setitimer(signal.ITIMER_REAL, timeout_s)
        t0 = time.time()
        try:
            if tag == "dht":
                ok = node.solve_sudoku(grid, 0, range(lo, hi))
            else:
                ok = node.solve_sudoku(grid, range(lo, hi))
        except Timeout:
            return None
        finally:
            signal.setitimer(signal.ITIMER_REAL, 0)
        out[tag] = (bool(ok), flat(grid), node.validations, time.time() - t0)
    d, m = out["dht"], out["main"]
    assert d[:3] == m[:3], ("reference twins disagree", cells, lo, hi)
    return {"ok": d[0], "board": d[1], "validations": d[2], "ref_seconds": round(d[3], 4)}


def ref_check(sudoku_mod, cells):
    S = sudoku_mod.Sudoku
    for g in ("i", "j"):
        if hasattr(sudoku_mod, g):
            delattr(sudoku_mod, g)
    try:
        raw = "True" if S(to_grid(cells)).check() else "False"
    except NameError:
        raw = "NameError"
    s = S(to_grid(cells))
    intended = all(s.check_row(r) for r in range(9)) and all(s.check_column(c) for c in range(9))
    if intended:
        for bi in range(3):
            for bj in range(3):
                sudoku_mod.i, sudoku_mod.j = bi, bj
                if not s.check_square(3 * bi, 3 * bj):
                    intended = False
                    break
            if not intended:
                break
    for g in ("i", "j"):
        if hasattr(sudoku_mod, g):
            delattr(sudoku_mod, g)
    return raw, bool(intended)


# ---------------------------------------------------------------- symmetry helpers
def random_transform(rng, cells):
    """Validity-preserving Sudoku symmetry (digit relabel, row/col perms, transpose)."""
    digits = list(range(1, 10))
    rng.shuffle(digits)
    relabel = [0] + digits

    def line_perm():
        bands = [0, 1, 2]
        rng.shuffle(bands)
        p = []
        for b in bands:
            inner = [0, 1, 2]
            rng.shuffle(inner)
            p += [3 * b + k for k in inner]
        return p

    rp, cp = line_perm(), line_perm()
    tr = rng.random() < 0.5
    out = [0] * 81
    for r in range(9):
        for c in range(9):
            rr, cc = (c, r) if tr else (r, c)
            v = cells[9 * rp[rr] + cp[cc]]
            out[9 * r + c] = relabel[v] if 0 <= v <= 9 else v
    return out


def main_():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--seed", type=int, default=20250614)
    args = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, args.ref)
    import DHT_Node  # noqa: E402
    import main as mainmod  # noqa: E402
    import sudoku as sudoku_mod  # noqa: E402
    sudoku_mod.Sudoku._limit_calls = lambda self, *a, **k: None
    signal.signal(signal.SIGALRM, _alarm)
    rng = random.Random(args.seed)

    # ------------------------------------------------------------ solve fixtures
    solve_cases = []

    def add(name, cells, lo=1, hi=10, timeout_s=5.0):
        r = run_solve(DHT_Node, mainmod, cells, lo, hi, timeout_s)
        if r is None:
            return False
        solve_cases.append({"name": name, "puzzle": list(cells), "range": [lo, hi], **r})
        return True

    # Appendix A vectors
    add("demo8", from_str(DEMO8))
    add("demo8_r1_5", from_str(DEMO8), 1, 5)
    add("demo8_r5_10", from_str(DEMO8), 5, 10)
    add("demo8_r1_2", from_str(DEMO8), 1, 2)
    add("wiki", from_str(WIKI))
    add("wiki_r5_10", from_str(WIKI), 5, 10)
    add("empty", [0] * 81)
    add("empty_r5_10", [0] * 81, 5, 10)
    add("empty_r9_10", [0] * 81, 9, 10)
    add("empty_r5_5", [0] * 81, 5, 5)          # empty digit range: first cell has no guess
    wiki_conflict = from_str(WIKI)
    wiki_conflict[1] = 5                        # clue conflict (0,0)=(0,1)=5
    add("wiki_clue_conflict", wiki_conflict, timeout_s=30.0)
    for name in ("S4", "S5"):
        add(name, from_str(SEEDS17[name]), timeout_s=60.0)

    # full boards (no empty cell -> True after 1 validation whatever the range)
    wiki_sol = solve_cases[4]["board"]
    add("full_valid", wiki_sol)
    bad = list(wiki_sol)
    bad[0], bad[1] = bad[1], bad[0]
    add("full_swapped", bad)
    dup = list(wiki_sol)
    dup[10] = dup[0]
    add("full_dup_clue", dup, 3, 4)

    # inert (out-of-domain) clues: never equal to a guess 1..9 (utils.py:36,44,53)
    inert = from_str(WIKI)
    inert[2], inert[40] = 10, 255
    add("wiki_inert_10_255", inert)
    inert2 = [0] * 81
    inert2[0], inert2[12], inert2[80] = 17, 200, 12
    add("empty_inert", inert2)

    # random puzzles from known solutions: symmetry + cell removal (fast for naive DFS)
    sol_pool = [wiki_sol] + [c["board"] for c in solve_cases if c["name"] in ("S4", "S5")]
    k = 0
    attempts = 0
    while k < 60 and attempts < 400:
        attempts += 1
        base = random_transform(rng, rng.choice(sol_pool))
        nclues = rng.randint(24, 50)
        keep = set(rng.sample(range(81), nclues))
        cells = [v if i in keep else 0 for i, v in enumerate(base)]
        if rng.random() < 0.35:
            lo = rng.randint(1, 9)
            hi = rng.randint(lo + 1, 10)
        else:
            lo, hi = 1, 10
        if add(f"rand{k:02d}_c{nclues}", cells, lo, hi, timeout_s=2.0):
            k += 1
    # random boards with a planted clue conflict (often fail fast, sometimes succeed)
    k = 0
    attempts = 0
    while k < 12 and attempts < 200:
        attempts += 1
        base = random_transform(rng, rng.choice(sol_pool))
        keep = set(rng.sample(range(81), rng.randint(30, 55)))
        cells = [v if i in keep else 0 for i, v in enumerate(base)]
        a, b = rng.sample(sorted(keep), 2)
        cells[b] = cells[a]
        if add(f"conflict{k:02d}", cells, timeout_s=2.0):
            k += 1
    # sparse random boards (many solutions: lex-first matters)
    k = 0
    attempts = 0
    while k < 16 and attempts < 200:
        attempts += 1
        base = random_transform(rng, rng.choice(sol_pool))
        keep = set(rng.sample(range(81), rng.randint(3, 14)))
        cells = [v if i in keep else 0 for i, v in enumerate(base)]
        lo = rng.randint(1, 9)
        hi = rng.randint(lo + 1, 10)
        if add(f"sparse{k:02d}", cells, lo, hi, timeout_s=2.0):
            k += 1

    # ------------------------------------------------------------ check fixtures
    check_cases = []

    def addc(name, cells):
        raw, intended = ref_check(sudoku_mod, cells)
        check_cases.append({"name": name, "board": list(cells), "raw": raw, "intended": intended})

    addc("valid", wiki_sol)
    rs = list(wiki_sol)
    rs[63:72], rs[72:81] = wiki_sol[72:81], wiki_sol[63:72]
    addc("rows_swapped_within_band", rs)
    addc("swap_cells_row0", [wiki_sol[1], wiki_sol[0]] + wiki_sol[2:])
    addc("latin_cyclic", [((r + c) % 9) + 1 for r in range(9) for c in range(9)])
    addc("swap_last_two", wiki_sol[:79] + [wiki_sol[80], wiki_sol[79]])
    addc("all_zeros", [0] * 81)
    for n in range(40):
        addc(f"valid_sym{n:02d}", random_transform(rng, rng.choice(sol_pool)))
    for n in range(60):
        g = random_transform(rng, rng.choice(sol_pool))
        kind = n % 3
        if kind == 0:      # swap two cells in a row
            r = rng.randrange(9)
            a, b = rng.sample(range(9), 2)
            g[9 * r + a], g[9 * r + b] = g[9 * r + b], g[9 * r + a]
        elif kind == 1:    # change one value to another in 1..9
            i = rng.randrange(81)
            g[i] = rng.choice([d for d in range(1, 10) if d != g[i]])
        else:              # permute columns arbitrarily: rows+cols stay latin, boxes may break
            perm = list(range(9))
            rng.shuffle(perm)
            g = [g[9 * r + perm[c]] for r in range(9) for c in range(9)]
        addc(f"corrupt{n:02d}_k{kind}", g)
    # literal-rule edge cases: sum==45 with 9 distinct values outside 1..9
    relabels = {
        "lit_0_10": {1: 0, 9: 10},
        "lit_0_17": {1: 0, 2: 1, 3: 2, 4: 3, 5: 4, 6: 5, 7: 6, 8: 7, 9: 17},
        "lit_0_16": {1: 0, 2: 1, 3: 2, 4: 3, 5: 4, 6: 5, 7: 6, 8: 8, 9: 16},
    }
    for name, mp in relabels.items():
        addc(name, [mp.get(v, v) for v in random_transform(rng, wiki_sol)])
    over = list(wiki_sol)
    over[0] = 200
    addc("value_200", over)
    addc("all_255", [255] * 81)
    addc("all_5", [5] * 81)
    for n in range(20):
        addc(f"random_vals{n:02d}", [rng.randrange(0, 20) for _ in range(81)])

    os.makedirs(HERE, exist_ok=True)
    meta = {
        "generator": "tests/golden/make_golden.py",
        "reference": "jsturm-11/distributed_sudoku_solver @ 2025-06-14 (imported read-only)",
        "seed": args.seed,
    }
    with open(os.path.join(HERE, "solve_cases.json"), "w") as f:
        json.dump({"meta": meta, "cases": solve_cases}, f, separators=(",", ":"))
    with open(os.path.join(HERE, "check_cases.json"), "w") as f:
        json.dump({"meta": meta, "cases": check_cases}, f, separators=(",", ":"))
    print(f"solve cases: {len(solve_cases)}  check cases: {len(check_cases)}")
    raws = {}
    for c in check_cases:
        raws[(c["raw"], c["intended"])] = raws.get((c["raw"], c["intended"]), 0) + 1
    print("check outcome histogram:", raws)
    print("solve ok histogram:", sum(c["ok"] for c in solve_cases), "True of", len(solve_cases))


if __name__ == "__main__":
    main_()
