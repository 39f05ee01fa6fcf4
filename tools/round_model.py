"""CPU model of the GPU solvers' round-synchronous propagation (dev tool, not a test).

Counts propagation rounds and search nodes per board for the rule set of solve4_kernel.h
(naked + hidden singles applied synchronously: every cell of a round sees the unit
summaries of the previous state) under LEX order, so that changes to the rule set can be
weighed in rounds before any kernel is written.

usage: python tools/round_model.py [--n N] [--workload solve17|solve30|minimal] [--variant base|...]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import synth  # noqa: E402

ALL = 0x1FF
UNITS = [[r * 9 + c for c in range(9)] for r in range(9)] + [[r * 9 + c for r in range(9)] for c in range(9)] + \
    [[(3 * (b // 3) + i // 3) * 9 + 3 * (b % 3) + i % 3 for i in range(9)] for b in range(9)]
CELL_UNITS = [[u for u in range(27) if cell in UNITS[u]] for cell in range(81)]


def single(x):
    return x != 0 and (x & (x - 1)) == 0


def propagate(X, S, variant):
    """Round-synchronous propagation to a fixpoint or contradiction.
    Returns (status, rounds): status 'contra' | 'open' | 'solved'."""
    rounds = 0
    while True:
        rounds += 1
        T = [0] * 27
        once = [0] * 27
        bad = False
        for u, cells in enumerate(UNITS):
            ox = os_ = tx = ts = 0
            for c in cells:
                tx |= ox & X[c]
                ox |= X[c]
                ts |= os_ & S[c]
                os_ |= S[c]
            if ts:
                bad = True
            if (ox | os_) != ALL:
                bad = True
            T[u] = os_
            once[u] = ox & ~tx
            if variant == "unit_naked":
                # unit lane anticipates naked singles w.r.t. its own T: X & ~T a single digit
                extra = 0
                for c in cells:
                    if X[c]:
                        v = X[c] & ~os_
                        if single(v):
                            extra |= v
                T[u] = (os_, extra)
        if bad:
            return "contra", rounds
        changed = False
        nX, nS = list(X), list(S)
        for c in range(81):
            if not X[c]:
                continue
            if variant == "unit_naked":
                t = 0
                for u in CELL_UNITS[c]:
                    t |= T[u][0]
                v = X[c] & ~t
                # a digit another cell of a unit is forced to (by that unit's T alone)
                ext = 0
                for u in CELL_UNITS[c]:
                    e = T[u][1]
                    own = X[c] & ~T[u][0]
                    if single(own):
                        e &= ~own   # ignore our own contribution (other cells may share it: conflict next round)
                    ext |= e
                v &= ~ext
            else:
                t = T[CELL_UNITS[c][0]] | T[CELL_UNITS[c][1]] | T[CELL_UNITS[c][2]]
                v = X[c] & ~t
            h = v & (once[CELL_UNITS[c][0]] | once[CELL_UNITS[c][1]] | once[CELL_UNITS[c][2]])
            if h and (h & (h - 1)):
                return "contra", rounds
            if h:
                v = h
            if v == 0:
                return "contra", rounds
            if single(v):
                nS[c] = v
                nX[c] = 0
            else:
                nX[c] = v
            if nX[c] != X[c]:
                changed = True
        X[:], S[:] = nX, nS
        if not changed:
            return ("open" if any(X) else "solved"), rounds


def locked(X):
    """One synchronous locked-candidates pass (pointing + claiming over the 54 box-line
    intersections).  Returns True if any candidate was removed."""
    rem = [0] * 81
    for b in range(9):
        br, bc = 3 * (b // 3), 3 * (b % 3)
        for k in range(3):
            # box b x row br+k, box b x col bc+k
            for line, inter in ((list(range((br + k) * 9, (br + k) * 9 + 9)), [(br + k) * 9 + bc + i for i in range(3)]),
                                (list(range(bc + k, 81, 9)), [(br + i) * 9 + bc + k for i in range(3)])):
                box = UNITS[18 + b]
                m_int = 0
                for c in inter:
                    m_int |= X[c]
                m_box_rest = 0
                for c in box:
                    if c not in inter:
                        m_box_rest |= X[c]
                m_line_rest = 0
                for c in line:
                    if c not in inter:
                        m_line_rest |= X[c]
                point = m_int & ~m_box_rest     # digits of the box only in this line: remove from line rest
                claim = m_int & ~m_line_rest    # digits of the line only in this box: remove from box rest
                for c in line:
                    if c not in inter:
                        rem[c] |= point
                for c in box:
                    if c not in inter:
                        rem[c] |= claim
    ch = False
    for c in range(81):
        if X[c] & rem[c]:
            X[c] &= ~rem[c]
            ch = True
    return ch


def solve(board, variant):
    X = [ALL if v == 0 else 0 for v in board]
    S = [0 if v == 0 else 1 << (v - 1) for v in board]
    stack = []
    nodes = 0
    rounds_per_node = []
    while True:
        st, r = propagate(X, S, variant)
        while st == "open" and variant == "locked" and locked(X):
            st, r2 = propagate(X, S, variant)
            r += r2 + 1
        nodes += 1
        rounds_per_node.append(r)
        if st == "solved":
            return nodes, rounds_per_node, [(S[c].bit_length()) for c in range(81)]
        if st == "open":
            cell = next(c for c in range(81) if X[c])
            m = X[cell]
            d = m & -m
            stack.append((list(X), list(S), cell, m ^ d))
            X[cell], S[cell] = 0, d
            continue
        while stack and stack[-1][3] == 0:
            stack.pop()
        if not stack:
            return nodes, rounds_per_node, None
        sx, ss, cell, rest = stack[-1]
        d = rest & -rest
        stack[-1] = (sx, ss, cell, rest ^ d)
        X[:], S[:] = list(sx), list(ss)
        X[cell], S[cell] = 0, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--workload", default="solve17")
    ap.add_argument("--variant", default="base")
    args = ap.parse_args()
    if args.workload == "minimal":
        p, s = synth.make_minimal(args.n)
    else:
        gen = synth.make_17clue if args.workload == "solve17" else synth.make_30clue
        p, s = gen(args.n, seed=11)
    tn = tr = 0
    first = []
    later = []
    for i in range(args.n):
        nodes, rpn, sol = solve([int(v) for v in p[i]], args.variant)
        assert sol is not None and sol == [int(v) for v in s[i]], i
        tn += nodes
        tr += sum(rpn)
        first.append(rpn[0])
        later.extend(rpn[1:])
    print(f"{args.variant} {args.workload} n={args.n}: nodes/board {tn / args.n:.3f}  rounds/board {tr / args.n:.2f}  "
          f"first-node rounds {np.mean(first):.2f}  later-node rounds {np.mean(later) if later else 0:.2f}")


if __name__ == "__main__":
    main()
