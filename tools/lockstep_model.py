"""CPU model of a bit-sliced, lockstep propagation pass (dev tool, not a test): 32 boards advance
together -- one synchronous singles round or one locked-candidates pass for all of them at a time --
until every board is solved, contradicted or stuck (a fixpoint that locked candidates cannot move).
Counts rounds and locked-candidates passes per group under a scheduling policy, beside the per-board
counts of solve4's own schedule (round_model's rule set: singles to a fixpoint, then one LC pass,
again until LC changes nothing), so a bit-sliced kernel can be priced before it is written.

usage: python tools/lockstep_model.py [--n 2048] [--workload solve17|minimal] [--group 32]
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
ROW_TRIADS = [[9 * r + 3 * k + i for i in range(3)] for r in range(9) for k in range(3)]     # (row, box column)
COL_TRIADS = [[9 * (3 * k + i) + c for i in range(3)] for c in range(9) for k in range(3)]   # (column, box row)


def single(x):
    return x != 0 and (x & (x - 1)) == 0


def singles_round(X):
    """One synchronous round (naked + hidden singles) on candidate masks X (closed cell = one bit).
    Returns (newX, changed, bad)."""
    T, once, bad = [0] * 27, [0] * 27, False
    for u, cells in enumerate(UNITS):
        ox = tx = taken = twice = 0
        for c in cells:
            x = X[c]
            if single(x):
                twice |= taken & x
                taken |= x
            else:
                tx |= ox & x
                ox |= x
        if twice or (ox | taken) != ALL:
            bad = True
        T[u], once[u] = taken, ox & ~tx
    new = list(X)
    for c in range(81):
        x = X[c]
        if single(x):
            continue
        U = T[CELL_UNITS[c][0]] | T[CELL_UNITS[c][1]] | T[CELL_UNITS[c][2]]
        H = once[CELL_UNITS[c][0]] | once[CELL_UNITS[c][1]] | once[CELL_UNITS[c][2]]
        v = x & ~U
        h = v & H
        if h:
            if not single(h):
                bad = True
            v = h
        if v == 0:
            bad = True
        new[c] = v
    return new, new != X, bad


def lc_pass(X):
    """Pointing and claiming over the 54 box-line triads."""
    def pres(tri):
        # every digit still possible in the triad, closed cells included: then the pass is valid at
        # any state, not only at a singles fixpoint (where the two are the same)
        m = 0
        for c in tri:
            m |= X[c]
        return m
    new = list(X)
    for triads in (ROW_TRIADS, COL_TRIADS):
        P = [pres(t) for t in triads]
        for line in range(9):
            for k in range(3):
                t = 3 * line + k
                others_line = P[3 * line + (k + 1) % 3] | P[3 * line + (k + 2) % 3]
                # the other triads of the same box: same k, the other two lines of the band/stack
                band = (line // 3) * 3
                others_box = 0
                for l2 in range(band, band + 3):
                    if l2 != line:
                        others_box |= P[3 * l2 + k]
                claim = P[t] & ~others_line          # digit of the line only in this box -> out of the box's other cells
                point = P[t] & ~others_box           # digit of the box only in this line -> out of the line's other cells
                for l2 in range(band, band + 3):
                    if l2 != line:
                        for c in triads[3 * l2 + k]:
                            if not single(new[c]):
                                new[c] &= ~claim
                for k2 in range(3):
                    if k2 != k:
                        for c in triads[3 * line + k2]:
                            if not single(new[c]):
                                new[c] &= ~point
    return new, new != X


def board_state(b):
    return [ALL if v == 0 else 1 << (int(v) - 1) for v in b]


def done_kind(X, bad):
    if bad:
        return "contra"
    if all(single(x) for x in X):
        return "solved"
    return None


def solo(b):
    """solve4's root schedule for one board: rounds and LC passes until solved / contra / stuck."""
    X, rounds, lcs = board_state(b), 0, 0
    while True:
        X, ch, bad = singles_round(X)
        rounds += 1
        k = done_kind(X, bad)
        if k:
            return rounds, lcs, k
        if not ch:
            X, lch = lc_pass(X)
            lcs += 1
            if not lch:
                return rounds, lcs, "stuck"


def lockstep(group, policy, lc_every):
    """All boards of the group take every step.  policy 'fix': an LC pass after a singles round in
    which some live board made no change; 'every': an LC pass after every lc_every-th round;
    'stall': after a round in which no live board closed a cell, or after lc_every rounds without a
    pass."""
    Xs = [board_state(b) for b in group]
    prev_closed = [sum(single(x) for x in X) for X in Xs]
    since = 0
    live = [True] * len(group)
    kinds = [None] * len(group)
    rounds = lcs = 0
    while any(live):
        fix = False
        for i, X in enumerate(Xs):
            if not live[i]:
                continue
            X, ch, bad = singles_round(X)
            Xs[i] = X
            k = done_kind(X, bad)
            if k:
                live[i], kinds[i] = False, k
            elif not ch:
                fix = True
                kinds[i] = "fix"
        rounds += 1
        since = locals().get("since", 0) + 1
        if policy == "stall":
            closed_any = any(sum(single(x) for x in Xs[i]) > prev_closed[i] for i in range(len(group)) if live[i])
            run_lc = (not closed_any) or since >= lc_every
        else:
            run_lc = fix if policy == "fix" else (rounds % lc_every == 0 or (fix and all(
                kinds[i] == "fix" for i in range(len(group)) if live[i])))
        prev_closed = [sum(single(x) for x in X) for X in Xs]
        if run_lc:
            since = 0
        if run_lc and any(live):
            lcs += 1
            for i, X in enumerate(Xs):
                if not live[i]:
                    continue
                X, lch = lc_pass(X)
                Xs[i] = X
                if kinds[i] == "fix" and not lch:
                    live[i], kinds[i] = False, "stuck"
                elif kinds[i] == "fix":
                    kinds[i] = None
        if rounds > 200:
            break
    return rounds, lcs, kinds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--workload", default="solve17")
    ap.add_argument("--group", type=int, default=32)
    args = ap.parse_args()
    if args.workload == "minimal":
        p, _ = synth.make_minimal_sym(args.n, threads=8)
    else:
        p, _ = synth.make_17clue(args.n, seed=11)
    res = [solo(b) for b in p]
    r = np.array([x[0] for x in res])
    lc = np.array([x[1] for x in res])
    kinds = [x[2] for x in res]
    print(f"solo: rounds mean {r.mean():.2f} max {r.max()}, LC passes mean {lc.mean():.2f}, "
          f"solved {kinds.count('solved')}, stuck {kinds.count('stuck')}, contra {kinds.count('contra')}")
    for policy, k in (("every", 1), ("every", 2), ("every", 3)):
        gr, gl, stuck = [], [], 0
        for g in range(0, len(p), args.group):
            rr, ll, kk = lockstep(p[g:g + args.group], policy, k)
            gr.append(rr)
            gl.append(ll)
            stuck += kk.count("stuck")
        gr, gl = np.array(gr), np.array(gl)
        print(f"lockstep {policy}{k or ''}: rounds per group mean {gr.mean():.2f} max {gr.max()}, "
              f"LC passes per group mean {gl.mean():.2f}, stuck boards {stuck}")


if __name__ == "__main__":
    main()
