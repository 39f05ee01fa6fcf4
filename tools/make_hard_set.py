"""Build the committed hard set (distributed_sudoku_solver_amd/data/hard_minimal.npz).

Scans the make_minimal stream (csrc/gen_minimal.c: random complete grid, clues removed
while the completion stays unique -> distinct minimal unique puzzles) in blocks, and
keeps every puzzle that a lowest-open-cell DFS with naked + hidden singles propagation
(lex_singles_nodes: the propagating solvers' own branching order) needs >= MIN_NODES
search nodes for, until COUNT are kept.  About 2 % of minimal puzzles pass at 20 nodes.

Stored: the stream indices (uint32), the clue masks (81 bits, packed), the seed, the
threshold and the filter's node counts; synth.load_hard rebuilds each puzzle as its
generating grid (= its unique answer) masked by its clue mask.

    python tools/make_hard_set.py [--count 100000] [--min-nodes 20] [--threads 8]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_sudoku_solver_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=100_000)
    ap.add_argument("--min-nodes", type=int, default=20)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--block", type=int, default=1 << 16)
    ap.add_argument("--out", default=synth.HARD_SET)
    args = ap.parse_args()
    seed = synth.DEFAULT_SEED + 3          # make_minimal's default stream
    idx, bits, nodes = [], [], []
    kept, lo, t0 = 0, 0, time.time()
    while kept < args.count:
        p, nd = synth.minimal_nodes(args.block, seed=seed, lo=lo, threads=args.threads)
        sel = np.flatnonzero(nd >= args.min_nodes)[: args.count - kept]
        idx.append((lo + sel).astype(np.uint32))
        bits.append(np.packbits(p[sel] != 0, axis=1))
        nodes.append(nd[sel])
        kept += len(sel)
        lo += args.block
        print(f"scanned {lo} kept {kept} ({time.time() - t0:.0f} s)", flush=True)
    idx, bits, nodes = np.concatenate(idx), np.concatenate(bits), np.concatenate(nodes)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.savez_compressed(args.out, idx=idx, clue_bits=bits, seed=np.uint64(seed),
                        min_nodes=np.uint32(args.min_nodes), filter_nodes=nodes, scanned=np.uint64(lo))
    print(f"wrote {args.out}: {len(idx)} puzzles from {lo} scanned, filter nodes mean {nodes.mean():.1f} "
          f"max {nodes.max()}", flush=True)


if __name__ == "__main__":
    main()
