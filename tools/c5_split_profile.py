"""Projected multi-GPU C5 count on ONE GPU (dev tool): every rank's work of a world-W split is
run in turn on this device and timed alone; the max over ranks is the wall a W-GPU node would
see (the all-reduce aside).  Two-stage (replicated 1024*W frontier + per-rank refinement) vs
single-stage (replicated frontier of W GPUs' size, interleaved slices)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L  # noqa: E402
from distributed_sudoku_solver_amd.shard import default_target  # noqa: E402

EXPECT = {"15": 3_481_026, "14": 18_204_270}
b15 = synth.SEEDS17["S1"][:-9] + "0" * 9
boards = {"15": synth.parse(b15), "14": synth.parse(b15[:63] + "000100000" + "0" * 9)}


def rank_work(eng, board, rank, world, two_stage, stage1=1024, rdiv=1):
    t0 = time.perf_counter()
    if two_stage:
        _, leaves0 = eng.frontier_build(board, mode=L.SDK_FRONTIER_COUNT, target=stage1 * world)
        size, leaves1 = eng.frontier_refine(rank, world, max(8192, default_target(eng, 1) // rdiv))
        first, step, end, own = 0, 1, size, leaves1 + (leaves0 if rank == 0 else 0)
    else:
        size, leaves = eng.frontier_build(board, mode=L.SDK_FRONTIER_COUNT, target=default_target(eng, world))
        first, step, end, own = rank, world, size, (leaves if rank == 0 else 0)
    res = eng.result_buffer(2, np.uint64)
    eng.frontier_count(first, step, end, 0, res)
    cnt = int(eng.read(res, 2, np.uint64)[0]) + own
    res.free()
    return cnt, time.perf_counter() - t0


with SudokuEngine(0) as eng:
    for name, board in boards.items():
        for world in (4, 8):
            for stage1, rdiv in ((1024, 1), (1024, 2), (1024, 4), (256, 1), (256, 2), (4096, 2)):
                rank_work(eng, board, 0, world, True, stage1, rdiv)          # warm-up
                times, total = [], 0
                for r in range(world):
                    c, t = rank_work(eng, board, r, world, True, stage1, rdiv)
                    total += c
                    times.append(t)
                print(f"{name}-clue W={world} stage1={stage1}/rank refine=target/{rdiv}: ok={total == EXPECT[name]} "
                      f"max-rank {1e3 * max(times):.2f} ms  mean {1e3 * np.mean(times):.2f} ms", flush=True)
