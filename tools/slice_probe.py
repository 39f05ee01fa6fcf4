"""Wall time of search.LexSearch slices on the GPU (dev tool): the conflict board '55'+79 zeros
(unrefutable by propagation), per slice: budget, width, the slice's time split into the launch
(engine.solve_batch: H2D + kernel + D2H), the expansion (engine.expand) and the host work around
them, and the worklist size.  Sizes the node's slice_target_s / node_budget (node.py).

    python tools/slice_probe.py [--slices 12] [--target 0.01] [--node]

--node: the search exactly as a SudokuNode continues a budget-hit board (node.py _run_batch).
"""
import argparse
import gc
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from distributed_sudoku_solver_amd import SudokuEngine  # noqa: E402
from distributed_sudoku_solver_amd.search import LexSearch, default_budget  # noqa: E402


class _Timed:
    """Engine proxy that adds up the wall time of solve_batch and expand calls."""

    def __init__(self, eng):
        self.eng = eng
        self.t_solve = self.t_expand = 0.0
        self.n_solve = self.n_expand = 0

    def solve_batch(self, *a, **k):
        t0 = time.perf_counter()
        try:
            r = self.eng.solve_batch(*a, **k)
            if r[2] is not None and len(r[2]):
                self.work_max = max(getattr(self, "work_max", 0), int(np.max(r[2])))
            return r
        finally:
            self.t_solve += time.perf_counter() - t0
            self.n_solve += len(a[0])

    def expand(self, *a, **k):
        t0 = time.perf_counter()
        try:
            r = self.eng.expand(*a, **k)
            self.n_expand += len(r)
            return r
        finally:
            self.t_expand += time.perf_counter() - t0

    def __getattr__(self, k):
        return getattr(self.eng, k)


def _throttled_us():
    """cgroup v2 CPU throttling of this process's group (0 if not available)."""
    for path, key, scale in (("/sys/fs/cgroup/cpu.stat", "throttled_usec", 1),
                             ("/sys/fs/cgroup/cpu/cpu.stat", "throttled_time", 1e-3),
                             ("/sys/fs/cgroup/cpu,cpuacct/cpu.stat", "throttled_time", 1e-3)):
        try:
            with open(path) as f:
                for line in f:
                    if line.startswith(key):
                        return int(int(line.split()[1]) * scale)
        except OSError:
            continue
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slices", type=int, default=12)
    ap.add_argument("--target", type=float, default=0.01)
    ap.add_argument("--node", action="store_true", help="only the node's configuration")
    ap.add_argument("--fork", action="store_true", help="run on a forked context (as a node does)")
    ap.add_argument("--timing", action="store_true",
                    help="per slice also the kernels' own time (SDK_OPT_TIMING HIP events) and the most nodes a board took")
    args = ap.parse_args()
    board = np.zeros(81, np.uint8)
    board[0] = board[1] = 5
    worst = {}
    with SudokuEngine(0) as eng0:
        eng = eng0.fork() if args.fork else eng0
        if args.timing:
            from distributed_sudoku_solver_amd import _lib as L
            eng.set_option(L.SDK_OPT_TIMING, 1)
        b0 = default_budget(eng)
        configs = [("node", args.target)] if args.node else [("free", None), ("node", args.target)]
        for name, target in configs:
            te = _Timed(eng)
            if name == "node":
                s = LexSearch.for_node(te, board, None, slice_target_s=target)
            else:
                s = LexSearch(te, board, budget=b0, hit=True, slice_target_s=target)
            worst[name] = 0.0
            for k in range(args.slices):
                te.t_solve = te.t_expand = 0.0
                te.n_solve = te.n_expand = 0
                te.work_max = 0
                if args.timing:
                    eng.timer_reset()
                tcpu0 = time.thread_time()
                thr0, cpu0, gc0 = _throttled_us(), time.process_time(), sum(g["collections"] for g in gc.get_stats())
                t0 = time.perf_counter()
                done = s.step()
                dt = time.perf_counter() - t0
                thr = _throttled_us() - thr0
                cpu = time.process_time() - cpu0
                tcpu = time.thread_time() - tcpu0
                gcs = sum(g["collections"] for g in gc.get_stats()) - gc0
                kern = ""
                if args.timing:
                    eng.synchronize()
                    kms, nl = eng.timer_read()
                    kern = f" kernel_ms={kms:.2f} ({nl} launches) work_max={te.work_max}"
                worst[name] = max(worst[name], dt)
                print(f"{name} target={target} slice={k} budget={s.budget} width={te.n_solve} pending={s.pending} "
                      f"nodes={s.nodes} ms={1e3 * dt:.2f} launch_ms={1e3 * te.t_solve:.2f} "
                      f"expand_ms={1e3 * te.t_expand:.2f} (kids {te.n_expand}) "
                      f"host_ms={1e3 * (dt - te.t_solve - te.t_expand):.2f} "
                      f"cpu_ms={1e3 * cpu:.2f} thread_cpu_ms={1e3 * tcpu:.2f} throttled_ms={thr / 1e3:.2f} gc={gcs}"
                      f"{kern} done={done}", flush=True)
                if done:
                    break
    for name, w in worst.items():
        print(f"worst slice {name}: {1e3 * w:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
