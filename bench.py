#!/usr/bin/env python3
"""Benchmark of the hot path on MI355X (contract: one JSON line from rank 0).

Headline (BASELINE.json metric): 17-clue hard puzzles solved per second, whole
job, config C4 = 10M transformed 17-clue puzzles SHARDED over the N GPUs (rank k
owns rows [k*10M/N, (k+1)*10M/N) of one seeded stream, resident in HBM; strong
scaling); one "step" = one sdk_solve_batch_dev pass of every rank over its
slice.  No collective on the data path; the ranks' barrier and max-over-ranks
time go over hostcomm.TcpComm (standard-library sockets: the product's own host
transport -- nothing here imports torch).  After timing, every solved board is
compared with its expected solution (known by construction) -- a mismatch fails
the run.  At N > 1 a secondary weak-scaling figure (10M puzzles per GPU) is
reported beside it.

`python bench.py --gpus N` without torchrun starts N rank processes itself (one
per GPU, before anything touches a GPU); under torchrun the ranks come from
RANK / WORLD_SIZE / LOCAL_RANK.

Side legs on the same run: the batched checker (config C3, 100M boards per GPU
by default, HBM-bound), config C2 (1M ~30-clue puzzles per GPU), config C5 (an
exhaustive count of one 15-clue board, its frontier split over all ranks, the
count combined by an RCCL all-reduce over xGMI), config C1 (POST /solve latency on
a GPU-backed node) and the CPU baseline (rank 0, N=1 only): the oracle's C port of
the reference's naive DFS on a bounded sample of the same puzzles.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "puzzles solved/sec (whole node, 17-clue hard) at 1/2/4/8 GPUs; checker HBM GB/s"
HBM_PEAK_GBPS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
SOLVE_BYTES_PER_PUZZLE = 163      # 81 in + 81 out + 1 status
CHECK_BYTES_PER_BOARD = 82        # 81 in + 1 verdict
# VALU issue peak: 256 CUs x 4 SIMD-32, one wave64 VALU instruction per 2 cycles per SIMD = 2 per
# SIMD quad-cycle (MI355X_MICROARCH.md:54: "issues each VALU instruction over 2 cycles (32 lanes/cycle
# x 2)"); at 2.4 GHz 1.23e12 wave-instr/s.  Round 4 priced it at one per quad-cycle.
VALU_PER_SIMD_QUAD = 2.0
VALU_PEAK_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 4 * VALU_PER_SIMD_QUAD
# --solver: (SDK_OPT_SOLVER value, kernel name, grid option) -- resolved after the library loads
SOLVERS = {
    "halfwave": (1, "sdk::solve2_kernel", 8),
    "wave": (0, "sdk::solve_kernel", 3),
    "quad": (2, "sdk::solve4_kernel", 8),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--inflight", type=int, default=2,
                    help="C4 headline: passes in flight per rank -- consecutive passes issued on this many engine "
                         "contexts in turn (own HIP stream, dequeue state and output buffer each), so one pass's "
                         "launch drain overlaps the next pass's start, as a serving node keeps batches in flight; "
                         "1 = one context.  The single-context figure and its per-launch kernel time (the "
                         "roofline's) are reported beside it as `single_stream`.  2 since the round-6 kernels "
                         "(1 / 2 / 3: 3.23-3.24 / 3.27-3.28 / 3.23-3.29 G/s, profiles/r06/ab_inflight_r06.log)")
    ap.add_argument("--workload", choices=["solve17", "solve30"], default="solve17")
    ap.add_argument("--batch", type=int, default=10_000_000, help="C4 puzzles, whole job (sharded over the GPUs)")
    ap.add_argument("--weak-leg", type=int, default=1, help="N > 1: also time --batch puzzles per GPU (weak scaling)")
    ap.add_argument("--check-boards", type=int, default=100_000_000, help="checker boards per GPU (0 = skip)")
    ap.add_argument("--check-steps", type=int, default=20)
    ap.add_argument("--check-warmup", type=int, default=10,
                    help="untimed checker launches first (the memory clocks ramp under sustained streaming)")
    ap.add_argument("--warm-ms", type=float, default=60.0,
                    help="untimed warm-up: beyond the W steps, passes back to back until this long (ms) -- the "
                         "GPU's clock ramps over its first ~40 ms of load (profiles/r06/clock_ramp_r06i.jsonl)")
    ap.add_argument("--order", choices=["mrv_unique", "lex"], default="lex")
    ap.add_argument("--solver", choices=sorted(SOLVERS), default="quad",
                    help="solve kernel: four boards per wave (solve4_kernel), two (solve2_kernel) or one (solve_kernel)")
    ap.add_argument("--waves-per-cu", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget per leg (0 = skip)")
    ap.add_argument("--cpu-cores", type=int, default=0,
                    help="CPU baseline processes/threads (0 = this process's CPU share: affinity, capped by "
                         "OMP_NUM_THREADS when set)")
    ap.add_argument("--cpu-puzzle-budget", type=int, default=2_000_000,
                    help="per-puzzle timeout of the Python baseline, in reference validations")
    ap.add_argument("--http-requests", type=int, default=20, help="C1 POST /solve leg (rank 0, N=1; 0 = skip)")
    ap.add_argument("--seed", type=int, default=20250614)
    ap.add_argument("--c2-puzzles", type=int, default=1_000_000,
                    help="C2 leg: ~30-clue unique puzzles per GPU (0 = skip)")
    ap.add_argument("--minimal-puzzles", type=int, default=1 << 20,
                    help="distinct minimal-puzzle leg, puzzles per GPU (0 = skip)")
    ap.add_argument("--hard-leg", type=int, default=1,
                    help="hard-search leg: the committed hard set (100k distinct puzzles that search) and its "
                         "1000 heaviest, one launch vs the phased solve with subtree donation (0 = skip)")
    ap.add_argument("--hard-reps", type=int, default=10, help="hard_1m: symmetries of the 100k hard set per GPU")
    ap.add_argument("--prop32", type=int, default=-1, help="SDK_OPT_PROP32 for every leg (-1 = library default)")
    ap.add_argument("--hard-split-inflight", type=int, default=0,
                    help="hard legs: split budget of the donation_in_flight mode (0 = the library's rule)")
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=VALUE: an SDK_OPT_* engine option for every leg (experiments), e.g. PROP32_LC=3")
    ap.add_argument("--hard-inflight", type=int, default=3,
                    help="hard legs: passes in flight of the donation_in_flight mode (0 = --inflight); 3: the "
                         "hard sets' launch tails are longer than C4's (profiles/r05/bench_hard_inflight_r05z.log)")
    ap.add_argument("--count-leg", type=int, default=1, help="C5 leg: frontier-split count over all ranks (0 = skip)")
    ap.add_argument("--c5-boards", default="15,14",
                    help="C5 boards: 16/15/14 clues (S1 with clues removed; counts 7,309 / 3,481,026 / 18,204,270); "
                         "the first is counted by the two-stage split, the second by the rebalanced one")
    ap.add_argument("--first-boards", default="heaviest,antibt,S1",
                    help="first-solution leg (sharded_solve over all ranks): boards -- heaviest, antibt (the "
                         "anti-backtracking 17-clue puzzle) or S1..S5 ('' = skip); each at the default frontier "
                         "and split (4 boards per rank, 16-node rounds)")
    ap.add_argument("--frontier-probe", type=int, default=1_000_000,
                    help="boards of the timed one-board frontier build beside the rebalanced count (0 = skip)")
    ap.add_argument("--lane-puzzles", type=int, default=200_000,
                    help="per-lane reference-DFS leg on a C2 prefix (rank 0, N=1; 0 = skip)")
    ap.add_argument("--leg-timeout", type=float, default=120.0,
                    help="watchdog for the side legs: print what was measured and exit")
    ap.add_argument("--pmc-pipe", default=os.path.join(ROOT, "profiles", "r06", "pmc_pipe.json"),
                    help="per-SIMD pipe counters of the solve kernel (tools/pmc_r04.sh; '' = none)")
    ap.add_argument("--issue-calib", default=os.path.join(ROOT, "profiles", "r06", "issue_calib_pmc.json"),
                    help="VALU issue ceilings of the solve kernel's instruction mix (tools/issue_calib.hip under "
                         "rocprofv3, tools/issue_calib_summary.py; '' = none)")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "r06", "pmc_c4.json"),
                    help="per-launch PMC figures of the C4 solve kernel and the C3 checker from rocprofv3 passes "
                         "of this bench at its default sizes (tools/pmc_c4.sh); '' = report traffic null")
    ap.add_argument("--engine-factory", default="", help=argparse.SUPPRESS)
    return ap.parse_args()


class Dist:
    """The ranks' host exchanges (barrier, max/sum of one number) over hostcomm.TcpComm: the
    product's own standard-library transport, the one that also hands out the RCCL id of the C5
    legs.  Ranks come from RANK / WORLD_SIZE / LOCAL_RANK (torchrun or launch_ranks), the
    rendezvous from MASTER_ADDR and SDK_RDZV_PORT (else MASTER_PORT + 1)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.comm = None
        if self.world > 1:
            from distributed_sudoku_solver_amd.hostcomm import TcpComm
            self.comm = TcpComm(self.rank, self.world, addr=os.environ.get("MASTER_ADDR", "127.0.0.1"))

    def barrier(self):
        if self.world > 1:
            self.comm.barrier()

    def _reduce(self, x, op):
        if self.world == 1:
            return x
        buf = np.array([float(x)], dtype=np.float64)
        self.comm.allreduce(buf, 1, np.float64, op)
        return float(buf[0])

    def max(self, x):
        return self._reduce(x, "max")

    def sum(self, x):
        return self._reduce(x, "sum")

    def close(self):
        if self.comm is not None:
            self.comm.close()


def pmc_record(path, kernel, units):
    """Per-launch PMC figures of `kernel` from the committed rocprofv3 passes of this bench
    (tools/pmc_c4.sh -> tools/pmc_summary.py), or None.  Only used when the record was taken at
    the same units per launch as this run (puzzles or boards per launch)."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        recs = json.load(f)
    # a kernel's record is keyed by its full name (template arguments included: the plain
    # sdk::solve4_kernel<false, false, false>) or by the bare name
    rec = recs.get(kernel) or next((v for k, v in recs.items() if k.startswith(kernel + "<")
                                    and k.endswith("<false, false, false>")), None)
    if rec is None or int(rec.get("units_per_launch", -1)) != int(units):
        return None
    return rec


def mix_ceiling(path):
    """VALU issue ceiling of the solve kernel's own instruction mix (tools/issue_calib.hip k_mix: the
    exact-wave round's VALU -- unit4x and three upd4x, 3-source VOP3 and packed VOP3P ops -- on
    registers, every SIMD full), VALU wave-instructions per SIMD quad-cycle, or None."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        recs = json.load(f)
    out = {}
    for key in ("k_mix@8", "k_round<true>@8", "k_int2@8", "k_or3@8", "k_b3@8", "k_pk@8"):
        r = recs.get(key, {}).get("pipe")
        if r and r.get("valu_per_quad") is not None:
            out[key] = {"valu_per_quad": r["valu_per_quad"], "dual_frac": r.get("valu_dual_frac"),
                        "waves_per_simd": r.get("waves_per_simd")}
    return out or None


def pipe_record(path, run, units):
    """Per-SIMD pipe figures of the solve kernel from tools/pmc_r04.sh (pmc_pipe.json), or None;
    only for a launch of the same size as this run's."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        rec = json.load(f).get(run)
    if rec is None or int(rec.get("units_per_launch", -1)) != int(units):
        return None
    keep = ("kernel_ms", "clock_ghz", "valu_busy_frac", "valu_dual_frac", "valu_per_quad", "salu_per_cu_cycle",
            "lds_busy_frac", "lds_insts_per_cu_cycle", "lds_bank_conflict_frac", "lds_data_fifo_full_frac",
            "lds_cmd_fifo_full_frac", "waves_per_simd")
    out = {}
    for part in ("pipe", "lds"):
        for k, v in rec.get(part, {}).items():
            if k in keep and k not in out:
                out[k] = v
        ctr = rec.get(part, {}).get("counters", {})
        for k, c in (("valu_insts", "SQ_INSTS_VALU"), ("salu_insts", "SQ_INSTS_SALU"), ("lds_insts", "SQ_INSTS_LDS")):
            if c in ctr and k not in out:
                out[k] = ctr[c]
    out["source"] = os.path.relpath(path, ROOT)
    return out


def cpu_share():
    """CPU cores this process may use: its affinity set, capped by OMP_NUM_THREADS when set
    (the GPU box exports its per-GPU CPU share there; os.cpu_count() is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline_c(puzzles, seconds, threads):
    """Oracle's C port of the reference naive DFS (DHT_Node.py:474-538), timed on this
    host on a bounded prefix of the SAME puzzle batch, `threads` puzzles at a time."""
    from oracle import oracle as O
    budget = 2_000_000_000
    done = solved = timeouts = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done + threads <= len(puzzles):
        chunk = puzzles[done:done + threads]
        _, st, _ = O.naive_solve_batch(chunk, budget=budget, threads=threads)
        solved += int((st == 1).sum())
        timeouts += int((st == -2).sum())
        done += threads
    wall = time.perf_counter() - t0
    return {
        "value": solved / wall if wall > 0 else 0.0,
        "unit": "puzzles/s",
        "cores": threads,
        "kind": "port",
        "attempted": done, "solved": solved, "capped": timeouts,
        "sample": (f"first {done} puzzles of the rank-0 batch, naive DFS in C (oracle/sudoku_oracle.c, "
                   f"restates DHT_Node.py:474-538, validations-exact), {threads} threads, "
                   f"{wall:.1f} s wall, {timeouts} hit the 2e9-validation budget"),
    }


def cpu_baseline_python(puzzles, seconds, procs, budget, what):
    """The oracle's line-by-line Python restatement of DHTNode.solve_sudoku
    (oracle.py_naive_solve, DHT_Node.py:474-538) -- the closest stand-in for the
    reference's own Python solver, which cannot travel to the GPU box -- one process
    per core (like one DHT node per core, -d 0), each on its own slice of the batch,
    every puzzle capped at `budget` validations (the per-puzzle timeout)."""
    import multiprocessing as mp
    from oracle import oracle as O
    per = max(1, -(-len(puzzles) // procs))
    slices = [[list(map(int, puzzles[i])) for i in range(k * per, min((k + 1) * per, len(puzzles)))]
              for k in range(procs)]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.starmap(O.py_solve_timed, [(sl, seconds, budget) for sl in slices])
    wall = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    solved = sum(r[1] for r in res)
    busy = max(r[2] for r in res)
    timeouts = sum(r[3] for r in res)
    return {
        "value": solved / busy if busy > 0 else 0.0,
        "unit": "puzzles/s",
        "cores": procs,
        "kind": "port",
        "attempted": done, "solved": solved, "capped": timeouts,
        # puzzles stopped at the per-puzzle cap are not counted and their time is: with capped > 0 the
        # sample's solved puzzles are its easiest, and the rate an upper bound of the CPU's rate on them
        "value_is": ("an upper bound: solved puzzles per second of a sample whose capped puzzles were dropped "
                     "(the easiest slice)" if timeouts else "solved puzzles per second, every puzzle solved"),
        "sample": (f"{what}: {done} puzzles attempted in {procs} disjoint slices, one process per core, "
                   f"pure-Python naive DFS (oracle/oracle.py py_naive_solve, restates DHT_Node.py:474-538 "
                   f"line by line, -d 0), {solved} solved, {timeouts} stopped at the {budget:,}-validation "
                   f"per-puzzle timeout, {busy:.1f} s solving per process ({wall:.1f} s incl. process start)"),
    }


# The reference's own CPU numbers, measured by the survey in the build container (SURVEY §6,
# BASELINE.md; not published anywhere): quoted beside the GPU figures they compare with.
REFERENCE_MEASURED = {
    "solve_17clue": {"value": 0.0059, "unit": "puzzles/s/core",
                     "how": "DHT_Node.solve_sudoku, -d 0, 5 seeds S1-S5 in 844 core-s (SURVEY §6)"},
    "check": {"value": 20_400.0, "unit": "boards/s/core",
              "how": "Sudoku.check intended semantics, _limit_calls disabled, 49 us/board (SURVEY §3.3)"},
    "post_solve_ms": {"dht": 87.0, "main": 100.0, "unit": "ms",
                      "how": "wiki 30-clue POST /solve, one node on loopback, -d 0 (SURVEY §3.1)"},
}


def cpu_baseline_check(boards, seconds, procs):
    """Config C3 on the host: the oracle's line-by-line Python restatement of Sudoku.check
    (oracle.py_check, sudoku.py:43-94, limiter off) one process per core on disjoint slices of a
    fixed sample, and the C port (oracle check_batch) with `procs` threads on the whole sample."""
    import multiprocessing as mp
    from oracle import oracle as O
    n = len(boards)
    per = max(1, -(-n // procs))
    # a bounded sample: about `seconds` of Python work per process at ~50 us per board
    per = min(per, max(1000, int(seconds / 50e-6)))
    slices = [[list(map(int, b)) for b in boards[k * per: min((k + 1) * per, n)]] for k in range(procs)]
    slices = [sl for sl in slices if sl]
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(len(slices)) as pool:
        res = pool.map(O.py_check_timed, slices)
    wall = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    busy = max(r[2] for r in res)
    t1 = time.perf_counter()
    v = O.check_batch(boards, threads=procs)
    cwall = time.perf_counter() - t1
    return {
        "value": done / busy if busy > 0 else 0.0, "unit": "boards/s", "cores": len(slices), "kind": "port",
        "per_core": done / busy / len(slices) if busy > 0 else 0.0,
        "sample": (f"{done} boards of the C3 stream in {len(slices)} disjoint slices, one process per core, "
                   f"pure-Python Sudoku.check restatement (oracle/oracle.py py_check, sudoku.py:43-94, "
                   f"limiter off), {busy:.1f} s per process ({wall:.1f} s incl. process start)"),
        "c_port": {"value": n / cwall, "unit": "boards/s", "threads": procs, "boards": n,
                   "valid": int((v & 1).sum())},
        "reference_measured": REFERENCE_MEASURED["check"],
    }


def c2_leg(eng, d, args, synth):
    """Config C2: ~30-clue unique puzzles, resident in HBM, one launch per step."""
    from distributed_sudoku_solver_amd import _lib as L
    n = args.c2_puzzles
    p, sol = synth.make_30clue(n, seed=args.seed + 31, lo=d.rank * n)
    d_in, d_out, d_st = eng.alloc(n * 81), eng.alloc(n * 81), eng.alloc(n)
    d_in.upload(p)
    _warm(args, [eng], lambda e, k: e.solve_batch_dev(d_in, d_out, d_st, n))
    eng.timer_reset()
    d.barrier()
    t0 = time.perf_counter()
    steps = 5
    for _ in range(steps):
        eng.solve_batch_dev(d_in, d_out, d_st, n)
    eng.synchronize()
    d.barrier()
    el = d.max(time.perf_counter() - t0)
    spans = timer_spans(eng)
    eng.timer_stop()
    if len(spans) == 2 * steps and eng.get_option(L.SDK_OPT_PROP32):
        spans = spans[0::2]         # a prop32 solve is two spans: the pass (the roofline's) and its fallback
    out = np.empty((n, 81), np.uint8)
    st = np.empty(n, np.int8)
    d_out.download(out)
    d_st.download(st)
    bad = int(d.sum(int(((out != sol).any(axis=1) | (st != 1)).sum())))
    for b in (d_in, d_out, d_st):
        b.free()
    k_s = sum(spans) / 1000.0 / max(len(spans), 1)
    leg = {"workload": f"C2: {n} ~30-clue unique puzzles per GPU (seeds S1-S5 solutions + 13 cells, symmetries)",
           "value": d.world * n * steps / el, "unit": "puzzles/s", "avg_kernel_ms": k_s * 1000.0,
           "roofline": {"bound": "hbm", "achieved": SOLVE_BYTES_PER_PUZZLE * n / k_s / 1e9, "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": SOLVE_BYTES_PER_PUZZLE * n / k_s / 1e9 / HBM_PEAK_GBPS,
                        "kernel": args.solve_kernel},
           "parity": {"mismatched_boards": bad, "checked_boards": d.world * n}}
    if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0:
        cores = args.cpu_cores or cpu_share()
        leg["cpu_baseline"] = cpu_baseline_python(p[:200_000], min(5.0, args.cpu_seconds), cores,
                                                  args.cpu_puzzle_budget, "C2 ~30-clue sample")
        leg["cpu_baseline_c_port"] = cpu_baseline_c(p, min(5.0, args.cpu_seconds), cores)
    return leg


C5_BOARD_SOLUTIONS = 3_481_026    # S1 with its last row cleared (15 clues)
C5_14CLUE_SOLUTIONS = 18_204_270   # the 15-clue board minus one more clue (C probe)


def c5_board(synth, clues):
    """SURVEY §8(d) C5 boards: S1 with clues removed -> (board, expected count, description)."""
    b15 = synth.SEEDS17["S1"][:-9] + "0" * 9
    spec = {"16": (synth.SEEDS17["S1"][:-9] + "000800000", 7_309, "S1 minus its last row but one clue (16 clues)"),
            "15": (b15, C5_BOARD_SOLUTIONS, "S1 minus its last row (15 clues)"),
            "14": (b15[:63] + "000100000" + "0" * 9, C5_14CLUE_SOLUTIONS,
                   "S1 minus its last row and one more clue (14 clues)")}[str(clues)]
    return synth.parse(spec[0]), spec[1], spec[2]


def c5_leg(eng, d, args, synth):
    """Config C5: exhaustive count of one 15-clue board.  Every rank expands the same frontier
    and counts its interleaved share; one RCCL all-reduce (device memory, xGMI) combines them.
    The RCCL id travels over the ranks' TcpComm."""
    from distributed_sudoku_solver_amd.shard import RcclComm, sharded_count
    board, expected, what = c5_board(synth, args.c5_boards.split(",")[0])
    comm = RcclComm(eng, d.rank, d.world, transport=d.comm) if d.world > 1 else None
    try:
        sharded_count(eng, board, d.rank, d.world, comm=comm)            # warm-up
        walls = []
        for _ in range(3):
            d.barrier()
            t0 = time.perf_counter()
            total, st, size = sharded_count(eng, board, d.rank, d.world, comm=comm)
            walls.append(d.max(time.perf_counter() - t0))
    finally:
        if comm is not None:
            comm.close()
    w = min(walls)
    return {"workload": f"C5: count every completion of {what}, frontier split over "
                        f"{d.world} GPU(s)" + (", RCCL all-reduce" if d.world > 1 else ""),
            "solutions": total, "expected": expected, "ok": total == expected and st == 1,
            "frontier_boards": size, "wall_ms": w * 1000.0, "value": total / w, "unit": "solutions/s"}


def c5_rebalanced_leg(eng, d, args, synth):
    """Config C5 on the 14-clue board with dynamic rebalancing: ranks start on equal blocks of the
    replicated frontier and, after every round, all-gather their live ranges over RCCL (xGMI) so dry
    ranks take half of the largest remaining one (shard.sharded_count_rebalanced)."""
    from distributed_sudoku_solver_amd.shard import RcclComm, sharded_count_rebalanced
    specs = args.c5_boards.split(",")
    board, expected, what = c5_board(synth, specs[1] if len(specs) > 1 else specs[0])
    comm = RcclComm(eng, d.rank, d.world, transport=d.comm) if d.world > 1 else None
    try:
        sharded_count_rebalanced(eng, board, d.rank, d.world, comm=comm)   # warm-up
        walls = []
        for _ in range(3):
            info = {}
            d.barrier()
            t0 = time.perf_counter()
            total, st, size = sharded_count_rebalanced(eng, board, d.rank, d.world, comm=comm, info=info)
            walls.append(d.max(time.perf_counter() - t0))
    finally:
        if comm is not None:
            comm.close()
    w = min(walls)
    # frontier scale: a ~1M-board frontier of the same board (tile scan over the chip,
    # device-side level loop), timed alone
    if args.frontier_probe > 0:
        fw = []
        for _ in range(3):
            eng.synchronize()
            t0 = time.perf_counter()
            fsize, _ = eng.frontier_build(board, target=args.frontier_probe)
            fw.append(time.perf_counter() - t0)
        info["frontier_1m"] = {"boards": fsize, "build_ms": 1000 * min(fw)}
    return {"frontier_1m": info.get("frontier_1m"),
            "workload": f"C5: count every completion of {what}, rebalanced frontier over {d.world} GPU(s)"
                        + (", RCCL all-gather of live ranges + all-reduce" if d.world > 1 else ""),
            "solutions": total, "expected": expected,
            "ok": total == expected and st == 1, "frontier_boards": size,
            "rounds": info.get("rounds"), "steals": info.get("steals"),
            "wall_ms": w * 1000.0, "value": total / w, "unit": "solutions/s"}


def first_board(synth, name):
    """A first-solution board of the sharded_solve leg -> (board, its lex-first completion, what).
    `heaviest`: the committed hard set's heaviest puzzle (most singles-DFS nodes, unique);
    `S1`..`S5`: the survey's 17-clue seeds (0.67M-83M reference validations each)."""
    if name == "heaviest":
        hp, hs = synth.make_hard_heaviest(1, threads=cpu_share())
        return hp[0], hs[0], "the committed hard set's heaviest puzzle"
    if name == "antibt":
        return (synth.parse(ANTI_BACKTRACKING), synth.parse(ANTI_BACKTRACKING_SOLUTION),
                "the 17-clue puzzle built against brute-force backtracking (first row 987654321; "
                "138,350,633 reference validations by the oracle's C port)")
    return (synth.parse(synth.SEEDS17[name]), synth.parse(synth.SEED_SOLUTIONS[name]),
            f"17-clue seed {name} (SURVEY App. A)")


# Wikipedia "Sudoku solving algorithms": a puzzle built so that row-major ascending backtracking
# needs as many steps as possible (its solution's first row is 987654321)
ANTI_BACKTRACKING = "000000000000003085001020000000507000004000100090000000500000073002010000000040009"
ANTI_BACKTRACKING_SOLUTION = ("987654321246173985351928746128537694634892157795461832519286473472319568"
                              "863745219")


def first_solution_leg(eng, d, args, synth):
    """North star's single hard search split over the GPUs (the reference splits one
    search between ring nodes, DHT_Node.py:491-510): shard.sharded_solve on each board -- every
    rank builds the same lex-ordered frontier, searches its block in rounds, all-gathers (lo, hi,
    keys, best) over RCCL (xGMI) as the found flag and rebalances by moving frontier records
    (grouped ncclSend/ncclRecv) -- answer checked against the board's known completion."""
    from distributed_sudoku_solver_amd.shard import RcclComm, sharded_solve
    comm = RcclComm(eng, d.rank, d.world, transport=d.comm) if d.world > 1 else None
    res, ok = {}, True
    # each board twice: at the default frontier (CUs x waves x 8 boards per GPU: these boards are then
    # usually decided inside the frontier build) and split -- a frontier of 4 boards per rank and a
    # 16-node round budget, so the search runs in rounds, refines its heavy boards and (N > 1)
    # rebalances by moving records: the collective path, on a one-board workload
    cases = []
    for name in args.first_boards.split(","):
        cases += [(name, name, {}), (name + "_split", name, {"target": 4 * d.world, "round_budget": 16})]
    try:
        for key, name, kw in cases:
            board, sol, what = first_board(synth, name)
            sharded_solve(eng, board, d.rank, d.world, comm=comm, **kw)      # warm-up
            best = None
            for _ in range(3):
                info = {}
                d.barrier()
                t0 = time.perf_counter()
                out, st = sharded_solve(eng, board, d.rank, d.world, comm=comm, info=info, **kw)
                w = d.max(time.perf_counter() - t0)
                good = st == 1 and bool(np.array_equal(np.asarray(out, np.uint8), sol))
                ok &= good
                if best is None or w < best[0]:
                    best = (w, info, good)
            w, info, good = best
            res[key] = {"board": what, "wall_ms": 1000.0 * w, "ok": good, "rounds": info.get("rounds"),
                        "moved_records": info.get("moved_records"), "refines": info.get("refines"),
                        "steals": info.get("steals"), "frontier_boards": info.get("frontier"),
                        "target": kw.get("target", "default"), "round_budget": kw.get("round_budget", "default")}
    finally:
        if comm is not None:
            comm.close()
    res["workload"] = (f"first (lex-first) completion of one board, its lex frontier split over {d.world} GPU(s)"
                       + (": RCCL all-gather found flag + record moves" if d.world > 1 else ""))
    res["ok"] = ok
    return res


def minimal_leg(eng, d, args, synth, L):
    """Robustness leg beside C4: DISTINCT minimal unique puzzles (random grids, clues removed while
    the completion stays unique, 21-29 clues; csrc/gen_minimal.c), resident in HBM, checked against
    their generating grids, with the search-tail statistics (nodes, max DFS depth) of the same set."""
    n = args.minimal_puzzles
    p, s = synth.make_minimal_sym(n, base=65536, lo=d.rank * 65536, threads=cpu_share())
    el, k_s, bad = solve_leg(eng, d, args, p, s, 3, 1)
    stats = {}
    for kind, name in ((L.SDK_WORK_NODES, "nodes"), (L.SDK_WORK_ROUNDS, "rounds"), (L.SDK_WORK_DEPTH, "depth")):
        eng.set_option(L.SDK_OPT_WORK_COUNTER, kind)
        _, _, w = eng.solve_batch(p, want_work=True)
        stats[name] = {"mean": float(w.mean()), "p50": float(np.percentile(w, 50)),
                       "p99": float(np.percentile(w, 99)), "max": int(w.max())}
    eng.set_option(L.SDK_OPT_WORK_COUNTER, L.SDK_WORK_NODES)
    return {"workload": f"{n} minimal unique puzzles per GPU: 65536 distinct random-grid puzzles "
                        f"({int((p > 0).sum(1).mean())} clues on average) x seeded symmetries",
            "value": d.world * n * 3 / el, "unit": "puzzles/s", "avg_kernel_ms": k_s * 1000.0,
            "search": stats, "parity": {"mismatched_boards": bad, "checked_boards": d.world * n}}


def _warm(args, engines, launch, at_least=1):
    """Untimed passes before a timed region: at least one per engine context, then on, back to back,
    until --warm-ms of load (the GPU's clock ramps over its first ~40 ms of load)."""
    t_w, i = time.perf_counter(), 0
    while i < max(at_least, len(engines)) or (time.perf_counter() - t_w) * 1000.0 < args.warm_ms:
        k = i % len(engines)
        launch(engines[k], k)
        engines[k].synchronize()
        i += 1
    for e in engines:
        e.synchronize()
    return i


def _timed_solves(eng, d, p, s, steps, args, contexts=1):
    """Wall time of `steps` solve_batch_dev passes over resident boards (+ 1 warm-up per context),
    max over ranks; every board of every output buffer checked against its known answer afterwards.
    contexts > 1: consecutive passes on that many engine contexts in turn (own stream and output
    buffers each, engine.fork()), as the headline's passes in flight -- one pass's launch tail (a few
    heavy boards on a nearly idle GPU) overlaps the next pass."""
    n = len(p)
    engines = [eng] + [eng.fork() for _ in range(max(1, contexts) - 1)]
    d_in = eng.alloc(n * 81)
    bufs = [(e.alloc(n * 81), e.alloc(n)) for e in engines]
    d_in.upload(p)
    _warm(args, engines, lambda e, k: e.solve_batch_dev(d_in, bufs[k][0], bufs[k][1], n))
    d.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        k = i % len(engines)
        engines[k].solve_batch_dev(d_in, bufs[k][0], bufs[k][1], n)
    for e in engines:
        e.synchronize()
    d.barrier()
    el = d.max(time.perf_counter() - t0) / steps
    out = np.empty((n, 81), np.uint8)
    st = np.empty(n, np.int8)
    bad = 0
    for d_out, d_st in bufs:
        d_out.download(out)
        d_st.download(st)
        bad += int(((out != s).any(axis=1) | (st != 1)).sum())
    bad = int(d.sum(bad))
    d_in.free()
    for d_out, d_st in bufs:
        d_out.free()
        d_st.free()
    for e in engines[1:]:
        e.close()
    return el, bad


def hard_leg(eng, d, args, synth, L):
    """Puzzles that actually search: the committed hard set
    (distributed_sudoku_solver_amd/data/hard_minimal.npz: 100k distinct minimal unique puzzles that a
    singles-propagating lowest-cell DFS needs >= 20 nodes for; rank r > 0 takes a seeded symmetry of
    each), and its 1000 heaviest -- a batch that is all launch tail.  Each timed one launch per board
    (SDK_OPT_DONATE 0) and with the phased solve (split phase, then the boards over the split budget
    with subtree donation: exhaustive MRV count-to-2, LEX re-solve of multi-solution boards)."""
    p, s, _ = synth.load_hard(threads=cpu_share())
    hp, hs = synth.make_hard_heaviest(1000, threads=cpu_share())
    if d.rank:
        rng = np.random.default_rng([args.seed, d.rank, 5])
        g, rl = synth.random_symmetries(rng, len(p))
        p, s = synth.apply_symmetries(p, g, rl), synth.apply_symmetries(s, g, rl)
        g, rl = synth.random_symmetries(rng, len(hp))
        hp, hs = synth.apply_symmetries(hp, g, rl), synth.apply_symmetries(hs, g, rl)
    # hard_1m: the 100k set x 10 seeded symmetries (a throughput-bound batch that searches,
    # VERDICT r3 item 5); symmetries keep every board's solution count and its search shape
    # (synth.make_hard_sym: the same boards tools/pmc_r04.sh profiles; rank r > 0 a symmetry of each)
    reps = max(1, args.hard_reps)
    mp, ms = synth.make_hard_sym(len(p) * reps, threads=cpu_share())
    if d.rank:
        g, rl = synth.random_symmetries(np.random.default_rng([args.seed, d.rank, 7]), len(mp))
        mp, ms = synth.apply_symmetries(mp, g, rl), synth.apply_symmetries(ms, g, rl)
    res, bad, checked = {}, 0, 0
    old_max = eng.get_option(L.SDK_OPT_DONATE_MAX)
    # modes: LEX order (the reference's branching after propagation) and MRV order counting to two
    # completions (a unique completion is the lex-first one; boards with two are re-searched in
    # LEX), each as one launch and as the phased solve with donation.  Same boards in every mode.
    split_dn = {"heaviest_1000": 16}
    for name, (bp, bs) in (("hard_100k", (p, s)), ("heaviest_1000", (hp, hs)), ("hard_1m", (mp, ms))):
        legs = {}
        for mode, order, dn, ctx in (("one_launch", L.SDK_ORDER_LEX, 0, 1),
                                     ("donation", L.SDK_ORDER_LEX, split_dn.get(name, 1), 1),
                                     ("mrv_one_launch", L.SDK_ORDER_MRV_UNIQUE, 0, 1),
                                     ("mrv_donation", L.SDK_ORDER_MRV_UNIQUE, split_dn.get(name, 1), 1),
                                     ("donation_in_flight", L.SDK_ORDER_LEX,
                                      args.hard_split_inflight or split_dn.get(name, 1),
                                      args.hard_inflight or args.inflight)):
            if ctx < 2 and mode == "donation_in_flight":
                continue
            eng.set_option(L.SDK_OPT_ORDER, order)
            eng.set_option(L.SDK_OPT_DONATE, dn)
            eng.set_option(L.SDK_OPT_DONATE_MAX, 0)       # phased at any size (hard_1m is above the default)
            el, b = _timed_solves(eng, d, bp, bs, 6 if ctx > 1 else 5, args, contexts=ctx)
            bad += b
            checked += d.world * len(bp) * ctx
            legs[mode] = {"value": d.world * len(bp) / el, "unit": "puzzles/s", "ms": el * 1000.0, "contexts": ctx,
                          "order": "lex" if order == L.SDK_ORDER_LEX else "mrv_unique",
                          "split_budget": dn if dn > 1 else ((256 if len(bp) > (1 << 19) else 128) if dn else None),
                          "split_boards": eng.get_option(L.SDK_OPT_SPLIT_BOARDS),
                          "lex_boards": eng.get_option(L.SDK_OPT_LEX_BOARDS),
                          "donated": eng.get_option(L.SDK_OPT_DONATED)}
        eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if args.order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
        eng.set_option(L.SDK_OPT_DONATE, 1)
        eng.set_option(L.SDK_OPT_DONATE_MAX, old_max)
        base = legs["one_launch"]["value"]
        legs["donation_speedup"] = legs["donation"]["value"] / base
        best = max((m for m in ("donation", "mrv_one_launch", "mrv_donation", "donation_in_flight") if m in legs),
                   key=lambda m: legs[m]["value"])
        legs["best"] = {"mode": best, "speedup_vs_lex_one_launch": legs[best]["value"] / base}
        res[name] = legs
    res["hard_1m"]["workload"] = f"the {len(p)} hard puzzles x {reps} seeded symmetries ({len(mp)} boards) per GPU"
    res["hard_1m"]["roofline"] = pipe_record(args.pmc_pipe, "hard1m", len(mp))
    stats = {}
    eng.set_option(L.SDK_OPT_DONATE, 0)     # per-board work of one slot per board
    for kind, nm in ((L.SDK_WORK_NODES, "nodes"), (L.SDK_WORK_ROUNDS, "rounds"), (L.SDK_WORK_DEPTH, "depth")):
        eng.set_option(L.SDK_OPT_WORK_COUNTER, kind)
        _, _, w = eng.solve_batch(p, want_work=True)
        stats[nm] = {"mean": float(w.mean()), "p50": float(np.percentile(w, 50)), "p99": float(np.percentile(w, 99)),
                     "p99.9": float(np.percentile(w, 99.9)), "max": int(w.max())}
    eng.set_option(L.SDK_OPT_WORK_COUNTER, L.SDK_WORK_NODES)
    eng.set_option(L.SDK_OPT_DONATE, 1)
    res["workload"] = (f"{len(p)} distinct hard puzzles per GPU ({int((p > 0).sum(1).mean())} clues on average, "
                       f"committed set) and their 1000 heaviest, resident in HBM")
    res["search"] = stats
    res["parity"] = {"mismatched_boards": bad, "checked_boards": checked}   # every mode, every output buffer
    if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0:
        res["cpu_baseline_c_port"] = cpu_baseline_c(p, min(args.cpu_seconds, 5.0), cpu_share())
    return res


def lane_dfs_leg(eng, args, synth, L):
    """North-star part (3) beside the propagating solvers: the reference's own naive DFS, ONE
    BOARD PER LANE with its stack in LDS (SDK_SOLVER_LANE, csrc/solve_lane_kernel.h), on a
    prefix of the C2 30-clue stream.  Its work counter is the reference's `validations`, so
    the leg reports validations/s of the same algorithm on the GPU and on the host cores (the
    oracle's C port), and checks the counts against the port on a sample."""
    from oracle import oracle as O
    n = args.lane_puzzles
    p, sol = synth.make_30clue(n, seed=args.seed + 31)
    budget = 50_000_000
    eng.set_option(L.SDK_OPT_SOLVER, L.SDK_SOLVER_LANE)
    eng.set_option(L.SDK_OPT_NODE_BUDGET, budget)
    try:
        eng.solve_batch(p[:4096])
        eng.synchronize()
        t0 = time.perf_counter()
        out, st, val = eng.solve_batch(p, want_work=True)
        wall = time.perf_counter() - t0
    finally:
        eng.set_option(L.SDK_OPT_NODE_BUDGET, 0)
        eng.set_option(L.SDK_OPT_SOLVER, SOLVERS[args.solver][0])
    if args.prop32 >= 0:
        eng.set_option(L.SDK_OPT_PROP32, args.prop32)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        eng.set_option(getattr(L, "SDK_OPT_" + k), int(v))
    # the same batch with the per-puzzle budget cut to 20k validations: the wave-parallel bulk
    # rate without the serial tail of the few boards that need a million validations
    eng.set_option(L.SDK_OPT_SOLVER, L.SDK_SOLVER_LANE)
    eng.set_option(L.SDK_OPT_NODE_BUDGET, 20_000)
    try:
        t0 = time.perf_counter()
        _, bst, bval = eng.solve_batch(p, want_work=True)
        bwall = time.perf_counter() - t0
    finally:
        eng.set_option(L.SDK_OPT_NODE_BUDGET, 0)
        eng.set_option(L.SDK_OPT_SOLVER, SOLVERS[args.solver][0])
    if args.prop32 >= 0:
        eng.set_option(L.SDK_OPT_PROP32, args.prop32)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        eng.set_option(getattr(L, "SDK_OPT_" + k), int(v))
    m = min(n, 4096)
    cores = args.cpu_cores or cpu_share()
    t1 = time.perf_counter()
    ref_out, ref_st, ref_val = O.naive_solve_batch(p[:m], budget=budget, threads=cores)
    cwall = time.perf_counter() - t1
    ok = st == 1
    return {"workload": f"{n} C2 ~30-clue puzzles, one board per lane: the reference's naive DFS "
                        "(lowest empty cell, digits ascending), LDS-resident digit stack, host-pointer call",
            "value": n / wall, "unit": "puzzles/s", "validations_per_s": float(val.sum()) / wall,
            "validations_per_puzzle": {"mean": float(val.mean()), "p99": float(np.percentile(val, 99)),
                                       "max": int(val.max())},
            "budget_hits": int((st == -2).sum()),
            "bulk_20k_budget": {"solved_per_s": float((bst == 1).sum()) / bwall,
                                "validations_per_s": float(bval.sum()) / bwall,
                                "stopped_at_budget": int((bst == -2).sum()), "wall_ms": 1000.0 * bwall},
            "parity": {"mismatched_boards": int(((out != sol).any(axis=1) & ok).sum() + (~ok & (st != -2)).sum()),
                       "checked_boards": n,
                       "validations_vs_c_port": {"sample": m, "equal": int((val[:m] == ref_val).sum()),
                                                 "status_equal": int((st[:m] == ref_st).sum())}},
            "c_port_same_dfs": {"validations_per_s": float(ref_val.sum()) / cwall, "cores": cores,
                                "puzzles_per_s": m / cwall, "sample": m}}


def http_leg(requests, api="dht"):
    """Config C1: one puzzle POSTed to a single node's /solve (wiki 30-clue puzzle), end to end
    over loopback HTTP, on a GPU-backed node (distributed_sudoku_solver_amd.node) serving
    DHT_Node.py's HTTP surface (api="dht") or main.py's (api="main", main.py:356-375)."""
    import urllib.request
    from distributed_sudoku_solver_amd import synth
    from distributed_sudoku_solver_amd.engine import SudokuEngine
    from distributed_sudoku_solver_amd.node import SudokuNode
    eng = SudokuEngine(0)
    node = SudokuNode("127.0.0.1", 0, 0, engine=eng, delay_ms=0, api=api).start()
    grid = [[int(c) for c in synth.WIKI[9 * r: 9 * r + 9]] for r in range(9)]
    body = json.dumps({"sudoku": grid}).encode()
    lat, ok = [], True
    try:
        for _ in range(requests + 2):
            req = urllib.request.Request(f"http://127.0.0.1:{node.http_port}/solve", data=body, method="POST")
            t0 = time.perf_counter()
            with urllib.request.urlopen(req, timeout=60) as r:
                out = json.loads(r.read())
            lat.append(time.perf_counter() - t0)
            ok &= "".join(str(v) for row in out["solution"] for v in row) == synth.WIKI_SOLUTION
    finally:
        node.stop(graceful=False)
        eng.close()
    lat = sorted(lat[2:])
    ref = "DHT_Node.py" if api == "dht" else "main.py"
    return {"workload": f"C1: wiki 30-clue puzzle POSTed to /solve on one node, {ref} HTTP surface (loopback)",
            "median_ms": 1000 * lat[len(lat) // 2], "min_ms": 1000 * lat[0], "requests": len(lat),
            "solution_ok": bool(ok), "reference_ms": REFERENCE_MEASURED["post_solve_ms"][api],
            "reference_note": f"{ref} single node, -d 0, measured in the build container (SURVEY §3.1)"}


def _checker_last(result, leg):
    """The C3 checker leg goes at the END of the line (the driver keeps only
    the tail of stdout), with its headline figures first in a compact summary."""
    # the headline kernel's rooflines first, compact (visible in the driver's tail)
    rf = result.get("roofline") or {}
    v = rf.get("valu") or {}
    if rf:
        result.pop("roofline_summary", None)
        result["roofline_summary"] = {
            "kernel": rf.get("kernel"), "avg_kernel_ms": rf.get("avg_kernel_ms"), "hbm_frac": rf.get("frac"),
            "valu_frac": v.get("frac"), "valu_per_quad": v.get("valu_per_quad"),
            "mix_ceiling_frac": (v.get("mix_ceiling") or {}).get("frac"), "clock_ghz": v.get("clock_ghz"),
            "clock_measured_live": bool(v.get("clock")),
            "valu_frac_at_2p4ghz": (v.get("at_2p4ghz_cap") or {}).get("frac")}
    if leg is None:
        return
    result.pop("checker", None)
    result.pop("checker_summary", None)
    result["checker"] = leg
    rf = leg["roofline"]
    result["checker_summary"] = {"metric": "checker HBM GB/s (C3, 82 algorithmic B per board)",
                                 "boards_per_s": leg["value"], "avg_kernel_ms": leg["avg_kernel_ms"],
                                 "achieved_gbps": rf["achieved"], "peak_gbps": rf["peak"], "frac": rf["frac"],
                                 "mismatched_boards": leg["parity"]["mismatched_boards"],
                                 "checked_boards": leg["parity"]["checked_boards"]}


def launch_ranks(args):
    """`--gpus N` without torchrun: start N rank processes of this script (one per GPU) with
    the torchrun environment, before this process touches any GPU; rank 0 prints the line."""
    import socket
    import subprocess
    ports = []
    socks = [socket.socket() for _ in range(2)]
    try:
        for sk in socks:
            sk.bind(("127.0.0.1", 0))
            ports.append(sk.getsockname()[1])
    finally:
        for sk in socks:
            sk.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(ports[0]),
                   SDK_RDZV_PORT=str(ports[1]))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    codes = [p.wait() for p in procs]
    return max(codes, key=abs)


def timer_spans(e):
    """The context's timed spans since timer_reset, ms each (sdk_debug_timer_list; an engine without
    the library -- the CPU tests' stub -- reports its total as equal spans)."""
    if not hasattr(e, "lib"):
        ms, nl = e.timer_read()
        return [ms / max(nl, 1)] * nl
    cap = 1 << 16
    arr = (ctypes.c_double * cap)()
    cnt = ctypes.c_int64()
    if e.lib.sdk_debug_timer_list(e.ctx, arr, ctypes.c_int64(cap), ctypes.byref(cnt)) != 0:
        raise RuntimeError("sdk_debug_timer_list failed")
    return list(arr[:min(cnt.value, cap)])


def kernel_clock(e, d_in, d_out, d_st, n, launches=20):
    """In-kernel shader clock of the prop32 pass, measured live: `launches` more back-to-back passes
    over the same resident boards with the diagnostic twin of the kernel (prop32_clock_kernel:
    s_memtime / s_memrealtime stamped at each workgroup's entry and exit, nothing else changed;
    MI355X_MICROARCH.md "DVFS give-back" item 6); the last pass's workgroups give the median
    clock.  None for an engine without the diagnostic (the CPU tests' stub)."""
    from distributed_sudoku_solver_amd import _lib as L
    lib = getattr(e, "lib", None)
    if lib is None or not hasattr(lib, "sdk_debug_clock_arm"):
        return None
    L.check(lib.sdk_debug_clock_arm(e.ctx, 1), "sdk_debug_clock_arm")
    try:
        for _ in range(launches):
            e.solve_batch_dev(d_in, d_out, d_st, n)
        e.synchronize()
        out4 = (ctypes.c_double * 4)()
        wgs = ctypes.c_int64()
        L.check(lib.sdk_debug_clock_read(e.ctx, out4, ctypes.byref(wgs)), "sdk_debug_clock_read")
    finally:
        lib.sdk_debug_clock_arm(e.ctx, 0)
    if wgs.value == 0:
        return None
    return {"ghz": out4[0], "ghz_p10": out4[1], "ghz_p90": out4[2], "ghz_mean": out4[3], "workgroups": wgs.value,
            "launches": launches,
            "source": "s_memtime / s_memrealtime per workgroup of the last of these back-to-back passes "
                      "(prop32_clock_kernel, the stamped twin of the timed kernel), median"}


def solve_leg(eng, d, args, puzzles, expected, steps, warmup, contexts=1, timed=True, clock=False):
    """Time `steps` sdk_solve_batch_dev passes over this rank's resident slice (barrier +
    device sync on both sides, max over ranks); verify every board afterwards.  Each rank's clock
    runs from the release of the opening barrier to its own device sync at the end, and the job's
    time is the maximum over ranks: the closing barrier's host round trip (a TCP exchange, ~0.1 ms,
    several % of a 1.25M-board shard's step at 8 GPUs) is not the workload's.

    With `contexts` > 1 the passes are issued on that many engine contexts in turn
    (engine.fork(): each its own HIP stream, dequeue state, DFS stacks and output buffer), so that
    one pass's launch drain -- the last chunks finishing while most of the GPU idles, ~0.3 ms at
    every batch size -- overlaps the next pass's start: batches in flight, as a serving node keeps
    them.  Every pass solves the whole slice; every output buffer is checked.  (The headline's
    `value` uses three contexts; its `single_stream` figure, one context, supplies the per-launch
    HIP events -- the kernel's own duration, the roofline's denominator: overlapped launches'
    events would also hold their wait for the GPU.)"""
    from distributed_sudoku_solver_amd import _lib as L
    n = len(puzzles)
    nctx = max(1, min(int(contexts), max(1, steps)))
    engines = [eng] + [eng.fork() for _ in range(nctx - 1)]
    d_in = eng.alloc(max(n, 1) * 81)
    outs = [(e.alloc(max(n, 1) * 81), e.alloc(max(n, 1))) for e in engines]
    d_in.upload(puzzles)
    # untimed: W passes, and on until the GPU has run passes back to back for --warm-ms (its clock
    # ramps from ~1.9 to ~2.35 GHz over the first ~40 ms of load, profiles/r06/clock_ramp_r06i.jsonl)
    t_w, i = time.perf_counter(), 0
    while i < max(warmup, nctx) or (time.perf_counter() - t_w) * 1000.0 < args.warm_ms:
        o, st = outs[i % nctx]
        engines[i % nctx].solve_batch_dev(d_in, o, st, n)
        if i >= max(warmup, nctx) - 1:
            engines[i % nctx].synchronize()       # paces the time-based part
        i += 1
    solve_leg.warm_passes = i
    for e in engines:
        e.synchronize()
        if timed:          # per-launch HIP events (the roofline's kernel time); off: wall clock only
            e.timer_reset()
    d.barrier()
    for e in engines:
        e.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        o, st = outs[i % nctx]
        engines[i % nctx].solve_batch_dev(d_in, o, st, n)
    for e in engines:
        e.synchronize()
    elapsed = time.perf_counter() - t0
    d.barrier()
    kernel_ms, launches = 0.0, 0
    fallback = []
    for e in engines:
        if timed:
            spans = timer_spans(e)
            e.timer_stop()
            if len(spans) == 2 * steps and e.get_option(L.SDK_OPT_PROP32):
                # a prop32 solve is two spans: the propagation pass (the roofline's kernel) and its
                # fallback (search of the undecided boards + scatter)
                fallback += spans[1::2]
                spans = spans[0::2]
            kernel_ms += sum(spans)
            launches += len(spans)
    # the clock the timed passes ran at: more passes of the same kind straight after them (events off)
    solve_leg.clock = kernel_clock(eng, d_in, outs[0][0], outs[0][1], n) if clock else None
    elapsed_max = d.max(elapsed)
    bad = 0
    out = np.empty((n, 81), np.uint8)
    st_h = np.empty(n, np.int8)
    for o, st in outs:
        o.download(out)
        st.download(st_h)
        bad += int(((out != expected).any(axis=1) | (st_h != 1)).sum())
    bad_total = int(d.sum(bad))
    d_in.free()
    for o, st in outs:
        o.free()
        st.free()
    for e in engines[1:]:
        e.close()
    avg_kernel_s = kernel_ms / 1000.0 / max(launches, 1)
    solve_leg.fallback_ms = sum(fallback) / len(fallback) if fallback else None
    return elapsed_max, avg_kernel_s, bad_total


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    d = Dist()
    if d.rank == 0 and d.world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={d.world}; reporting n_gpus={d.world}", file=sys.stderr)
    from distributed_sudoku_solver_amd import SudokuEngine, synth, _lib as L
    from distributed_sudoku_solver_amd.shard import shard_bounds

    if args.engine_factory:      # CPU tests of the rank / shard logic (tests/test_bench_cpu.py)
        import importlib
        mod, fn = args.engine_factory.split(":")
        eng = getattr(importlib.import_module(mod), fn)(d.local_rank)
    else:
        # one GPU per rank; more ranks than GPUs (a 1-GPU rehearsal of the rank path) share them
        ndev = ctypes.c_int(0)
        L.check(L.load().sdk_device_count(ctypes.byref(ndev)), "sdk_device_count")
        eng = SudokuEngine(d.local_rank % max(1, ndev.value))
        args.shared_gpus = d.world > ndev.value
    eng.set_option(L.SDK_OPT_ORDER, L.SDK_ORDER_LEX if args.order == "lex" else L.SDK_ORDER_MRV_UNIQUE)
    eng.set_option(L.SDK_OPT_SOLVER, SOLVERS[args.solver][0])
    if args.prop32 >= 0:
        eng.set_option(L.SDK_OPT_PROP32, args.prop32)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        eng.set_option(getattr(L, "SDK_OPT_" + k), int(v))
    if args.waves_per_cu:
        eng.set_option(SOLVERS[args.solver][2], args.waves_per_cu)
    solve_kernel = SOLVERS[args.solver][1]
    if args.solver == "quad" and eng.get_option(L.SDK_OPT_PROP32):
        # the QUAD solve's first pass, which decides every C4 board (prop32_kernel.h)
        solve_kernel = "sdk::prop32_kernel"
    args.solve_kernel = solve_kernel

    # -------------------------------------------------------------- checker
    # Runs before the solver leg, on a fresh allocation: measured after the solver leg the same
    # kernel read ~9% slower on the same box (profiles/r01/check_variants.txt).
    checker_leg = None
    if args.check_boards > 0:
        nb = args.check_boards
        pool_n = min(nb, 1 << 20)
        pool, pool_exp = synth.make_check_boards(pool_n, seed=args.seed + 7, lo=d.rank * pool_n)
        d_b = eng.alloc(nb * 81)
        d_v = eng.alloc(nb)
        # tile the pool through HBM (content repeats; every byte is still streamed from HBM)
        for s in range(0, nb, pool_n):
            d_b.upload(pool[:min(pool_n, nb - s)], offset=s * 81)
        t_w, cw = time.perf_counter(), 0
        while cw < max(1, args.check_warmup) or (time.perf_counter() - t_w) * 1000.0 < args.warm_ms:
            eng.check_batch_dev(d_b, d_v, nb)
            if cw >= max(1, args.check_warmup) - 1:
                eng.synchronize()
            cw += 1
        eng.synchronize()
        eng.timer_reset()
        d.barrier()
        eng.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.check_steps):
            eng.check_batch_dev(d_b, d_v, nb)
        eng.synchronize()
        cel = time.perf_counter() - t0       # the rank's own clock, as in solve_leg
        d.barrier()
        cel = d.max(cel)
        cms, cl = eng.timer_read()
        eng.timer_stop()
        v = np.empty(nb, np.uint8)
        d_v.download(v)
        reps = (nb + pool_n - 1) // pool_n
        exp = np.tile(pool_exp, reps)[:nb]
        cbad = int(d.sum(int((v != exp).sum())))
        d_b.free()
        d_v.free()
        ck_s = cms / 1000.0 / max(cl, 1)
        ach = CHECK_BYTES_PER_BOARD * nb / ck_s / 1e9
        crec = pmc_record(args.pmc_summary, "sdk::check_kernel", nb)
        checker_leg = {
            "workload": f"C3: {nb} complete boards per GPU (50% valid), literal sudoku.py:43-94 rule",
            "value": d.world * nb * args.check_steps / cel,
            "unit": "boards/s",
            "avg_kernel_ms": ck_s * 1000.0,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBPS,
                         "traffic": crec["traffic_bytes"] if crec else None,
                         "traffic_note": crec.get("traffic_note") if crec else None,
                         "kernel": "sdk::check_kernel"},
            "parity": {"mismatched_boards": cbad, "checked_boards": d.world * nb},
            "warm_launches": cw,
        }
        if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0:
            checker_leg["cpu_baseline"] = cpu_baseline_check(pool[:1_000_000], min(5.0, args.cpu_seconds),
                                                             args.cpu_cores or cpu_share())

    # ------------------------------------------------- C4 solve (headline)
    total = args.batch
    lo, hi = shard_bounds(total, d.rank, d.world)
    gen = synth.make_17clue if args.workload == "solve17" else synth.make_30clue
    puzzles, expected = gen(hi - lo, seed=args.seed, lo=lo)
    n = hi - lo
    # one context first: its per-launch HIP events are the kernel's own duration (the roofline's
    # denominator); then the headline with `inflight` passes in flight (every pass solves the whole
    # slice, every output buffer is checked)
    s_el, avg_kernel_s, bad_total = solve_leg(eng, d, args, puzzles, expected, args.steps, args.warmup,
                                              clock=args.solver == "quad" and "prop32" in solve_kernel)
    single_stream = {"value": total * args.steps / s_el, "unit": "puzzles/s", "ms_per_step": s_el / args.steps * 1e3,
                     "avg_kernel_ms": avg_kernel_s * 1e3, "contexts": 1,
                     "avg_fallback_ms": solve_leg.fallback_ms, "clock": solve_leg.clock,
                     "warm_passes": solve_leg.warm_passes,
                     "parity": {"mismatched_boards": bad_total, "checked_boards": total}}
    inflight = max(1, args.inflight)
    if inflight > 1:
        elapsed_max, _, bad_if = solve_leg(eng, d, args, puzzles, expected, args.steps, args.warmup,
                                           contexts=inflight, timed=False)
        bad_total += bad_if
    else:
        elapsed_max = s_el

    value = total * args.steps / elapsed_max
    achieved = SOLVE_BYTES_PER_PUZZLE * n / avg_kernel_s / 1e9
    srec = pmc_record(args.pmc_summary, solve_kernel, n)
    roofline = {
        "bound": "hbm",
        "achieved": achieved,
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBPS,
        "traffic": srec["traffic_bytes"] if srec else None,
        "traffic_note": srec.get("traffic_note") if srec else None,
        "traffic_source": (os.path.relpath(args.pmc_summary, ROOT) if srec else None),
        # the counters themselves beside the calibrated figure: the raw write is ~1.37x the 82 B
        # per puzzle because each 81-B record is written on its own (solver traffic)
        "traffic_raw": srec.get("traffic_raw") if srec else None,
        "kernel": solve_kernel,
        "avg_kernel_ms": avg_kernel_s * 1000.0,
        "note": "the kernel is bound by its LDS pipe (roofline.valu.pipe.lds_busy_frac, the stall counters in "
                "roofline.valu.stalls; VALU issue against the 2-per-quad-cycle peak and the ceiling of the "
                "kernel's own instruction mix in roofline.valu); HBM fraction reported per contract (163 "
                "algorithmic B per puzzle)",
    }
    prec = pipe_record(args.pmc_pipe, "c4", n) if args.workload == "solve17" else None
    clk = single_stream.get("clock")
    if prec and prec.get("valu_insts"):
        # VALU wave-instructions per launch from a PMC pass of this exact launch (tools/pmc_r04.sh,
        # tools/pmc_pipe_summary.py; an instruction count does not depend on the clock) over the
        # timed kernel's duration, priced at the issue peak of 2 wave64 VALU per SIMD quad-cycle AT
        # THE CLOCK THE TIMED PASSES RAN AT (measured live in this run, kernel_clock; the profiled
        # run's clock is lower and would overstate every fraction), and beside it
        # at the 2.4 GHz cap.  Next to the peak: the ceiling this kernel's own instruction mix reaches
        # on this GPU (tools/issue_calib.hip under rocprofv3: legacy 3-source VOP3 ops -- v_or3,
        # v_and_or -- and packed VOP3P ops do not dual-issue and top out near one per quad-cycle;
        # v_bitop3 and 2-operand ops dual-issue, ~1.7 per quad-cycle with every SIMD full)
        rate = prec["valu_insts"] / avg_kernel_s
        mix = mix_ceiling(args.issue_calib)
        # the kernel's own mix: prop32's step is v_bitop3 / 2-operand ops throughout since round 6
        # (solve_kernel.h SDK_OR3) -- tools/issue_calib.hip k_b3; solve4's round is k_mix
        p32 = "prop32" in solve_kernel
        mix_key = "k_b3@8" if p32 else "k_mix@8"
        mix_q = (mix or {}).get(mix_key, {}).get("valu_per_quad")

        def priced(ghz):
            quads_per_s = 256 * 4 * ghz * 1e9 / 4
            peak = quads_per_s * VALU_PER_SIMD_QUAD
            return {"clock_ghz": ghz, "peak": peak, "frac": rate / peak, "valu_per_quad": rate / quads_per_s,
                    "mix_ceiling_frac": rate / (mix_q * quads_per_s) if mix_q else None}
        at = priced(clk["ghz"]) if clk else priced(2.4)
        cap = priced(2.4)
        roofline["valu"] = {
            "bound": "valu-issue", "achieved": rate, "unit": "wave-instr/s", "peak": at["peak"],
            "clock_ghz": at["clock_ghz"],
            "clock_source": (clk["source"] if clk else "no live clock: the 2.4 GHz cap (fractions are then lower bounds)"),
            "clock": clk,
            "peak_note": "2 wave64 VALU per SIMD quad-cycle (one per 2 cycles on a SIMD-32, MI355X_MICROARCH.md:54) "
                         "x 1024 SIMDs at clock_ghz",
            "frac": at["frac"],
            "valu_per_quad": at["valu_per_quad"],
            "at_2p4ghz_cap": cap,
            "mix_ceiling": ({"valu_per_quad": mix_q, "wave_instr_per_s": mix_q * 256 * at["clock_ghz"] * 1e9,
                             "frac": at["mix_ceiling_frac"], "calibration_kernel": mix_key,
                             "note": ("tools/issue_calib.hip k_b3 (independent v_bitop3_b32 chains, every SIMD "
                                      "full): prop32's step is v_bitop3 and 2-operand ops throughout; they dual-"
                                      "issue in ~79 % of quad-cycles (v_or3_b32 chains: 7 %, ~0.98 per quad-cycle, "
                                      "k_or3@8 in the same calibration)" if p32 else
                                      "tools/issue_calib.hip k_mix at 8 waves/SIMD: the exact round's VALU "
                                      "(unit4x + 3 upd4x) on registers; VOP3 3-source and VOP3P packed ops "
                                      "dual-issue in ~7 % of quad-cycles (2-operand VOP2 ops: 78 %)"),
                             "calibration": mix, "source": os.path.relpath(args.issue_calib, ROOT)}
                            if mix_q else None),
            "profiled_clock_ghz": prec.get("clock_ghz"),
            "issue_busy_frac": prec["valu_busy_frac"],
            "issue_busy_note": "SIMD quad-cycles with any VALU issue in the profiled run: (SQ_INSTS_VALU - "
                               "SQ_ACTIVE_INST_VALU2) / quad-cycles; dual issue in valu_dual_frac of them",
            "valu_insts_per_puzzle": prec["valu_insts"] / n,
            "lds_insts_per_puzzle": (prec.get("lds_insts") or 0) / n,
            "salu_insts_per_puzzle": (prec.get("salu_insts") or 0) / n,
            "pipe": prec,
            "stalls": srec.get("stalls") if srec else None,
        }
    elif srec and srec.get("valu_insts"):
        # older PMC record (no per-SIMD counters): VALU wave-instructions per launch over the issue
        # peak of 2 per SIMD quad-cycle at 2.4 GHz
        peak = VALU_PEAK_WAVE_INSTR_PER_S
        rate = srec["valu_insts"] / avg_kernel_s
        roofline["valu"] = {
            "bound": "valu-issue", "achieved": rate, "peak": peak, "unit": "wave-instr/s", "frac": rate / peak,
            "valu_insts_per_puzzle": srec["valu_insts"] / n,
            "lds_insts_per_puzzle": srec.get("lds_insts", 0) / n,
            "stalls": srec.get("stalls"),
            "source": os.path.relpath(args.pmc_summary, ROOT),
        }
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "puzzles/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1000.0,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": ("C4: 17-clue hard puzzles (seeds S1-S5 x seeded Sudoku symmetries), "
                         if args.workload == "solve17" else
                         "C2: ~30-clue unique puzzles (17 seed givens + 13 solution cells, symmetries), ")
                        + f"{total} puzzles sharded over {d.world} GPU(s), resident in HBM",
            "puzzles_total": total,
            "puzzles_per_gpu": n,
            "order": args.order,
            "solver": args.solver,
            "parallelism": f"batch-shard x{d.world} (contiguous slices, no collectives)",
            "passes_in_flight_per_gpu": inflight,
            "warmup_policy": (f"W = {args.warmup} untimed passes, continued back to back until {args.warm_ms:g} ms "
                              "of load before each timed region (the clock ramps from ~1.9 to ~2.35 GHz over "
                              "the first ~40 ms; profiles/r06/clock_ramp_r06i.jsonl); exactly `steps` passes "
                              "timed"),
        },
        "single_stream": single_stream,
        "roofline": roofline,
        "parity": {"mismatched_boards": bad_total, "checked_boards": total * (1 + inflight if inflight > 1 else 1)},
    }

    # side legs run under a watchdog: if one stalls (e.g. a collective), rank 0
    # still prints the line with everything measured so far
    import threading

    def _watchdog():
        if d.rank == 0:
            result["watchdog"] = f"side legs stopped after {args.leg_timeout} s"
            _checker_last(result, checker_leg)
            print(json.dumps(result), flush=True)
        os._exit(3 if bad_total else 0)
    dog = threading.Timer(args.leg_timeout, _watchdog)
    dog.daemon = True
    dog.start()

    def side(name, fn):
        # a side leg that raises (e.g. a collective refused on some node) is recorded, not fatal:
        # the headline line above is measured and still printed
        try:
            result[name] = fn()
        except Exception as e:  # noqa: BLE001
            result[name] = {"error": f"{type(e).__name__}: {e}"}
        return result[name]

    # ------------------------------------------------ weak-scaling figure
    if d.world > 1 and args.weak_leg:
        wp, we = gen(total, seed=args.seed, lo=d.rank * total)
        w_el, w_k, w_bad = solve_leg(eng, d, args, wp, we, args.steps, 1, contexts=inflight, timed=inflight == 1)
        del wp, we
        result["weak_scaling"] = {
            "workload": f"C4 with {total} puzzles PER GPU (rows [rank*{total}, (rank+1)*{total}) of the same stream)",
            "value": d.world * total * args.steps / w_el, "unit": "puzzles/s",
            "ms_per_step": w_el / args.steps * 1000.0, "avg_kernel_ms": w_k * 1000.0,
            "parity": {"mismatched_boards": w_bad, "checked_boards": d.world * total}}
        bad_total += w_bad

    # ------------------------------------------------------------ C2 leg
    if args.c2_puzzles > 0:
        side("c2_30clue", lambda: c2_leg(eng, d, args, synth))

    # ------------------------------------------------ distinct minimal puzzles
    if args.minimal_puzzles > 0:
        leg = side("minimal_puzzles", lambda: minimal_leg(eng, d, args, synth, L))
        bad_total += leg.get("parity", {}).get("mismatched_boards", 0)

    # ------------------------------------------------ puzzles that search
    if args.hard_leg:
        leg = side("hard_search", lambda: hard_leg(eng, d, args, synth, L))
        bad_total += leg.get("parity", {}).get("mismatched_boards", 0)

    # ------------------------------------------------------------ C5 leg
    if args.count_leg and getattr(args, "shared_gpus", False):
        # RCCL refuses two ranks on one device ("invalid usage"): a rehearsal with more ranks than
        # GPUs has no C5 leg (on a node every rank has its own GPU)
        result["c5_count"] = {"skipped": "more ranks than GPUs: RCCL needs one device per rank"}
    elif args.count_leg:
        side("c5_count", lambda: c5_leg(eng, d, args, synth))
        side("c5_count_rebalanced", lambda: c5_rebalanced_leg(eng, d, args, synth))

    # ------------------------------------- one hard search split over the GPUs
    if args.first_boards and getattr(args, "shared_gpus", False):
        result["first_solution"] = {"skipped": "more ranks than GPUs: RCCL needs one device per rank"}
    elif args.first_boards:
        leg = side("first_solution", lambda: first_solution_leg(eng, d, args, synth))
        bad_total += 1 if leg.get("ok") is False else 0       # a wrong answer fails the run

    # ---------------------------------------------------------- CPU baseline
    if d.rank == 0 and d.world == 1 and args.cpu_seconds > 0:
        cores = args.cpu_cores or cpu_share()
        # fixed C4 sample: the first 8 puzzles of every core's slice are the same on every run
        result["cpu_baseline"] = cpu_baseline_python(puzzles[:cores * 64], args.cpu_seconds, cores,
                                                     args.cpu_puzzle_budget, "C4 17-clue sample")
        result["cpu_baseline"]["reference_measured"] = REFERENCE_MEASURED["solve_17clue"]
        # the same DFS in C, uncapped (every attempted puzzle solved), on the same stream
        result["cpu_baseline"]["c_port"] = cpu_baseline_c(puzzles, args.cpu_seconds, cores)
        hs = result.get("hard_search", {}).get("cpu_baseline_c_port")
        if hs:     # the hard set's C-port rate, beside the GPU's hard_search figures
            result["cpu_baseline"]["hard_set_c_port"] = {k: hs[k] for k in ("value", "unit", "cores", "attempted",
                                                                             "solved", "capped") if k in hs}

    if d.rank == 0 and d.world == 1 and args.http_requests > 0:
        side("post_solve_latency", lambda: http_leg(args.http_requests))
        side("post_solve_latency_main", lambda: http_leg(args.http_requests, api="main"))

    # -------------------------------------------- per-lane reference DFS (north star part 3)
    if d.rank == 0 and d.world == 1 and args.lane_puzzles > 0:
        leg = side("lane_dfs", lambda: lane_dfs_leg(eng, args, synth, L))
        bad_total += leg.get("parity", {}).get("mismatched_boards", 0)

    dog.cancel()
    eng.close()
    _checker_last(result, checker_leg)
    if d.rank == 0:
        print(json.dumps(result), flush=True)
    d.close()
    if bad_total or result.get("checker", {}).get("parity", {}).get("mismatched_boards", 0):
        sys.exit(3)


if __name__ == "__main__":
    main()
