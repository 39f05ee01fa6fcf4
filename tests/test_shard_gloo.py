"""N>1 batch-sharding path on CPU: world_size-2 gloo processes, each with a stand-in
engine (the oracle plays the GPU here; the product path is the same host code)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_sudoku_solver_amd.shard import (HostComm, MultiDeviceEngine, ShardedBatch, rebalance_ranges,
                                                 shard_bounds, sharded_count, sharded_count_rebalanced, sharded_solve)
from distributed_sudoku_solver_amd import synth, _lib as L

from doubles import OracleEngine


S4_SOLUTION = "679835412123694758548217936416723895892561374735489621287956143961342587354178269"


def O_range_mask(lo, hi):
    from oracle import oracle as O
    return O.range_mask(lo, hi)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, s = synth.make_30clue(301, seed=5)            # odd size: ragged shards
        b, exp = synth.make_check_boards(1001, seed=6)
        eng = OracleEngine()
        sb = ShardedBatch(eng, rank, world)
        out, st = sb.solve(p)
        v = sb.check(b)
        if rank == 0:
            q.put(("solve", bool((out == s).all() and (st == 1).all())))
            q.put(("check", bool((v == exp).all())))
        comm = HostComm(rank, world)
        s1 = synth.SEEDS17["S1"]
        q.put(("calls", rank, list(eng.calls)))
        eng.calls = []
        # two-stage split (default): shares of a small replicated frontier, refined per rank
        total, st, size = sharded_count(eng, synth.parse(s1[:-9] + "000800000"), rank, world, comm=comm)
        ref = [c for c in eng.calls if c[0] == "refine"]
        q.put(("count_refine", rank, ref[0][1:] if ref else None, total == 7309 and st == 1))
        # single stage: interleaved boards of one replicated frontier
        eng.calls = []
        total, st, size = sharded_count(eng, synth.parse(s1[:-9] + "000800000"), rank, world, comm=comm,
                                        refine=False)
        counted = [c[1] for c in eng.calls if c[0] == "count"][0]
        if rank == 0:
            q.put(("count", total == 7309 and st == 1 and size >= 32))
        q.put(("count_split", rank, counted, size))
        # rebalanced count: rank 0 starts with the whole frontier, rank 1 must steal over gloo
        eng.calls = []
        info = {}
        b16 = synth.parse(s1[:-9] + "000800000")
        total, st, size = sharded_count_rebalanced(eng, b16, rank, world, comm=comm, chunk=2, info=info,
                                                   ranges=[(0, 10 ** 9), (0, 0)], move_records=False)
        idx = sorted(i for c in eng.calls if c[0] == "count" for i in c[1])
        q.put(("rebal", rank, total == 7309 and st == 1, idx, size, info["steals"]))
        # record moves: rank 0 holds ONE heavy board (the whole 16-clue board, a
        # one-board frontier), rank 1 nothing.  Rank 0 refines it into second-level records, sends
        # half of them to rank 1 (p2p), and rank 1 counts part of that board's subtree
        eng.calls = []
        info = {}
        total, st, size = sharded_count_rebalanced(eng, b16, rank, world, comm=comm, chunk=2, info=info, target=1,
                                                   ranges=[(0, 1), (1, 1)])
        loads = [c[1] for c in eng.calls if c[0] == "load"]
        counted = sum(len(c[1]) for c in eng.calls if c[0] == "count")
        q.put(("records", rank, total == 7309 and st == 1, size, loads, counted, info["refines"],
               info["moved_records"]))
        # first solution of the multi-solution demo board (sudoku.py:99-109) = reference golden
        demo = synth.parse("000100000000320000000009000000000070000000000000900000000000900000000003000000000")
        golden = "234156789179328456568479132391245678425687391687913245752831964816794523943562817"
        out, st = sharded_solve(eng, demo, rank, world, comm=comm)
        q.put(("first", rank, "".join(map(str, out)) == golden and st == 1))
        # TASK range(5, 10) on the same board (golden: reference solve_sudoku with arr=range(5,10))
        out, st = sharded_solve(eng, demo, rank, world, comm=comm, mask=O_range_mask(5, 10))
        q.put(("first_range", rank, "".join(map(str, out)) ==
               "523146789179328456468579132291435678345687291687912345712853964954761823836294517" and st == 1))
        # unsolvable (clue conflict), the wiki board with (0,1) = 5: input comes back, status 0
        bad = synth.parse("55" + synth.WIKI[2:])
        out, st = sharded_solve(eng, bad, rank, world, comm=comm, target=4)
        q.put(("unsolvable", rank, st == 0 and (out == bad).all()))
        # first solution with rebalancing: rank 0 holds ONE board (a one-board
        # lex frontier), rank 1 nothing.  Rank 0 splits it into lex-ordered sub-boards, sends the
        # upper half as records, rank 1 searches part of it; the answer is the reference's
        eng.calls = []
        info = {}
        out, st = sharded_solve(eng, demo, rank, world, comm=comm, target=1, ranges=[(0, 1), (1, 1)], info=info)
        loads = [c[1] for c in eng.calls if c[0] == "load"]
        scanned = sum(c[2] - c[1] for c in eng.calls if c[0] == "first")
        q.put(("first_moved", rank, "".join(map(str, out)) == golden and st == 1, loads, scanned,
               info["refines"], info["moved_records"]))
        # a heavy 17-clue board (919,763 reference validations) under a 1-node round budget: every
        # round's budget hits are split again (refine_head) and handed on; answer = golden S4
        info = {}
        s4 = synth.parse(synth.SEEDS17["S4"])
        out, st = sharded_solve(eng, s4, rank, world, comm=comm, round_budget=1, info=info)
        q.put(("first_heavy", rank, "".join(map(str, out)) == S4_SOLUTION and st == 1, info["refines"],
               info["rounds"]))

    finally:
        dist.destroy_process_group()


def test_shard_bounds_partition():
    for n in (0, 1, 7, 100, 10_000_001):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_world2_gloo_gather():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = [q.get(timeout=5) for _ in range(3 + 10 * world)]
    res = {g[0]: g[1:] for g in got if g[0] not in ("calls", "count_split", "count_refine", "first", "first_range", "unsolvable",
                                                    "rebal", "records", "first_moved", "first_heavy")}
    fm = {g[1]: g[2:] for g in got if g[0] == "first_moved"}
    assert fm[0][0] and fm[1][0], fm                                       # the golden board on both ranks
    assert fm[0][3] >= 1 and fm[0][4] > 0, fm                               # rank 0 split its board, records moved
    assert fm[1][1] and fm[1][2] > 0, fm                                   # rank 1 loaded records and searched them
    fh = {g[1]: g[2:] for g in got if g[0] == "first_heavy"}
    assert fh[0][0] and fh[1][0], fh
    assert fh[0][1] + fh[1][1] >= 1, fh                                     # budget hits were split
    rec = {g[1]: g[2:] for g in got if g[0] == "records"}
    assert rec[0][0] and rec[1][0], rec                                   # exact total (7,309) on both ranks
    assert rec[0][1] == 1                                                  # a one-board frontier
    assert rec[0][4] >= 1 and rec[0][5] > 0                                # rank 0 refined, records moved
    assert rec[1][2] and rec[1][3] > 0, rec                                # rank 1 loaded records and counted
    rebal = {g[1]: g[2:] for g in got if g[0] == "rebal"}
    assert rebal[0][0] and rebal[1][0]                                      # same total on both ranks
    fsize = rebal[0][2]
    assert sorted(rebal[0][1] + rebal[1][1]) == list(range(fsize))         # disjoint and complete
    assert len(rebal[1][1]) > 0 and rebal[1][3] >= 1                        # rank 1 stole work
    assert res["solve"] == (True,) and res["check"] == (True,) and res["count"] == (True,)
    for key in ("first", "first_range", "unsolvable"):
        assert sorted(g[1:] for g in got if g[0] == key) == [(r, True) for r in range(world)], key
    refs = {g[1]: g[2:] for g in got if g[0] == "count_refine"}
    assert refs[0][1] and refs[1][1]                                  # exact total on both ranks
    assert refs[0][0][:2] == (0, 2) and refs[1][0][:2] == (1, 2)      # interleaved shares of stage 1
    split = {g[1]: g[2:] for g in got if g[0] == "count_split"}
    size = split[0][1]
    assert sorted(split[0][0] + split[1][0]) == list(range(size))     # interleaved, disjoint, complete
    calls = {g[1]: g[2] for g in got if g[0] == "calls"}
    assert calls[0] == [150, 500] and calls[1] == [151, 501]     # each rank ran only its slice


def test_multi_device_engine_threads():
    engines = [OracleEngine() for _ in range(3)]
    mde = MultiDeviceEngine(engines)
    p, s = synth.make_30clue(100, seed=8)
    out, st, _ = mde.solve_batch(p)
    assert (out == s).all() and (st == 1).all()
    b, exp = synth.make_check_boards(1000, seed=9)
    assert (mde.check_batch(b) == exp).all()
    assert [e.calls for e in engines] == [[33, 333], [33, 333], [34, 334]]


def test_rebalance_ranges():
    # dry ranks take the upper half of the largest live range, in rank order; ties -> lowest rank
    assert rebalance_ranges([[5, 5], [0, 100], [10, 20]]) == [[50, 100], [0, 50], [10, 20]]
    assert rebalance_ranges([[0, 0], [0, 0], [0, 64]]) == [[32, 48], [48, 64], [0, 32]]
    assert rebalance_ranges([[0, 8], [0, 8], [3, 3]]) == [[0, 4], [0, 8], [4, 8]]
    assert rebalance_ranges([[0, 3], [7, 7]], min_split=4) == [[0, 3], [7, 7]]   # too short to split
    assert rebalance_ranges([[1, 1], [2, 2]]) == [[1, 1], [2, 2]]                 # all done
    rng = np.random.default_rng(0)
    for _ in range(200):                           # conservation: the live work is only re-partitioned
        w = int(rng.integers(1, 9))
        R = []
        for _ in range(w):
            lo = int(rng.integers(0, 1000))
            R.append([lo, lo + int(rng.integers(0, 50)) * int(rng.integers(0, 2))])
        N = rebalance_ranges(R)
        before = sorted(i for a, b in R for i in range(a, b))
        after = sorted(i for a, b in N for i in range(a, b))
        assert before == after


def test_rebalance_plan():
    from distributed_sudoku_solver_amd.shard import rebalance_plan
    # replicated frontiers on both sides: an index move, no records
    S, moves, ref = rebalance_plan([[0, 100, 0], [5, 5, 0]])
    assert S == [[0, 50, 0], [50, 100, 0]] and moves == [(0, 1, 50, 100, False)] and ref == []
    # a donor that holds its own records: they travel, the receiver's frontier becomes them
    S, moves, ref = rebalance_plan([[3, 11, 1], [5, 5, 0]])
    assert S == [[3, 7, 1], [0, 4, 1]] and moves == [(0, 1, 7, 11, True)] and ref == []
    # one board left, a rank dry: the holder refines (no move this step)
    S, moves, ref = rebalance_plan([[0, 1, 0], [1, 1, 0], [4, 4, 0]])
    assert moves == [] and ref == [0] and S[0] == [0, 1, 0]
    # a rank that takes records this step does not give any
    S, moves, ref = rebalance_plan([[0, 0, 0], [0, 0, 0], [0, 64, 1]])
    assert [m[:2] for m in moves] == [(2, 0), (2, 1)]
    assert S == [[0, 32, 1], [0, 16, 1], [0, 16, 1]]
    # all done: nothing to do
    assert rebalance_plan([[1, 1, 0], [2, 2, 1]]) == ([[1, 1, 0], [2, 2, 1]], [], [])
    rng = np.random.default_rng(1)
    for _ in range(300):                            # conservation: live boards are only re-partitioned
        w = int(rng.integers(1, 9))
        st = []
        for _ in range(w):
            lo = int(rng.integers(0, 100))
            st.append([lo, lo + int(rng.integers(0, 40)) * int(rng.integers(0, 2)), int(rng.integers(0, 2))])
        S, moves, ref = rebalance_plan(st, min_split=int(rng.integers(2, 6)))
        assert sum(b - a for a, b, _ in S) == sum(b - a for a, b, _ in st)
        recv = [m[1] for m in moves]
        assert len(recv) == len(set(recv)) and not set(recv) & {m[0] for m in moves}
        assert all(st[m[1]][1] <= st[m[1]][0] for m in moves)              # only dry ranks receive
