"""Torch-free multi-process path: hostcomm.TcpComm (standard-library sockets) as the
host transport of ShardedBatch and as the comm of the one-board frontier searches,
world size 3 on the CPU with the oracle standing in for the GPUs."""
import multiprocessing as mp
import os
import socket
import subprocess
import sys

import numpy as np

from distributed_sudoku_solver_amd import synth
from distributed_sudoku_solver_amd.hostcomm import TcpComm
from distributed_sudoku_solver_amd.shard import ShardedBatch, sharded_count, sharded_count_rebalanced, sharded_solve

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = "000100000000320000000009000000000070000000000000900000000000900000000003000000000"
DEMO_FIRST = "234156789179328456568479132391245678425687391687913245752831964816794523943562817"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    from doubles import OracleEngine
    comm = TcpComm(rank, world, "127.0.0.1", port, timeout=60)
    try:
        # byte-level collectives, any root
        got = comm.broadcast_bytes(b"id-from-1" if rank == 1 else None, root=1)
        parts = comm.gather_bytes(bytes([rank]) * (rank + 1), root=2)
        every = comm.allgather_bytes(str(rank).encode())
        buf = np.array([rank + 1, -rank, 7 * rank], np.int64)
        comm.allreduce(buf, 3, np.int64, "min")
        s = np.array([rank + 1], np.uint64)
        comm.allreduce(s, 1, np.uint64, "sum")
        q.put(("bytes", rank, got == b"id-from-1", parts if rank == 2 else None, every, buf.tolist(), int(s[0])))
        comm.barrier()
        # sharded batch gathered over TcpComm (ragged shards)
        eng = OracleEngine()
        p, sol = synth.make_30clue(101, seed=5)
        out, st = ShardedBatch(eng, rank, world, comm=comm).solve(p)
        if rank == 0:
            q.put(("batch", bool((out == sol).all() and (st == 1).all())))
        # one-board searches with TcpComm as the comm
        b16 = synth.parse(synth.SEEDS17["S1"][:-9] + "000800000")
        total, st, _ = sharded_count(eng, b16, rank, world, comm=comm)
        rt, rst, _ = sharded_count_rebalanced(eng, b16, rank, world, comm=comm, chunk=3)
        o, fst = sharded_solve(eng, synth.parse(DEMO), rank, world, comm=comm)
        q.put(("search", rank, total == 7309 and st == 1, rt == 7309 and rst == 1,
               "".join(map(str, o)) == DEMO_FIRST and fst == 1))
        # point-to-point through the star (non-root to non-root) and the record-moving count:
        # rank 2 holds the whole 16-clue board as a one-board frontier, ranks 0 and 1 nothing
        from distributed_sudoku_solver_amd import _lib as L
        recv = np.zeros(5, np.uint8)
        ops = {1: [(L.SDK_COMM_SEND, 2, np.arange(5, dtype=np.uint8), 5)],
               2: [(L.SDK_COMM_RECV, 1, recv, 5)]}.get(rank, [])
        comm.p2p(ops)
        info = {}
        mt, mst, _ = sharded_count_rebalanced(eng, b16, rank, world, comm=comm, chunk=2, target=1,
                                              ranges=[(1, 1), (1, 1), (0, 1)], info=info)
        loads = sum(1 for c in eng.calls if isinstance(c, tuple) and c[0] == "load")
        q.put(("records", rank, recv.tolist() if rank == 2 else None, mt == 7309 and mst == 1, loads,
               info["refines"]))
    finally:
        comm.close()


def test_tcpcomm_world3():
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    got = [q.get(timeout=5) for _ in range(3 * world + 1)]
    by = {}
    for g in got:
        by.setdefault(g[0], []).append(g[1:])
    assert by["batch"] == [(True,)]
    for rank, ok_bcast, parts, every, mins, total in by["bytes"]:
        assert ok_bcast and every == [b"0", b"1", b"2"] and mins == [1, -2, 0] and total == 6
        if rank == 2:
            assert parts == [b"\x00", b"\x01\x01", b"\x02\x02\x02"]
    assert sorted(by["search"]) == [(r, True, True, True) for r in range(world)]
    rec = {g[0]: g[1:] for g in by["records"]}
    assert rec[2][0] == [0, 1, 2, 3, 4]
    assert all(rec[r][1] for r in range(world))                    # exact total on every rank
    assert rec[2][3] >= 1 and rec[0][2] >= 1 and rec[1][2] >= 1      # rank 2 refined, both others got records


def test_product_path_imports_no_torch():
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import distributed_sudoku_solver_amd.shard, distributed_sudoku_solver_amd.hostcomm\n"
            "import distributed_sudoku_solver_amd.node, distributed_sudoku_solver_amd.solver\n"
            "import distributed_sudoku_solver_amd.engine, distributed_sudoku_solver_amd.sudoku\n"
            "assert 'torch' not in sys.modules, 'torch was imported'\n" % ROOT)
    subprocess.run([sys.executable, "-c", code], check=True, timeout=120)


def test_tcpcomm_world1_is_local():
    c = TcpComm(0, 1)
    buf = np.array([3, 4], np.int64)
    c.allreduce(buf, 2, np.int64, "sum")
    assert buf.tolist() == [3, 4]
    assert c.broadcast_bytes(b"x") == b"x" and c.allgather_bytes(b"y") == [b"y"]
    assert (c.gather(np.arange(6).reshape(3, 2)) == np.arange(6).reshape(3, 2)).all()
    c.close()
