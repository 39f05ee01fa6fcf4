"""Host node protocol (HTTP + UDP ring) on 127.0.0.1.  The engine is a test double
computed by the oracle on CPU tests; tests/test_gpu_node.py runs the same flows
on the HIP engine."""
import json
import pickle
import socket
import time
import urllib.request

import numpy as np
import pytest

from distributed_sudoku_solver_amd import synth
from distributed_sudoku_solver_amd.node import SudokuNode, decode_datagram, encode_datagram


class OracleEngine:
    def __init__(self):
        from oracle import oracle as O
        self.O = O
        self.batches = []

    def solve_batch(self, boards, masks=None, want_work=False):
        self.batches.append(len(boards))
        out, st, val = self.O.naive_solve_batch(boards, masks, budget=100_000_000, threads=2)
        return out, st, val


def _post(port, grid, timeout=30):
    req = urllib.request.Request(f"http://127.0.0.1:{port}/solve", data=json.dumps({"sudoku": grid}).encode(),
                                 headers={"Content-Type": "application/json"}, method="POST")
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, json.loads(r.read())


def _get(port, path):
    with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=30) as r:
        return r.status, json.loads(r.read())


def _grid(s):
    v = [int(c) for c in s]
    return [v[9 * r: 9 * r + 9] for r in range(9)]


def _ring(n, engine_factory=OracleEngine, **kw):
    nodes = [SudokuNode("127.0.0.1", 0, 0, engine=engine_factory(), delay_ms=0, stats_wait_s=0.5, **kw).start()]
    for _ in range(n - 1):
        nodes.append(SudokuNode("127.0.0.1", 0, 0, anchor=nodes[0].me, engine=engine_factory(), delay_ms=0,
                                stats_wait_s=0.5, **kw).start())
        assert nodes[-1].wait_joined()
    time.sleep(0.2)
    return nodes


def _stop(nodes):
    for nd in nodes:
        if nd.running:
            nd.stop(graceful=False)


def test_single_node_http_api():
    (node,) = _ring(1)
    try:
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201
        assert "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
        assert isinstance(body["duration"], float)
        code, st = _get(node.http_port, "/stats")
        assert code == 200 and st["all"]["solved"] == 1 and st["all"]["validations"] > 0
        assert st["nodes"] == [{"address": f"127.0.0.1:{node.port}", "validations": st["all"]["validations"]}]
        code, net = _get(node.http_port, "/network")
        me = str(node.me)
        assert net == {me: [me, me]}
        # unsolvable puzzle answers instead of hanging (reference: DHT_Node.py:553 spins forever)
        bad = _grid(synth.WIKI)
        bad[0][2] = 5
        code, body = _post(node.http_port, bad)
        assert code == 201 and body["solution"] is None
        # malformed request
        req = urllib.request.Request(f"http://127.0.0.1:{node.http_port}/solve", data=b"{}", method="POST")
        with pytest.raises(urllib.error.HTTPError):
            urllib.request.urlopen(req, timeout=10)
    finally:
        _stop([node])


def test_three_node_ring_join_network_stats():
    nodes = _ring(3)
    try:
        order = nodes[0].network
        assert [nd.network for nd in nodes] == [order] * 3
        for i, nd in enumerate(nodes):
            k = order.index(nd.me)
            assert nd.predecessor == order[(k - 1) % 3] and nd.neighbor == order[(k + 1) % 3]
        code, net = _get(nodes[1].http_port, "/network")
        assert list(net) == [str(a) for a in order]
        assert net[str(order[1])] == [str(order[0]), str(order[2])]
        code, body = _post(nodes[2].http_port, _grid(synth.WIKI))
        assert code == 201
        time.sleep(0.2)
        code, st = _get(nodes[0].http_port, "/stats")
        assert len(st["nodes"]) == 3
        assert all("validation" in e for e in st["nodes"][1:])          # reference key for remote entries
        assert st["all"]["solved"] >= 1
    finally:
        _stop(nodes)


def test_batched_tasks_one_launch():
    """Queued TASKs are drained into one engine call."""
    (node,) = _ring(1)
    try:
        with node.lock:
            node.busy = True                     # hold the worker while we enqueue
        p, s = synth.make_30clue(20, seed=3)
        from distributed_sudoku_solver_amd.engine import SudokuEngine  # noqa: F401  (import path check only)
        node.engine.batches.clear()
        with node._work:
            for i in range(20):
                node.tasks.put({"method": "TASK", "sudoku": [list(map(int, p[i][9 * r: 9 * r + 9])) for r in range(9)],
                                "range": range(1, 10), "uuid": i})
            node._work.notify()
        with node.lock:
            node.busy = False
        t0 = time.time()
        while node.solved_count < 20 and time.time() - t0 < 20:
            time.sleep(0.01)
        assert node.solved_count == 20
        assert max(node.engine.batches) > 1
    finally:
        _stop([node])


def test_failure_detection_repairs_ring():
    nodes = _ring(3, heartbeat_s=0.2)
    try:
        order = list(nodes[0].network)
        victim = next(nd for nd in nodes if nd.me == order[1])
        victim.stop(graceful=False)              # crash: no NODE_FAILED sent
        t0 = time.time()
        alive = [nd for nd in nodes if nd is not victim]
        while time.time() - t0 < 10:
            if all(len(nd.network) == 2 for nd in alive):
                break
            time.sleep(0.05)
        assert all(victim.me not in nd.network for nd in alive)
        a, b = alive
        assert a.neighbor == b.me and b.neighbor == a.me
        code, body = _post(alive[1].http_port, _grid(synth.WIKI))
        assert code == 201 and body["solution"] is not None
    finally:
        _stop(nodes)


def test_wire_format_and_safe_unpickler():
    msg = {"method": "TASK", "sudoku": _grid(synth.WIKI), "range": range(1, 5), "uuid": __import__("uuid").uuid4(),
           "initial_node": ("127.0.0.1", 7000)}
    data = encode_datagram(msg)
    assert len(data) <= 1024                     # fits the reference's recvfrom(1024)
    assert decode_datagram(data) == msg
    assert pickle.loads(data) == msg             # a reference node reads it with plain pickle

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))

    with pytest.raises(pickle.UnpicklingError):
        decode_datagram(pickle.dumps({"method": "TASK", "x": Evil()}))


def test_accepts_reference_style_task_over_udp():
    (node,) = _ring(1)
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        uid = __import__("uuid").uuid4()
        s.sendto(pickle.dumps({"method": "TASK", "sudoku": _grid(synth.WIKI), "range": range(1, 10), "uuid": uid}),
                 node.me)
        t0 = time.time()
        while node.solved_count < 1 and time.time() - t0 < 10:
            time.sleep(0.01)
        assert node.solved_count == 1 and uid in node.done_uuids
    finally:
        _stop([node])
