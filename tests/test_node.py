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

from doubles import naive_expand, validation_budget


class OracleEngine:
    def __init__(self):
        from oracle import oracle as O
        self.O = O
        self.batches = []
        self.expansions = 0

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        self.batches.append(len(boards))
        out, st, val = self.O.naive_solve_batch(boards, masks, budget=validation_budget(budget, 100_000_000),
                                                threads=2)
        return out, st, val

    def expand(self, boards, masks=None, target=64):
        self.expansions += 1
        return naive_expand(boards, masks, target)


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
        node.pause()                             # hold the worker while we enqueue
        p, s = synth.make_30clue(20, seed=3)
        node.engine.batches.clear()
        for i in range(20):
            node.enqueue({"method": "TASK", "sudoku": [list(map(int, p[i][9 * r: 9 * r + 9])) for r in range(9)],
                          "range": range(1, 10), "uuid": i})
        node.resume()
        t0 = time.time()
        while node.solved_count < 20 and time.time() - t0 < 20:
            time.sleep(0.01)
        assert node.solved_count == 20
        assert node.engine.batches == [20]          # one launch for the whole queue
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


DEMO8 = "000100000000320000000009000000000070000000000000900000000000900000000003000000000"
DEMO8_FIRST = "234156789179328456568479132391245678425687391687913245752831964816794523943562817"


def test_bad_task_is_dropped_and_node_keeps_working():
    """a malformed TASK (descending range, short rows) must not kill the worker."""
    (node,) = _ring(1)
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        uid = __import__("uuid").uuid4()
        s.sendto(pickle.dumps({"method": "TASK", "sudoku": _grid(synth.WIKI), "range": [5, 3], "uuid": uid}), node.me)
        s.sendto(pickle.dumps({"method": "TASK", "sudoku": [[0] * 3] * 9, "range": range(1, 10), "uuid": uid}),
                 node.me)
        time.sleep(0.2)
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
    finally:
        _stop([node])


class _FlakyEngine(OracleEngine):
    def __init__(self):
        super().__init__()
        self.fail_next = True

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        if self.fail_next:
            self.fail_next = False
            raise RuntimeError("simulated launch failure")
        return super().solve_batch(boards, masks, want_work, budget)


def test_engine_error_answers_500_and_worker_survives():
    (node,) = _ring(1, engine_factory=_FlakyEngine)
    try:
        with pytest.raises(urllib.error.HTTPError) as ei:
            _post(node.http_port, _grid(synth.WIKI))
        assert ei.value.code == 500
        assert not node.busy
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201 and body["solution"] is not None
    finally:
        _stop([node])


def _diag(*nodes):
    return [dict(me=n.me, nb=n.neighbor, pred=n.predecessor, free=n.neighborfree, busy=n.busy, q=n.tasks.qsize(),
                 alive=[t.is_alive() for t in n._threads], trace=list(n.trace or [])) for n in nodes]


def _two_ring(**kw):
    a = SudokuNode("127.0.0.1", 0, 0, engine=OracleEngine(), delay_ms=0, stats_wait_s=0.5, trace=True, **kw).start()
    b = SudokuNode("127.0.0.1", 0, 0, anchor=a.me, engine=OracleEngine(), delay_ms=0, stats_wait_s=0.5,
                   trace=True, **kw).start()
    assert b.wait_joined()
    t0 = time.time()
    while not a.neighborfree and time.time() - t0 < 10:      # b's NEEDWORK after joining (DHT_Node.py:322-326)
        time.sleep(0.01)
    assert a.neighborfree, "the joined neighbour never asked for work"
    return a, b


def test_split_range_goes_to_free_neighbor_and_answer_is_lex_first():
    """DHT_Node.py:491-510: the free neighbour gets half of the digit range (utils.py:1-9);
    the multi-solution demo board still answers the reference's golden (lex-first) board."""
    a, b = _two_ring()
    try:
        assert a.neighborfree
        code, body = _post(a.http_port, _grid(DEMO8))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == DEMO8_FIRST
        sent = [t for t in a.trace if t[0] == "TASK"]
        assert sent and sent[0][1] == b.me and sent[0][2] == range(5, 10), _diag(a, b)
    finally:
        _stop([a, b])


def test_unsolvable_split_answers_null():
    """Both halves fail on different nodes: NO_SOLUTION reports let the origin answer 201 null."""
    a, b = _two_ring()
    try:
        bad = _grid(synth.WIKI)
        bad[0][2] = 5                                     # clue conflict: no completion
        assert a.neighborfree
        code, body = _post(a.http_port, bad, timeout=60)
        assert any(t[0] == "TASK" and t[1] == b.me for t in a.trace), list(a.trace)
        assert code == 201 and body["solution"] is None
        assert any(t[0] == "NO_SOLUTION" and t[1] == a.me for t in b.trace)
    finally:
        _stop([a, b])


def test_unsolvable_task_delegated_whole_answers_null():
    """a full-range task that runs on the neighbour (handed over while the origin is
    busy) and has no completion must still wake the origin's POST."""
    a, b = _two_ring(split=False)
    try:
        bad = _grid(synth.WIKI)
        bad[0][2] = 5
        with a.lock:
            a.busy = True                                 # origin busy: the new task goes to the free neighbour
        res = {}

        def post():
            res["r"] = _post(a.http_port, bad, timeout=60)
        import threading
        th = threading.Thread(target=post)
        th.start()
        t0 = time.time()
        while not any(t[0] == "TASK" for t in a.trace) and time.time() - t0 < 10:
            time.sleep(0.01)
        with a.lock:
            a.busy = False
        th.join(60)
        assert res["r"][0] == 201 and res["r"][1]["solution"] is None
        assert any(t[0] == "TASK" and t[1] == b.me and t[2] == range(1, 10) for t in a.trace)
        assert b.validations > 0
    finally:
        _stop([a, b])


def test_two_node_ring_spreads_tasks():
    a, b = _two_ring()
    try:
        for name in ("S4", "S5", "S4", "S5"):
            code, body = _post(a.http_port, _grid(synth.SEEDS17[name]))
            assert "".join(str(v) for row in body["solution"] for v in row) == synth.SEED_SOLUTIONS[name]
        t0 = time.time()
        while b.validations == 0 and time.time() - t0 < 10:      # the neighbour's halves may still run
            time.sleep(0.01)
        assert a.validations > 0 and b.validations > 0, _diag(a, b)
        code, st = _get(a.http_port, "/stats")
        assert len(st["nodes"]) == 2 and st["all"]["validations"] > 0
    finally:
        _stop([a, b])


def test_main_py_http_surface():
    """api='main' = main.py:356-406: POST -> {"solution"} only; /network -> node/predecessor/neighbor."""
    (node,) = _ring(1, api="main")
    try:
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201 and list(body) == ["solution"]
        assert "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
        code, net = _get(node.http_port, "/network")
        assert net == {"node": f"127.0.0.1:{node.port}", "predecessor": list(node.me), "neighbor": list(node.me)}
        code, st = _get(node.http_port, "/stats")
        assert st["all"]["solved"] == 1 and st["nodes"][0]["address"] == f"127.0.0.1:{node.port}"
    finally:
        _stop([node])


class _RefNodeStub:
    """The attributes DHT_Node.DHTNode's solve path touches (DHT_Node.py:474-510)."""

    def __init__(self, inbox=()):
        import queue
        self.task = {"uuid": 0}
        self.neighbor = None
        self.neighborfree = False
        self.validations = 0
        self.task_queue = queue.Queue()
        self.neighbor_tasks = queue.Queue()
        self.inbox = list(inbox)
        self.sent = []

    def non_blocking_receive(self):
        return (self.inbox.pop(0), ("127.0.0.1", 1)) if self.inbox else (None, None)

    def handleMessage(self, data, addr):
        if data["method"] == "SOLUTION_FOUND":          # DHT_Node.py:348-387: abort the running task
            self.task = []

    def send_data(self, data, addr):
        self.sent.append((data, addr))


def test_mixin_cancel_after_poll():
    """a SOLUTION_FOUND read by the poll cancels the solve (reference returns False)."""
    from distributed_sudoku_solver_amd.solver import HipSolveMixin

    class Node(HipSolveMixin, _RefNodeStub):
        pass
    eng = OracleEngine()
    nd = Node([{"method": "SOLUTION_FOUND", "uuid": 0}])
    nd.sudoku_engine = eng
    grid = _grid(synth.WIKI)
    assert nd.solve_sudoku(grid, 0, range(1, 10)) is False
    assert eng.batches == [] and grid == _grid(synth.WIKI)


def test_main_mixin_on_stub_matches_golden(solve_cases):
    """HipSolveMixinMain in a main.DHTNode-shaped stub (main.py:301-354) with the split hand-off."""
    from distributed_sudoku_solver_amd.solver import HipSolveMixinMain

    class Node(HipSolveMixinMain, _RefNodeStub):
        pass
    for c in solve_cases[:20]:
        nd = Node()
        nd.sudoku_engine = OracleEngine()
        grid = [list(c["puzzle"][9 * r: 9 * r + 9]) for r in range(9)]
        assert nd.solve_sudoku(grid, range(*c["range"])) == c["ok"], c["name"]
        assert [v for row in grid for v in row] == (c["board"] if c["ok"] else c["puzzle"]), c["name"]
    nd = Node()
    nd.sudoku_engine = OracleEngine()
    nd.neighbor, nd.neighborfree = ("127.0.0.1", 9), True
    grid = _grid(DEMO8)
    assert nd.solve_sudoku(grid) is True                  # keeps range(5, 10) like main.py:313-325
    assert nd.sent[0][0]["range"] == range(1, 5) and nd.neighborfree is False
    assert "".join(str(v) for row in grid for v in row) == \
        "523146789179328456468579132291435678345687291687912345712853964954761823836294517"


class _SlowEngine(OracleEngine):
    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        time.sleep(0.5)
        return super().solve_batch(boards, masks, want_work, budget)


def test_lex_first_even_when_upper_half_finishes_first():
    """The neighbour's upper-range completion arrives first; the origin still answers with the
    lower range's (lexicographically first) completion, as the reference's single node does."""
    a = SudokuNode("127.0.0.1", 0, 0, engine=_SlowEngine(), delay_ms=0, trace=True).start()
    b = SudokuNode("127.0.0.1", 0, 0, anchor=a.me, engine=OracleEngine(), delay_ms=0, trace=True).start()
    try:
        assert b.wait_joined()
        t0 = time.time()
        while not a.neighborfree and time.time() - t0 < 10:
            time.sleep(0.01)
        code, body = _post(a.http_port, _grid(DEMO8))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == DEMO8_FIRST
        assert any(t[0] == "SOLUTION_FOUND" and t[1] == a.me and t[2] == range(5, 10) for t in b.trace), _diag(a, b)
    finally:
        _stop([a, b])


def test_http_burst_is_one_launch():
    """64 concurrent POST /solve (listen backlog > socketserver's 5) drain into one launch."""
    import threading
    node = SudokuNode("127.0.0.1", 0, 0, engine=OracleEngine(), delay_ms=0).start()
    try:
        p, s = synth.make_30clue(64, seed=123)
        res = [None] * 64
        node.pause()
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, _post(node.http_port, _grid("".join(map(str, p[i]))))))
               for i in range(64)]
        for t in ths:
            t.start()
        t0 = time.time()
        while node.tasks.qsize() < 64 and time.time() - t0 < 30:
            time.sleep(0.01)
        node.resume()
        for t in ths:
            t.join(60)
        assert all(r is not None and r[0] == 201 for r in res)
        assert ["".join(str(v) for row in r[1]["solution"] for v in row) for r in res] == \
            ["".join(map(str, x)) for x in s]
        assert node.engine.batches == [64]
    finally:
        _stop([node])


# ------------------------------------------------------------- bounded solves (SURVEY §7 hard parts 2, 7)
CONFLICT55 = "55" + "0" * 79          # unsolvable, propagation cannot refute it


class _TinyBudget(OracleEngine):
    """A node budget of b allows only 50 b naive validations: every real search hits it."""

    def solve_batch(self, boards, masks=None, want_work=False, budget=None, donate=None):
        self.batches.append(len(boards))
        v = 100_000_000 if budget is None else (0 if budget == 0 else 50 * int(budget))
        return self.O.naive_solve_batch(boards, masks, budget=v, threads=2)


def _post_any(port, grid, timeout=60):
    """_post that also returns error statuses with their JSON body."""
    try:
        return _post(port, grid, timeout)
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def test_unrefutable_board_does_not_block_the_node():
    """'55'+79 zeros beside the wiki puzzle: the wiki answer comes back at once, /stats answers while
    the conflict board's search runs, and the conflict board gets the documented 504 "exhausted"."""
    import threading
    node = SudokuNode("127.0.0.1", 0, 0, engine=OracleEngine(), delay_ms=0, node_budget=1, search_width=64,
                      search_max_pending=20_000, search_limit_s=3.0).start()
    try:
        res = {}
        node.pause()
        th = threading.Thread(target=lambda: res.__setitem__("c", _post_any(node.http_port, _grid(CONFLICT55))))
        th.start()
        t0 = time.time()
        while node.tasks.qsize() < 1 and time.time() - t0 < 10:
            time.sleep(0.01)
        node.resume()
        while node.engine.expansions == 0 and time.time() - t0 < 10:   # the conflict board is being continued
            time.sleep(0.01)
        assert node.engine.expansions > 0
        t1 = time.time()
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
        assert time.time() - t1 < 2.0
        code, st = _get(node.http_port, "/stats")
        assert code == 200 and st["all"]["solved"] >= 1
        th.join(30)
        code, body = res["c"]
        assert code == 504 and body["exhausted"] is True and body["solution"] is None
        assert not node.hard
    finally:
        _stop([node])


def test_budget_hits_still_answer_lex_first():
    """Every launch hits the budget (50 validations): the continued search still returns the
    reference's golden boards, and unsolvable boards still answer null (not exhausted)."""
    node = SudokuNode("127.0.0.1", 0, 0, engine=_TinyBudget(), delay_ms=0, node_budget=1, search_width=16).start()
    try:
        for puzzle, want in ((DEMO8, DEMO8_FIRST), (synth.WIKI, synth.WIKI_SOLUTION)):
            code, body = _post(node.http_port, _grid(puzzle))
            assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == want
        bad = _grid(synth.WIKI)
        bad[0][2] = 5
        code, body = _post(node.http_port, bad)
        assert code == 201 and body["solution"] is None
        assert node.engine.expansions > 0
    finally:
        _stop([node])


def test_split_with_budget_hit_lower_half_returns_golden():
    """The origin keeps range(1, 5) of DEMO8, whose launch hits the budget; the neighbour's
    range(5, 10) completion arrives first but is not taken: the answer is the golden lex-first one."""
    a = SudokuNode("127.0.0.1", 0, 0, engine=_TinyBudget(), delay_ms=0, trace=True, node_budget=1,
                   search_width=8).start()
    b = SudokuNode("127.0.0.1", 0, 0, anchor=a.me, engine=OracleEngine(), delay_ms=0, trace=True).start()
    try:
        assert b.wait_joined()
        t0 = time.time()
        while not a.neighborfree and time.time() - t0 < 10:
            time.sleep(0.01)
        code, body = _post(a.http_port, _grid(DEMO8))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == DEMO8_FIRST
        assert [t for t in a.trace if t[0] == "TASK"][0][1:] == (b.me, range(5, 10))
        assert a.engine.expansions > 0                       # the lower half was continued, not failed
        assert not any(t[0] == "NO_SOLUTION" for t in a.trace)
    finally:
        _stop([a, b])


def test_exhausted_lower_range_blocks_upper_completion():
    """Origin rule (node._decide): an exhausted range below a found completion means no answer can
    be proved lex-first -> 504 exhausted; an exhausted range above the accepted one is irrelevant."""
    import threading
    import uuid as U
    node = SudokuNode("127.0.0.1", 0, 0, engine=OracleEngine(), delay_ms=0)
    try:
        board = _grid(DEMO8)
        for lower_exhausted, expect in ((True, "exhausted"), (False, "solution")):
            uid = U.uuid4()
            ev, box = threading.Event(), []
            from distributed_sudoku_solver_amd.engine import encode_solve_grid
            node.waiters[uid] = (ev, box, encode_solve_grid(board), [0, 0])
            if lower_exhausted:
                node._failed(uid, range(1, 5), board, exhausted=True)
                node._solution(uid, _grid(DEMO8_FIRST), range(5, 10))
            else:
                node._solution(uid, _grid(DEMO8_FIRST), range(1, 5))
                node._failed(uid, range(5, 10), board, exhausted=True)
            assert ev.is_set()
            from distributed_sudoku_solver_amd import node as N
            assert (box[0] is N._EXHAUSTED) == (expect == "exhausted")
    finally:
        node.httpd.server_close()
        node.sock.close()


# ------------------------------------------------------- failure re-execution
def failure_rerun_scenario(engine_a, engine_b):
    """DHT_Node.py:158-209: A (the HTTP origin) splits S1, keeping range(1, 5) -- no completion there
    -- and handing range(5, 10) -- the answer -- to B.  B crashes (no NODE_FAILED) before solving
    it; A's heartbeat check finds B dead, re-runs the delegated half itself (neighbor_tasks) and
    the POST returns the reference's answer.  Returns A's trace."""
    a = SudokuNode("127.0.0.1", 0, 0, engine=engine_a, delay_ms=0, trace=True, heartbeat_s=0.2).start()
    b = SudokuNode("127.0.0.1", 0, 0, anchor=a.me, engine=engine_b, delay_ms=0, trace=True, heartbeat_s=0.2).start()
    try:
        assert b.wait_joined()
        t0 = time.time()
        while not a.neighborfree and time.time() - t0 < 10:
            time.sleep(0.01)
        assert a.neighborfree
        b.pause()                                          # B queues the half it gets and never runs it
        import threading
        res = {}
        th = threading.Thread(target=lambda: res.__setitem__("r", _post(a.http_port, _grid(synth.SEEDS17["S1"]))))
        th.start()
        while b.tasks.qsize() < 1 and time.time() - t0 < 10:
            time.sleep(0.01)
        assert b.tasks.qsize() == 1 and not res                 # B holds range(5, 10); nothing answered yet
        b.stop(graceful=False)                             # crash
        th.join(30)
        code, body = res["r"]
        assert code == 201
        assert "".join(str(v) for row in body["solution"] for v in row) == synth.SEED_SOLUTIONS["S1"]
        assert b.me not in a.network and a.neighbor == a.me
        sent = [t for t in a.trace if t[0] == "TASK"]
        assert sent[0][1:] == (b.me, range(5, 10))
        return a
    finally:
        _stop([a, b])


def graceful_stop_scenario(engine_a, engine_b):
    """DHT_Node.py:137-156: B (the HTTP origin, busy) hands a task to its free neighbour A; A stops
    gracefully before running it: its queued task goes back to its neighbour and NODE_FAILED to
    the coordinator, and the POST on B still answers the reference's board."""
    b = SudokuNode("127.0.0.1", 0, 0, engine=engine_b, delay_ms=0, trace=True, split=False).start()
    a = SudokuNode("127.0.0.1", 0, 0, anchor=b.me, engine=engine_a, delay_ms=0, trace=True, split=False).start()
    try:
        assert a.wait_joined()
        t0 = time.time()
        while not b.neighborfree and time.time() - t0 < 10:
            time.sleep(0.01)
        assert b.neighborfree
        a.pause()
        with b.lock:
            b.busy = True                                  # B busy: a new task goes to the free neighbour
        import threading
        res = {}
        th = threading.Thread(target=lambda: res.__setitem__("r", _post(b.http_port, _grid(synth.SEEDS17["S2"]))))
        th.start()
        while a.tasks.qsize() < 1 and time.time() - t0 < 10:
            time.sleep(0.01)
        assert a.tasks.qsize() == 1
        a.stop(graceful=True)
        with b.lock:
            b.busy = False
        with b._work:
            b._work.notify()
        th.join(30)
        code, body = res["r"]
        assert code == 201
        assert "".join(str(v) for row in body["solution"] for v in row) == synth.SEED_SOLUTIONS["S2"]
        assert any(t[0] == "TASK" and t[1] == b.me for t in a.trace)          # handed back
        assert any(t[0] == "NODE_FAILED" and t[1] == b.me for t in a.trace)   # coordinator told
        t0 = time.time()
        while a.me in b.network and time.time() - t0 < 5:
            time.sleep(0.01)
        assert b.network == [b.me]
    finally:
        _stop([a, b])


def test_failure_reruns_delegated_half():
    failure_rerun_scenario(OracleEngine(), OracleEngine())


def test_graceful_stop_hands_queue_to_neighbour():
    graceful_stop_scenario(OracleEngine(), OracleEngine())


# ------------------------------------------------ every GPU of the box (north_star: sharding, N3)
def test_node_on_multi_device_engine():
    """A SudokuNode on a 3-device MultiDeviceEngine (oracle doubles): batches and the continued
    search of a budget-hit board are sharded over the devices, and the answers are the reference's:
    the wiki puzzle, DEMO8's golden lex-first board (a budget-hit, continued search) and the
    documented 504 "exhausted" for '55'+79 zeros."""
    import threading
    from distributed_sudoku_solver_amd.shard import MultiDeviceEngine
    devs = [_TinyBudget() for _ in range(3)]
    mde = MultiDeviceEngine(devs)
    node = SudokuNode("127.0.0.1", 0, 0, engine=mde, delay_ms=0, node_budget=1, search_width=8,
                      search_max_pending=20_000, search_limit_s=3.0).start()
    try:
        assert node.search_engine is mde                      # doubles cannot fork: shared
        code, body = _post(node.http_port, _grid(synth.WIKI))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
        code, body = _post(node.http_port, _grid(DEMO8))
        assert code == 201 and "".join(str(v) for row in body["solution"] for v in row) == DEMO8_FIRST
        res = {}
        th = threading.Thread(target=lambda: res.__setitem__("c", _post_any(node.http_port, _grid(CONFLICT55))))
        th.start()
        th.join(60)
        code, body = res["c"]
        assert code == 504 and body["exhausted"] is True and body["solution"] is None
        # the continued searches' launches used every device (width 8 per device: 24 sub-boards a slice)
        assert all(len(d.batches) > 3 for d in devs), [d.batches for d in devs]
        assert sum(d.expansions for d in devs) > 0
    finally:
        _stop([node])


def test_multi_device_expand_is_an_ordered_partition():
    """MultiDeviceEngine.expand splits the parents contiguously over the devices and concatenates
    the children in order: solving them in order gives the parents' completions in lex order."""
    from distributed_sudoku_solver_amd.shard import MultiDeviceEngine
    from oracle import oracle as O
    mde = MultiDeviceEngine([OracleEngine() for _ in range(3)])
    b = synth.parse(DEMO8)
    kids = mde.expand(np.stack([b, b, b, b]), None, target=40)
    one = naive_expand(b[None], None, target=10)
    assert len(kids) >= 40
    out, st, _ = O.naive_solve_batch(kids, budget=10_000_000, threads=2)
    sols = ["".join(map(str, o)) for o, s_ in zip(out, st) if s_ == 1]
    ref_out, ref_st, _ = O.naive_solve_batch(one, budget=10_000_000, threads=2)
    ref = ["".join(map(str, o)) for o, s_ in zip(ref_out, ref_st) if s_ == 1]
    assert sols[0] == DEMO8_FIRST and sorted(set(sols)) == sorted(set(ref))


def test_task_in_flight_at_graceful_stop_goes_to_neighbour():
    """a budget-hit task whose search slice (or batch launch) is in flight when a graceful
    stop() drains the queues comes back after the drain; it must go to the neighbour like the rest
    instead of waiting in a queue nobody serves."""
    from distributed_sudoku_solver_amd import node as N
    node = SudokuNode("127.0.0.1", 0, 0, engine=OracleEngine(), delay_ms=0)
    try:
        sent = []
        node.send = lambda msg, to: sent.append((msg, to))
        task = {"method": "TASK", "sudoku": _grid(synth.WIKI), "uuid": "u1"}
        h = N._HardTask(task, None, time.monotonic() + 10)
        assert node._keep_hard(h) and node.hard == [h]               # running: queued for the search thread
        node.hard = []
        node.neighbor = ("127.0.0.1", 1)
        with node.lock:
            node._leaving = True                                    # what stop(graceful=True) sets
        assert not node._keep_hard(h) and node.hard == []
        assert sent == [(task, ("127.0.0.1", 1))]
    finally:
        node.httpd.server_close()
        node.sock.close()
