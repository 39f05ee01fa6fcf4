"""Host node on the HIP engine: POST /solve end to end (config C1) and a 3-node ring."""
import time

import pytest

from distributed_sudoku_solver_amd import synth
from distributed_sudoku_solver_amd.node import SudokuNode

from test_node import _get, _grid, _post, _stop

pytestmark = pytest.mark.gpu


def test_post_solve_on_gpu_node(engine):
    node = SudokuNode("127.0.0.1", 0, 0, engine=engine, delay_ms=0).start()
    try:
        lat = []
        for _ in range(5):
            code, body = _post(node.http_port, _grid(synth.WIKI))
            assert code == 201
            assert "".join(str(v) for row in body["solution"] for v in row) == synth.WIKI_SOLUTION
            lat.append(body["duration"])
        assert min(lat) < 0.05                           # reference: 0.087 s
        for name in ("S1", "S2", "S3"):
            code, body = _post(node.http_port, _grid(synth.SEEDS17[name]))
            assert "".join(str(v) for row in body["solution"] for v in row) == synth.SEED_SOLUTIONS[name]
    finally:
        _stop([node])


def test_gpu_ring(engine):
    nodes = [SudokuNode("127.0.0.1", 0, 0, engine=engine, delay_ms=0, stats_wait_s=0.5).start()]
    for _ in range(2):
        nodes.append(SudokuNode("127.0.0.1", 0, 0, anchor=nodes[0].me, engine=engine, delay_ms=0,
                                stats_wait_s=0.5).start())
        assert nodes[-1].wait_joined()
    try:
        time.sleep(0.2)
        for nd in nodes:
            code, body = _post(nd.http_port, _grid(synth.SEEDS17["S4"]))
            assert code == 201
            assert "".join(str(v) for row in body["solution"] for v in row) == synth.SEED_SOLUTIONS["S4"]
        code, st = _get(nodes[0].http_port, "/stats")
        assert len(st["nodes"]) == 3 and st["all"]["solved"] >= 3
    finally:
        _stop(nodes)
