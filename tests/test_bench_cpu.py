"""bench.py's rank launcher and C4 sharding on the CPU: `--gpus 2` without torchrun starts two
rank processes (gloo barrier / max), each solves its contiguous slice of the SAME seeded stream
(strong scaling), and rank 0 prints one JSON line with n_gpus == 2.  The oracle stands in for the
GPU (tests/doubles.BenchStubEngine)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(gpus, extra=()):
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests")]))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--workload", "solve30", "--batch", "301", "--check-boards", "2000", "--check-steps", "1",
           "--check-warmup", "1", "--c2-puzzles", "0", "--minimal-puzzles", "0", "--count-leg", "0", "--lane-puzzles", "0",
           "--cpu-seconds", "0",
           "--http-requests", "0", "--pmc-summary", "", "--engine-factory", "doubles:BenchStubEngine", *extra]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout     # exactly one JSON line on stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks():
    r = _run_bench(2)
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["puzzles_total"] == 301 and r["config"]["puzzles_per_gpu"] in (150, 151)
    assert r["parity"] == {"mismatched_boards": 0, "checked_boards": 301}
    assert r["checker"]["parity"] == {"mismatched_boards": 0, "checked_boards": 4000}
    assert r["weak_scaling"]["parity"]["mismatched_boards"] == 0
    assert r["value"] > 0 and r["steps"] == 2 and r["warmup"] == 1


def test_bench_gpus1_single_process():
    r = _run_bench(1)
    assert r["n_gpus"] == 1 and "weak_scaling" not in r
    assert r["parity"] == {"mismatched_boards": 0, "checked_boards": 301}
