"""bench.py's rank launcher and C4 sharding on the CPU: `--gpus 2` without torchrun starts two
rank processes (TcpComm barrier / max), each solves its contiguous slice of the SAME seeded stream
(strong scaling), and rank 0 prints one JSON line with n_gpus == 2.  The oracle stands in for the
GPU (tests/doubles.BenchStubEngine, whose RCCL stub is a TcpComm set up from the exchanged id).
Every run blocks `import torch` in every process (a sitecustomize on PYTHONPATH): the bench and
its multi-rank path are torch-free."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


NO_TORCH = """
import sys


class _NoTorch:
    def find_spec(self, name, path=None, target=None):
        if name == "torch" or name.startswith("torch."):
            raise ImportError("bench.py must not import torch (VERDICT r2 item 5)")
        return None


sys.meta_path.insert(0, _NoTorch())
"""


def _run_bench(gpus, extra=(), tmp=None):
    paths = [ROOT, os.path.join(ROOT, "tests")]
    if tmp is not None:
        with open(os.path.join(tmp, "sitecustomize.py"), "w") as f:
            f.write(NO_TORCH)
        paths.insert(0, str(tmp))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join(paths))
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "2", "--warmup", "1",
           "--workload", "solve30", "--batch", "301", "--check-boards", "2000", "--check-steps", "1",
           "--check-warmup", "1", "--c2-puzzles", "0", "--minimal-puzzles", "0", "--hard-leg", "0", "--count-leg", "0", "--lane-puzzles", "0",
           "--first-boards", "",
           "--cpu-seconds", "0",
           "--http-requests", "0", "--pmc-summary", "", "--engine-factory", "doubles:BenchStubEngine", *extra]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout     # exactly one JSON line on stdout
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks(tmp_path):
    r = _run_bench(2, tmp=tmp_path)
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["puzzles_total"] == 301 and r["config"]["puzzles_per_gpu"] in (150, 151)
    # the single-context pass and every in-flight context's output are checked
    k = r["config"]["passes_in_flight_per_gpu"]
    assert k == 2 and r["parity"] == {"mismatched_boards": 0, "checked_boards": (1 + k) * 301}
    assert r["single_stream"]["parity"]["mismatched_boards"] == 0
    assert r["checker"]["parity"] == {"mismatched_boards": 0, "checked_boards": 4000}
    assert list(r)[-3:] == ["roofline_summary", "checker", "checker_summary"]   # the tail the driver keeps
    assert r["weak_scaling"]["parity"]["mismatched_boards"] == 0
    assert r["value"] > 0 and r["steps"] == 2 and r["warmup"] == 1


def test_bench_gpus1_single_process(tmp_path):
    r = _run_bench(1, tmp=tmp_path)
    assert r["n_gpus"] == 1 and "weak_scaling" not in r
    k = r["config"]["passes_in_flight_per_gpu"]
    assert r["parity"] == {"mismatched_boards": 0, "checked_boards": (1 + k) * 301}


def test_bench_gpus2_count_legs_over_tcp_rccl_stub(tmp_path):
    """the C5 legs at world 2 -- RCCL id over the ranks' TcpComm, the two-stage
    count's all-reduce and the rebalanced count's all-gathers through the stub -- with torch blocked."""
    r = _run_bench(2, extra=["--count-leg", "1", "--c5-boards", "16,16", "--frontier-probe", "0"], tmp=tmp_path)
    for leg in ("c5_count", "c5_count_rebalanced"):
        assert r[leg].get("ok") is True, r[leg]
        assert r[leg]["solutions"] == 7309
    assert r["c5_count_rebalanced"]["rounds"] >= 1


def test_bench_gpus2_first_solution_leg(tmp_path):
    """the first-solution leg (shard.sharded_solve over the ranks' RCCL stub) at
    world 2 on a heavy 17-clue seed: the known completion, and its rounds / moves / refinements."""
    r = _run_bench(2, extra=["--first-boards", "S4"], tmp=tmp_path)
    leg = r["first_solution"]
    assert leg["ok"] is True and leg["S4"]["ok"] is True, leg
    for key in ("wall_ms", "rounds", "moved_records", "refines", "steals", "frontier_boards"):
        assert leg["S4"][key] is not None, key
    assert leg["S4"]["rounds"] >= 1 and leg["S4_split"]["ok"] is True and leg["S4_split"]["refines"] >= 1


def test_no_torch_blocker_works(tmp_path):
    """The blocker the bench tests rely on does stop a torch import."""
    import subprocess
    with open(os.path.join(tmp_path, "sitecustomize.py"), "w") as f:
        f.write(NO_TORCH)
    env = dict(os.environ, PYTHONPATH=str(tmp_path))
    p = subprocess.run([sys.executable, "-c", "import torch"], env=env, capture_output=True, text=True)
    assert p.returncode != 0 and "must not import torch" in p.stderr


def test_mix_ceiling_calibration_has_the_kernels_keys():
    """The bench prices prop32 against k_b3 (its ORs are v_bitop3 since round 6) and solve4 against
    k_mix; both come from the committed rocprofv3 calibration, and v_bitop3 chains pair (dual-issue)
    where v_or3 chains do not."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    mix = bench.mix_ceiling(os.path.join(ROOT, "profiles", "r06", "issue_calib_pmc.json"))
    assert mix and {"k_b3@8", "k_or3@8", "k_mix@8"} <= set(mix)
    assert mix["k_b3@8"]["valu_per_quad"] > 1.5 * mix["k_or3@8"]["valu_per_quad"]
    assert mix["k_b3@8"]["dual_frac"] > 0.5 > mix["k_or3@8"]["dual_frac"]
