import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libsudoku_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def solve_cases():
    return load_golden("solve_cases.json")


@pytest.fixture(scope="session")
def check_cases():
    return load_golden("check_cases.json")


@pytest.fixture(scope="session")
def engine():
    from distributed_sudoku_solver_amd import SudokuEngine
    eng = SudokuEngine(0)
    yield eng
    eng.close()
