"""distributed_sudoku_solver_amd -- MI355X-native (gfx950) engine for the hot path of
jsturm-11/distributed_sudoku_solver: DHTNode.solve_sudoku (DHT_Node.py:474-538) and
Sudoku.check (sudoku.py:43-94), behind the reference's own call contracts.

    from distributed_sudoku_solver_amd import SudokuEngine          # numpy batches
    from distributed_sudoku_solver_amd.solver import solve_sudoku   # list-of-lists drop-in
    from distributed_sudoku_solver_amd.sudoku import Sudoku         # Sudoku(grid).check()
"""
from .engine import SudokuEngine, encode_solve_grid, encode_check_grid, range_to_mask  # noqa: F401
from . import _lib  # noqa: F401

__all__ = ["SudokuEngine", "encode_solve_grid", "encode_check_grid", "range_to_mask"]
