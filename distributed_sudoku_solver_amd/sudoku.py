"""Drop-in for the reference checker class `Sudoku` (sudoku.py:5-94).

`Sudoku(grid).check()` is evaluated by the HIP checker kernel (one board here;
use SudokuEngine.check_batch for batches).  Differences from the reference,
all deliberate:
  * no `_limit_calls` rate limiter (sudoku.py:10-17 sleeps up to seconds per
    board; SURVEY §0.5 -- benchmarks run with it disabled);
  * check() returns the INTENDED verdict (each 3x3 box tests its own cells).
    The reference's check() raises NameError whenever rows, columns and the
    box(0,0) sum pass (sudoku.py:68); check(raw=True) reproduces that.
Grid values must be integers (|v| < 2^59; 5.0 counts as 5): the literal
`sum == 45 and len(set) == 9` rule is evaluated exactly -- boards within 0..255
on the streaming uint8 kernel, others on its int64 twin (sdk_check_batch_i64).
"""
from .engine import encode_check_grid
from . import _lib as L


class Sudoku:
    def __init__(self, sudoku, engine=None):
        self.grid = sudoku
        self.engine = engine

    def _engine(self):
        if self.engine is None:
            from .solver import default_engine
            self.engine = default_engine()
        return self.engine

    def __str__(self):
        bar = "| - - - - - - - - - - - |\n"
        lines = [bar]
        for r in range(9):
            cells = [str(self.grid[r][c]) + (" | " if c % 3 == 2 else " ") for c in range(9)]
            lines.append("| " + "".join(cells) + "\n")
            if r % 3 == 2:
                lines.append(bar)
        return "".join(lines)

    def update_row(self, row, values):
        self.grid[row] = values

    def update_column(self, col, values):
        for r in range(9):
            self.grid[r][col] = values[r]

    def verdict(self):
        """Raw verdict byte: SDK_CHECK_OK | SDK_CHECK_RAW_NAMEERROR."""
        board = encode_check_grid(self.grid)
        return int(self._engine().check_batch(board[None, :])[0])

    def check(self, base_delay=0.01, interval=10, threshold=5, raw=False):
        v = self.verdict()
        if raw and (v & L.SDK_CHECK_RAW_NAMEERROR):
            raise NameError("name 'i' is not defined")
        if raw:
            return False
        return bool(v & L.SDK_CHECK_OK)
