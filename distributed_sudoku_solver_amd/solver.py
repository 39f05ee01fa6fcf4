"""Drop-in for the reference solve path: DHTNode.solve_sudoku (DHT_Node.py:474-538) and
its main.py twin (main.py:301-354).

Call contract kept from the reference:
  * `puzzle` is a list of 9 lists of 9 numbers and is mutated in place:
    completed (lexicographically first completion = the reference's row-major,
    ascending-digit DFS result) when True is returned, untouched when False;
  * `arr` (a TASK digit `range`) restricts only the lowest-index empty cell;
  * returns a bool.
The search itself runs in libsudoku_hip.so; this module only converts the grid.

Node protocol side effects of the reference's recursive solver are applied once,
before the (micro-second) device call instead of once per recursion level:
cancellation (`task == []`, DHT_Node.py:481), one non-blocking UDP poll
(DHT_Node.py:485-488), and the hand-off of half the digit range to a free
neighbour (DHT_Node.py:491-510).  `validations` is advanced by the engine's work counter:
search nodes for the propagating solvers (the naive-DFS count is not defined for a
propagating search), or exactly the reference's validations when the
engine runs the one-board-per-lane reference DFS (SDK_OPT_SOLVER = SDK_SOLVER_LANE;
slow on hard boards, exact /stats accounting).

Every solve is bounded (search.LexSearch): launches of DEFAULT_BUDGET nodes per board,
a board that needs more is continued in slices over its lex-ordered frontier until it
is decided or `time_limit` passes.  Then solve_grid raises SearchExhausted, and the
mixins return False WITHOUT any side effect -- exactly what a reference node whose
solve_sudoku is still running shows its peers (perform_solving sends nothing on
False, DHT_Node.py:424-470), but its node thread is free again.
"""
import threading
import time

import numpy as np

from .engine import SudokuEngine, encode_solve_grid, range_to_mask
from .search import DEFAULT_BUDGET, LexSearch, default_budget
from .utils import split_array_in_middle
from . import _lib as L

DEFAULT_TIME_LIMIT_S = 60.0


class SearchExhausted(L.SudokuHipError):
    """The bounded search gave up (time limit or worklist size): the board is undecided."""

_engines = {}
_engines_lock = threading.Lock()


def default_engine(device=0):
    with _engines_lock:
        eng = _engines.get(device)
        if eng is None:
            # bounded by default: a direct solve_batch on it never runs unbounded either
            eng = _engines[device] = SudokuEngine(device, node_budget=DEFAULT_BUDGET)
        return eng


def _empty_cells(puzzle):
    return [(r, c) for r in range(9) for c in range(9) if puzzle[r][c] == 0]


def solve_grid(puzzle, arr=range(1, 10), engine=None, budget=None, time_limit=DEFAULT_TIME_LIMIT_S):
    """Core drop-in: mutate `puzzle` like the reference solver and return (ok, work).

    Bounded (module docstring): raises SearchExhausted when the search gives up.  budget =
    per-launch budget (None: search.default_budget of the engine)."""
    eng = engine or default_engine()
    board = encode_solve_grid(puzzle)
    search = LexSearch(eng, board, range_to_mask(arr), budget=default_budget(eng) if budget is None else budget)
    st, sol = search.run(None if time_limit is None else time.monotonic() + time_limit)
    if st == L.SDK_BUDGET_HIT:
        raise SearchExhausted(f"search exhausted after {search.nodes} nodes in {search.launches} launches; "
                              "the reference would still be searching (DHT_Node.py:474-538)")
    if st == L.SDK_SOLVED:
        for r, c in _empty_cells(puzzle):
            puzzle[r][c] = int(sol[9 * r + c])
        return True, search.nodes
    return False, search.nodes


def _solve_or_idle(node, puzzle, arr):
    """solve_grid for the mixins: an exhausted search is reported as False with no side
    effect (the reference node would still be searching and would have sent nothing)."""
    try:
        ok, work = solve_grid(puzzle, arr, node.sudoku_engine)
    except SearchExhausted:
        return False
    node.validations += work
    return ok


def solve_sudoku(puzzle, arr=range(1, 10), engine=None):
    """Function form of the solve contract (no node attached)."""
    return solve_grid(puzzle, arr, engine)[0]


class HipSolveMixin:
    """Mix into DHT_Node.DHTNode: `class Node(HipSolveMixin, DHTNode)`.

    Replaces solve_sudoku(self, puzzle, uuid, arr=range(1, 10)) (DHT_Node.py:474)."""

    sudoku_engine = None

    def solve_sudoku(self, puzzle, uuid=None, arr=range(1, 10)):
        if self.task == []:                                   # DHT_Node.py:481-482
            return False
        data, addr = self.non_blocking_receive()              # DHT_Node.py:485-488
        if data:
            self.handleMessage(data, addr)
            if self.task == []:      # the poll may have cancelled this task (SOLUTION_FOUND, DHT_Node.py:348-387)
                return False
        if self.neighbor and self.neighborfree:               # DHT_Node.py:491-510
            if not self.task_queue.empty():
                task = self.task_queue.get()
                self.send_data(task, self.neighbor)
                self.neighborfree = False
                self.neighbor_tasks.put(task)
            elif len(arr) > 1:
                first_half, arr = split_array_in_middle(arr)
                task = {"method": "TASK", "sudoku": puzzle, "range": first_half, "uuid": uuid}
                self.send_data(task, self.neighbor)
                self.neighbor_tasks.put(task)
                self.neighborfree = False
        return _solve_or_idle(self, puzzle, arr)


class HipSolveMixinMain:
    """Mix into main.DHTNode: replaces solve_sudoku(self, puzzle, arr=range(1, 10)) (main.py:301)."""

    sudoku_engine = None

    def solve_sudoku(self, puzzle, arr=range(1, 10)):
        if self.task == []:                                   # main.py:306-307
            return False
        data, addr = self.non_blocking_receive()              # main.py:308-311
        if data:
            self.handleMessage(data, addr)
            if self.task == []:
                return False
        if self.neighbor and self.neighborfree and len(arr) > 1:   # main.py:313-325
            first_half, arr = split_array_in_middle(arr)
            self.send_data({"method": "TASK", "sudoku": puzzle, "range": first_half}, self.neighbor)
            self.neighborfree = False
        return _solve_or_idle(self, puzzle, arr)
