"""Resumable, budgeted lex-first search of one board (SURVEY §7 hard parts 2 and 7).

The reference's solve_sudoku (DHT_Node.py:474-538) searches until its DFS ends -- on
a board that propagation cannot refute (e.g. '55' + 79 zeros) that is
never, and its POST /solve waits forever (DHT_Node.py:553-554).  A GPU launch that
never ends is worse still: it holds every other board of its batch.  So every
product-path solve here is bounded:

  * a launch gives each board a node budget (sdk_solve_batch_budget); a board that
    runs out comes back as SDK_BUDGET_HIT -- a state of its own, never "no solution" --
    and its launch ends with the rest of the batch answered;
  * such a board is continued by LexSearch, in slices of bounded time: an ordered
    worklist of sub-boards whose completions, taken in worklist order, are exactly the
    board's completions in lex order.  Each slice solves the first `width` sub-boards in
    ONE launch (each with the budget) and replaces every sub-board that hit the budget by
    its children (sdk_expand_boards: the reference's branching -- lowest open cell,
    digits ascending -- after propagation, one batched call on the GPU).  The first
    SOLVED sub-board whose predecessors are all refuted holds the reference's answer
    (its lex-first completion); later sub-boards are dropped as soon as one solves.
    Only the first width/EXPAND_SHARE hits of a slice are expanded (the front of the lex
    order, where the answer is decided first); later hits go back unexpanded, and when
    most of a slice hits, the budget doubles (up to `max_budget`) -- so the worklist
    grows by about one slice per slice instead of nine.
  * the worklist only ever goes deeper, so the search ends on every board the engine
    can finish; a board whose worklist outgrows `max_pending` sub-boards, or whose caller's
    deadline passes, ends as SDK_BUDGET_HIT ("search exhausted"): a defined answer that
    is never confused with "no completion" (node.py keeps digit ranges lex-ordered on it).

A slice is one launch plus at most one expansion call.  With a slice target (a node's
continued search, LexSearch.for_node) every part of a slice is bounded before it runs, and
the whole slice -- launch, expansion, host copies -- is what is measured against it:
  * the first slice runs at the smallest budget;
  * the launch's node budget is capped by the measured wall time per search node on a
    launch's critical path (launch time / most nodes any board took), so budget x that
    time stays within LAUNCH_SHARE of the target; at budget 1 the width shrinks instead;
  * the number of budget hits expanded per slice halves while an expansion takes more than
    EXPAND_SHARE_OF_TARGET of the target.
A node runs these slices on their own thread and engine context (node.py), so new requests
never wait behind one.  The search runs on whatever engine it is given: SudokuEngine
(libsudoku_hip.so) in the product, a MultiDeviceEngine (the slice's launch and expansion
sharded over every GPU of the node), an oracle double in the CPU tests.
"""
import collections
import time

import numpy as np

from . import _lib as L
from .engine import ALL_DIGITS_MASK

DEFAULT_BUDGET = 2048          # search nodes per board per launch (a ~10 ms bound on MI355X)
DEFAULT_WIDTH = 16384          # sub-boards per slice (fills the solver's resident slots)
DEFAULT_MAX_PENDING = 1 << 20  # sub-boards the worklist may hold (81 MB of host memory)
BUDGET_GROWTH_CAP = 8          # the per-launch budget may double up to this multiple of the first
EXPAND_SHARE = 32              # a slice expands at most width / this of its hits (the lex front)
LANE_VALIDATIONS_PER_NODE = 4096   # SDK_SOLVER_LANE budgets count the reference's validations
SLICE_TARGET_S = 0.01          # a node's continued search: wall time of one slice (search + expansion + copies)
LAUNCH_SHARE = 0.5             # ... of which the launch may take this much (budget x node time)
EXPAND_SHARE_OF_TARGET = 0.3   # ... and an expansion this much before fewer hits are expanded
MIN_WIDTH = 256                # sub-boards per slice, at least (per device)


def n_devices(engine):
    """GPUs an engine drives (MultiDeviceEngine: all of them; anything else: one)."""
    return max(1, int(getattr(engine, "n_devices", 1)))


def default_budget(engine):
    """Per-launch budget for `engine`: DEFAULT_BUDGET search nodes, or as many of the reference's
    validations for the per-lane reference DFS (SDK_SOLVER_LANE counts its budget in those)."""
    try:
        lane = engine.get_option(L.SDK_OPT_SOLVER) == L.SDK_SOLVER_LANE
    except (AttributeError, KeyError, L.SudokuHipError):
        lane = False
    return DEFAULT_BUDGET * (LANE_VALIDATIONS_PER_NODE if lane else 1)


class LexSearch:
    """The reference's answer for one board, found in bounded slices.

    engine   anything with solve_batch(boards, masks, want_work, budget, donate) and
             expand(boards, masks, target) -- SudokuEngine on the GPU
    board    uint8[81] (0 empty, 1..9 given, 10..255 inert given)
    mask     first-cell digit mask (the TASK `range`, engine.range_to_mask), None = all
    hit      the board already hit the budget in a batch launch: start by expanding it

    After step() returned True, `status` is SDK_SOLVED (board = the lex-first completion),
    SDK_UNSOLVABLE (board = the input: the reference restores it) or SDK_BUDGET_HIT
    (exhausted: the worklist outgrew max_pending, or run()'s deadline passed)."""

    def __init__(self, engine, board, mask=None, budget=DEFAULT_BUDGET, width=DEFAULT_WIDTH,
                 max_pending=DEFAULT_MAX_PENDING, hit=False, max_budget=None, slice_target_s=None):
        if budget < 1 or width < 1:
            raise ValueError("budget and width must be >= 1")
        self.engine = engine
        self.input = np.ascontiguousarray(board, dtype=np.uint8).reshape(81).copy()
        self.budget = int(budget)
        self.max_budget = max(self.budget, int(max_budget) if max_budget else BUDGET_GROWTH_CAP * self.budget)
        self.width = int(width)
        # wall-time target of one slice's launch (None: no target).  A launch over it halves the
        # budget (down to 1/BUDGET_GROWTH_CAP of the first), and the budget only grows while
        # launches stay under half of it -- so a node's worker never waits on a search slice
        # much longer than this between two batches of new puzzles.
        self.slice_target_s = None if slice_target_s is None else float(slice_target_s)
        self.min_budget = max(1, self.budget // BUDGET_GROWTH_CAP)
        self.t_node = None        # wall time per search node on a launch's critical path (measured)
        self.expand_cap = max(1, self.width // EXPAND_SHARE)   # budget hits expanded per slice, at most
        self.last_slice_s = 0.0   # wall time of the last slice, all of it
        self.max_slice_s = 0.0
        self.max_pending = int(max_pending)
        root_mask = ALL_DIGITS_MASK if mask is None else int(mask)
        # worklist: chunks (boards uint8[k,81], masks uint16[k]) in lex order of their subtrees
        self._chunks = collections.deque([(self.input[None].copy(), np.array([root_mask], np.uint16))])
        self._pending = 1
        self._expand_first = bool(hit)
        self.best = None          # lex-first completion found so far (only unrefuted boards precede it)
        self.status = None
        self.nodes = 0            # engine work (search nodes) spent
        self.launches = 0
        self.expansions = 0
        self.slices = 0

    @classmethod
    def for_node(cls, engine, board, mask=None, budget=None, width=None, max_pending=DEFAULT_MAX_PENDING,
                 slice_target_s=SLICE_TARGET_S):
        """A board whose batch launch hit the node budget, continued in slices of about
        slice_target_s each (node.py): DEFAULT_WIDTH sub-boards per device and slice, the first
        slice at the smallest budget, the later ones at what the measured node time allows."""
        b = default_budget(engine) if budget is None else int(budget)
        w = (DEFAULT_WIDTH if width is None else int(width)) * n_devices(engine)
        s = cls(engine, board, mask, budget=b, width=w, max_pending=max_pending, hit=True,
                slice_target_s=slice_target_s)
        s.budget = s.min_budget
        return s

    # ----------------------------------------------------------------- worklist
    def _take(self, k):
        boards, masks, got = [], [], 0
        while self._chunks and got < k:
            b, m = self._chunks.popleft()
            if got + len(b) > k:
                cut = k - got
                self._chunks.appendleft((b[cut:], m[cut:]))
                b, m = b[:cut], m[:cut]
            boards.append(b)
            masks.append(m)
            got += len(b)
        self._pending -= got
        if len(boards) == 1:
            return boards[0], masks[0]
        return np.concatenate(boards), np.concatenate(masks)

    def _push_front(self, boards, masks):
        if len(boards):
            self._chunks.appendleft((boards, masks))
            self._pending += len(boards)

    def _expand(self, boards, masks):
        t0 = time.monotonic()
        kids = self.engine.expand(boards, masks, target=max(self.width, 2 * len(boards)))
        self.expansions += 1
        if self.slice_target_s is not None:
            # fewer hits per expansion while one takes a large share of the slice
            dt = time.monotonic() - t0
            if dt > EXPAND_SHARE_OF_TARGET * self.slice_target_s:
                self.expand_cap = max(1, self.expand_cap // 2)
            elif 3 * dt < EXPAND_SHARE_OF_TARGET * self.slice_target_s:
                self.expand_cap = min(max(1, self.width // EXPAND_SHARE), 2 * self.expand_cap)
        return kids, np.full(len(kids), ALL_DIGITS_MASK, np.uint16)   # a mask lives in level 0 only

    @property
    def pending(self):
        return self._pending

    @property
    def done(self):
        return self.status is not None

    @property
    def board(self):
        return self.best.copy() if self.status == L.SDK_SOLVED else self.input.copy()

    def _finish(self, status):
        self.status = status
        self._chunks.clear()
        self._pending = 0

    # -------------------------------------------------------------------- slice
    def step(self):
        """One slice: one launch over the worklist's front (+ one expansion call).  Returns done."""
        if self.status is not None:
            return True
        t_slice = time.monotonic()
        try:
            return self._step()
        finally:
            self.last_slice_s = time.monotonic() - t_slice
            self.max_slice_s = max(self.max_slice_s, self.last_slice_s)

    def _step(self):
        self.slices += 1
        if self._expand_first:
            self._expand_first = False
            b, m = self._take(self._pending)
            self._push_front(*self._expand(b, m))
        if self._pending == 0:
            self._finish(L.SDK_SOLVED if self.best is not None else L.SDK_UNSOLVABLE)
            return True
        boards, masks = self._take(self.width)
        t0 = time.monotonic()
        # one bounded launch (no phased solve: this search is the continuation of heavy boards)
        out, st, work = self.engine.solve_batch(boards, masks, want_work=True, budget=self.budget, donate=0)
        elapsed = time.monotonic() - t0
        self.launches += 1
        if work is not None:
            work = np.asarray(work, dtype=np.uint64)
            self.nodes += int(work.sum())
            if self.slice_target_s is not None and len(work):
                # launch wall time per node of its longest board (its critical path): an upper
                # bound of the node time, so the budget derived from it keeps the launch short
                tn = elapsed / max(1, int(work.max()))
                self.t_node = tn if self.t_node is None else max(tn, 0.5 * (self.t_node + tn))
                self._cap_budget()
        st = np.asarray(st)
        decided = np.flatnonzero(st != L.SDK_UNSOLVABLE)          # refuted sub-boards simply vanish
        solved = decided[st[decided] == L.SDK_SOLVED]
        first = int(solved[0]) if len(solved) else None
        hits = decided if first is None else decided[decided < first]
        if first is not None:
            # every sub-board after it (the rest of the slice and the worklist) is lex-greater
            self.best = np.array(out[first], dtype=np.uint8)
            self._chunks.clear()
            self._pending = 0
        if len(hits):
            k = min(len(hits), self.expand_cap if self.slice_target_s is not None else max(1, self.width // EXPAND_SHARE))
            self._push_front(boards[hits[k:]], masks[hits[k:]])           # retried later, unexpanded
            self._push_front(*self._expand(boards[hits[:k]], masks[hits[:k]]))
            if self.slice_target_s is None:
                if 2 * len(hits) > len(boards):
                    self.budget = min(2 * self.budget, self.max_budget)
            else:
                self._bound_budget(elapsed, 2 * len(hits) > len(boards))
        if self._pending == 0:
            self._finish(L.SDK_SOLVED if self.best is not None else L.SDK_UNSOLVABLE)
            return True
        if self._pending > self.max_pending:
            self._finish(L.SDK_BUDGET_HIT)
            return True
        return False

    def _cap_budget(self):
        """budget x (measured node time) <= LAUNCH_SHARE x the slice target, before the next launch."""
        if self.slice_target_s is not None and self.t_node:
            self.budget = max(1, min(self.budget, int(LAUNCH_SHARE * self.slice_target_s / self.t_node)))

    def _bound_budget(self, launch_s, mostly_hits):
        """The next launch's budget (and width) under the slice target: grow while launches are
        fast and mostly hit the budget, halve after a slow one, and never above what the
        measured node time allows for LAUNCH_SHARE of the target."""
        target = self.slice_target_s
        if launch_s > LAUNCH_SHARE * target:
            self.budget = max(1, self.budget // 2)
        elif 2 * launch_s < LAUNCH_SHARE * target and mostly_hits:
            self.budget = min(2 * self.budget, self.max_budget)
        self._cap_budget()
        if self.budget == 1 and launch_s > LAUNCH_SHARE * target:
            # one node per board is still too long: the launch's fixed costs (copies) dominate
            self.width = max(MIN_WIDTH * n_devices(self.engine), self.width // 2)

    def run(self, deadline=None):
        """Slices until done or time.monotonic() passes `deadline` (then SDK_BUDGET_HIT)."""
        while not self.step():
            if deadline is not None and time.monotonic() >= deadline:
                self._finish(L.SDK_BUDGET_HIT)
                break
        return self.status, self.board


def solve_bounded(engine, boards, masks=None, budget=DEFAULT_BUDGET, time_limit=None, width=DEFAULT_WIDTH,
                  max_pending=DEFAULT_MAX_PENDING, max_budget=None):
    """solve_batch with every board bounded: one launch at `budget` nodes per board, then a
    LexSearch per board that hit it, each until done or `time_limit` seconds (None = no limit).
    Returns (out, status, work) like solve_batch; status SDK_BUDGET_HIT = search exhausted."""
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 81)
    out, st, work = engine.solve_batch(boards, masks, want_work=True, budget=budget, donate=0)
    out, st = np.array(out), np.array(st)
    work = np.zeros(len(boards), np.uint64) if work is None else np.array(work, dtype=np.uint64)
    for i in np.flatnonzero(st == L.SDK_BUDGET_HIT):
        m = None if masks is None else int(np.asarray(masks)[i])
        s = LexSearch(engine, boards[i], m, budget=budget, width=width, max_pending=max_pending, hit=True,
                      max_budget=max_budget)
        s.run(None if time_limit is None else time.monotonic() + time_limit)
        out[i], st[i] = s.board, s.status
        work[i] += np.uint64(s.nodes)
    return out, st, work
