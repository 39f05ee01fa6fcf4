"""GPU-backed Sudoku node speaking the reference's HTTP and UDP protocol.

Wire compatibility with DHT_Node.py (protocolo.pdf):
  * UDP datagrams are pickled dicts with a 'method' key, the same 14 methods and
    fields as DHT_Node.py:221-416 (TASK carries 'sudoku', 'range', 'uuid' and,
    from an HTTP front end, 'initial_node').  Incoming datagrams go through a
    restricted unpickler that only admits the builtins and uuid.UUID the
    protocol uses (the reference's bare pickle.loads executes arbitrary code).
  * HTTP: POST /solve -> 201 {"solution": grid, "duration": s};
    GET /stats -> {"all": {"solved", "validations"}, "nodes": [...]} with the
    reference's "validation" key for remote entries (DHT_Node.py:591);
    GET /network -> {str(node): [str(pred), str(succ)]} (indent=4).
  * Ring membership, coordinator join, heartbeats to the predecessor, failure
    repair by the coordinator and re-execution of delegated tasks follow
    DHT_Node.py:52-62, 137-209, 260-330.

What changes (GPU-first):
  * TASKs are executed by a worker thread that drains the whole queue into ONE
    sdk_solve_batch launch (the reference serialises them on the UDP thread,
    DHT_Node.py:225-250); the UDP loop never blocks on a solve.
  * POST /solve hands its task straight to the worker and waits on an event
    instead of a 10-ms polling loop (DHT_Node.py:553-554).
  * No `sleep(2)` after a solution (DHT_Node.py:354,467) and an unsolvable
    puzzle answers 201 {"solution": null} instead of hanging.
  * `-d/--delay` keeps its role as a slow-node knob: milliseconds per search
    node spent by the engine (the reference sleeps per guess, DHT_Node.py:524).
  * Work splitting (DHT_Node.py:491-510): when the neighbour is free, a queued
    TASK is handed over whole (at NEEDWORK time, or when a TASK arrives while
    this node is busy); otherwise the next task's digit `range` is halved with
    split_array_in_middle (utils.py:1-9) just before the launch.  Unlike the
    reference, the node keeps the LOWER half and sends the upper half: its own
    half is solved in microseconds, so the lexicographically first completion
    (the single-node answer) is the one reported first.
  * A task without a completion is reported back: NO_SOLUTION {uuid, range,
    sudoku} to its `initial_node` (a new method; reference nodes ignore it).
    The HTTP origin answers 201 {"solution": null} once the failed ranges of
    its puzzle cover every digit, instead of hanging.
  * api="main" serves main.py's HTTP surface instead (main.py:356-406): POST
    /solve -> 201 {"solution"}; GET /stats (local counters only); GET /network
    -> {"node": "h:p", "predecessor": [h, p] | null, "neighbor": [h, p] | null}.
  * Every launch is bounded (SURVEY §7 hard parts 2 and 7): a batch gives each
    board `node_budget` search nodes (sdk_solve_batch_ex), so one hard board
    cannot hold back the others; a board that hits it is continued by a
    search.LexSearch in bounded slices (~SLICE_TARGET_S each: launch, expansion and
    copies) on a search thread of its own, with an engine context of its own
    (engine.fork(): its own HIP stream), so a new batch never waits behind a slice --
    the GPU runs both launches at once, and the node keeps answering POSTs, /stats
    and the ring.  A budget hit is never reported as NO_SOLUTION: the range stays
    open.  If the continued search gives up (`search_limit_s`, or its worklist
    outgrows search.DEFAULT_MAX_PENDING) the range is reported as EXHAUSTED {uuid,
    range, sudoku} (a new method; reference nodes ignore it) and the HTTP origin
    answers 504 {"solution": null, "exhausted": true, "error": ...} once no
    completion below that range can still arrive -- never a completion that might
    not be the lex-first one.
"""
import argparse
import collections
import io
import json
import pickle
import queue
import socket
import threading
import time
import uuid as uuidlib
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

from .engine import ALL_DIGITS_MASK, encode_solve_grid, range_to_mask
from .search import DEFAULT_MAX_PENDING, DEFAULT_WIDTH, SLICE_TARGET_S, LexSearch, default_budget
from .utils import split_array_in_middle
from . import _lib as L

RECV_BYTES = 1024          # DHT_Node.py:82,94
HEARTBEAT_S = 5.0          # DHT_Node.py:43
STATS_WAIT_S = 1.0         # DHT_Node.py:571
SEARCH_LIMIT_S = 10.0      # a budget-hit task's continued search gives up after this (EXHAUSTED)
DONE_UUIDS_KEPT = 1 << 16  # answered puzzles remembered (late duplicates are dropped)


class _RecentSet:
    """A set that forgets its oldest members beyond `cap` (the reference keeps no such
    state at all; unbounded it would grow with every puzzle the ring ever solved)."""

    def __init__(self, cap=DONE_UUIDS_KEPT):
        self.cap = cap
        self._d = collections.OrderedDict()

    def add(self, x):
        self._d[x] = None
        self._d.move_to_end(x)
        while len(self._d) > self.cap:
            self._d.popitem(last=False)

    def __contains__(self, x):
        return x in self._d

    def __len__(self):
        return len(self._d)


class _HardTask:
    """A TASK whose launch hit the node budget, continued by a LexSearch between batches."""

    def __init__(self, task, search, deadline):
        self.task, self.search, self.deadline = task, search, deadline


class _ProtocolUnpickler(pickle.Unpickler):
    """Admits exactly the types the protocol's dicts contain."""

    _ALLOWED = {("builtins", "range"), ("builtins", "tuple"), ("builtins", "list"), ("builtins", "dict"),
                ("builtins", "set"), ("builtins", "frozenset"), ("uuid", "UUID"), ("uuid", "SafeUUID")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing {module}.{name}")


def decode_datagram(data):
    return _ProtocolUnpickler(io.BytesIO(data)).load()


def encode_datagram(msg):
    return pickle.dumps(msg)


def _addr(a):
    return (a[0], int(a[1])) if a is not None else None


class SudokuNode:
    """One ring member.  `engine` is a SudokuEngine, a shard.MultiDeviceEngine (every GPU of
    the box: each drained batch and each search slice is sharded over them), or anything with
    solve_batch / expand.  `search_engine` continues budget-hit boards (default: engine.fork(),
    a second context on the same devices, or the engine itself if it cannot fork)."""

    def __init__(self, host, p2p_port, http_port, anchor=None, engine=None, delay_ms=0.0,
                 heartbeat_s=HEARTBEAT_S, stats_wait_s=STATS_WAIT_S, solve_timeout_s=600.0, log=False,
                 api="dht", split=True, trace=False, node_budget=None, search_limit_s=SEARCH_LIMIT_S,
                 search_width=DEFAULT_WIDTH, search_max_pending=DEFAULT_MAX_PENDING, search_engine=None,
                 slice_target_s=SLICE_TARGET_S):
        if api not in ("dht", "main"):
            raise ValueError("api must be 'dht' (DHT_Node.py) or 'main' (main.py)")
        self.api = api
        self.split = split
        self.host = host
        self.port = p2p_port
        self.http_port = http_port
        self.anchor = _addr(anchor)
        self.me = (host, p2p_port)
        self.delay_ms = float(delay_ms)
        self.heartbeat_s = heartbeat_s
        self.stats_wait_s = stats_wait_s
        self.solve_timeout_s = solve_timeout_s
        if node_budget is not None and node_budget < 1:
            raise ValueError("node_budget must be >= 1: an unbounded launch can hold the GPU forever")
        self._node_budget = None if node_budget is None else int(node_budget)
        self.search_limit_s = float(search_limit_s)
        self.search_width = int(search_width)
        self.search_max_pending = int(search_max_pending)
        self.slice_target_s = float(slice_target_s)
        self.log = log
        if engine is None:
            from .solver import default_engine
            engine = default_engine()
        self.engine = engine
        if search_engine is None:
            search_engine = engine.fork() if hasattr(engine, "fork") else engine
            self._own_search_engine = search_engine is not engine      # made here: closed by stop()
        else:
            self._own_search_engine = False
        self.search_engine = search_engine
        self.node_budget = self._node_budget or default_budget(engine)   # per board per launch
        # ring state (guarded by self.lock)
        self.lock = threading.RLock()
        self.network = []
        self.coordinator = None
        self.predecessor = None
        self.neighbor = None
        self.neighborfree = False
        self.inside = False
        self.last_heartbeat = time.time()
        # work state
        self.tasks = queue.Queue()               # pending TASK dicts
        self.neighbor_tasks = []                 # tasks handed to the neighbour (re-run on its failure)
        self.hard = []                           # _HardTask: budget-hit tasks (the search thread's round robin)
        self._leaving = False                    # graceful stop(): tasks still in hand go to the neighbour
        self.busy = False                        # the worker runs a batch
        self.searching = False                   # the search thread runs a slice
        self.done_uuids = _RecentSet()           # uuids already solved somewhere in the ring
        self.best = {}                           # uuid -> (lowest digit, grid): best ordered completion (origin only)
        self.waiters = {}                        # uuid -> (Event, [solution], puzzle, [failed mask, exhausted mask])
        self.trace = collections.deque(maxlen=4096) if trace else None   # (method, addr, range) sent
        self.validations = 0
        self.solved_count = 0
        self.stats_replies = {}
        self.running = False
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((host, p2p_port))
        self.sock.settimeout(0.2)
        self.port = self.sock.getsockname()[1]
        self.me = (host, self.port)
        self.httpd = _Server((host, http_port), _Handler)
        self.httpd.node = self
        self.httpd.daemon_threads = True
        self.http_port = self.httpd.server_address[1]
        self._threads = []
        self._work = threading.Condition()
        self._go = threading.Event()             # cleared by pause(): the worker holds its queue
        self._go.set()

    # ------------------------------------------------------------------ utils
    def _log(self, *a):
        if self.log:
            print(f"[node {self.port}]", *a, flush=True)

    def send(self, msg, addr):
        if self.trace is not None:
            self.trace.append((msg.get("method"), _addr(addr), msg.get("range")))
        try:
            self.sock.sendto(encode_datagram(msg), _addr(addr))
        except OSError as e:
            self._log("send failed", e)

    # -------------------------------------------------------------- lifecycle
    def start(self):
        self.running = True
        with self.lock:
            if self.anchor:
                self.send({"method": "JOIN_REQ", "requestor": self.me}, self.anchor)
            else:
                self.network = [self.me]
                self.coordinator = self.predecessor = self.neighbor = self.me
                self.inside = True
        for target in (self._udp_loop, self._worker_loop, self._search_loop, self._heartbeat_loop,
                       self.httpd.serve_forever):
            t = threading.Thread(target=target, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def wait_joined(self, timeout=5.0):
        t0 = time.time()
        while not self.inside and time.time() - t0 < timeout:
            time.sleep(0.01)
        return self.inside

    def stop(self, graceful=True):
        """Leave the ring: queued tasks go to the neighbour, the coordinator is told
        (DHT_Node.py:137-156); graceful=False simulates a crash."""
        if graceful and self.running:
            with self.lock:
                # from here on a task the worker or the search thread still holds (a slice or a
                # batch in flight) is handed on when it comes back (_keep_hard), not re-queued
                self._leaving = True
                pending = self._drain_queue() + [h.task for h in self.hard]
                self.hard = []
                if self.neighbor and self.neighbor != self.me:
                    for t in pending:
                        self.send(t, self.neighbor)
                if self.coordinator and self.coordinator != self.me:
                    self.send({"method": "NODE_FAILED", "node": self.me}, self.coordinator)
        self.running = False
        with self._work:
            self._work.notify_all()
        self.httpd.shutdown()
        self.httpd.server_close()
        self.sock.close()
        if self._own_search_engine:
            # the search thread ends after its current (bounded) slice; then its context goes
            for t in self._threads:
                if t is not threading.current_thread():
                    t.join(timeout=5.0)
            if not any(t.is_alive() for t in self._threads if t is not threading.current_thread()):
                self.search_engine.close()

    # ------------------------------------------------------------- UDP side
    def _udp_loop(self):
        while self.running:
            try:
                data, addr = self.sock.recvfrom(RECV_BYTES)
            except socket.timeout:
                continue
            except OSError:
                break
            try:
                msg = decode_datagram(data)
            except Exception as e:  # malformed or refused datagram
                self._log("dropped datagram:", e)
                continue
            if isinstance(msg, dict) and "method" in msg:
                try:
                    self.handle(msg, addr)
                except Exception as e:
                    self._log("handler error", msg.get("method"), e)

    def handle(self, msg, addr):
        fn = getattr(self, "_on_" + str(msg["method"]), None)
        if fn is None:
            return
        fn(msg)

    def _on_TASK(self, msg):
        try:
            _validate_task(msg)
        except (KeyError, TypeError, ValueError) as e:     # the reference catches per message too
            self._log("dropped malformed TASK:", e)
            return
        self.enqueue(msg)

    def _on_NEEDWORK(self, msg):
        with self.lock:
            self.neighborfree = True
        self._maybe_delegate()

    def _on_HEARTBEAT(self, msg):
        self.last_heartbeat = time.time()

    def _on_SOMETHING(self, msg):
        pass

    def _on_STOP(self, msg):
        threading.Thread(target=self.stop, daemon=True).start()

    def _on_NODE_FAILED(self, msg):
        self._node_failed(_addr(msg["node"]))

    def _on_JOIN_REQ(self, msg):
        joiner = _addr(msg["requestor"])
        with self.lock:
            if self.coordinator != self.me:
                self.send(msg, self.coordinator)
                return
            if joiner not in self.network:
                self.network.append(joiner)
            net = list(self.network)
            for node in net:
                if node != self.me:
                    self.send({"method": "UPDATE_NETWORK", "network": net, "coordinator": self.coordinator}, node)
            # joiner is appended last: it follows net[-2] and precedes net[0]; updates meant
            # for this node are applied below, not sent to itself (a late self-datagram
            # would reset neighborfree after the joiner's NEEDWORK arrived)
            if net[0] != self.me:
                self.send({"method": "UPDATE_PREDECESSOR", "predecessor": joiner}, net[0])
            if net[-2] != self.me:
                self.send({"method": "UPDATE_NEIGHBOR", "neighbor": joiner}, net[-2])
            self.send({"method": "JOIN_RES", "predecessor": net[-2], "neighbor": net[0], "network": net,
                       "coordinator": self.coordinator}, joiner)
            if net[0] == self.me:
                self.predecessor = joiner
            if net[-2] == self.me:
                self.neighbor = joiner
                self.neighborfree = False
                self.last_heartbeat = time.time()

    def _on_JOIN_RES(self, msg):
        with self.lock:
            self.predecessor = _addr(msg["predecessor"])
            self.neighbor = _addr(msg["neighbor"])
            self.network = [_addr(a) for a in msg["network"]]
            self.coordinator = _addr(msg["coordinator"])
            self.inside = True
            self.neighborfree = False
            self.last_heartbeat = time.time()
            idle = self._idle_locked()
        if idle and self.predecessor != self.me:
            self.send({"method": "NEEDWORK"}, self.predecessor)

    def _on_UPDATE_PREDECESSOR(self, msg):
        with self.lock:
            self.predecessor = _addr(msg["predecessor"])
            idle = self._idle_locked()
        if idle and self.predecessor != self.me:
            self.send({"method": "NEEDWORK"}, self.predecessor)

    def _on_UPDATE_NEIGHBOR(self, msg):
        with self.lock:
            self.neighbor = _addr(msg["neighbor"])
            self.neighborfree = False
            self.last_heartbeat = time.time()

    def _on_UPDATE_NETWORK(self, msg):
        with self.lock:
            self.network = [_addr(a) for a in msg["network"]]
            self.coordinator = _addr(msg["coordinator"])

    def _on_SOLUTION_FOUND(self, msg):
        with self.lock:
            self.solved_count += 1
        self._solution(msg.get("uuid"), msg.get("solution"), msg.get("range"))

    def _on_NO_SOLUTION(self, msg):
        self._failed(msg.get("uuid"), msg.get("range"), msg.get("sudoku"))

    def _on_EXHAUSTED(self, msg):
        self._failed(msg.get("uuid"), msg.get("range"), msg.get("sudoku"), exhausted=True)

    def _on_STATS_REQ(self, msg):
        with self.lock:
            peers = [n for n in self.network if n != self.me]
            v = self.validations
        for node in peers:
            self.send({"method": "STATS_RES", "validations": v, "address": self.me}, node)

    def _on_STATS_RES(self, msg):
        a = _addr(msg["address"])
        with self.lock:
            self.stats_replies[f"{a[0]}:{a[1]}"] = int(msg["validations"])

    # ----------------------------------------------------- membership repair
    def _heartbeat_loop(self):
        while self.running:
            with self.lock:
                pred, nb = self.predecessor, self.neighbor
            if pred and pred != self.me:
                self.send({"method": "HEARTBEAT"}, pred)
            else:
                self.last_heartbeat = time.time()
            if nb and nb != self.me and time.time() - self.last_heartbeat > 2 * self.heartbeat_s:
                self.last_heartbeat = time.time()
                self._node_failed(nb)
            time.sleep(self.heartbeat_s / 4)

    def _node_failed(self, dead):
        with self.lock:
            if self.coordinator == dead:
                self.coordinator = self.me
            if self.coordinator == self.me:
                if dead in self.network and len(self.network) > 1:
                    i = self.network.index(dead)
                    before = self.network[(i - 1) % len(self.network)]
                    after = self.network[(i + 1) % len(self.network)]
                    self.network.remove(dead)
                    if before == self.me:
                        self.neighbor, self.neighborfree = after, False
                        self.last_heartbeat = time.time()
                    else:
                        self.send({"method": "UPDATE_NEIGHBOR", "neighbor": after}, before)
                    if after == self.me:
                        self.predecessor = before
                    else:
                        self.send({"method": "UPDATE_PREDECESSOR", "predecessor": before}, after)
                    for node in self.network:
                        if node != self.me:
                            self.send({"method": "UPDATE_NETWORK", "network": list(self.network),
                                       "coordinator": self.coordinator}, node)
            else:
                self.send({"method": "NODE_FAILED", "node": dead}, self.coordinator)
            # re-run whatever was delegated to the (possibly dead) neighbour
            rerun, self.neighbor_tasks = self.neighbor_tasks, []
        for t in rerun:
            self.enqueue(t)

    # --------------------------------------------------------- task execution
    def enqueue(self, task):
        self.tasks.put(task)
        with self.lock:
            busy = self.busy
        if busy:                 # an idle neighbour takes what would wait behind the running batch
            self._maybe_delegate()
        with self._work:
            self._work.notify_all()

    def _drain_queue(self):
        out = []
        while True:
            try:
                out.append(self.tasks.get_nowait())
            except queue.Empty:
                return out

    def _purge(self, uid, above=None):
        """Drop the tasks of puzzle `uid` (only those whose lowest digit is above `above`, if given)."""
        def drop(t):
            return t.get("uuid") == uid and (above is None or _lowest_digit(t.get("range")) > above)
        keep = [t for t in self._drain_queue() if not drop(t)]
        for t in keep:
            self.tasks.put(t)
        self.neighbor_tasks = [t for t in self.neighbor_tasks if not drop(t)]
        self.hard = [h for h in self.hard if not drop(h.task)]

    def _maybe_delegate(self):
        """A free neighbour gets one queued task (DHT_Node.py:491-498) -- only while this node
        is busy (the reference hands work over from inside solve_sudoku); an idle node's
        worker takes its queue itself."""
        with self.lock:
            if not (self.busy and self.neighborfree and self.neighbor and self.neighbor != self.me):
                return
            try:
                t = self.tasks.get_nowait()
            except queue.Empty:
                return
            self.neighborfree = False
            self.neighbor_tasks.append(t)
            self.send(t, self.neighbor)

    def pause(self):
        """Hold the worker: TASKs queue up (and are batched together on resume())."""
        self._go.clear()

    def resume(self):
        self._go.set()
        with self._work:
            self._work.notify_all()

    def _idle_locked(self):
        return self.tasks.empty() and not self.hard and not self.busy and not self.searching

    def _worker_loop(self):
        """New TASKs: one batched launch per drained queue.  Budget-hit boards go to the search
        thread, so a batch never waits for a long search."""
        while self.running:
            with self._work:
                while self.running and (self.tasks.empty() or not self._go.is_set()):
                    self._work.wait(0.5)
            if not self.running:
                return
            with self.lock:
                batch = [t for t in self._drain_queue() if t.get("uuid") not in self.done_uuids]
                self.busy = bool(batch)
            if not batch:
                continue
            try:
                self._run_batch(batch)
            except Exception as e:      # the worker must survive a failed launch
                self._log("launch failed:", repr(e))
                for t in batch:
                    self._wake(t.get("uuid"), "error", error=repr(e))
            finally:
                with self.lock:
                    self.busy = False
                    pred = self.predecessor
                    idle = self._idle_locked()
            if idle and pred and pred != self.me:
                self.send({"method": "NEEDWORK"}, pred)        # DHT_Node.py:245-248

    def _search_loop(self):
        """Budget-hit searches, one bounded slice at a time, round robin (search.LexSearch on the
        node's search engine: its own context and stream, beside the worker's batches)."""
        while self.running:
            with self._work:
                while self.running and not self.hard:
                    self._work.wait(0.5)
            if not self.running:
                return
            with self.lock:
                h = self.hard.pop(0) if self.hard else None
                self.searching = h is not None
            if h is None:
                continue
            try:
                self._run_slice(h)
            except Exception as e:      # a failed slice answers its POST with 500; the thread goes on
                self._log("search slice failed:", repr(e))
                self._wake(h.task.get("uuid"), "error", error=repr(e))
            finally:
                with self.lock:
                    self.searching = False
                    pred = self.predecessor
                    idle = self._idle_locked()
            if idle and pred and pred != self.me:
                self.send({"method": "NEEDWORK"}, pred)

    def _split_for_neighbor(self, batch):
        """DHT_Node.py:491-510 at launch time: a free neighbour gets the upper half of the
        first splittable task's digit range (split_array_in_middle, utils.py:1-9); this node
        keeps the lower half, so its own (first reported) answer stays the lex-first one."""
        if not self.split:
            return
        with self.lock:
            if not (self.neighborfree and self.neighbor and self.neighbor != self.me):
                return
            for i, t in enumerate(batch):
                arr = t.get("range", range(1, 10))
                if len(arr) < 2:
                    continue
                lower, upper = split_array_in_middle(arr)
                half = dict(t, range=upper)
                batch[i] = dict(t, range=lower)
                self.neighborfree = False
                self.neighbor_tasks.append(half)
                nb = self.neighbor
                break
            else:
                return
        self.send(half, nb)

    def _spent(self, nodes):
        if self.delay_ms > 0:
            time.sleep(self.delay_ms * nodes / 1000.0)
        with self.lock:
            self.validations += nodes

    def _run_batch(self, batch):
        """All queued TASKs in one bounded launch (node_budget nodes per board)."""
        self._split_for_neighbor(batch)
        boards = np.stack([encode_solve_grid(t["sudoku"]) for t in batch])
        masks = np.array([range_to_mask(t.get("range", range(1, 10))) for t in batch], dtype=np.uint16)
        # one bounded launch: budget hits continue in search.LexSearch slices between batches
        out, status, work = self.engine.solve_batch(boards, masks, want_work=True, budget=self.node_budget, donate=0)
        self._spent(int(np.asarray(work).sum()))
        for t, b, m, o, st in zip(batch, boards, masks, out, status):
            if st == L.SDK_BUDGET_HIT:
                # not "no solution": the subtree is unexplored.  Continue it on the search thread
                s = LexSearch.for_node(self.search_engine, b, int(m), budget=self.node_budget,
                                       width=self.search_width, max_pending=self.search_max_pending,
                                       slice_target_s=self.slice_target_s)
                if self._keep_hard(_HardTask(t, s, time.monotonic() + self.search_limit_s)):
                    with self._work:
                        self._work.notify_all()
                    self._log("budget hit, continuing", t.get("uuid"))
            else:
                self._task_done(t, int(st), o)

    def _run_slice(self, h):
        """One bounded slice of a budget-hit task's search (search.LexSearch.step)."""
        with self.lock:
            if h.task.get("uuid") in self.done_uuids:
                return
        before = h.search.nodes
        done = h.search.step()
        self._spent(h.search.nodes - before)
        if not done and time.monotonic() >= h.deadline:
            done = True
            h.search.status = L.SDK_BUDGET_HIT
        if done:
            self._task_done(h.task, int(h.search.status), h.search.board)
        else:
            self._keep_hard(h)

    def _keep_hard(self, h):
        """Queue a budget-hit task for the search thread -- or, once a graceful stop() has drained
        the queues, hand it to the neighbour like the rest (the task of a slice in flight
        used to come back after the drain and wait out its POST).  Returns whether it was queued."""
        with self.lock:
            if h.task.get("uuid") in self.done_uuids:
                return False
            if not self._leaving:
                self.hard.append(h)
                return True
            nb = self.neighbor if self.neighbor and self.neighbor != self.me else None
        if nb:
            self.send(h.task, nb)
        return False

    def _task_done(self, t, st, o):
        """Report a finished task: its completion, 'no completion in this range' (NO_SOLUTION) or
        'search exhausted' (EXHAUSTED; the range stays undecided, so no higher-range completion
        is ever taken for the lex-first one)."""
        uid = t.get("uuid")
        if st == L.SDK_SOLVED:
            grid = [list(row) for row in t["sudoku"]]
            for r in range(9):
                for c in range(9):
                    if grid[r][c] == 0:
                        grid[r][c] = int(o[9 * r + c])
            self._solved(t, grid)
            return
        exhausted = st == L.SDK_BUDGET_HIT
        if exhausted:
            self._log("search exhausted for", uid)
        # tell the HTTP origin, which answers once its puzzle's ranges are decided
        origin = _addr(t.get("initial_node"))
        if origin is None or origin == self.me:
            self._failed(uid, t.get("range"), t["sudoku"], exhausted=exhausted)
        else:
            self.send({"method": "EXHAUSTED" if exhausted else "NO_SOLUTION", "uuid": uid,
                       "range": t.get("range", range(1, 10)), "sudoku": t["sudoku"], "node": self.me}, origin)

    def _solved(self, task, grid):
        """This node completed `task`: SOLUTION_FOUND to every peer (and the HTTP origin).  A
        task that came from an HTTP origin (it carries `initial_node`) also reports its digit
        range, so the origin can keep the reference's single-node answer (see _solution)."""
        uid = task.get("uuid")
        origin = _addr(task.get("initial_node"))
        arr = task.get("range", range(1, 10)) if origin is not None else None
        with self.lock:
            if uid is not None and uid in self.done_uuids:
                return
            self.solved_count += 1                       # perform_solving, DHT_Node.py:428
            peers = [n for n in self.network if n != self.me]
        if origin is not None and origin != self.me and origin not in peers:
            peers.append(origin)
        msg = {"method": "SOLUTION_FOUND", "solution": grid, "node": self.me, "uuid": uid}
        if arr is not None:
            msg["range"] = arr
        for node in peers:
            self.send(msg, node)
        self._solution(uid, grid, arr)

    def _solution(self, uid, grid, arr):
        """A completion of puzzle `uid` was found with its first empty cell in digit range `arr`.

        arr None (a reference node's report, or a split of a partial board): final, as in the
        reference (DHT_Node.py:348-387).  Otherwise ranges of one puzzle are ordered: tasks
        whose digits all lie above `arr` are dropped, lower ones keep running, and the HTTP
        origin answers with the lowest-range completion once every lower digit has failed --
        the lexicographically first completion, whichever node finishes first."""
        if uid is None:                              # main.py TASKs carry no uuid (main.py:359-360)
            return
        lo = _lowest_digit(arr) if arr is not None else None
        with self.lock:
            if uid in self.done_uuids:
                return
            if lo is None:
                self.done_uuids.add(uid)
                self._purge(uid)
                self.best.pop(uid, None)
                final = ("solution", grid)
            else:
                if uid in self.waiters:              # only the HTTP origin orders completions
                    best = self.best.get(uid)
                    if best is None or lo < best[0]:
                        self.best[uid] = (lo, grid)
                self._purge(uid, above=lo)
                final = self._decide(uid)
        if final is not None:
            self._wake(uid, *final)

    def _decide(self, uid):
        """(under self.lock) The origin's answer once it is determined, else None:
          ("solution", grid)  the best completion, every digit below its range failed;
          ("none", None)      every digit of the first empty cell failed;
          ("exhausted", None) the lowest undecided digit lies in an exhausted range, so no
                              completion that could still arrive is provably the lex-first one."""
        w = self.waiters.get(uid)
        if w is None:
            return None
        failed, exhausted = w[3]
        best = self.best.get(uid)
        verdict = None
        if best is not None:
            need = ((1 << best[0]) - 1) & ALL_DIGITS_MASK      # digits 1 .. lo-1
            if (failed & need) == need:
                verdict = ("solution", best[1])
        if verdict is None:
            rest = ALL_DIGITS_MASK & ~failed
            if rest == 0:
                verdict = ("none", None)
            elif exhausted & rest & -rest:
                verdict = ("exhausted", None)
        if verdict is not None:
            self.done_uuids.add(uid)
            self._purge(uid)
            self.best.pop(uid, None)
        return verdict

    def _failed(self, uid, arr, sudoku, exhausted=False):
        """A range of puzzle `uid` has no completion (or, `exhausted`, its search gave up): the
        HTTP origin answers once the ranges are decided (_decide; only reports about its own
        board count)."""
        try:
            m = range_to_mask(arr if arr is not None else range(1, 10))
            board = encode_solve_grid(sudoku)
        except (TypeError, ValueError):
            return
        with self.lock:
            w = self.waiters.get(uid)
            if w is None or not np.array_equal(w[2], board):
                return
            w[3][1 if exhausted else 0] |= m
            final = self._decide(uid)
        if final is not None:
            self._wake(uid, *final)

    def _wake(self, uid, kind, solution=None, error=None):
        with self.lock:
            w = self.waiters.get(uid)
        if w is not None:
            w[1].append(_Failure(error) if error is not None else
                        (_EXHAUSTED if kind == "exhausted" else solution))
            w[0].set()

    # ------------------------------------------------------------- HTTP side
    def solve_http(self, puzzle):
        uid = uuidlib.uuid4()
        ev = threading.Event()
        box = []
        task = {"method": "TASK", "sudoku": puzzle, "range": range(1, 10), "uuid": uid, "initial_node": self.me}
        _validate_task(task)
        with self.lock:
            self.waiters[uid] = (ev, box, encode_solve_grid(puzzle), [0, 0])
        self.enqueue(task)
        ok = ev.wait(self.solve_timeout_s)
        with self.lock:
            self.waiters.pop(uid, None)
            self.best.pop(uid, None)
        if not ok:
            raise TimeoutError("no solution reported in time")
        res = box[0] if box else None
        if isinstance(res, _Failure):
            raise RuntimeError(f"solve failed: {res.error}")
        if res is _EXHAUSTED:
            raise SearchExhaustedError("search exhausted: no answer within the node's search limits "
                                       "(the reference would still be searching, DHT_Node.py:553-554)")
        return res

    def stats(self):
        with self.lock:
            peers = [n for n in self.network if n != self.me]
            self.stats_replies = {}
        for node in peers:
            self.send({"method": "STATS_REQ"}, node)
        t0 = time.time()
        while peers and time.time() - t0 < self.stats_wait_s:
            with self.lock:
                if len(self.stats_replies) >= len(peers):
                    break
            time.sleep(0.005)
        with self.lock:
            replies = dict(self.stats_replies)
            mine = int(self.validations)
            solved = self.solved_count
        nodes = [{"address": f"{self.host}:{self.port}", "validations": mine}]
        nodes += [{"address": a, "validation": v} for a, v in replies.items()]   # reference key, DHT_Node.py:591
        return {"all": {"solved": solved, "validations": mine + sum(replies.values())}, "nodes": nodes}

    def stats_local(self):
        """main.py's /stats: this node's counters only (main.py:378-395)."""
        with self.lock:
            return {"all": {"solved": self.solved_count, "validations": int(self.validations)},
                    "nodes": [{"address": f"{self.host}:{self.port}", "validations": int(self.validations)}]}

    def network_view_main(self):
        """main.py's /network (main.py:397-406): tuples serialise as JSON lists."""
        with self.lock:
            pred = None if self.predecessor is None else list(self.predecessor)
            nb = None if self.neighbor is None else list(self.neighbor)
        return {"node": f"{self.host}:{self.port}", "predecessor": pred, "neighbor": nb}

    def network_view(self):
        with self.lock:
            net = list(self.network)
        n = len(net)
        return {str(a): [str(net[(i - 1) % n]), str(net[(i + 1) % n])] for i, a in enumerate(net)}


def _lowest_digit(arr):
    """Lowest digit 1..9 of a TASK range (10 if none)."""
    try:
        m = range_to_mask(arr if arr is not None else range(1, 10))
    except (TypeError, ValueError):
        return 1
    return (m & -m).bit_length() - 1 if m else 10


class _Failure:
    def __init__(self, error):
        self.error = error


_EXHAUSTED = object()


class SearchExhaustedError(Exception):
    """POST /solve of a puzzle whose search gave up (HTTP 504, "exhausted": true)."""


def _validate_task(msg):
    """Raise unless a TASK can be launched: a 9x9 (or flat 81) grid and an ascending 0..9 range."""
    encode_solve_grid(msg["sudoku"])
    range_to_mask(msg.get("range", range(1, 10)))


class _Server(ThreadingHTTPServer):
    # bursts of concurrent POST /solve are what the batched launch is for: the
    # socketserver default listen backlog of 5 would drop their connections
    request_queue_size = 256


class _Handler(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def _reply(self, code, obj, indent=None):
        body = json.dumps(obj, indent=indent).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def do_POST(self):
        node = self.server.node
        if self.path != "/solve":
            return self._reply(404, {"error": "not found"})
        t0 = time.time()
        try:
            n = int(self.headers.get("Content-Length", 0))
            puzzle = json.loads(self.rfile.read(n))["sudoku"]
            if len(puzzle) != 9 or any(len(row) != 9 for row in puzzle):
                raise ValueError("sudoku must be 9 rows of 9 cells")
        except Exception as e:
            return self._reply(400, {"error": str(e)})
        try:
            solution = node.solve_http(puzzle)
        except SearchExhaustedError as e:
            return self._reply(504, {"error": str(e), "solution": None, "exhausted": True,
                                     "duration": time.time() - t0})
        except TimeoutError as e:
            return self._reply(504, {"error": str(e)})
        except (ValueError, TypeError) as e:
            return self._reply(400, {"error": str(e)})
        except RuntimeError as e:
            return self._reply(500, {"error": str(e)})
        if node.api == "main":                                  # main.py:375
            return self._reply(201, {"solution": solution})
        self._reply(201, {"solution": solution, "duration": time.time() - t0})

    def do_GET(self):
        node = self.server.node
        if self.path == "/stats":
            return self._reply(200, node.stats_local() if node.api == "main" else node.stats())
        if self.path == "/network":
            if node.api == "main":
                return self._reply(200, node.network_view_main())
            return self._reply(200, node.network_view(), indent=4)
        self._reply(404, {"error": "not found"})


def main(argv=None):
    ap = argparse.ArgumentParser(description="GPU-backed distributed Sudoku solver node")
    ap.add_argument("-p", "--port", type=int, required=True, help="HTTP port")
    ap.add_argument("-s", "--p2p-port", type=int, required=True, help="UDP port")
    ap.add_argument("-a", "--anchor", type=str, help="host:port of a ring member to join")
    ap.add_argument("-d", "--delay", type=float, default=1.0, help="ms per engine search node (slow-node knob)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--api", choices=["dht", "main"], default="dht", help="HTTP surface: DHT_Node.py or main.py")
    args = ap.parse_args(argv)
    anchor = None
    if args.anchor:
        h, p = args.anchor.rsplit(":", 1)
        anchor = (h, int(p))
    from .engine import SudokuEngine
    node = SudokuNode(args.host, args.p2p_port, args.port, anchor, SudokuEngine(args.device), args.delay, log=True,
                      api=args.api)
    node.start()
    try:
        while True:
            time.sleep(1)
    except KeyboardInterrupt:
        node.stop()


if __name__ == "__main__":
    main()
