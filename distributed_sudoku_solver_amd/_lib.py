"""ctypes binding of libsudoku_hip.so (C-ABI declared in include/sudoku_hip.h).

The shared library is built in-tree (distributed_sudoku_solver_amd/libsudoku_hip.so,
see csrc/Makefile or __graft_entry__.build()).  There is no fallback: if the
library is missing or fails to load, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDK_LIB_PATH", os.path.join(HERE, "libsudoku_hip.so"))
HEADER = os.path.join(os.path.dirname(HERE), "include", "sudoku_hip.h")

SDK_ABI_VERSION = 2
SDK_OK = 0
SDK_EINVAL = -1
SDK_EHIP = -2
SDK_ENOMEM = -3
SDK_ECOMM = -4

SDK_SOLVED = 1
SDK_UNSOLVABLE = 0
SDK_BUDGET_HIT = -2
SDK_BUDGET_CONTEXT = (1 << 64) - 1    # sdk_solve_batch_budget: use the context's SDK_OPT_NODE_BUDGET

SDK_CHECK_OK = 1
SDK_CHECK_RAW_NAMEERROR = 2

SDK_OPT_ORDER = 1
SDK_OPT_NODE_BUDGET = 2
SDK_OPT_WAVES_PER_CU = 3
SDK_OPT_CHECK_BLOCKS_PER_CU = 4
SDK_OPT_WORK_COUNTER = 5
SDK_OPT_DEVICE_CUS = 6
SDK_OPT_SOLVER = 7
SDK_OPT_WAVES_PER_CU2 = 8
SDK_OPT_CHECK_VARIANT = 9
SDK_OPT_SOLVE_CHUNK = 10
SDK_OPT_TIMING = 11
SDK_OPT_TIMER_EVENTS = 12
SDK_OPT_LOCKED = 13
SDK_OPT_XCD_HEADS = 14
SDK_OPT_DONATE = 15
SDK_OPT_DONATED = 16
SDK_OPT_SPLIT_BOARDS = 17
SDK_OPT_DONATE_MODE = 18
SDK_OPT_LEX_BOARDS = 19
SDK_OPT_DONATE_MAX = 20
SDK_OPT_DN_FAULT = 21
SDK_OPT_DONATE_HELPERS = 22
SDK_OPT_DONATE_RESUME = 23
SDK_OPT_RESUMED = 24
SDK_OPT_PROP32 = 25
SDK_OPT_PROP32_LC = 26
SDK_OPT_PROP32_MIN = 27
SDK_OPT_PROP32_UNDECIDED = 28
SDK_OPT_PROP32_HANDOVER = 29
SDK_OPT_PROP32_TAIL = 30
SDK_DONATE_CONTEXT = -1    # sdk_solve_batch_ex: use the context's SDK_OPT_DONATE
SDK_CHECK_REG1 = 0
SDK_CHECK_REG2 = 1
SDK_CHECK_GLDS2 = 2
SDK_CHECK_GLDS3 = 3
SDK_CHECK_GLDS4 = 4
SDK_CHECK_WAVE1 = 5
SDK_CHECK_WAVE2 = 6

SDK_SOLVER_WAVE = 0
SDK_SOLVER_HALFWAVE = 1
SDK_SOLVER_QUAD = 2
SDK_SOLVER_LANE = 3

SDK_WORK_NODES = 0
SDK_WORK_ROUNDS = 1
SDK_WORK_DEPTH = 2

SDK_ORDER_MRV_UNIQUE = 0
SDK_ORDER_LEX = 1

SDK_FRONTIER_COUNT = 0
SDK_FRONTIER_FIRST = 1

SDK_COMM_ID_BYTES = 128
SDK_COMM_U64 = 0
SDK_COMM_I64 = 1
SDK_COMM_U8 = 2
SDK_COMM_SUM = 0
SDK_COMM_MIN = 1
SDK_COMM_MAX = 2
SDK_COMM_SEND = 0
SDK_COMM_RECV = 1

# every symbol the header declares: name -> (restype, argtypes)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
SIGNATURES = {
    "sdk_abi_version": (ctypes.c_int, []),
    "sdk_last_error": (ctypes.c_char_p, []),
    "sdk_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "sdk_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "sdk_destroy": (ctypes.c_int, [_vp]),
    "sdk_set_option": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int64]),
    "sdk_get_option": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    "sdk_check_batch": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_check_batch_i64": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_solve_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz]),
    "sdk_solve_batch_budget": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint64]),
    "sdk_solve_batch_ex": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_uint64, ctypes.c_int64]),
    "sdk_frontier_boards_dev": (ctypes.c_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64)]),
    "sdk_frontier_load_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64]),
    "sdk_frontier_refine_range": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "sdk_frontier_refine_head": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_uint64)]),
    "sdk_comm_send_dev": (ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int]),
    "sdk_comm_recv_dev": (ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int]),
    "sdk_comm_p2p_dev": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, _vp]),
    "sdk_expand_boards": (ctypes.c_int, [_vp, _vp, _vp, _sz, ctypes.c_uint64, _vp, _sz,
                                         ctypes.POINTER(ctypes.c_uint64)]),
    "sdk_count_solutions": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_int8)]),
    "sdk_count_solutions_slice": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                                                 ctypes.POINTER(ctypes.c_int8)]),
    "sdk_frontier_build": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "sdk_frontier_refine": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp]),
    "sdk_frontier_count_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                              ctypes.c_uint64, _vp]),
    "sdk_frontier_first_dev": (ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp]),
    "sdk_comm_unique_id": (ctypes.c_int, [_vp]),
    "sdk_comm_init": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    "sdk_comm_init_all": (ctypes.c_int, [_vp, ctypes.c_int, _vp]),
    "sdk_comm_destroy": (ctypes.c_int, [_vp]),
    "sdk_comm_allreduce_dev": (ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int, ctypes.c_int]),
    "sdk_comm_broadcast_dev": (ctypes.c_int, [_vp, _vp, _sz, ctypes.c_int]),
    "sdk_comm_allgather_dev": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_dev_alloc": (ctypes.c_int, [_vp, _sz, ctypes.POINTER(_vp)]),
    "sdk_dev_free": (ctypes.c_int, [_vp, _vp]),
    "sdk_memcpy_h2d": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_memcpy_d2h": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_synchronize": (ctypes.c_int, [_vp]),
    "sdk_check_batch_dev": (ctypes.c_int, [_vp, _vp, _vp, _sz]),
    "sdk_solve_batch_dev": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _sz]),
    "sdk_timer_reset": (ctypes.c_int, [_vp]),
    "sdk_timer_read": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
}

_lib = None


class SudokuHipError(RuntimeError):
    pass


def load():
    """Load libsudoku_hip.so (once). Raises if it is missing: no CPU fallback exists."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SudokuHipError(
            f"{LIB_PATH} not found: build it with `make -C distributed_sudoku_solver_amd/csrc` "
            "or `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    # a library named by SDK_LIB_PATH (dev A/B builds of older commits) may predate newer
    # entry points; the in-tree library must export every one
    override = "SDK_LIB_PATH" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if override and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what=""):
    if rc != SDK_OK:
        msg = load().sdk_last_error()
        msg = msg.decode() if msg else ""
        raise SudokuHipError(f"{what} failed ({rc}): {msg}")
    return rc
