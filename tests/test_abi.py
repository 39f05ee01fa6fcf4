"""The C-ABI library loads and exports every symbol include/sudoku_hip.h declares.
No compute call is made (runs without a GPU)."""
import ctypes
import os
import re

from distributed_sudoku_solver_amd import _lib as L


def declared_symbols():
    text = open(L.HEADER).read()
    return sorted(set(re.findall(r"\b(sdk_[a-z0-9_]+)\s*\(", text)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(L.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert L.load().sdk_abi_version() == L.SDK_ABI_VERSION == 2


def test_library_is_gfx950_code_object():
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_library_does_not_link_the_oracle():
    data = open(L.LIB_PATH, "rb").read()
    assert b"orc_" not in data and b"liboracle" not in data


def test_error_path_without_gpu_is_clean():
    lib = L.load()
    n = ctypes.c_int(-1)
    assert lib.sdk_device_count(ctypes.byref(n)) == 0
    ctx = ctypes.c_void_p()
    if n.value == 0:
        assert lib.sdk_create(0, ctypes.byref(ctx)) != 0
        assert lib.sdk_last_error()
    assert lib.sdk_set_option(None, 1, 0) == L.SDK_EINVAL


def test_header_constants_match_binding():
    """Every #define SDK_* integer constant of the header has the same value in _lib.py."""
    text = open(L.HEADER).read()
    for name, value in re.findall(r"#define\s+(SDK_[A-Z0-9_]+)\s+(-?\d+)u?\b", text):
        if hasattr(L, name):
            assert getattr(L, name) == int(value), name
    for name in ("SDK_OPT_DONATE", "SDK_OPT_DONATED", "SDK_OPT_XCD_HEADS", "SDK_OPT_LOCKED"):
        assert hasattr(L, name), name
