"""The C-ABI library loads on the CPU-only build host and exports every declared symbol."""
import ctypes
import os
import re

import _hip as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "rwrt.h")).read()
    return sorted(set(re.findall(r"\b(rwrt_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding():
    assert header_symbols() == sorted(H.ABI_SYMBOLS)


def test_library_exports_every_symbol():
    lib = H.load()
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert "gfx950" in H.version()


def test_struct_layouts():
    # rwrt_grid: 2 x int32 + 4 x double; rwrt_params: 4 x double + 2 x int32 + double
    assert ctypes.sizeof(H.Grid) == 40
    assert ctypes.sizeof(H.Params) == 48


def test_argument_errors_are_reported_without_a_gpu():
    """Argument validation happens before any HIP call: NULL grid -> RWRT_ERR_ARG."""
    lib = H.load()
    st = lib.rwrt_rhs(None, None, 0, None, None, None)
    assert st == H.RWRT_ERR_ARG
    assert b"grid" in lib.rwrt_last_error()
    g = H.Grid(145, 73, 0.0, 0.04363323, -1.5707964, 0.04363323)
    p = H.Params(1e-6, 1e-6, 7.2, 0.2, 1081, 0, 7200.0)
    st = lib.rwrt_rk45_run(None, ctypes.byref(g), 16, 10, ctypes.byref(p), None, 0, 5, None, 0,
                           None, None, None, None, None, None)
    assert st == H.RWRT_ERR_ARG
    # the ray loop needs an execution context
    st = lib.rwrt_rk4_run(None, ctypes.byref(g), 16, 10, ctypes.byref(p), 1, 5, None, None, None,
                          None, None, None, None)
    assert st == H.RWRT_ERR_ARG and b"rwrt_ctx" in lib.rwrt_last_error()


def test_selftest_kinds_retired_are_errors():
    """Retired selftest kinds (17-22) are refused instead of aliasing another
    operation; a live kind with n = 0 is a no-op (no GPU needed)."""
    lib = H.load()
    for kind in range(17, 23):
        assert lib.rwrt_selftest_math(kind, 0, None, None, None, None) == H.RWRT_ERR_ARG
        assert b"retired" in lib.rwrt_last_error()
    for kind in (0, 12, 16, 23, 35):
        assert lib.rwrt_selftest_math(kind, 0, None, None, None, None) == H.RWRT_OK
    assert lib.rwrt_selftest_math(38, 0, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_selftest_math(36, 0, None, None, None, None) == H.RWRT_OK   # (jump verdicts, round 5)


def test_expand_tails_argument_errors():
    """rwrt_expand_tails (ABI 3) validates before touching the device."""
    lib = H.load()
    assert lib.rwrt_expand_tails(-1, 1, 5, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_expand_tails(16, 5, 5, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_expand_tails(16, 1, 5, None, None, None, None) == H.RWRT_ERR_ARG
    assert b"NULL" in lib.rwrt_last_error()
    assert lib.rwrt_expand_tails(0, 1, 5, None, None, None, None) == H.RWRT_OK


def test_row_slot_entry_points_validate():
    """ABI 4 (rwrt_row_slots, rwrt_rk45_run_slots, rwrt_expand_slots)
    validates before touching the device."""
    lib = H.load()
    assert lib.rwrt_row_slots(-1, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_row_slots(16, None, None, None, None) == H.RWRT_ERR_ARG
    assert b"NULL" in lib.rwrt_last_error()
    assert lib.rwrt_rk45_run_slots(None, None, None, 16, None, None, 1, 5, None, 0, None, None, None, None,
                                   None, None, None, None, None) == H.RWRT_ERR_ARG
    assert b"d_row_slot" in lib.rwrt_last_error()
    assert lib.rwrt_rk45_run_tv_slots(None, None, None, 16, None, None, 1, 5, None, 0, None, None, None, None,
                                      None, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_expand_slots(-1, 1, 5, None, None, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_expand_slots(16, 1, 5, None, None, None, None, None, None) == H.RWRT_ERR_ARG
    assert lib.rwrt_expand_slots(0, 1, 5, None, None, None, None, None, None) == H.RWRT_OK


def test_context_needs_a_device():
    """rwrt_ctx_create refuses a device that does not exist (none on the build
    host); destroying NULL is a no-op."""
    lib = H.load()
    h = ctypes.c_void_p()
    assert lib.rwrt_ctx_create(4096, ctypes.byref(h)) == H.RWRT_ERR_ARG
    assert not h.value
    assert lib.rwrt_ctx_destroy(None) == H.RWRT_OK


def test_host_fill_rows():
    """rwrt_host_fill_rows (host code, no GPU): the drop-in's row delivery
    equals copying the whole block, for scattered, edge, empty and full
    column sets; bad column lists are refused."""
    import numpy as np
    from hostio import fill_rows
    rng = np.random.default_rng(0)
    ncol, r = 1000, 9
    prev = rng.standard_normal(ncol)
    for cols in (np.array([], np.int64), np.array([0], np.int64), np.array([ncol - 1], np.int64),
                 np.array([0, 1, 2, 500, 998, 999], np.int64),
                 np.sort(rng.choice(ncol, 300, replace=False)).astype(np.int64),
                 np.arange(ncol, dtype=np.int64)):
        src = rng.standard_normal((r, len(cols)))
        want = np.tile(prev, (r, 1))
        want[:, cols] = src
        block = np.full((r + 2, ncol), np.nan)
        dst = block[1:1 + r]
        fill_rows(dst, prev, src, cols if len(cols) else None)
        assert np.array_equal(dst, want)
        assert np.isnan(block[0]).all() and np.isnan(block[-1]).all()
    lib = H.load()
    bad = np.array([3, 3], np.int64)
    dst = np.zeros((2, 10))
    src = np.zeros((2, 2))
    st = lib.rwrt_host_fill_rows(dst.ctypes.data, 2, 10, 10, prev.ctypes.data, src.ctypes.data, 2, 2,
                                 bad.ctypes.data)
    assert st == H.RWRT_ERR_ARG and b"ascending" in lib.rwrt_last_error()
