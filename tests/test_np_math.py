"""The kernel's transcendentals == the reference NumPy's, bit for bit (CPU).

csrc/np_math.h restates glibc 2.35's __sin_fma/__cos_fma and NumPy 2.2.6's
SVML __svml_tan8_ha/__svml_pow8_ha (what np.sin, np.cos, np.tan and
np.power run on an AVX-512 host, the reference's arithmetic: SURVEY.md
§8(c)) instruction by instruction; oracle/npmath.cpp compiles the same header
for the host.  Each function is compared with NumPy itself on >= 16 M
arguments: latitudes (the RHS's sin/cos/tan), half-differences of positions
(cal_dis), error norms ** -0.2 and (0.01 / d) ** 0.2 (the step control), plus
wide random ranges, table-boundary points and special values.  The GPU runs
the same header (tests/test_gpu_np_math.py).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_devmath", "libnpmath.so")


def _svml_host():
    try:
        from numpy._core._multiarray_umath import __cpu_features__ as cf
    except ImportError:
        return False
    return bool(cf.get("AVX512_SKX"))


pytestmark = pytest.mark.skipif(not _svml_host(),
                                reason="this host's NumPy does not dispatch SVML (no AVX512_SKX): "
                                       "its tan/power are not the reference's")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(LIB)
    P, I = ctypes.c_void_p, ctypes.c_int64
    for n in ("nm_sin_arr", "nm_cos_arr", "nm_tan_arr", "nm_rcp14_arr"):
        getattr(lib, n).argtypes = [P, P, I]
    lib.nm_sincos_arr.argtypes = [P, P, P, I]
    lib.nm_sincostan_arr.argtypes = [P, P, P, P, I]
    lib.nm_sincostan_split_arr.argtypes = [P, P, P, P, I]
    lib.nm_pow_arr.argtypes = [P, P, I, P, I]
    return lib


def unary(lib, name, x):
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    getattr(lib, name)(x.ctypes.data, out.ctypes.data, x.size)
    return out


def power(lib, x, y):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(np.broadcast_to(y, x.shape), np.float64)
    out = np.empty_like(x)
    lib.nm_pow_arr(x.ctypes.data, y.ctypes.data, 1, out.ctypes.data, x.size)
    return out


def assert_bitwise(got, want, x, what):
    g = np.where(np.isnan(got), np.nan, got).view(np.int64)
    w = np.where(np.isnan(want), np.nan, want).view(np.int64)
    bad = np.nonzero(g != w)[0]
    assert bad.size == 0, (f"{what}: {bad.size} of {got.size} differ, e.g. x={x[bad[0]]!r}: "
                           f"{got[bad[0]]!r} vs NumPy {want[bad[0]]!r}")


def trig_args(rng, n):
    half_pi = np.pi / 2
    k = np.arange(-500, 501, dtype=np.float64)
    edges = np.concatenate([k / 128.0, k * np.pi / 16.0, [0.126, 0.855469, 2.426265, half_pi, np.pi]])
    edges = np.concatenate([edges, -edges])
    near = np.concatenate([np.nextafter(edges, np.inf), np.nextafter(edges, -np.inf), edges])
    return np.concatenate([
        rng.uniform(-half_pi, half_pi, n),                        # latitudes
        rng.uniform(-0.2, 0.2, n // 4),                           # half position steps
        rng.standard_normal(n // 4) * 10.0 ** rng.uniform(-30, 0, n // 4),
        rng.uniform(-200.0, 200.0, n // 4),                       # unwrapped longitudes
        rng.uniform(-6.5e4, 6.5e4, n // 8),
        near, [0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 1e-300, np.nan, np.inf, -np.inf]])


@pytest.mark.parametrize("fn", ["sin", "cos", "tan"])
def test_trig_bitwise_vs_numpy(lib, fn):
    x = trig_args(np.random.default_rng(1), 1 << 24)
    if fn == "tan":
        x = x[~(np.abs(x) > 65536.0)]          # beyond: SVML's Payne-Hanek path (not restated)
    with np.errstate(all="ignore"):
        want = getattr(np, fn)(x)
    assert_bitwise(unary(lib, f"nm_{fn}_arr", x), want, x, fn)


@pytest.mark.parametrize("y", [-0.2, 0.2])
def test_pow_step_control_bitwise_vs_numpy(lib, y):
    """error_norm ** -0.2 (rkf45.py:454,475) and (0.01 / max(d1, d2)) ** 0.2
    (rkf45.py:97) over every positive double magnitude, plus 0, inf, NaN."""
    rng = np.random.default_rng(2)
    n = 1 << 24
    x = np.concatenate([10.0 ** rng.uniform(-12, 4, n // 2),   # error norms in practice
                        rng.uniform(0.0, 3.0, n // 4),
                        10.0 ** rng.uniform(-323, 308, n // 4),
                        [0.0, -0.0, 1.0, 5e-324, 2.2250738585072014e-308, 1.7976931348623157e308,
                         np.inf, np.nan, 1.0 - 2 ** -53, 1.0 + 2 ** -52]])
    with np.errstate(all="ignore"):
        want = np.power(x, y)
    assert_bitwise(power(lib, x, y), want, x, f"pow(x, {y})")


def test_pow_general_main_path(lib):
    """Random exponents: every result SVML computes on its main path (|y log2 x|
    <= 1021.5) is bitwise NumPy's; C99 special values for x <= 0 and inf."""
    rng = np.random.default_rng(3)
    n = 1 << 22
    x = np.abs(rng.standard_normal(n) * 10.0 ** rng.uniform(-30, 30, n))
    y = rng.standard_normal(n) * 10.0 ** rng.uniform(-2, 1.5, n)
    with np.errstate(all="ignore"):
        main = np.abs(y * np.log2(x)) < 1000.0
        x, y = x[main], y[main]
        assert_bitwise(power(lib, x, y), np.power(x, y), x, "pow(x, y)")
        sx = np.array([0.0, -0.0, np.inf, -np.inf, -2.0, -0.5, 1.0, np.nan])
        sy = np.array([-0.2, 0.2, -1.0, 2.0, 3.0, -np.inf, np.inf, 0.0, np.nan, 0.5])
        xx, yy = np.meshgrid(sx, sy)
        assert_bitwise(power(lib, xx.ravel(), yy.ravel()), np.power(xx.ravel(), yy.ravel()),
                       xx.ravel(), "pow special values")


def test_fused_sincos_is_sin_and_cos(lib):
    """nm_sincos (one do_sin + one do_cos per lane, the kernels' RHS form) ==
    np.sin and np.cos."""
    x = trig_args(np.random.default_rng(4), 1 << 23)
    s, c = np.empty_like(x), np.empty_like(x)
    lib.nm_sincos_arr(x.ctypes.data, s.ctypes.data, c.ctypes.data, x.size)
    with np.errstate(all="ignore"):
        assert_bitwise(s, np.sin(x), x, "sincos: sin")
        assert_bitwise(c, np.cos(x), x, "sincos: cos")


def test_fused_sincostan_is_sin_cos_tan(lib):
    """nm_sincostan (the RHS's latitude: one straight-line block, one
    rare-argument branch) == np.sin, np.cos and np.tan."""
    x = trig_args(np.random.default_rng(5), 1 << 22)
    x = x[~(np.abs(x) > 65536.0)]
    s, c, t = np.empty_like(x), np.empty_like(x), np.empty_like(x)
    lib.nm_sincostan_arr(x.ctypes.data, s.ctypes.data, c.ctypes.data, t.ctypes.data, x.size)
    with np.errstate(all="ignore"):
        assert_bitwise(s, np.sin(x), x, "sincostan: sin")
        assert_bitwise(c, np.cos(x), x, "sincostan: cos")
        assert_bitwise(t, np.tan(x), x, "sincostan: tan")


def test_split_sincostan_is_sin_cos_tan(lib):
    """The RHS's split form (nm_sincostan_begin before the lookup's refill
    branch, nm_sincostan_end after it) == np.sin, np.cos and np.tan."""
    x = trig_args(np.random.default_rng(6), 1 << 22)
    x = x[~(np.abs(x) > 65536.0)]
    s, c, t = np.empty_like(x), np.empty_like(x), np.empty_like(x)
    lib.nm_sincostan_split_arr(x.ctypes.data, s.ctypes.data, c.ctypes.data, t.ctypes.data, x.size)
    with np.errstate(all="ignore"):
        assert_bitwise(s, np.sin(x), x, "split sincostan: sin")
        assert_bitwise(c, np.cos(x), x, "split sincostan: cos")
        assert_bitwise(t, np.tan(x), x, "split sincostan: tan")


def test_rcp14_restatement(lib):
    """VRCP14PD as restated (top 16 fraction bits -> table) on this host's own
    instruction, if the Python process can reach it through NumPy's SVML: the
    SVML pow rounds it to 1/32 and the tests above exercise every bucket; here
    the table's shape: monotone, 16 fraction bits, exact at powers of two."""
    x = 1.0 + np.arange(65536) / 65536.0 + 2.0 ** -52
    r = unary(lib, "nm_rcp14_arr", x)
    assert np.all(np.diff(r) <= 0) and np.all(r * x < 1 + 2 ** -13) and np.all(r * x > 1 - 2 ** -13)
    assert np.all((r.view(np.int64) & ((1 << 36) - 1)) == 0)
    p2 = 2.0 ** np.arange(-1000, 1000, 7, dtype=np.float64)
    assert np.array_equal(unary(lib, "nm_rcp14_arr", p2), 1.0 / p2)
    assert np.array_equal(unary(lib, "nm_rcp14_arr", -x), -r)


def test_team_sin_or_cos_is_sin_and_cos(lib):
    """nm_sinorcostan_begin/_end (the ray teams' trigonometry: a lane pair or a
    quad shares a ray, each lane evaluates sin OR cos in one instruction
    stream from one table point) == NumPy's sin and cos bit for bit, with the
    same tan, on every argument class of the other tests."""
    lib.nm_sinorcos_arr.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int64]
    x = trig_args(np.random.default_rng(11), 1 << 23)
    x = x[~(np.abs(x) > 65536.0)]
    with np.errstate(all="ignore"):
        want = {0: np.sin(x), 1: np.cos(x)}
    want_tan = unary(lib, "nm_tan_arr", x)
    for flag in (0, 1):
        f = np.full(x.size, flag, np.int32)
        out, tn = np.empty_like(x), np.empty_like(x)
        lib.nm_sinorcos_arr(x.ctypes.data, f.ctypes.data, out.ctypes.data, tn.ctypes.data, x.size)
        assert_bitwise(out, want[flag], x, "cos" if flag else "sin")
        assert_bitwise(tn, want_tan, x, "tan")
