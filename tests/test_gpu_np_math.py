"""The kernels' transcendentals on the GPU == the reference NumPy's, bit for bit.

The device evaluates csrc/np_math.h (glibc 2.35 __sin_fma/__cos_fma, SVML
__svml_tan8_ha/__svml_pow8_ha restated; the host build of the same header is
checked against NumPy in tests/test_np_math.py).  Here the device's own
results -- the plain routines and the forms the kernels call (k_*: the RHS's
sin/cos/tan of a latitude, the step control's pow) -- are compared with
NumPy on the same kinds of arguments, bit for bit, and the one
target-dependent piece, SVML pow's round-toward-zero / -infinity steps
(MODE.FP_ROUND switches on the GPU, embedded rounding on the host), with the
host on arguments that exercise them.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.refhost]


def bitwise(a, b):
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    b = np.where(np.isnan(b), np.nan, np.asarray(b, np.float64))
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def first_diff(got, want, x):
    g = np.where(np.isnan(got), np.nan, got).view(np.int64)
    w = np.where(np.isnan(want), np.nan, want).view(np.int64)
    bad = np.nonzero(g != w)[0]
    return f"{bad.size} differ, e.g. x={x[bad[0]]!r}: {got[bad[0]]!r} vs {want[bad[0]]!r}" if bad.size else ""


def test_trig_on_device_equals_numpy():
    from engine import selftest_math as dev
    from test_np_math import trig_args
    x = trig_args(np.random.default_rng(11), 1 << 22)
    with np.errstate(all="ignore"):
        for name, ref in (("sin", np.sin), ("cos", np.cos), ("tan", np.tan)):
            xx = x[~(np.abs(x) > 65536.0)] if name == "tan" else x
            want = ref(xx)
            for kind in ("nm_" + name, "k_" + name):
                got = dev(kind, xx)
                assert bitwise(got, want), (kind, first_diff(got, want, xx))


def test_pow_on_device_equals_numpy():
    from engine import selftest_math as dev
    rng = np.random.default_rng(12)
    n = 1 << 22
    x = np.concatenate([10.0 ** rng.uniform(-12, 4, n), rng.uniform(0.0, 3.0, n // 4),
                        10.0 ** rng.uniform(-323, 308, n // 4),
                        [0.0, -0.0, 1.0, 5e-324, 1.7976931348623157e308, np.inf, np.nan]])
    with np.errstate(all="ignore"):
        for y in (-0.2, 0.2):
            want = np.power(x, y)
            for kind in ("nm_pow", "k_pow"):
                got = dev(kind, x, np.full(x.shape, y))
                assert bitwise(got, want), (kind, y, first_diff(got, want, x))
        xs = np.abs(rng.standard_normal(n) * 10.0 ** rng.uniform(-30, 30, n))
        ys = rng.standard_normal(n) * 10.0 ** rng.uniform(-2, 1.5, n)
        main = np.abs(ys * np.log2(xs)) < 1000.0
        xs, ys = xs[main], ys[main]
        got, want = dev("nm_pow", xs, ys), np.power(xs, ys)
        assert bitwise(got, want), first_diff(got, want, xs)


def test_rcp14_on_device_equals_host():
    import ctypes
    import rwrt_oracle as O
    from engine import selftest_math as dev
    rng = np.random.default_rng(13)
    x = np.concatenate([rng.uniform(0.5, 4.0, 1 << 20) * rng.choice([-1, 1], 1 << 20),
                        1.0 + np.arange(65536) / 65536.0, 2.0 ** np.arange(-60, 60)])
    lib = O._devmath_lib()
    want = np.empty_like(x)
    lib.nm_rcp14_arr(ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(want.ctypes.data), x.size)
    assert bitwise(dev("nm_rcp14", x), want)
