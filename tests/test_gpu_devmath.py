"""Bit-exact parity with libm taken out of the comparison.

The GPU path and the reference differ in one thing only: the last bit of
sin/cos/tan/pow (the device's ocml vs the reference NumPy's glibc/SVML).
The oracle can run with the device's transcendentals instead
(``rwrt_oracle.device_math()``, oracle/devmath.cpp = the kernel's
csrc/rwrt_math.h compiled for the host).  Then every operation on both sides
is the same IEEE operation in the same order, and whole 90-day C2 histories
-- 1 081 rows x 7 variables x 3 072 slots, RK45 and RK4 -- must agree BIT FOR
BIT, including every accept/reject decision (per-ray accepted-step counts).

1. the host restatement equals the device's functions bitwise (also the
   library routines the kernel replaces, and the reciprocal-refinement
   emulation ``RM_RECIP2``);
2. GPU histories == oracle(device math) histories, row by row (sha256 per row
   in tests/golden/devmath_C2_<kind>.npz, made by tests/golden/make_devmath.py).
"""
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from make_devmath import row_hashes  # noqa: E402

pytestmark = pytest.mark.gpu
KINDS = ["zonal", "nonzonal"]


def host(name, x, y=None):
    import rwrt_oracle as O
    lib = O._devmath_lib()
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty_like(x)
    if name == "pow":
        y = np.ascontiguousarray(np.broadcast_to(y, x.shape), np.float64)
        lib.dm_pow(x.ctypes.data, y.ctypes.data, 1, out.ctypes.data, x.size)
    else:
        getattr(lib, "dm_" + name)(x.ctypes.data, out.ctypes.data, x.size)
    return out


def same(a, b):
    """Bitwise equality (signed zeros distinguished, NaN payloads not)."""
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    b = np.where(np.isnan(b), np.nan, np.asarray(b, np.float64))
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def test_host_restatement_equals_device_math():
    from engine import selftest_math as dev
    rng = np.random.default_rng(11)
    n = 1 << 22
    lat = rng.uniform(-1.5707963267948966, 1.5707963267948966, n)
    wide = np.concatenate([rng.uniform(-8, 8, n // 4),
                           rng.standard_normal(n // 4) * 10.0 ** rng.uniform(-300, 9, n // 4),
                           np.pi / 4 * np.arange(-400, 401), np.nextafter(np.pi / 4 * np.arange(-400, 401), 9),
                           [0.0, -0.0, 5e-324, -1e-310, 2.0 ** 30 - 1, -2.0 ** 30 + 1]])
    wide = wide[np.abs(wide) < 2.0 ** 30]   # beyond: each side's library (Payne-Hanek), never a latitude
    for x in (lat, wide):
        for name in ("sin", "cos", "tan"):
            h = host(name, x)
            assert same(dev("sct_" + name, x), h), name       # the kernel's fused routine
            assert same(dev(name, x), h), name                # the device library's
    # pow at the step control's arguments (error norms ** -0.2, the initial
    # step's (0.01 / d) ** 0.2) and at random ones
    en = np.concatenate([10.0 ** rng.uniform(-20, 12, n), rng.uniform(0, 2, n // 4),
                         [0.0, 1.0, 1e-320, 1.7e308, np.inf, np.nan]])
    for y in (-0.2, 0.2):
        yy = np.full(en.shape, y)
        with np.errstate(all="ignore"):
            h = host("pow", en, yy)
            assert same(dev("rm_pow", en, yy), h), y
            assert same(dev("pow", en, yy), h), y
    xs = rng.standard_normal(n // 4) * 10.0 ** rng.uniform(-30, 30, n // 4)
    ys = rng.standard_normal(n // 4) * 10.0 ** rng.uniform(-2, 2, n // 4)
    ys[::7] = np.round(ys[::7])
    with np.errstate(all="ignore"):
        h = host("pow", xs, ys)
        assert same(dev("rm_pow", xs, ys), h)
        assert same(dev("pow", xs, ys), h)
    # RM_RECIP2: v_rcp_f64 + two Newton steps == the IEEE reciprocal on the
    # ranges where the routines use it (1 + mantissa in [5/3, 7/3) for log;
    # the reduced tangent in [-1.01, 1.01] for tan)
    for lo, hi in ((5.0 / 3.0, 7.0 / 3.0), (-1.01, 1.01)):
        b = rng.uniform(lo, hi, 4 * n)
        b = b[b != 0.0]
        assert same(dev("recip2", b), 1.0 / b), (lo, hi)
    ex = np.concatenate([rng.uniform(-745, 709, n // 4), [-1076.0, 1025.0, 0.0, np.nan]])
    assert same(dev("rm_exp", ex), host("exp", ex))


def run_rk45(kind, nt):
    from test_gpu_parity import run_c2
    hist, res = run_c2(kind, nt)
    return np.transpose(hist[:, :, :7], (2, 1, 0)), res.nacc.cpu().numpy()


def check_rows(got_sha, want_sha, hist, last):
    bad = np.nonzero(got_sha != want_sha)[0]
    if bad.size:
        i = int(bad[0])
        d = ~((hist[:, -1] == last) | (np.isnan(hist[:, -1]) & np.isnan(last)))
        raise AssertionError(f"{bad.size} of {len(want_sha)} rows differ, first row {i}; "
                             f"{int(d.any(0).sum())} of {last.shape[1]} slots differ in the last row")


@pytest.mark.parametrize("kind", KINDS)
def test_rk45_c2_90d_bitwise_with_device_math(kind):
    g = golden(f"devmath_C2_{kind}.npz")
    nt = int(g["nt"])
    hist, nacc = run_rk45(kind, nt)
    check_rows(row_hashes(hist), g["row_sha"], hist, g["last"])
    assert np.array_equal(nacc, g["nacc"])


@pytest.mark.parametrize("kind", KINDS)
def test_rk4_c2_90d_bitwise_with_device_math(kind):
    from test_gpu_parity import run_wr
    g = golden(f"devmath_C2_{kind}.npz")
    nt = int(g["nt"])
    hist = run_wr(kind, "C2", nt, "")
    check_rows(row_hashes(hist), g["rk4_row_sha"], hist, g["rk4_last"])


@pytest.mark.parametrize("fp32", [False, True])
def test_time_varying_c2_bitwise_with_device_math(fp32):
    """The time-varying path (fp64 levels: one level in the LDS cache, the
    other gathered; fp32 levels: both cached) over 2 days -- past the last
    level, where the time weight clips -- equals the oracle bit for bit."""
    import torch
    import rwrt_oracle as O
    import synthetic as S
    from test_gpu_time_varying import tv
    eng, ob, ob0 = tv(fp32)
    cfg = S.config("C2")
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = eng.initial_rows(slon, slat, cfg.zwn, cfg.freq).cpu().numpy()
    y0 = rows[:5].reshape(5, -1)
    nt = 25
    got = {}
    res = eng.integrate(torch.as_tensor(y0), nt, 7200.0, ttotal=(nt - 1) * 7200.0,
                        sink=lambda a, b, o: got.__setitem__(a, o.cpu().numpy().copy()))
    hist = np.concatenate([got[k] for k in sorted(got)], axis=1)       # rows 1..nt-1
    with np.errstate(all="ignore"), O.device_math():
        ref, nacc, _, st = O.ray_run(ob, y0.copy(), nt, 7200.0)
    assert st == 0
    g = np.transpose(hist[:, :, :7], (2, 1, 0))
    assert same(g, ref[:, 1:]), int((~((g == ref[:, 1:]) | (np.isnan(g) & np.isnan(ref[:, 1:])))).sum())
    assert np.array_equal(res.nacc.cpu().numpy(), nacc)


def test_interleaved_division_pair_is_ieee():
    """div2 (two IEEE divisions interleaved in inline asm) == a / b bit for bit,
    as either quotient of the pair, on random, extreme and special operands."""
    from engine import selftest_math as dev
    rng = np.random.default_rng(5)
    n = 1 << 21
    a = rng.standard_normal(n) * 10.0 ** rng.uniform(-308, 308, n)
    b = rng.standard_normal(n) * 10.0 ** rng.uniform(-308, 308, n)
    phys_a = rng.standard_normal(n) * 10.0 ** rng.uniform(-15, 8, n)
    phys_b = rng.uniform(0.01, 1.0, n) * rng.choice([-1, 1], n)
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
                   1.7976931348623157e308, -1.7976931348623157e308, 1.0, -1.0, 6.3712e6, 3.0, 0.1])
    ea, eb = np.meshgrid(sp, sp)
    a = np.concatenate([a, phys_a, ea.ravel(), rng.standard_normal(1000) * 1e-310,
                        np.full(1000, 1e308)])
    b = np.concatenate([b, phys_b, eb.ravel(), rng.standard_normal(1000) * 1e300,
                        rng.standard_normal(1000) * 1e-10])
    with np.errstate(all="ignore"):
        want = a / b
    assert same(dev("div2_first", a, b), want)
    assert same(dev("div2_second", a, b), want)
