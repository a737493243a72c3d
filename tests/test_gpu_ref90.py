"""90-day histories on the GPU == the reference's arithmetic, bit for bit.

tests/golden/ref90_C2_<kind>.npz hold the per-row sha256 of the oracle's C2
histories (1 081 rows x 7 variables x 3 072 slots) computed with NumPy's own
transcendentals -- the reference's arithmetic (the oracle is pinned bit-exact
to the reference, tests/test_oracle_golden.py).  The GPU must reproduce every
row, RK45 (with every accept/reject decision: per-ray accepted-step counts)
and RK4, on both backgrounds; the time-varying extension the same way against
the oracle's restatement of it.
"""
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from make_devmath import row_hashes  # noqa: E402

pytestmark = pytest.mark.gpu
KINDS = ["zonal", "nonzonal"]


def same(a, b):
    """Bitwise equality (signed zeros distinguished, NaN payloads not)."""
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    b = np.where(np.isnan(b), np.nan, np.asarray(b, np.float64))
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def check_rows(got_sha, want_sha, hist, last):
    bad = np.nonzero(got_sha != want_sha)[0]
    if bad.size:
        i = int(bad[0])
        d = ~((hist[:, -1] == last) | (np.isnan(hist[:, -1]) & np.isnan(last)))
        raise AssertionError(f"{bad.size} of {len(want_sha)} rows differ, first row {i}; "
                             f"{int(d.any(0).sum())} of {last.shape[1]} slots differ in the last row")


@pytest.mark.parametrize("kind", KINDS)
def test_rk45_c2_90d_bitwise_with_reference_arithmetic(kind):
    from test_gpu_parity import run_c2
    g = golden(f"ref90_C2_{kind}.npz")
    nt = int(g["nt"])
    hist, res = run_c2(kind, nt)
    hist = np.transpose(hist[:, :, :7], (2, 1, 0))
    check_rows(row_hashes(hist), g["row_sha"], hist, g["last"])
    assert np.array_equal(res.nacc.cpu().numpy(), g["nacc"])


@pytest.mark.parametrize("kind", KINDS)
def test_rk4_c2_90d_bitwise_with_reference_arithmetic(kind):
    from test_gpu_parity import run_wr
    g = golden(f"ref90_C2_{kind}.npz")
    nt = int(g["nt"])
    hist = run_wr(kind, "C2", nt, "")
    check_rows(row_hashes(hist), g["rk4_row_sha"], hist, g["rk4_last"])


@pytest.mark.refhost
@pytest.mark.parametrize("fp32", [False, True])
def test_time_varying_c2_bitwise_with_oracle(fp32):
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
    with np.errstate(all="ignore"):
        ref, nacc, _, st = O.ray_run(ob, y0.copy(), nt, 7200.0)
    assert st == 0
    g = np.transpose(hist[:, :, :7], (2, 1, 0))
    assert same(g, ref[:, 1:]), int((~((g == ref[:, 1:]) | (np.isnan(g) & np.isnan(ref[:, 1:])))).sum())
    assert np.array_equal(res.nacc.cpu().numpy(), nacc)


# The time-varying kernels on a basic state held constant in time: one fp64
# level (the C2 background, built on the device by rwrt_bs_ready) valid from
# t0 = 1e9 s, so that every ray time lies before it and the time weight clips
# to 0: g = g_0 (1 - 0) + g_0 0 == g_0 bit for bit (x + x * 0 == x for every
# finite x, signed zeros included).  The reference integrates exactly that
# state (fun ignores t, wr.py:784-789), so the rwrt_rk45_*_tv kernels --
# 64 rays per wave (VaryingBG<double>: one level in the LDS cache, one
# gathered), 32 (PairVaryingBG64: lane pairs), and the latency waves
# (BlockVaryingBG<double>) -- must give the reference's own rows and
# accepted-step counts ("reduce bitwise to the
# reference for a constant-in-time background").
TV_HELD = [(32, 0), (64, 0), (32, (64, 1))]


def held_engine(kind, lanes):
    import synthetic as S
    from engine import RayEngine
    from levels import Levels
    b = S.background(kind)
    lv = Levels(b["lat"], b["lon"], 1, t0=1e9, dt=6 * 3600.0)
    lv.set_level(0, b["u"], b["v"])
    eng = RayEngine.from_levels(lv, time_varying=True)
    assert eng.bg is not None
    eng.tv_lanes = lanes
    return eng


@pytest.mark.parametrize("lanes,team", TV_HELD, ids=["pair32", "lanes64", "latency_waves"])
@pytest.mark.parametrize("kind", KINDS)
def test_time_varying_kernels_held_state_equal_reference(kind, lanes, team):
    from test_gpu_parity import bitwise, run_c2
    eng = held_engine(kind, lanes)
    kw = dict(order_policy="cell", first_chunk=[6], team=team) if team else {}
    # the reference's own rows at 2 h, 1 d, 10 d and accepted steps (golden)
    g = golden(f"traj_C2_{kind}.npz")
    hist, res = run_c2(kind, int(g["nt"]), chunk=40 if team else None, eng=eng, **kw)
    for j, row in enumerate(g["rows"]):
        assert bitwise(hist[:, row, :7].T, g["hist"][:, j]), row
    assert np.array_equal(res.nacc.cpu().numpy(), g["nacc"])
    if team:
        assert any(l["n_heavy"] for l in eng.launch_log), eng.launch_log
    # every row of 90 days (the reference's arithmetic, oracle row hashes)
    g = golden(f"ref90_C2_{kind}.npz")
    nt = int(g["nt"])
    hist, res = run_c2(kind, nt, chunk=120 if team else None, eng=eng, **kw)
    hist = np.transpose(hist[:, :, :7], (2, 1, 0))
    check_rows(row_hashes(hist), g["row_sha"], hist, g["last"])
    assert np.array_equal(res.nacc.cpu().numpy(), g["nacc"])


def test_interleaved_division_pair_is_ieee():
    """div2 (two IEEE divisions interleaved in inline asm) == a / b bit for bit,
    as either quotient of the pair, on random, extreme and special operands."""
    from engine import selftest_math as dev
    rng = np.random.default_rng(5)
    n = 1 << 21
    with np.errstate(all="ignore"):
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
