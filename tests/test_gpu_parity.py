"""GPU parity: the HIP ray integrator against the reference's golden vectors.

The golden vectors were produced by the reference itself (tests/golden/
make_golden.py imports /root/reference).  The kernels evaluate every
operation in the reference's order with IEEE division/sqrt and no FMA
contraction, and their sin/cos/tan/pow are the reference NumPy's own
(csrc/np_math.h: glibc's __sin_fma/__cos_fma and SVML's tan/pow, bitwise on
16 M+ arguments, tests/test_np_math.py).  So every tier is BIT-EXACT:
  T0  element kernels (Mercator point, RHS);
  T1  one DP5(4) attempt (stages, y_new, error norm);
  T2  trajectories: C2 at 2 h, 1 d, 10 d; C1 for all 90 days (1 081 rows);
  RK4 C2 10 days and C1 90 days.
(BASELINE.md's north-star tolerance, 1e-6 rad at the endpoints, is met with
margin: the difference is zero.)
"""

import numpy as np
import pytest
import torch

from conftest import golden
import synthetic as S

pytestmark = pytest.mark.gpu

KINDS = ["zonal", "nonzonal"]
_ENG = {}


def bs_of(kind):
    from bs import BS
    bg = S.background(kind)
    bs = BS(len(bg["lon"]), len(bg["lat"]))
    bs.load_arrays(**bg)
    bs.ready(xcyclic=True)
    return bs


def engine(kind):
    if kind not in _ENG:
        from engine import RayEngine
        _ENG[kind] = RayEngine.from_bs(bs_of(kind))
    return _ENG[kind]


def ulps(a, b):
    """Distance in units of the last place of max(|a|, |b|) (NaN == NaN -> 0)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    nan_a, nan_b = np.isnan(a), np.isnan(b)
    assert np.array_equal(nan_a, nan_b), "NaN pattern differs"
    a, b = np.where(nan_a, 0, a), np.where(nan_b, 0, b)
    scale = np.spacing(np.maximum(np.abs(a), np.abs(b)))
    with np.errstate(invalid="ignore", divide="ignore"):
        d = np.abs(a - b) / scale
    d[(a == b)] = 0
    return d


def test_library_is_the_hip_build():
    import _hip as H
    assert torch.cuda.is_available()
    assert "gfx950" in H.version()


# ------------------------------------------------------------------------ T0
@pytest.mark.parametrize("kind", KINDS)
def test_t0_mercator_point(kind):
    g = golden(f"merc_{kind}.npz")
    out = engine(kind).mercator_point(g["lon"], g["lat"]).cpu().numpy()
    assert bitwise(out, g["out"][:12])


@pytest.mark.parametrize("kind", KINDS)
def test_t0_rhs(kind):
    g = golden(f"rhs_{kind}.npz")
    out = engine(kind).rhs(g["y"]).cpu().numpy()
    assert bitwise(out, g["dydt"])


# ------------------------------------------------------------------------ T1
@pytest.mark.parametrize("kind", KINDS)
def test_t1_single_attempt(kind):
    g = golden(f"step_{kind}.npz")
    K, yn, err = engine(kind).attempt(g["y"], g["f"], g["h"])
    K, yn, err = K.cpu().numpy(), yn.cpu().numpy(), err.cpu().numpy()
    assert bitwise(K, g["K"])
    assert bitwise(yn, g["y_new"])
    assert bitwise(err, g["err_norm"])


@pytest.mark.parametrize("kind", KINDS)
def test_initial_step(kind):
    g = golden(f"init_C2_{kind}.npz")
    eng = engine(kind)
    y0 = g["rows"][:5].reshape(5, -1)
    p = eng.params(121, 7200.0)
    st = eng.init(torch.as_tensor(y0), p)
    state = st["state"].cpu().numpy()
    f0, h = state[5:10], state[11]
    assert bitwise(h, g["h_abs"])
    assert bitwise(f0, g["f0"])
    live = st["live"].cpu().numpy()
    assert live.sum() == int(st["summary"][0])


def bitwise(a, b):
    """Equal bit for bit (signed zeros distinguished; NaN == NaN)."""
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    b = np.where(np.isnan(b), np.nan, np.asarray(b, np.float64))
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


# ------------------------------------------------------------ initial rays
def same_bits(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("kind", KINDS)
def test_initial_rows_gpu_bitwise_c2(kind):
    """rwrt_ray_initial (Mercator point, np.roots restated, change_roots_order,
    t = 0 group velocity) == the reference's row 0 of C2, bit for bit."""
    from wr import WR
    g = golden(f"init_C2_{kind}.npz")
    cfg = S.config("C2")
    w = WR(cfg.nzwn, cfg.nsource, 7200.0, 7200.0, cfg.freq, nx=144, ny=73)
    w.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = engine(kind).initial_rows(w.source_lon, w.source_lat, cfg.zwn, cfg.freq)
    assert same_bits(rows.cpu().numpy(), g["rows"])


@pytest.mark.parametrize("kind", KINDS)
def test_initial_rows_gpu_bitwise_c3_golden(kind):
    """The reference's C3 roots subsample (stationary and 10-day waves): m, amp,
    ug, vg bit-identical -- including the ORDER of the three roots."""
    g = golden("roots_C3.npz")
    cfg = S.config("C3")
    for tag in ("stat", "p10"):
        src = g[f"{tag}_{kind}_src"]
        rows = engine(kind).initial_rows(src[0], src[1], cfg.zwn, float(g[f"{tag}_{kind}_freq"]))
        got = rows.cpu().numpy()[[3, 4, 5, 6]]
        assert same_bits(got, g[f"{tag}_{kind}_rows"]), tag


@pytest.mark.refhost
@pytest.mark.parametrize("kind", KINDS)
def test_initial_rows_gpu_equals_host_full_c3(kind):
    """All 2.40 M C3 slots (5 periods): GPU rows == host rows (the host path is
    bit-exact with the reference, tests/test_host_prep.py)."""
    from wr import initial_rows
    cfg = S.config("C3")
    bs = bs_of(kind)
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * (np.pi / 180.0)
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * (np.pi / 180.0)
    for P in S.C3_PERIODS_DAYS:
        f = S.c3_freq(P)
        with np.errstate(all="ignore"):
            host = np.array(initial_rows(bs, lon, lat, cfg.zwn, f))
        dev = engine(kind).initial_rows(lon, lat, cfg.zwn, f).cpu().numpy()
        bad = ~((dev == host) | (np.isnan(dev) & np.isnan(host)))
        assert not bad.any(), (P, int(bad.sum()))


# ------------------------------------------------------------------- T2 / T3
def run_c2(kind, nt, chunk=None, order=None, eng=None, **kw):
    from engine import t_eval_of
    g = golden(f"init_C2_{kind}.npz")
    eng = eng or engine(kind)
    y0 = torch.as_tensor(g["rows"][:5].reshape(5, -1))
    rows = {}

    def sink(i0, i1, out):
        rows[(i0, i1)] = out.cpu().numpy().copy()

    res = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=chunk, sink=sink, **kw)
    nray = y0.shape[1]
    hist = np.full((nray, nt, 8), np.nan)
    hist[:, 0, :7] = g["rows"].reshape(7, -1).T
    for (i0, i1), r in rows.items():
        hist[:, i0:i1] = r
    return hist, res


@pytest.mark.parametrize("kind", KINDS)
def test_t2_c2_trajectories(kind):
    """C2 (3 072 slots) against the reference's own rows at 2 h, 1 d and 10 d
    and its per-ray accepted-step counts: identical bit for bit."""
    g = golden(f"traj_C2_{kind}.npz")
    hist, res = run_c2(kind, int(g["nt"]))
    ref = g["hist"]                          # (7, len(rows), nray)
    for j, row in enumerate(g["rows"]):
        assert bitwise(hist[:, row, :7].T, ref[:, j]), row
    assert np.array_equal(res.nacc.cpu().numpy(), g["nacc"])


def test_t2_c1_90d_bitwise():
    """C1 through the reference's entry point: every one of the 1 081 rows of
    the reference's own 90-day history, bit for bit."""
    g = golden("traj_C1.npz")
    nt = int(g["nt"])
    from wr import WR
    cfg = S.config("C1")
    bs = bs_of("zonal")
    wr = WR(cfg.nzwn, cfg.nsource, 7200.0, 90 * 86400.0, 0.0, nx=bs.nlon, ny=bs.nlat)
    wr.bs = bs
    wr.set_zwn(cfg.zwn)
    wr.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        res = wr.ray_run(mode="hip", inte_method="rk45")
    hist = np.array([wr.rlon, wr.rlat, wr.rzwn, wr.rmwn, wr.ramp, wr.rug, wr.rvg]).reshape(7, nt, -1)
    assert bitwise(hist, g["hist"])
    assert np.array_equal(res.nacc.cpu().numpy(), np.asarray(g["nacc"]).reshape(-1))


# --------------------------------------------------------- structural props
def test_time_chunking_is_bitwise_invisible():
    h1, r1 = run_c2("nonzonal", 25)
    h2, r2 = run_c2("nonzonal", 25, chunk=5)
    assert np.array_equal(h1, h2, equal_nan=True)
    assert torch.equal(r1.nacc, r2.nacc)


def test_frozen_rays_filled_like_the_run_kernel():
    """Rays frozen at a launch start (dead slots, rays masked in an earlier
    chunk) are written by frozen_fill_kernel on a side stream; chunked runs,
    where many rays enter later chunks frozen, equal one launch bit for bit
    (rows, accepted/rejected counts, first-NaN rows, the early-exit row)."""
    h1, r1 = run_c2("nonzonal", 241)
    h2, r2 = run_c2("nonzonal", 241, chunk=40)
    frozen_later = np.isnan(h1[:, 40, 0]) & ~np.isnan(h1[:, 0, 3])
    assert frozen_later.sum() > 0            # rays masked in the first chunk exist
    assert np.array_equal(h1, h2, equal_nan=True)
    assert torch.equal(r1.nacc, r2.nacc) and torch.equal(r1.nrej, r2.nrej)
    assert torch.equal(r1.nanrow, r2.nanrow) and r1.break_row == r2.break_row


def test_sharding_is_bitwise_invisible():
    """Rays are independent: any split into shards reproduces the unsharded run."""
    g = golden("init_C2_nonzonal.npz")
    eng = engine("nonzonal")
    y0 = torch.as_tensor(g["rows"][:5].reshape(5, -1))
    full = {}
    eng.integrate(y0, 13, 7200.0, sink=lambda a, b, o: full.setdefault(0, o.cpu().numpy().copy()))
    parts = []
    for s in range(3):
        idx = torch.arange(s, y0.shape[1], 3)
        out = {}
        eng.integrate(y0[:, idx].contiguous(), 13, 7200.0,
                      sink=lambda a, b, o: out.setdefault(0, o.cpu().numpy().copy()))
        parts.append((idx.numpy(), out[0]))
    for idx, o in parts:
        assert np.array_equal(full[0][idx], o, equal_nan=True)


# ----------------------------------------------------------------- KATs
def test_kat_stepper():
    from engine import kat_rk45
    g = golden("kat_stepper.npz")
    ts = g["t_eval"]
    lin = kat_rk45(0, g["lin_y0"], ts, 1e-3, 1e-6, 0.001).cpu().numpy()
    assert np.max(np.abs(lin[:, 0, 0] - (ts ** 2 + 0.1))) < 1e-10
    assert np.max(np.abs(lin - g["lin_ys"])) < 1e-10
    ex = kat_rk45(1, g["exp_y0"], ts, 1e-14, 1e-15, 0.001).cpu().numpy()
    exact = 10 * np.exp(0.1 * ts) + 0.0
    assert np.max(np.abs(ex[:, 0, 0] - exact) / exact) < 1e-13
    assert np.max(np.abs(ex - g["exp_ys"]) / np.abs(g["exp_ys"])) < 1e-13
    lo = kat_rk45(2, g["lorenz_y0"], ts, 1e-3, 1e-6, 0.001).cpu().numpy()
    k = np.searchsorted(ts, 2.0)
    assert np.max(np.abs(lo[:k] - g["lorenz_ys"][:k])) < 1e-6


# ------------------------------------------------------------ device math
def test_device_math_exactness():
    """IEEE division, sqrt, floor and the Python modulo are bit-exact on the GPU;
    sin/cos/tan/pow/atan2 agree with NumPy in the last bit for most inputs
    (the residual is what bounds trajectory parity; rates recorded in DESIGN.md)."""
    from engine import selftest_math
    rng = np.random.default_rng(7)
    n = 1 << 20
    a = rng.uniform(-1e3, 1e3, n) * 10 ** rng.uniform(-6, 2, n)
    b = rng.uniform(0.1, 10, n) * rng.choice([-1, 1], n)
    assert np.array_equal(selftest_math("div", a, b), a / b)
    pos = np.abs(a)
    assert np.array_equal(selftest_math("sqrt", pos), np.sqrt(pos))
    assert np.array_equal(selftest_math("floor", a), np.floor(a))
    lon = np.concatenate([rng.uniform(-60, 80, n), [-0.0, 0.0, -1e-300, 2 * np.pi, -2 * np.pi]])
    assert np.array_equal(selftest_math("mod", lon, np.full(lon.shape, 2 * np.pi)),
                          lon % (2 * np.pi))
    lat = rng.uniform(-1.5707963, 1.5707963, n)
    # the kernels' shortcuts are bit-identical to the operations they replace
    assert np.array_equal(selftest_math("sincos_sin", lat), selftest_math("sin", lat))
    assert np.array_equal(selftest_math("sincos_cos", lat), selftest_math("cos", lat))
    wide = rng.standard_normal(4 * n) * 10.0 ** rng.uniform(-300, 300, 4 * n)
    wide = np.concatenate([wide, [0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -1e-310,
                                  1.7e308, 6.3712e6, -6.3712e6 * 3]])
    with np.errstate(all="ignore"):
        assert np.array_equal(selftest_math("div_rearth", wide), wide / 6.3712e6, equal_nan=True)
    phys = rng.standard_normal(4 * n) * 10.0 ** rng.uniform(-12, 4, 4 * n)
    assert np.array_equal(selftest_math("div_rearth", phys), phys / 6.3712e6)
    zeros = np.array([0.0, -0.0, 1e-300, -1e-300, 2.0 ** -900, -(2.0 ** -900), 2.0 ** 900])
    with np.errstate(all="ignore"):
        dz = selftest_math("div_rearth", zeros)
        assert np.array_equal(dz.view(np.int64), (zeros / 6.3712e6).view(np.int64))
    tp = 2 * np.pi
    near = np.concatenate([np.arange(-200, 200) * tp, np.nextafter(np.arange(-200, 200) * tp, np.inf),
                           np.nextafter(np.arange(-200, 200) * tp, -np.inf),
                           rng.uniform(-1e4, 1e4, n), rng.uniform(-1e13, 1e13, 1000),
                           [1e300, -1e300, np.inf, np.nan, 0.0, -0.0]])
    with np.errstate(all="ignore"):
        assert np.array_equal(selftest_math("fmod", near, np.full(near.shape, tp)),
                              np.fmod(near, tp), equal_nan=True)
    # the kernels' x % (2 pi) (reciprocal quotient) and the second reduction
    # of interpolation.py:80 (a clamp) equal NumPy's
    wrap = np.concatenate([lon, near[np.isfinite(near)], -near[np.isfinite(near)],
                           np.nextafter(-0.0, -1) * np.arange(1, 50), [np.inf, np.nan]])
    with np.errstate(all="ignore"):
        assert np.array_equal(selftest_math("mod2pi", wrap), wrap % tp, equal_nan=True)
        assert np.array_equal(selftest_math("mod2pi_twice", wrap), (wrap % tp) % tp, equal_nan=True)
    # shared-reciprocal division (lookup cell coordinates): bit-identical to
    # IEEE division for every numerator/divisor, including the fallbacks
    num = np.concatenate([wide, phys, a, [0.0, -0.0, 2.0 ** -900, -2.0 ** -901, 2.0 ** 600,
                                          2.0 ** 599, 5e-324]])
    for den in (0.04363323259353638, -2.5, 1.0, 3.0, 2.0 ** -100, 2.0 ** 100, 2.0 ** -101,
                7.3e-200, 1e300, 5e-324, 0.0, -0.0, np.inf, np.nan):
        dd = np.full(num.shape, den)
        with np.errstate(all="ignore"):
            assert np.array_equal(selftest_math("div_hw", num, dd), num / dd, equal_nan=True), den
    both = rng.standard_normal(n) * 10.0 ** rng.uniform(-150, 150, n)
    assert np.array_equal(selftest_math("div_hw", phys[:n], both), phys[:n] / both)
    assert np.array_equal(np.signbit(selftest_math("div_hw", num, np.full(num.shape, -2.5))),
                          np.signbit(num / -2.5))
    # the RHS's shared-reciprocal division (qdiv, csrc/rwrt.hip): wherever
    # DivGuard admits it, bit-identical to IEEE division -- signed zeros,
    # inf and NaN numerators (v_div_fixup) and NaN / inf / zero divisors
    # included; physical operands are always admitted
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -2.0 ** -1000, 2.0 ** -899,
                         -2.0 ** -900, 2.0 ** 599, -2.0 ** 600, 1.7e308, 1.0, -3.0])
    dens = np.array([0.0175, 0.5, 1.0, 6.3712e6, 2.5, -2.5, 2.0 ** -99, 2.0 ** -100, 2.0 ** 99,
                     2.0 ** 100, 2.0 ** 101, 1e-300, 1e300, 0.0, -0.0, np.inf, -np.inf, np.nan])
    nn = np.concatenate([wide, phys, np.repeat(specials, 64)])
    for den in dens:
        dd = np.full(nn.shape, den)
        inr = selftest_math("qdiv_exact_range", nn, dd) == 1.0
        with np.errstate(all="ignore"):
            want = nn / dd
        got = selftest_math("qdiv", nn, dd)
        assert np.array_equal(got[inr], want[inr], equal_nan=True), den
        m = inr & ~np.isnan(want)
        assert np.array_equal(np.signbit(got[m]), np.signbit(want[m])), den
        if 2.0 ** -99 <= abs(den) <= 2.0 ** 99:
            sp = np.isin(nn, specials[:5]) | np.isnan(nn)
            assert inr[sp].all(), den              # zeros, inf, NaN: on the fast path
    ph = rng.standard_normal(n) * 10.0 ** rng.uniform(-40, 40, n)
    pd = rng.uniform(0.0175, 1.0, n) * 10.0 ** rng.integers(-20, 20, n)
    assert (selftest_math("qdiv_exact_range", ph, pd) == 1.0).all()
    assert np.array_equal(selftest_math("qdiv", ph, pd), ph / pd)
    # np.floor(x).astype('int32') (x86 semantics: NaN / out of range -> INT32_MIN)
    fx = np.concatenate([a, [2.0 ** 31 - 1, 2.0 ** 31 - 0.5, 2.0 ** 31, -2.0 ** 31, -2.0 ** 31 - 1,
                             1e300, -1e300, np.inf, -np.inf]])
    with np.errstate(all="ignore"):
        want = np.floor(fx).astype(np.int32).astype(np.float64)
    assert np.array_equal(selftest_math("floor_i32", fx), want)



@pytest.mark.gpu
def test_jump_verdict_fast_path_near_threshold():
    """The jump mask's polynomial "no jump" shortcut (no_jump_fast, used by
    cal_dis_reaches and quad_dis_reaches) gives the exact path's verdict on
    steps straddling the threshold: with cut_off = 0.05 rad the
    threshold lies inside the shortcut's |x| <= 1/16 window, which the bench's
    0.1 rad x 2 h never reaches.  Steps of every direction are scaled so the
    haversine distance (NumPy, wr.py:97-112) is cut_off (1 + eps) for eps from
    -1e-3 to 1e-3 down to 1e-15 and exactly at the threshold."""
    from engine import selftest_math
    rng = np.random.default_rng(36)
    lat_p, lon_p, cut = 0.6, 1.0, 0.05

    def dist(dlat, dlon):
        lat_c, lon_c = lat_p + dlat, lon_p + dlon
        a = np.sin((lat_c - lat_p) / 2.0) ** 2 + (np.cos(lat_p) * np.cos(lat_c)) * np.sin((lon_c - lon_p) / 2.0) ** 2
        return np.abs(2.0 * np.arctan2(np.sqrt(a), np.sqrt(1.0 - a)))

    th = rng.uniform(0, 2 * np.pi, 512)
    u, v = np.cos(th), np.sin(th) / np.cos(lat_p)
    lo, hi = np.zeros_like(th), np.full_like(th, 0.2)
    for _ in range(200):                       # bisect the scale to the threshold
        mid = 0.5 * (lo + hi)
        far = dist(mid * u, mid * v) >= cut
        hi, lo = np.where(far, mid, hi), np.where(far, lo, mid)
    eps = np.concatenate([-np.logspace(-3, -15, 25), [0.0], np.logspace(-15, -3, 25)])
    s = (hi[:, None] * (1.0 + eps[None, :])).ravel()
    dlat, dlon = s * np.repeat(u, eps.size), s * np.repeat(v, eps.size)
    dlat = np.concatenate([dlat, np.nextafter(dlat, 0), np.nextafter(dlat, 1)])
    dlon = np.concatenate([dlon, dlon, dlon])
    fast = selftest_math("jump_verdict_fast", dlat, dlon)
    exact = selftest_math("jump_verdict_exact", dlat, dlon)
    assert np.array_equal(fast, exact)
    assert 0.3 < exact.mean() < 0.7            # both verdicts occur
    assert (np.abs(dlat / 2) <= 1 / 16).all() and (np.abs(dlon / 2) <= 1 / 16).all()   # inside the window


# ------------------------------------------------------------------- RK4 mode
def run_wr(kind, cfg_name, nt, inte_method):
    from wr import WR
    cfg = S.config(cfg_name)
    bs = bs_of(kind)
    w = WR(cfg.nzwn, cfg.nsource, 7200.0, (nt - 1) * 7200.0, cfg.freq, nx=bs.nlon, ny=bs.nlat)
    w.bs = bs
    w.set_zwn(cfg.zwn)
    w.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        w.ray_run(mode="hip", inte_method=inte_method)
    return np.array([w.rlon, w.rlat, w.rzwn, w.rmwn, w.ramp, w.rug, w.rvg]).reshape(7, nt, -1)


@pytest.mark.parametrize("kind", KINDS)
def test_rk4_c2_bitwise(kind):
    """The reference's default integrator, RK4: C2 rows at the reference's
    checkpoints over 10 days, bit for bit."""
    g = golden(f"rk4_C2_{kind}.npz")
    nt = int(g["nt"])
    hist = run_wr(kind, "C2", nt, "")
    for j, row in enumerate(g["rows"]):
        assert bitwise(hist[:, row], g["hist"][:, j]), row


def test_rk4_c1_90d_bitwise():
    """RK4 on C1: all 1 081 rows of the reference's 90-day history."""
    g = golden("rk4_C1.npz")
    nt = int(g["nt"])
    hist = run_wr("zonal", "C1", nt, "")
    assert bitwise(hist, g["hist"])


# ------------------------------------------------------------ drop-in delivery
def test_history_sink_delivers_bitwise():
    """hostio.HistorySink on synthetic chunks (rays that change, rays frozen
    from a row on -- NaN payloads of either sign included -- and a chunk where
    nothing changes): the host arrays equal the device rows bit for bit, and
    only changed rays were shipped."""
    from hostio import HistorySink
    rng = np.random.default_rng(5)
    nray, nt, rows_shape = 500, 30, (5, 100)
    full = rng.standard_normal((nray, nt, 8))
    freeze = rng.integers(1, nt + 8, nray)            # row from which a ray repeats itself
    for i in range(nray):
        if freeze[i] < nt:
            full[i, freeze[i]:] = full[i, freeze[i]]
    neg_nan = np.frombuffer(np.uint64(0xFFF8000000000001).tobytes(), np.float64)[0]
    full[::7, 3:, 3] = neg_nan                        # frozen NaN with a payload
    full[:, 20:25] = full[:, 19:20]                   # chunk [20, 25): every ray repeats row 19
    hist = tuple(np.full((nt,) + rows_shape, np.nan) for _ in range(7))
    for v in range(7):
        hist[v][0] = full[:, 0, v].reshape(rows_shape)
    sink = HistorySink(hist, rows_shape, nray, 8, torch.device("cuda"))
    bufs = sink.buffers()
    for k, (i0, i1) in enumerate([(1, 5), (5, 13), (13, 20), (20, 25), (25, 30)]):
        view = bufs[k % 2].view(-1)[: nray * (i1 - i0) * 8].view(nray, i1 - i0, 8)
        torch.cuda.current_stream().synchronize()
        view.copy_(torch.as_tensor(full[:, i0:i1]))
        sink(i0, i1, view)
    sink.finish()
    got = np.stack([h.reshape(nt, nray) for h in hist], axis=2)       # [nt, nray, 7]
    want = np.transpose(full[:, :, :7], (1, 0, 2))
    assert np.array_equal(got.view(np.int64), want.view(np.int64))
    assert sink.shipped < sink.delivered == (nt - 1) * nray


@pytest.mark.parametrize("inte_method", ["rk45", ""])
def test_dropin_history_matches_engine_rows(inte_method):
    """WR.ray_run(mode='hip') delivers every chunk into rlon..rvg through
    hostio.HistorySink (alternating device buffers, copy stream, pinned
    staging, threaded host copies): with 7-row chunks over 3 days the host
    arrays equal the rows of one unchunked engine run bit for bit."""
    from wr import WR
    cfg = S.config("C2")
    bs = bs_of("nonzonal")
    nt = 37
    w = WR(cfg.nzwn, cfg.nsource, 7200.0, (nt - 1) * 7200.0, cfg.freq, nx=bs.nlon, ny=bs.nlat,
           chunk_rows=7)
    w.bs = bs
    w.set_zwn(cfg.zwn)
    w.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        w.ray_run(mode="hip", inte_method=inte_method)
    got = np.array([w.rlon, w.rlat, w.rzwn, w.rmwn, w.ramp, w.rug, w.rvg]).reshape(7, nt, -1)
    y0 = torch.as_tensor(got[:5, 0])
    eng = bs.engine()
    if inte_method == "rk45":
        out = torch.empty((y0.shape[1], nt - 1, 8), dtype=torch.float64, device="cuda")
        eng.integrate(y0, nt, 7200.0, w.rtol, w.atol, w.MinStepFactor, ttotal=(nt - 1) * 7200.0,
                      out=out, cut_rad=float(w.cut_off[0]))
    else:
        out = torch.empty((y0.shape[1], nt - 1, 8), dtype=torch.float64, device="cuda")
        eng.integrate_rk4(y0, nt, 7200.0, out=out, cut_rad=float(w.cut_off[0]))
    want = out[:, :, :7].permute(2, 1, 0).cpu().numpy()
    a, b = got[:, 1:], want
    assert np.array_equal(np.where(np.isnan(a), np.nan, a).view(np.int64),
                          np.where(np.isnan(b), np.nan, b).view(np.int64))
    # frozen rays (NaN-root slots, rays masked on the way) were filled on the host
    d = w.last_delivery
    assert 0 < d["shipped_ray_rows"] < d["delivered_ray_rows"] == (nt - 1) * y0.shape[1]
