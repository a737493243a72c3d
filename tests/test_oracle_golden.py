"""The CPU oracle is bit-for-bit equal to the reference on its golden vectors.

Fixtures come from the reference itself (tests/golden/make_golden.py); this
file pins ``oracle/rwrt_oracle.py`` before any GPU result is compared with it.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden
import rwrt_oracle as O
import synthetic as S

KINDS = ["zonal", "nonzonal"]


def same(a, b):
    """Bitwise equality treating NaN == NaN."""
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a, b, equal_nan=True)


_BG = {}


def bg(kind):
    if kind not in _BG:
        _BG[kind] = O.Background(**S.background(kind))
    return _BG[kind]


@pytest.mark.parametrize("kind", KINDS)
def test_fields_bitwise(kind):
    g = golden(f"bg_{kind}.npz")
    F = bg(kind).fields
    assert tuple(g["shape"]) == F.shape
    assert same(F[::7, ::5, :], g["sample"])
    assert hashlib.sha256(np.ascontiguousarray(F).tobytes()).hexdigest() == str(g["sha256"])
    assert same(bg(kind).lat, g["lat"]) and same(bg(kind).lon, g["lon"])


@pytest.mark.parametrize("kind", KINDS)
def test_mercator_point_bitwise(kind):
    g = golden(f"merc_{kind}.npz")
    assert same(O.mercator_point(bg(kind), g["lon"].copy(), g["lat"].copy()), g["out"])


@pytest.mark.parametrize("kind", KINDS)
def test_rhs_bitwise(kind):
    g = golden(f"rhs_{kind}.npz")
    with np.errstate(all="ignore"):
        d, bad = O.rhs(bg(kind), g["y"].copy())
    assert same(bad, g["bad"])
    assert same(d, g["dydt"])


@pytest.mark.parametrize("kind", KINDS)
def test_single_step_bitwise(kind):
    g = golden(f"step_{kind}.npz")
    fun = lambda t, y: O.rhs(bg(kind), y)[0]
    y, h = g["y"], g["h"]
    with np.errstate(all="ignore"):
        yn, K = O.dp54_attempt(fun, np.zeros(len(h)), y, g["f"], h)
        en = O.error_norm(K, h, y, yn, 1e-6, 1e-6)
    assert same(K, g["K"])
    assert same(yn, g["y_new"])
    ref = g["err_norm"].copy()
    ref[np.isnan(ref)] = 0
    assert same(en, ref)


@pytest.mark.parametrize("kind", KINDS)
def test_initial_rows_and_step_bitwise(kind):
    g = golden(f"init_C2_{kind}.npz")
    cfg = S.config("C2")
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        rows = np.array(O.ray_initial(bg(kind), slon, slat, cfg.zwn, cfg.freq))
    assert same(rows, g["rows"])
    y0 = rows[:5].reshape(5, -1)
    fun = lambda t, y: O.rhs(bg(kind), y)[0]
    with np.errstate(all="ignore"):
        f0 = fun(0, y0)
        h = O.initial_step(fun, np.zeros(y0.shape[1]), y0, f0, 1e-6, 1e-6)
    assert same(f0, g["f0"])
    assert same(h, g["h_abs"])


def test_roots_c3_subsample_bitwise():
    g = golden("roots_C3.npz")
    cfg = S.config("C3")
    for tag in ["stat", "p10"]:
        for kind in KINDS:
            src = g[f"{tag}_{kind}_src"]
            with np.errstate(all="ignore"):
                rows = O.ray_initial(bg(kind), src[0], src[1], cfg.zwn, float(g[f"{tag}_{kind}_freq"]))
            assert same(np.array([rows[3], rows[4], rows[5], rows[6]]), g[f"{tag}_{kind}_rows"]), (tag, kind)


def test_c1_trajectory_bitwise():
    g = golden("traj_C1.npz")
    with np.errstate(all="ignore"):
        hist, nacc, nrej, st = O.run_config(bg("zonal"), S.config("C1"), nt=int(g["nt"]))
    assert st == 0
    assert same(hist, g["hist"])
    assert same(nacc, g["nacc"])
    assert int(nacc.sum() + nrej.sum()) == int(g["attempts"])


@pytest.mark.parametrize("kind", KINDS)
def test_reference_loop_shape_bitwise(kind):
    """The oracle's reference-structured loop (f recomputed for every column at
    each step start, rkf45.py:378; bench.py's cpu_baseline) gives the same
    bits as the FSAL loop, and evaluates the RHS on about twice the columns."""
    g = golden(f"traj_C2_{kind}.npz")
    cols = [0]
    with np.errstate(all="ignore"):
        hist, nacc, nrej, st = O.run_config(bg(kind), S.config("C2"), nt=13, fsal=False, columns=cols)
        h2, nacc2, _, _ = O.run_config(bg(kind), S.config("C2"), nt=13)
    assert st == 0
    assert same(hist, h2) and same(nacc, nacc2)
    assert same(hist[:, 1], g["hist"][:, 0]) and same(hist[:, 12], g["hist"][:, 1])
    per_acc = cols[0] / nacc.sum()
    assert 10.0 < per_acc < 30.0, per_acc


@pytest.mark.parametrize("kind", KINDS)
def test_c2_trajectory_bitwise(kind):
    g = golden(f"traj_C2_{kind}.npz")
    with np.errstate(all="ignore"):
        hist, nacc, nrej, st = O.run_config(bg(kind), S.config("C2"), nt=int(g["nt"]))
    assert st == 0
    assert same(hist[:, g["rows"]], g["hist"])
    assert same(nacc, g["nacc"])
    assert int(nacc.sum() + nrej.sum()) == int(g["attempts"])


def _kat(name, fun, rtol=1e-3, atol=1e-6):
    g = golden("kat_stepper.npz")
    ts = g["t_eval"]
    y0 = g[f"{name}_y0"]
    sol = O.DP54(fun, 0, y0.astype(float), ts[-1], rtol, atol, 0.001, autonomous=False)
    ys = np.full((len(ts),) + y0.shape, np.nan)
    ys[0] = y0
    for i in range(1, len(ts)):
        sol.advance_to(ts[i])
        ys[i] = sol.y
    assert same(ys, g[f"{name}_ys"])


def test_kat_linear():
    _kat("lin", lambda t, u: np.array([2 * t + u[0] * 0]))


def test_kat_exp():
    _kat("exp", lambda t, u: np.array([np.e ** (0.1 * t) + u[0] * 0]), rtol=1e-14, atol=1e-15)


def test_kat_lorenz():
    def lorenz(t, u, p=10, b=8 / 3, r=28):
        x, y, z = u
        return np.array([-p * x + p * y, -x * z + r * x - y, x * y - b * z])
    _kat("lorenz", lorenz)


def test_rk4_c1_bitwise():
    g = golden("rk4_C1.npz")
    with np.errstate(all="ignore"):
        hist, st = O.run_config_rk4(bg("zonal"), S.config("C1"), nt=int(g["nt"]))
    assert same(hist, g["hist"])


@pytest.mark.parametrize("kind", KINDS)
def test_rk4_c2_bitwise(kind):
    g = golden(f"rk4_C2_{kind}.npz")
    with np.errstate(all="ignore"):
        hist, st = O.run_config_rk4(bg(kind), S.config("C2"), nt=int(g["nt"]))
    assert same(hist[:, g["rows"]], g["hist"])
