"""The time-varying extension's oracle (oracle/rwrt_oracle.py TimeVaryingBackground).

Time-varying basic states are not in the reference (its ``fun`` ignores ``t``,
wr.py:784-789), so their parity is stated against this
restatement.  What pins it to the reference: at a level time ``t0 + j*dt``
the RHS is the reference's RHS on level ``j``'s basic state, bit for bit, and
between levels it is the documented linear blend of two such lookups.
"""
import numpy as np
import pytest

import rwrt_oracle as O
import synthetic as S


def levels(n, res=2.5):
    return [O.Background(**S.background_level(j, res=res)) for j in range(n)]


def sample_y(n, seed=0):
    rng = np.random.default_rng(seed)
    y = np.empty((5, n))
    y[0] = rng.uniform(-1.0, 8.0, n)
    y[1] = rng.uniform(-1.5, 1.5, n)
    y[2] = rng.integers(1, 8, n).astype(float)
    y[3] = rng.uniform(-6, 6, n)
    y[4] = 1.0
    return y


@pytest.mark.parametrize("fp32", [False, True])
def test_level_times_reduce_to_the_static_rhs(fp32):
    lv = levels(3)
    tv = O.TimeVaryingBackground(lv, t0=0.0, dt=6 * 3600.0, fp32=fp32)
    y = sample_y(2000)
    for j in range(3):
        t = np.full(y.shape[1], j * 6 * 3600.0)
        got, _ = O.rhs(tv, y, t)
        if fp32:
            bg = lv[j]
            hot = O.TimeVaryingBackground.HOT
            f = bg.fields.copy()
            f[..., hot] = f[..., hot].astype(np.float32).astype(np.float64)
            bg = O.Background.__new__(O.Background)
            bg.fields, bg.lat, bg.lon = f, lv[j].lat, lv[j].lon
        else:
            bg = lv[j]
        ref, _ = O.rhs(bg, y)
        assert np.array_equal(got, ref, equal_nan=True), j


def test_between_levels_is_the_linear_blend():
    lv = levels(2)
    tv = O.TimeVaryingBackground(lv, t0=0.0, dt=6 * 3600.0)
    rng = np.random.default_rng(3)
    n = 500
    lon, lat = rng.uniform(0, 6.2, n), rng.uniform(-1.4, 1.4, n)
    w = 0.25
    t = np.full(n, w * 6 * 3600.0)
    g = O.mercator_point(tv, lon, lat, t)[[0, 1, 6, 7]]
    a = O.mercator_point(lv[0], lon, lat)[[0, 1, 6, 7]]
    b = O.mercator_point(lv[1], lon, lat)[[0, 1, 6, 7]]
    # the blend happens before the Mercator factors (linear in the fields)
    assert np.allclose(g, a * (1 - w) + b * w, rtol=1e-12, atol=1e-18)
    # outside [t0, t0 + (nlev-1) dt] the first / last level is held
    t_out = np.full(n, -3600.0)
    assert np.array_equal(O.mercator_point(tv, lon, lat, t_out)[:12],
                          O.mercator_point(lv[0], lon, lat)[:12], equal_nan=True)
