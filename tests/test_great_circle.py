"""Physical KAT: the docs' Great-Circle example (Hoskins &
Karoly 1981).  In solid-body super-rotation U = U0 cos(phi), V = 0,
stationary Rossby-wave rays follow great circles.  Sources at 0 E, 0-20 N
every 5 degrees, k = 1..5, 30 days (the docs' Figure 1 set-up; the docs'
``ideal basic flow.nc`` is not shipped, synthetic.background('superrotation')
stands in).

Measure: each live ray's positions as unit vectors, distance (rad) from the
best-fit plane through the origin.  On the 2.5-degree grid with rtol = 1e-6
the oracle's rays stay within 7e-4 rad of a great circle over 30 days
(median ray 1e-5): the bound below is 1e-3 / 4e-5.  The GPU's rays must meet
the same bound, through the drop-in ``WR.ray_run(mode='hip')``.
"""
import numpy as np
import pytest

import synthetic as S

NT = 361          # 30 days at 2 h
ZWN = np.arange(1.0, 6.0)


def great_circle_deviation(lon, lat, live):
    """Per live ray: max distance (rad) of its positions from the best-fit great circle."""
    out = []
    for r in np.nonzero(live)[0]:
        ok = ~np.isnan(lon[:, r])
        la, lo = lat[ok, r], lon[ok, r]
        pts = np.stack([np.cos(la) * np.cos(lo), np.cos(la) * np.sin(lo), np.sin(la)], axis=1)
        n = np.linalg.svd(pts, full_matrices=False)[2][-1]
        out.append(np.max(np.arcsin(np.minimum(np.abs(pts @ n), 1.0))))
    return np.array(out)


def check(dev, n_live):
    assert len(dev) == n_live
    assert dev.max() < 1e-3, dev.max()
    assert np.median(dev) < 4e-5, np.median(dev)


def test_great_circle_oracle():
    import rwrt_oracle as O
    ob = O.Background(**S.background("superrotation"))
    slon, slat = O.source_matrix(0.0, 0.0, 5.0, 5.0, 1, 5)
    rows = np.array(O.ray_initial(ob, slon, slat, ZWN, 0.0)).reshape(7, -1)
    n_live = int(np.sum(~np.isnan(rows[3])))
    assert n_live == 50          # two real roots (+-l) per source and k
    with np.errstate(all="ignore"):
        hist, nacc, _, st = O.ray_run(ob, rows[:5].copy(), NT, 7200.0, row0=rows)
    assert st == 0
    check(great_circle_deviation(hist[0], hist[1], ~np.isnan(rows[3])), n_live)


@pytest.mark.gpu
def test_great_circle_gpu_dropin():
    from bs import BS
    from wr import WR
    bg = S.background("superrotation")
    bs = BS(len(bg["lon"]), len(bg["lat"]))
    bs.load_arrays(**bg)
    bs.ready(xcyclic=True)
    w = WR(len(ZWN), 5, 7200.0, (NT - 1) * 7200.0, 0.0, nx=bs.nlon, ny=bs.nlat)
    w.bs = bs
    w.set_zwn(ZWN)
    w.set_source_matrix(0.0, 0.0, 5.0, 5.0, 1, 5)
    with np.errstate(all="ignore"):
        w.ray_run(mode="hip", inte_method="rk45")
    lon = np.asarray(w.rlon).reshape(NT, -1)
    lat = np.asarray(w.rlat).reshape(NT, -1)
    live = ~np.isnan(np.asarray(w.rmwn)[0].reshape(-1))
    check(great_circle_deviation(lon, lat, live), int(live.sum()))
