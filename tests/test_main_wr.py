"""The reference's entry point end to end: ``real2d_hnf(**parameters)``
(``main_wr.py:31-89``) with a basic-flow file in, the basic-state and ray files
out, only ``mode='hip'`` changed.

* CPU: the file path (netCDF-3 written here, read by ``BS.loadbs_ncfile``)
  gives the same field stack as the in-memory arrays, bit for bit; the
  writers round-trip.
* GPU: ``real2d_hnf`` on C1 (1 source at 120E 30N, k = 5) for the reference's
  full 90 days; the ray file holds exactly the returned history (lon/lat in
  degrees, ``wr.py:916-959``) and EVERY row of all seven arrays equals the
  reference's own C1 history (tests/golden/traj_C1.npz) bit for bit; C2
  (16 x 16 sources x k = 3..6, both backgrounds) through the same entry point
  for 10 days equals the reference's rows at 2 h, 1 d and 10 d bit for bit.
"""
import numpy as np
import pytest

import ncio
import synthetic as S
from conftest import golden


def write_flow(path, kind="zonal"):
    bg = S.background(kind)
    ncio.write(path, {"lat": len(bg["lat"]), "lon": len(bg["lon"])},
               {"lat": (("lat",), bg["lat"]), "lon": (("lon",), bg["lon"]),
                "u": (("lat", "lon"), bg["u"]), "v": (("lat", "lon"), bg["v"])})
    return bg


def test_loadbs_ncfile_equals_in_memory(tmp_path):
    from bs import BS
    f = str(tmp_path / "flow.nc")
    bg = write_flow(f, "nonzonal")
    a = BS(len(bg["lon"]), len(bg["lat"]))
    a.loadbs_ncfile(f)
    a.ready(xcyclic=True)
    b = BS(len(bg["lon"]), len(bg["lat"]))
    b.load_arrays(**bg)
    b.ready(xcyclic=True)
    assert np.array_equal(a.fields, b.fields, equal_nan=True)
    out = str(tmp_path / "bs.nc")
    a.output(out)
    d = ncio.read(out)
    assert np.array_equal(d["qy"], np.asarray(a.qy, dtype=a.all_dtype_))


def _real2d_hnf(tmp_path, kind, cfg_name, days):
    """real2d_hnf(**parameters) with only the seed set, the horizon, the files
    and mode='hip' changed (main_wr.py:5-30, 31-89)."""
    from main_wr import parameters, real2d_hnf
    flow = str(tmp_path / f"flow_{kind}.nc")
    write_flow(flow, kind)
    cfg = S.config(cfg_name)
    p = dict(parameters)
    p.update(SW_lon=cfg.SW_lon, SW_lat=cfg.SW_lat, dlon=cfg.dlon, dlat=cfg.dlat, nnx=cfg.nnx, nny=cfg.nny,
             zwn=np.array(cfg.zwn), nzwn=len(cfg.zwn), ttotal=float(days), inputuv=flow,
             bsfile=str(tmp_path / f"bs_{kind}.nc"), ncfile=str(tmp_path / f"rays_{kind}.nc"),
             mode="hip", inte_method="rk45")
    with np.errstate(all="ignore"):
        w = real2d_hnf(**p)
    return w, p


def _history(w, nt):
    return np.array([w.rlon, w.rlat, w.rzwn, w.rmwn, w.ramp, w.rug, w.rvg]).reshape(7, nt, -1)


@pytest.mark.gpu
def test_real2d_hnf_c1_files(tmp_path):
    """C1 through the reference's entry point for its full 90 days: every row
    of all 7 history arrays equals the reference's own real2d_hnf output."""
    w, p = _real2d_hnf(tmp_path, "zonal", "C1", 90)
    d = ncio.read(p["ncfile"])
    nt = 1081
    assert d["rlon"].shape == (nt, 3, 1, 1)
    rad2deg = 180.0 / np.pi
    for name, arr, scale in (("rlon", w.rlon, rad2deg), ("rlat", w.rlat, rad2deg),
                             ("rzwn", w.rzwn, 1.0), ("rmwn", w.rmwn, 1.0), ("ramp", w.ramp, 1.0),
                             ("rug", w.rug, 1.0), ("rvg", w.rvg, 1.0)):
        assert np.array_equal(d[name], arr * scale, equal_nan=True), name
    g = golden("traj_C1.npz")
    ref = np.asarray(g["hist"]).reshape(7, nt, -1)
    got = _history(w, nt)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), f"{int((~same).sum())} of {same.size} values differ from the reference (first row " \
                       f"{int(np.where(~same.all(axis=(0, 2)))[0][0])})"


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_real2d_hnf_c2_rows(tmp_path, kind):
    """C2 (3 072 slots) through real2d_hnf for 10 days: the rows the reference
    kept (2 h, 1 d, 10 d; tests/golden/traj_C2_<kind>.npz) bit for bit."""
    w, _ = _real2d_hnf(tmp_path, kind, "C2", 10)
    g = golden(f"traj_C2_{kind}.npz")
    got = _history(w, 121)[:, np.asarray(g["rows"])]
    ref = np.asarray(g["hist"]).reshape(got.shape)
    same = (got == ref) | (np.isnan(got) & np.isnan(ref))
    assert same.all(), f"{int((~same).sum())} of {same.size} values differ"
