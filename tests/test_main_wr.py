"""The reference's entry point end to end: ``real2d_hnf(**parameters)``
(``main_wr.py:31-89``) with a basic-flow file in, the basic-state and ray files
out, only ``mode='hip'`` changed.

* CPU: the file path (netCDF-3 written here, read by ``BS.loadbs_ncfile``)
  gives the same field stack as the in-memory arrays, bit for bit; the
  writers round-trip.
* GPU: ``real2d_hnf`` on C1 (1 source at 120E 30N, k = 5) for 3 days; the ray
  file holds exactly the returned history (lon/lat in degrees,
  ``wr.py:916-959``) and its first rows match the reference's own C1 history
  (tests/golden/traj_C1.npz) -- row 0 bit for bit, 2 h within 1e-6 rad.
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


@pytest.mark.gpu
def test_real2d_hnf_c1_files(tmp_path):
    from main_wr import parameters, real2d_hnf
    flow = str(tmp_path / "flow.nc")
    write_flow(flow, "zonal")
    p = dict(parameters)
    p.update(SW_lon=120.0, SW_lat=30.0, nnx=1, nny=1, zwn=np.array([5.0]), nzwn=1,
             ttotal=3.0, inputuv=flow, bsfile=str(tmp_path / "bs.nc"),
             ncfile=str(tmp_path / "rays.nc"), mode="hip", inte_method="rk45")
    with np.errstate(all="ignore"):
        w = real2d_hnf(**p)
    d = ncio.read(p["ncfile"])
    nt = 37
    assert d["rlon"].shape == (nt, 3, 1, 1)
    rad2deg = 180.0 / np.pi
    for name, arr, scale in (("rlon", w.rlon, rad2deg), ("rlat", w.rlat, rad2deg),
                             ("rzwn", w.rzwn, 1.0), ("rmwn", w.rmwn, 1.0), ("ramp", w.ramp, 1.0),
                             ("rug", w.rug, 1.0), ("rvg", w.rvg, 1.0)):
        assert np.array_equal(d[name], arr * scale, equal_nan=True), name
    g = golden("traj_C1.npz")
    ref = g["hist"] if "hist" in g.files else None
    assert ref is not None
    got = np.array([w.rlon, w.rlat, w.rzwn, w.rmwn, w.ramp, w.rug, w.rvg]).reshape(7, nt, -1)
    ref = np.asarray(ref).reshape(7, ref.shape[1], -1)
    assert np.array_equal(got[:, 0], ref[:, 0], equal_nan=True)          # initial rows
    ok = ~np.isnan(ref[0, 1])
    assert np.max(np.abs(got[:2, 1, ok] - ref[:2, 1, ok])) <= 1e-6      # 2 h
