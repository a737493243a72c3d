"""Entry point with the reference's parameter dict and ``real2d_hnf`` (main_wr.py:5-100).

Identical keys and flow; the ray loop runs on the GPU (``mode='hip'``,
``inte_method='rk45'``).  Files: netCDF-3 or ``.npz`` (see ncio.py).
"""
import warnings

import numpy as np

warnings.filterwarnings("ignore")
parameters = {
    "freq": 0.,            # frequency; 0 for stationary Rossby waves
    "mm": None,            # nlon (None: from the file)
    "nn": None,            # nlat (None: from the file)
    "SW_lon": 70., "SW_lat": -4.,
    "dlon": 4, "dlat": 2,
    "nnx": 21, "nny": 15,
    "zwn": np.array([1., 2., 3., 4., 5., 6., 7.]),
    "nzwn": 7,
    "tstep": 2,            # hours
    "ttotal": 90.,         # days
    "mode": "hip",
    "root_method": "numpy",
    "inte_method": "rk45",
    "xcyclic": True,
    "cal_dtype": "float64",
    "read_dtype": "float32",
    "inputuv": "basic_flow.nc",
    "bsfile": "bs_out.nc",
    "ncfile": "rays_out.nc",
    "rtol": 1e-6,
    "atol": 1e-6,
    "MinStepFactor": 1e-3,
}


def real2d_hnf(nzwn, mm, nn, freq, zwn, inputuv, ncfile, bsfile, SW_lon, SW_lat, dlon, dlat,
               nnx, nny, mode, tstep, ttotal, xcyclic, root_method, read_dtype, cal_dtype,
               inte_method, atol, rtol, MinStepFactor):
    """Read the basic flow, trace every ray, write the results (main_wr.py:31-89)."""
    from constants import hour, day
    from wr import WR

    nsource = nnx * nny
    wr1 = WR(nzwn, nsource, tstep * hour, ttotal * day, freq, nx=mm, ny=nn,
             read_dtype=read_dtype, cal_dtype=cal_dtype, rtol=rtol, atol=atol,
             ncfile=inputuv, MinStepFactor=MinStepFactor)
    wr1.bs.loadbs_ncfile(inputuv)
    wr1.bs.ready(xcyclic=xcyclic)
    if bsfile:
        wr1.bs.output(bsfile)
    wr1.set_zwn(zwn)
    wr1.set_source_matrix(SW_lon, SW_lat, dlon, dlat, nnx, nny)
    wr1.ray_info()
    wr1.ray_run(mode=mode, root_method=root_method, inte_method=inte_method)
    if ncfile:
        wr1.output(ncfile)
    return wr1


if __name__ == "__main__":
    real2d_hnf(**parameters)
