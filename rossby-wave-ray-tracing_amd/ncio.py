"""Array file I/O for the drop-in: netCDF-3 (scipy.io.netcdf_file) or NumPy .npz.

The reference reads and writes through ``netCDF4.Dataset`` (bs.py:202-262,
461-511; wr.py:916-959).  ``netCDF4`` is not installed in this image, so files
ending in ``.npz`` use NumPy and everything else the classic netCDF-3 format
(readable by netCDF4 and xarray).
"""
import numpy as np


def read(path):
    """``{name: array}`` of every variable in ``path``."""
    if str(path).endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: np.array(z[k]) for k in z.files}
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        return {k: np.array(v[:]) for k, v in f.variables.items()}


def write(path, dims, variables, attrs=None):
    """``dims``: ``{name: size}``; ``variables``: ``{name: (dim_names, array[, units])}``."""
    if str(path).endswith(".npz"):
        np.savez(path, **{k: np.asarray(v[1]) for k, v in variables.items()})
        return
    from scipy.io import netcdf_file
    with netcdf_file(path, "w", version=2) as f:
        for name, size in dims.items():
            f.createDimension(name, size)
        for name, spec in variables.items():
            dn, arr = spec[0], np.asarray(spec[1])
            typ = "i4" if np.issubdtype(arr.dtype, np.integer) else ("f8" if arr.dtype == np.float64 else "f4")
            var = f.createVariable(name, typ, dn)
            var[...] = arr
            if len(spec) > 2:
                var.units = spec[2]
        for k, v in (attrs or {}).items():
            setattr(f, k, v)
