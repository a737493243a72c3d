"""Import the read-only Python reference with in-memory stubs (generation only).

Used ONLY by ``make_golden.py`` in the build container, where
``/root/reference`` exists.  Nothing on the GPU box imports this module.

The reference imports two modules this image lacks:

* ``numba`` -- replaced by an identity ``jit`` decorator, so the five
  ``@nb.jit`` functions (``wr.py:44,89,97``, ``wn.py:266``, ``bs.py:38``) run as
  plain NumPy with the same IEEE fp64 element operations (no fastmath);
* ``netCDF4`` -- replaced by a ``Dataset`` that serves and stores in-memory
  dicts, so ``BS.loadbs_ncfile`` (``bs.py:202-262``), ``BS.output`` and
  ``WR.output`` run unchanged.
"""
import sys
import types

REF_DIR = "/root/reference"

_STORE = {}


class _Var:
    def __init__(self, data=None):
        self._data = data

    def __getitem__(self, key):
        return self._data[key]

    def __setitem__(self, key, value):
        import numpy as np
        if self._data is None:
            self._data = np.array(value)
        else:
            self._data[key] = value


class _Dataset:
    def __init__(self, path, mode="r", **kw):
        self.path = path
        self.mode = mode
        if mode == "r":
            self.variables = {k: _Var(v) for k, v in _STORE[path].items()}
        else:
            self.variables = {}
            self.dimensions = {}

    def createDimension(self, name, size):
        self.dimensions[name] = size

    def createVariable(self, name, dtype, dims=(), **kw):
        import numpy as np
        shape = tuple(self.dimensions[d] for d in dims)
        v = _Var(np.zeros(shape, dtype=dtype))
        self.variables[name] = v
        return v

    def close(self):
        if self.mode != "r":
            _STORE[self.path] = {k: v._data for k, v in self.variables.items()}

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def put_nc(path, **arrays):
    """Register an in-memory 'netCDF file' readable by the stubbed Dataset."""
    _STORE[path] = dict(arrays)


def get_nc(path):
    return _STORE[path]


def load_reference():
    """Install the stubs and import the reference modules; returns a namespace."""
    if "wr" in sys.modules and getattr(sys.modules["wr"], "__file__", "").startswith(REF_DIR):
        return _ns()
    nb = types.ModuleType("numba")
    nb.jit = lambda *a, **k: (lambda f: f)
    nb.njit = nb.jit
    sys.modules["numba"] = nb
    nc = types.ModuleType("netCDF4")
    nc.Dataset = _Dataset
    sys.modules["netCDF4"] = nc
    try:
        import matplotlib
        matplotlib.use("Agg")
    except Exception:   # matplotlib only used by rkf45's __main__ demos
        mpl = types.ModuleType("matplotlib")
        mpl.pyplot = types.ModuleType("matplotlib.pyplot")
        sys.modules["matplotlib"] = mpl
        sys.modules["matplotlib.pyplot"] = mpl.pyplot
    sys.dont_write_bytecode = True
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import constants, interpolation, rkf45, bs, wn, wr, main_wr  # noqa: F401
    return _ns()


def _ns():
    import constants, interpolation, rkf45, bs, wn, wr, main_wr
    return types.SimpleNamespace(constants=constants, interpolation=interpolation,
                                 rkf45=rkf45, bs=bs, wn=wn, wr=wr, main_wr=main_wr)
