"""Basic state: the reference's ``BS`` (bs.py:69-887) as a drop-in.

Host-side prerequisite of the ray loop (SURVEY.md §2 "(★ host)"): reading
``u, v``, building absolute vorticity and the finite-difference stack
``fields[nlon+1, nlat, 18]`` (``BS.ready``), and the initial meridional
wavenumbers (``cal_ky``).  These run once per background in NumPy and are
bit-identical to the reference (pinned by tests/test_host_prep.py against
golden vectors).  ``cal_bs_mercator_point(mode='hip')`` evaluates on the GPU.

Reference quirks kept on purpose (they change numbers):
* the radian axes are computed in float32 (bs.py:225-236);
* a descending-latitude file flips ``u, v`` but not ``lat`` (bs.py:251-256);
* ``smth9`` smooths ``[1:-2, 1:-2]`` in place after the third derivatives
  were taken (bs.py:291-305, 338-347); ``qyx`` keeps the unsmoothed copy.
"""
import numpy as np
from scipy.ndimage import convolve

from constants import pi, rearth, omega, undef, delt
import ncio

__all__ = ["BS", "cal_ky", "change_roots_order"]

FIELD_NAMES = ["u", "v", "ux", "uy", "vx", "vy", "qx", "qy", "qxx", "qxy", "qyx", "qyy",
               "qxxx", "qxxy", "qxyy", "qyyy", "qyxx", "qyyx"]


class BS:
    """Basic flow on a regular lat-lon grid (``BS(nlon, nlat, read_dtype, cal_dtype)``)."""

    def __init__(self, nlon, nlat, read_dtype="float32", cal_dtype="float64"):
        self.all_dtype = read_dtype
        self.all_dtype_ = cal_dtype
        self.nlon, self.nlat = nlon, nlat
        self.dx = np.array([2.0 * pi / nlon], dtype=cal_dtype)       # bs.py:77-78
        self.dy = np.array([pi / (nlat - 1)], dtype=cal_dtype)
        shape = (nlon, nlat)
        self.u = np.zeros(shape, dtype=read_dtype)
        self.v = np.zeros(shape, dtype=read_dtype)
        self.lat = np.zeros(nlat, dtype=cal_dtype)
        self.lon = np.zeros(nlon, dtype=cal_dtype)
        self.fields = None
        self.xcyclic = True
        self._engine = None

    def getlon(self):
        return self.lon

    def getlat(self):
        return self.lat

    # ---------------------------------------------------------------- input
    def loadbs_ncfile(self, ncfile):
        """Read ``u, v`` (+ ``lat``/``lon`` if present) from a netCDF-3 or .npz file."""
        d = ncio.read(ncfile)
        lat = next((d[k] for k in ("lat", "latitude", "Lat", "Latitude") if k in d), None)
        lon = next((d[k] for k in ("lon", "longitude", "Lon", "Longitude") if k in d), None)
        self.load_arrays(d["u"], d["v"], lat, lon)

    def load_arrays(self, u, v, lat=None, lon=None):
        """``loadbs_ncfile`` on in-memory arrays: ``u, v`` as ``(nlat, nlon)``, degrees."""
        u = np.array(u, dtype=self.all_dtype)
        v = np.array(v, dtype=self.all_dtype)
        if lat is not None:
            lat = np.array(lat, dtype=self.all_dtype)
            self.lat[:] = (lat * pi / 180).astype(self.all_dtype_)   # float32 arithmetic
        else:
            self.lat = -pi * 0.5 + np.arange(self.nlat) * self.dy
        if lon is not None:
            lon = np.array(lon, dtype=self.all_dtype)
            self.lon[:] = (lon * pi / 180).astype(self.all_dtype_)
        else:
            self.lon = np.arange(self.nlon) * self.dx
        self.u, self.v = u.T, v.T
        if lat is None or lon is None:
            print("###WARNING: lon and lat not found. Make sure your lats are from 90S to 90N "
                  "and lons are from 0E to 360E###")
        elif lat[0] > lat[-1]:
            # the reference flips the winds but keeps the descending lat axis
            self.u, self.v = u[::-1, :].T, v[::-1, :].T

    # ------------------------------------------------------- derivatives
    def _px(self, f):
        """Periodic padding along longitude (axis 0)."""
        return np.concatenate([f[-1:], f, f[:1]], axis=0)

    def gradient_x(self, f):
        g = self._px(np.asarray(f).astype(self.all_dtype_))
        return (g[2:] - g[:-2]) / (2.0 * self.dx)

    def gradient_y(self, f):
        f = np.asarray(f).astype(self.all_dtype_)
        out = np.empty_like(f)
        out[:, 1:-1] = (f[:, 2:] - f[:, :-2]) / (2.0 * self.dy)
        out[:, 0] = (f[:, 1] - f[:, 0]) / self.dy
        out[:, -1] = (f[:, -1] - f[:, -2]) / self.dy
        return out

    def gradient_xx(self, f):
        g = self._px(np.asarray(f).astype(self.all_dtype_))
        return (g[2:] - 2.0 * g[1:-1] + g[:-2]) / (self.dx ** 2)

    def gradient_yy(self, f):
        f = np.asarray(f).astype(self.all_dtype_)
        out = np.empty_like(f)
        out[:, 1:-1] = (f[:, 2:] - 2.0 * f[:, 1:-1] + f[:, :-2]) / (self.dy ** 2)
        out[:, 0], out[:, -1] = out[:, 1], out[:, -2]
        return out

    def gradient_xy(self, f):
        """Mixed derivative; evaluated in the input's dtype (float32 for u, v)."""
        g = self._px(np.asarray(f))
        out = np.empty(np.shape(f), dtype=self.all_dtype_)
        out[:, 1:-1] = (g[2:, 2:] - g[2:, :-2] - g[:-2, 2:] + g[:-2, :-2]) / (4.0 * self.dx * self.dy)
        out[:, 0], out[:, -1] = out[:, 1], out[:, -2]
        return out

    gradient_yx = gradient_xy

    @staticmethod
    def smth9(field, p=0.5, q=0.25):
        """Nine-point smoother, in place on ``[1:-2, 1:-2]`` (bs.py:291-305)."""
        w = np.array([[q / 4, p / 4, q / 4], [p / 4, -(p + q), p / 4], [q / 4, p / 4, q / 4]])
        field[1:-2, 1:-2] = field[1:-2, 1:-2] + convolve(field, w, mode="constant", cval=0.0)[1:-2, 1:-2]
        return field

    def calc_absolute_vorticity(self):
        ucos = (self.u * np.cos(self.lat[None, :])).astype(self.all_dtype_)
        vx = self.gradient_x(self.v)
        uy = self.gradient_y(ucos)
        q = np.zeros((self.nlon, self.nlat), dtype=self.all_dtype_)
        q[:, 1:-1] = (vx[:, 1:-1] - uy[:, 1:-1]) / np.cos(self.lat[1:-1])[None, :] \
            + 2.0 * omega * np.sin(self.lat[1:-1])[None, :] * rearth
        q[:, 0], q[:, -1] = q[:, 1], q[:, -2]
        self.q = q

    def ready(self, xcyclic=False):
        """Vorticity, derivatives, smoothing and the 18-field stack (bs.py:318-407)."""
        self.xcyclic = xcyclic
        self.calc_absolute_vorticity()
        u, v, q = self.u, self.v, self.q
        d = dict(u=u, v=v)
        d["ux"], d["uy"] = self.gradient_x(u), self.gradient_y(u)
        d["vx"], d["vy"] = self.gradient_x(v), self.gradient_y(v)
        d["qx"], d["qy"] = self.gradient_x(q), self.gradient_y(q)
        self.uxx, self.uyy = self.gradient_xx(u), self.gradient_yy(u)
        self.vxx, self.vyy = self.gradient_xx(v), self.gradient_yy(v)
        d["qxx"], d["qyy"] = self.gradient_xx(q), self.gradient_yy(q)
        self.uxy, self.vxy = self.gradient_xy(u), self.gradient_xy(v)
        d["qxy"] = self.gradient_xy(q)
        d["qyx"] = d["qxy"].copy()
        d["qxxx"], d["qxxy"] = self.gradient_x(d["qxx"]), self.gradient_y(d["qxx"])
        d["qxyy"], d["qyyy"] = self.gradient_y(d["qxy"]), self.gradient_y(d["qyy"])
        d["qyxx"], d["qyyx"] = self.gradient_x(d["qxy"]), self.gradient_x(d["qyy"])
        for k in ("qxx", "qyy", "qxy"):
            self.smth9(d[k])
        for k in FIELD_NAMES[2:]:
            setattr(self, k, d[k])
        f = np.stack([d[k] for k in FIELD_NAMES], axis=-1).astype(self.all_dtype_)
        if xcyclic:
            f = np.concatenate([f, f[0:1]], axis=0)
        self.fields = f
        self._engine = None
        self._diagnostics()

    def _diagnostics(self):
        """beta_M and K_S (bs.py:379-407); written by ``output`` only."""
        c = np.cos(self.lat[None, 1:-1])
        s = np.sin(self.lat[None, 1:-1])
        betam = np.zeros((self.nlon, self.nlat), dtype=self.all_dtype_)
        betam[:, 1:-1] = (2 * omega * (c ** 2) + (-c * self.uyy[:, 1:-1] + s * self.uy[:, 1:-1]
                                                  + self.u[:, 1:-1] / c) / rearth) / rearth
        betam[:, 0] = betam[:, -1] = undef
        ks = np.zeros_like(betam)
        with np.errstate(invalid="ignore", divide="ignore"):
            ks[:, 1:-1] = np.sqrt(betam[:, 1:-1] * c / self.u[:, 1:-1]) * rearth
        ok = (betam > 0) & (self.u > 0)
        ks = ks * ok
        ks[~ok] = undef
        ks[:, 0] = ks[:, -1] = undef
        self.betam, self.KS = betam, ks

    # --------------------------------------------------------------- output
    def output(self, ncfile):
        """Write the basic state and its diagnostics (netCDF-3 or .npz by suffix)."""
        names = ["u", "v", "q", "ux", "uxx", "uy", "vx", "vxx", "vy", "qx", "qy", "qxx", "qxy",
                 "qyx", "qyy", "qxxx", "qxxy", "qxyy", "qyyy", "qyxx", "qyyx", "betam", "KS"]
        vars_ = {"lon": (("lon",), self.lon), "lat": (("lat",), self.lat)}
        for n in names:
            vars_[n] = (("lon", "lat"), np.asarray(getattr(self, n), dtype=self.all_dtype_))
        ncio.write(ncfile, {"lon": self.nlon, "lat": self.nlat}, vars_)

    def clean(self):
        for k in ["u", "v", "q", "fields", "betam", "KS"] + FIELD_NAMES[2:]:
            if hasattr(self, k):
                delattr(self, k)
        self._engine = None

    # ------------------------------------------------------ interpolation
    def engine(self):
        """The GPU engine holding this basic state (built lazily)."""
        if self._engine is None:
            from engine import RayEngine
            self._engine = RayEngine.from_bs(self)
        return self._engine

    def cal_bs_mercator_point(self, lon, lat, mode="numpy"):
        """Fields + Mercator conversion at points (bs.py:513-519,781-887).

        ``mode='numpy'``: host NumPy, all 18 outputs (used for ray
        initialisation, bit-identical to the reference).  ``mode='hip'``: the
        12 outputs of the hot path on the GPU.
        """
        if mode == "hip":
            return self.engine().mercator_point(np.asarray(lon, np.float64),
                                                np.asarray(lat, np.float64)).cpu().numpy()
        if mode != "numpy":
            raise ValueError(f"mode must be 'numpy' or 'hip', got {mode!r}")
        lon = np.asarray(lon, dtype=np.float64) % (2 * pi)
        lat = np.asarray(lat, dtype=np.float64)
        F = self.fields
        inr = np.where(np.abs(lat) <= 0.5 * pi)[0]
        vals = np.full((F.shape[-1], len(lat)), np.nan)
        x = (lon[inr] % (2 * np.pi) - self.lon[0]) / (self.lon[1] - self.lon[0])
        y = (lat[inr] - self.lat[0]) / (self.lat[1] - self.lat[0])
        W, Hh = F.shape[0], F.shape[1]
        xi, yi = np.floor(x).astype("int32"), np.floor(y).astype("int32")
        x0, x1 = np.clip(xi, 0, W - 1), np.clip(xi + 1, 0, W - 1)
        y0, y1 = np.clip(yi, 0, Hh - 1), np.clip(yi + 1, 0, Hh - 1)
        sx, sy = x - x0, y - y0
        w = [(1 - sx) * sy, sx * sy, (1 - sx) * (1 - sy), sx * (1 - sy)]
        vals[:, inr] = (F[x0, y1] * w[0][:, None] + F[x1, y1] * w[1][:, None]
                        + F[x0, y0] * w[2][:, None] + F[x1, y0] * w[3][:, None]).T
        g = dict(zip(FIELD_NAMES, vals))
        c, s, t = np.cos(lat), np.sin(lat), np.tan(lat)
        m = np.ones(c.shape, dtype=self.all_dtype_)
        m[np.abs(c) <= 0.0175] = 0
        c = c * m + (1 - m) * 1e-6
        fmqyx = g["qxy"] * c * m
        out = [g["u"] / c * m, g["v"] / c * m, g["ux"] / c * m, (g["uy"] + t * g["u"]) * m,
               g["vx"] / c * m, (g["vy"] + t * g["v"]) * m, g["qx"] * m, g["qy"] * c * m,
               g["qxx"] * m, fmqyx * m, fmqyx, (g["qyy"] * c - g["qy"] * s) * c * m,
               g["qxxx"] * m, g["qxxy"] * c * m, (g["qxyy"] * c - g["qxy"] * s) * c * m,
               g["qyyy"] * m, g["qyxx"] * c * m, (g["qyyx"] * c - g["qxy"] * s) * c * m]
        return np.array(out, dtype=self.all_dtype_)


# ----------------------------------------------------------------------------
# dispersion relation at t = 0
# ----------------------------------------------------------------------------
def _batched_roots(coef, deg):
    """``np.roots`` of each row's polynomial ``coef[i, :deg+1]`` (lowest order first).

    Rows are grouped by companion-matrix size so that one ``eigvals`` call
    serves thousands of sources; each matrix goes through the same LAPACK
    ``zgeev`` as ``np.roots`` would run on it alone (bs.py:38-40).
    Returns ``(roots[n, 3] complex, count[n])`` in np.roots' order.
    """
    n = coef.shape[0]
    roots = np.full((n, 3), np.nan + 0j)
    count = np.zeros(n, np.int64)
    p_all = coef[:, ::-1] + 0j                        # highest order first, width 4
    for d in (1, 2, 3):
        rows = np.where(deg == d)[0]
        if len(rows) == 0:
            continue
        p = p_all[rows][:, 3 - d:]                    # (m, d+1), p[:, 0] != 0
        nz = p != 0
        last_nz = d - np.argmax(nz[:, ::-1], axis=1)  # index of the last non-zero
        for last in np.unique(last_nz):
            sel = np.where(last_nz == last)[0]
            q = p[sel, :last + 1]
            trailing = d - last
            N = q.shape[1]
            if N > 1:
                A = np.zeros((len(sel), N - 1, N - 1), dtype=q.dtype)
                if N > 2:
                    A[:, np.arange(1, N - 1), np.arange(N - 2)] = 1
                A[:, 0, :] = -q[:, 1:] / q[:, :1]
                r = np.linalg.eigvals(A)
            else:
                r = np.zeros((len(sel), 0), dtype=q.dtype)
            r = np.concatenate([r, np.zeros((len(sel), trailing), dtype=q.dtype)], axis=1)
            roots[rows[sel], :r.shape[1]] = r
            count[rows[sel]] = r.shape[1]
    return roots, count


def change_roots_order(mwn, deg):
    """Vectorised ``change_roots_order`` (bs.py:942-982) on ``mwn[n, 3]``; returns reversed."""
    m = np.array(mwn, dtype=np.float64, copy=True)
    deg = np.asarray(deg)
    # deg == 3: slot 2 moves before slot 1 when smaller and non-negative, ...
    s3 = deg == 3
    sw = s3 & (m[:, 2] >= 0.) & (m[:, 2] < m[:, 1])
    m[sw, 1], m[sw, 2] = m[sw, 2], m[sw, 1].copy()
    sw = s3 & (m[:, 0] < 0)
    m[sw, 0], m[sw, 1] = m[sw, 1], m[sw, 0].copy()
    sw = s3 & (((m[:, 1] < 0) & (m[:, 2] < 0) & (m[:, 1] < m[:, 2])) | ((m[:, 1] > 0) & (m[:, 2] < 0.)))
    m[sw, 1], m[sw, 2] = m[sw, 2], m[sw, 1].copy()
    # deg == 2: only slot 0 is inspected (both branches break)
    sw = (deg == 2) & ~(m[:, 0] > 0)
    m[sw, 0], m[sw, 1] = m[sw, 1], m[sw, 0].copy()
    # deg == 1: a negative root ends up in slot 1, zero or positive in slot 0
    sw = (deg == 1) & (m[:, 0] < 0)
    m[sw, 0], m[sw, 1] = m[sw, 1], m[sw, 0].copy()
    big = ~np.isnan(m) & (np.abs(m) > 100.)
    m[big] = np.nan
    return m[:, ::-1]


def cal_ky(fu, fv, fqx, fqy, freq, zwn, iz=0, mode="numpy", root_method="numpy"):
    """Meridional wavenumbers at t = 0 (``cal_ky_numpy``, bs.py:985-1040).

    Returns ``(mwn[n, 3], nroots[n])``.  ``root_method`` is accepted for
    signature compatibility; the Fortran ``cmplx_roots_sg`` module is absent in
    the reference too and it falls back to ``np.roots`` (bs.py:1048-1053).
    """
    fu = np.asarray(fu, np.float64)
    n = len(fu)
    mwn = np.full((n, 3), np.nan)
    lens = np.zeros(n)
    if zwn == 0:
        return mwn, lens
    ps = freq / zwn * rearth
    coef = np.stack([(zwn ** 3) * (fu - ps - (fqy / zwn ** 2)), (zwn ** 2) * fv + fqx,
                     zwn * (fu - ps), fv * np.ones_like(fu)], axis=-1)
    deg = np.full(n, 3)
    for d in (3, 2, 1):                       # trailing exact-zero degree reduction
        deg = np.where((deg == d) & (np.abs(coef[:, d]) == 0), d - 1, deg)
    roots, count = _batched_roots(coef, deg)
    real = (np.abs(roots.imag) < delt) & (np.arange(3)[None, :] < count[:, None])
    # compact the real roots to the front, keeping np.roots' order
    order = np.argsort(~real, axis=1, kind="stable")
    vals = np.take_along_axis(roots.real, order, axis=1)
    nreal = real.sum(axis=1)
    vals[np.arange(3)[None, :] >= nreal[:, None]] = np.nan
    mwn = change_roots_order(vals, nreal)
    mwn[deg < 1] = np.nan
    lens = (~np.isnan(mwn)).sum(axis=1).astype(np.float64)
    return mwn, lens
