"""CPU oracle: NumPy restatement of the reference's RK45 ray loop.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline.  The product path (the HIP library behind
``rossby-wave-ray-tracing_amd/``) never imports or calls it.

Parity status: PINNED.  ``tests/test_oracle_golden.py`` checks this module
bit-for-bit against golden vectors produced by the reference itself
(``tests/golden/make_golden.py`` imports ``/root/reference`` with in-memory
``numba``/``netCDF4`` stubs).

What is restated (reference ``file:line`` per function):

* field preparation ``BS.ready``            -- ``bs.py:121-200,264-279,291-305,318-372``
* ``cal_bs_mercator_point(mode='numpy')``   -- ``bs.py:513-519,781-887``
  with ``batch_linint2_metpy``/``bilinear_interpolation_`` -- ``interpolation.py:77-135``
* group velocity ``cal_ugvg(mode='extent')`` -- ``wn.py:266-294,318-342``
* RHS ``WR.diffun_numpy`` + ``core_diffun``  -- ``wr.py:492-556,44-82``
* DP5(4) tableau / ``select_initial_step`` / ``norm`` -- ``rkf45.py:601-615,34-99,29-31``
* ``RungeKutta._step_impl`` + ``rk_step``    -- ``rkf45.py:375-514,259-321``
* interval loop ``WR.core_ray_run_rk45``     -- ``wr.py:767-887`` (+ ``cal_dis`` ``wr.py:97-112``)
* initial rays ``ray_initial_numpy``/``cal_ky_numpy``/``change_roots_order``/
  ``cal_ugvg_numpy`` -- ``wr.py:344-395``, ``bs.py:942-1040``, ``wn.py:209-259``

The element-wise operation order is the reference's: every sum is evaluated
left to right exactly as the reference's expression / reduction does it (the
``einsum('snf,s->nf')`` stage sums and the ``norm`` reduction over the 5
variables are sequential in the summed index for every batch size; probed
with NumPy 2.2).  The vectorisation differs (masks instead of index subsets),
which does not change any element's value.
"""
import numpy as np
from scipy.ndimage import convolve

# constants.py:13-29
PI = 3.14159265358979323846264338327950288419716939937510
R_EARTH = 6.3712e6
OMEGA = 7.2921e-5
HOUR = 3600.0
DAY = 24.0 * HOUR
DELT = 1.0e-8

# rkf45.py:601-615 -- Dormand-Prince 5(4)
DP_C = np.array([0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1])
DP_A = np.array([
    [0, 0, 0, 0, 0],
    [1 / 5, 0, 0, 0, 0],
    [3 / 40, 9 / 40, 0, 0, 0],
    [44 / 45, -56 / 15, 32 / 9, 0, 0],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729, 0],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]])
DP_B = np.array([35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84])
DP_E = np.array([-71 / 57600, 0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40])
SAFETY, MIN_FACTOR, MAX_FACTOR = 0.9, 0.2, 10
ERR_EXP = -1 / (4 + 1)        # rkf45.py:360, error_estimator_order = 4


# ----------------------------------------------------------------------------
# transcendentals of the ray loop: NumPy's (glibc sin/cos, SVML tan/power on
# AVX-512 hosts -- what the reference computes with) by default;
# ``device_math()`` swaps in the GPU kernel's own restatement of them
# (oracle/npmath.cpp: the kernel's csrc/np_math.h compiled for the host,
# bitwise equal to NumPy's: tests/test_np_math.py), so that the oracle
# computes with exactly the kernel's functions on any AVX-512 host.
# ----------------------------------------------------------------------------
class _LibM:
    sin = staticmethod(np.sin)
    cos = staticmethod(np.cos)
    tan = staticmethod(np.tan)
    power = staticmethod(np.power)


LIBM = _LibM()
_DEVMATH = None


def _devmath_lib():
    global _DEVMATH
    if _DEVMATH is None:
        import ctypes
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_devmath", "libnpmath.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: build it with `make -C oracle`")
        lib = ctypes.CDLL(path)
        P, I = ctypes.c_void_p, ctypes.c_int64
        for name in ("nm_sin_arr", "nm_cos_arr", "nm_tan_arr", "nm_rcp14_arr"):
            getattr(lib, name).argtypes = [P, P, I]
        lib.nm_pow_arr.argtypes = [P, P, I, P, I]
        _DEVMATH = lib
    return _DEVMATH


def _dm_unary(name):
    def f(x):
        x = np.asarray(x, np.float64)
        xc = np.ascontiguousarray(x)
        out = np.empty_like(xc)
        getattr(_devmath_lib(), name)(xc.ctypes.data, out.ctypes.data, xc.size)
        return out.reshape(x.shape)
    return f


def _dm_power(x, y):
    x, y = np.broadcast_arrays(np.asarray(x, np.float64), np.asarray(y, np.float64))
    xc, yc = np.ascontiguousarray(x), np.ascontiguousarray(y)
    out = np.empty(xc.shape)
    _devmath_lib().nm_pow_arr(xc.ctypes.data, yc.ctypes.data, 1, out.ctypes.data, xc.size)
    return out


class device_math:
    """Context manager: the oracle uses the kernel's sin/cos/tan/power inside."""

    def __enter__(self):
        _devmath_lib()
        self._saved = (LIBM.sin, LIBM.cos, LIBM.tan, LIBM.power)
        LIBM.sin, LIBM.cos = _dm_unary("nm_sin_arr"), _dm_unary("nm_cos_arr")
        LIBM.tan = _dm_unary("nm_tan_arr")
        LIBM.power = _dm_power
        return LIBM

    def __exit__(self, *exc):
        LIBM.sin, LIBM.cos, LIBM.tan, LIBM.power = self._saved
        return False


# ----------------------------------------------------------------------------
# basic state  (bs.py)
# ----------------------------------------------------------------------------
class Background:
    """The 18-field stack ``fields[nlon+1, nlat, 18]`` plus its float32-rounded grid."""

    def __init__(self, u, v, lat, lon, xcyclic=True):
        """``u, v``: float32 ``(nlat, nlon)``; ``lat, lon``: float32 degrees (ascending lat)."""
        nlat, nlon = u.shape
        # bs.py:225-236: degrees -> radians evaluated in float32, then upcast.
        self.lat = (np.asarray(lat, np.float32) * PI / 180).astype(np.float64)
        self.lon = (np.asarray(lon, np.float32) * PI / 180).astype(np.float64)
        self.u = np.asarray(u, np.float32).T          # (nlon, nlat) views, bs.py:245-247
        self.v = np.asarray(v, np.float32).T
        self.dx = np.array([2.0 * PI / nlon])          # bs.py:77-78
        self.dy = np.array([PI / (nlat - 1)])
        self.fields = self._prepare(xcyclic)

    # periodic-x / one-sided-y finite differences, bs.py:121-200
    def _dx1(self, f):
        f = f.astype(np.float64)
        g = np.concatenate([f[-1:], f, f[:1]], axis=0)
        return (g[2:] - g[:-2]) / (2.0 * self.dx)

    def _dy1(self, f):
        f = f.astype(np.float64)
        out = np.empty_like(f)
        out[:, 1:-1] = (f[:, 2:] - f[:, :-2]) / (2.0 * self.dy)
        out[:, 0] = (f[:, 1] - f[:, 0]) / self.dy
        out[:, -1] = (f[:, -1] - f[:, -2]) / self.dy
        return out

    def _dx2(self, f):
        f = f.astype(np.float64)
        g = np.concatenate([f[-1:], f, f[:1]], axis=0)
        return (g[2:] - 2.0 * g[1:-1] + g[:-2]) / (self.dx ** 2)

    def _dy2(self, f):
        f = f.astype(np.float64)
        out = np.empty_like(f)
        out[:, 1:-1] = (f[:, 2:] - 2.0 * f[:, 1:-1] + f[:, :-2]) / (self.dy ** 2)
        out[:, 0] = out[:, 1]
        out[:, -1] = out[:, -2]
        return out

    def _dxy(self, f):
        # NB: no upcast -- for float32 u, v the 4-point numerator is float32 (bs.py:168-195)
        g = np.concatenate([f[-1:], f, f[:1]], axis=0)
        out = np.empty(f.shape, np.float64)
        out[:, 1:-1] = (g[2:, 2:] - g[2:, :-2] - g[:-2, 2:] + g[:-2, :-2]) / (4.0 * self.dx * self.dy)
        out[:, 0] = out[:, 1]
        out[:, -1] = out[:, -2]
        return out

    @staticmethod
    def _smooth9(f, p=0.5, q=0.25):
        """bs.py:291-305 (in place on [1:-2, 1:-2], scipy convolve, constant mode)."""
        w = np.array([[q / 4, p / 4, q / 4], [p / 4, -(p + q), p / 4], [q / 4, p / 4, q / 4]])
        f[1:-2, 1:-2] = f[1:-2, 1:-2] + convolve(f, w, mode="constant", cval=0.0)[1:-2, 1:-2]
        return f

    def _vorticity(self):
        """bs.py:264-279."""
        ucos = (self.u * np.cos(self.lat[None, :])).astype(np.float64)
        q = np.zeros(self.u.shape)
        c = np.cos(self.lat[1:-1])[None, :]
        s = np.sin(self.lat[1:-1])[None, :]
        q[:, 1:-1] = (self._dx1(self.v)[:, 1:-1] - self._dy1(ucos)[:, 1:-1]) / c \
            + 2.0 * OMEGA * s * R_EARTH
        q[:, 0] = q[:, 1]
        q[:, -1] = q[:, -2]
        return q

    def _prepare(self, xcyclic):
        """bs.py:318-372."""
        u, v = self.u, self.v
        q = self._vorticity()
        d = {}
        d["ux"], d["uy"] = self._dx1(u), self._dy1(u)
        d["vx"], d["vy"] = self._dx1(v), self._dy1(v)
        d["qx"], d["qy"] = self._dx1(q), self._dy1(q)
        qxx, qyy, qxy = self._dx2(q), self._dy2(q), self._dxy(q)
        qyx = qxy.copy()
        third = [self._dx1(qxx), self._dy1(qxx), self._dy1(qxy), self._dy1(qyy),
                 self._dx1(qxy), self._dx1(qyy)]
        qxx, qyy, qxy = self._smooth9(qxx), self._smooth9(qyy), self._smooth9(qxy)
        stack = [u, v, d["ux"], d["uy"], d["vx"], d["vy"], d["qx"], d["qy"],
                 qxx, qxy, qyx, qyy] + third
        f = np.stack(stack, axis=-1).astype(np.float64)
        if xcyclic:
            f = np.concatenate([f, f[0:1]], axis=0)
        return f


class TimeVaryingBackground:
    """Time-varying basic state -- THIS FRAMEWORK'S EXTENSION, not in the reference
    (its ``fun`` ignores ``t``, wr.py:784-789).  Parity of
    the extension is against this restatement; its building blocks are the
    reference's (``Background`` per level, bilinear ``_cell``), and at a level
    time ``t0 + j*dt`` it returns level ``j``'s values bit for bit.

    Per point: ``s = (t - t0)/dt``, ``j = clip(floor(s), 0, nlev-2)``,
    ``w = clip(s - j, 0, 1)``, ``g = g_j (1 - w) + g_{j+1} w`` after the bilinear
    lookup of each level (include/rwrt.h ``rwrt_background``).  ``fp32``: the
    levels are stored in float32 (rounded once), arithmetic stays float64.
    Only the 11 fields the ray path reads are carried (the others are NaN).
    """
    HOT = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11]

    def __init__(self, levels, t0=0.0, dt=6 * HOUR, fp32=False):
        self.lat, self.lon = levels[0].lat, levels[0].lon
        F = np.stack([b.fields for b in levels])                    # (nlev, W, H, 18)
        if fp32:
            F = F.astype(np.float32).astype(np.float64)
        mask = np.zeros(F.shape[-1], bool)
        mask[self.HOT] = True
        F[..., ~mask] = np.nan
        self.F = F
        self.fields = F[0]
        self.nlev, self.t0, self.dt = len(levels), float(t0), float(dt)

    def interp_time(self, c, t):
        s = (t - self.t0) / self.dt
        j = np.floor(s).astype("int32")
        j = np.clip(j, 0, self.nlev - 2) if self.nlev > 1 else np.zeros_like(j)
        w = np.clip(s - j, 0.0, 1.0)
        jb = j + 1 if self.nlev > 1 else j
        ok, x0, x1, y0, y1, wa, wb, wc, wd = c
        F = self.F
        ga = (F[j, x0, y1] * wa[:, None] + F[j, x1, y1] * wb[:, None]
              + F[j, x0, y0] * wc[:, None] + F[j, x1, y0] * wd[:, None])
        gb = (F[jb, x0, y1] * wa[:, None] + F[jb, x1, y1] * wb[:, None]
              + F[jb, x0, y0] * wc[:, None] + F[jb, x1, y0] * wd[:, None])
        return ga * (1.0 - w)[:, None] + gb * w[:, None]


# ----------------------------------------------------------------------------
# interpolation + Mercator conversion
# ----------------------------------------------------------------------------
def _cell(bg, lon, lat):
    """Bilinear cell of ``batch_linint2_metpy`` (interpolation.py:77-135) for the
    in-range points: ``(ok, x0, x1, y0, y1, wa, wb, wc, wd)``."""
    lon = lon % (2 * PI)                                  # bs.py:519
    ok = np.where(np.abs(lat) <= 0.5 * PI)[0]             # bs.py:787
    xs = lon[ok] % (2 * np.pi)                            # interpolation.py:80
    fx = (xs - bg.lon[0]) / (bg.lon[1] - bg.lon[0])
    fy = (lat[ok] - bg.lat[0]) / (bg.lat[1] - bg.lat[0])
    W, H = bg.fields.shape[-3], bg.fields.shape[-2]
    ix = np.floor(fx).astype("int32")
    iy = np.floor(fy).astype("int32")
    x0, x1 = np.clip(ix, 0, W - 1), np.clip(ix + 1, 0, W - 1)
    y0, y1 = np.clip(iy, 0, H - 1), np.clip(iy + 1, 0, H - 1)
    sx, sy = fx - x0, fy - y0
    wa, wb = (1 - sx) * sy, sx * sy
    wc, wd = (1 - sx) * (1 - sy), sx * (1 - sy)
    return ok, x0, x1, y0, y1, wa, wb, wc, wd


def _bilinear(F, c):
    ok, x0, x1, y0, y1, wa, wb, wc, wd = c
    return (F[x0, y1] * wa[:, None] + F[x1, y1] * wb[:, None]
            + F[x0, y0] * wc[:, None] + F[x1, y0] * wd[:, None])


def mercator_point(bg, lon, lat, t=None):
    """``BS.cal_bs_mercator_point(lon, lat, mode='numpy')``: returns ``(18, N)``.

    ``t`` (per point) is read only by a ``TimeVaryingBackground``."""
    c = _cell(bg, lon, lat)
    ok = c[0]
    vals = np.full((bg.fields.shape[-1], len(lat)), np.nan)
    if isinstance(bg, TimeVaryingBackground):
        vals[:, ok] = bg.interp_time(c, np.broadcast_to(t, lat.shape)[ok]).T
    else:
        vals[:, ok] = _bilinear(bg.fields, c).T
    (fu, fv, fux, fuy, fvx, fvy, fqx, fqy, fqxx, fqxy, fqyx, fqyy,
     fqxxx, fqxxy, fqxyy, fqyyy, fqyxx, fqyyx) = vals
    c, s, t = LIBM.cos(lat), LIBM.sin(lat), LIBM.tan(lat)
    m = np.ones(c.shape)
    m[np.abs(c) <= 0.0175] = 0
    c = c * m + (1 - m) * 1e-6
    out = [fu / c * m, fv / c * m, fux / c * m, (fuy + t * fu) * m,
           fvx / c * m, (fvy + t * fv) * m, fqx * m, fqy * c * m,
           fqxx * m, fqxy * c * m * m, fqxy * c * m,
           (fqyy * c - fqy * s) * c * m,
           fqxxx * m, fqxxy * c * m, (fqxyy * c - fqxy * s) * c * m,
           fqyyy * m, fqyxx * c * m, (fqyyx * c - fqxy * s) * c * m]
    return np.array(out)


def ugvg_extent(fu, fv, fqx, fqy, k, l):
    """wn.py:266-294 (group velocity, Mercator)."""
    kap = l / k
    kap2 = kap * kap
    kap1 = 1.0 + kap2
    den = k * k * kap1 * kap1
    ug = fu + ((1. - kap2) * fqy - 2. * kap * fqx) / den
    vg = fv + (2. * kap * fqy + (1. - kap2) * fqx) / den
    return ug, vg


def rhs(bg, y, t=None):
    """``WR.diffun_numpy`` on ``y[5, N]`` -> ``(dydt[5, N], bad[N])`` (``t``: time
    of each column, read only by a ``TimeVaryingBackground``)."""
    lon, lat, kx, ky, amp = y[0], y[1], y[2], y[3], y[4]
    bad = (np.abs(lat) >= 0.5 * PI) | (np.abs(ky) >= 100.0)          # wr.py:508-510
    ky = ky.copy()
    ky[bad] = np.nan
    M = mercator_point(bg, lon.reshape(-1), lat.reshape(-1), t)
    fmu, fmv, fmux, fmuy, fmvx, fmvy, fmqx, fmqy, fmqxx, fmqxy, fmqyx, fmqyy = M[:12]
    ug, vg = ugvg_extent(fmu, fmv, fmqx, fmqy, kx, ky)
    # wr.py:44-82 core_diffun
    kap = ky / kx
    kap2 = kap * kap
    kap1 = 1 + kap * kap
    kk = kx * kx * kap1
    dk = -kx * ((fmux + kap * fmvx) + (kap * fmqxx - fmqyx) / kk)
    dl = -kx * ((fmuy + kap * fmvy) + (kap * fmqxy - fmqyy) / kk)
    damp = (2.0 * (fmux + fmvy + kap * (fmvx + fmuy)) / kap1
            + 2.0 * (kap * (fmqxx - fmqyy) + (kap2 - 1.0) * fmqxy) / (kk * kap1)
            + -2.0 * LIBM.sin(lat) * fmv)
    d = np.array([ug / R_EARTH, vg * LIBM.cos(lat) / R_EARTH, dk / R_EARTH,
                  dl / R_EARTH, damp * amp / R_EARTH])
    d[:, bad] = np.nan
    return d, bad


def norm5(x):
    """``rkf45.norm``: RMS over axis 0 (sequential sum of squares)."""
    return np.linalg.norm(x, axis=0) / x.shape[0] ** 0.5


# ----------------------------------------------------------------------------
# the batched DP5(4) stepper
# ----------------------------------------------------------------------------
def initial_step(fun, t0, y0, f0, rtol, atol):
    """``select_initial_step`` (rkf45.py:34-99), direction = +1."""
    scale = atol + np.abs(y0) * rtol
    d0, d1 = norm5(y0 / scale), norm5(f0 / scale)
    h0 = 0.01 * d0 / d1
    h0[d0 < 1e-5] = 1e-6
    h0[d1 < 1e-5] = 1e-6
    f1 = fun(t0 + h0, y0 + h0 * f0)
    d2 = norm5((f1 - f0) / scale) / h0
    with np.errstate(all="ignore"):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            h1 = LIBM.power(0.01 / np.nanmax([d1, d2], axis=0), 1 / 5)
    tiny = ~(d1 > 1e-15) & ~(d2 > 1e-15)
    h1[tiny] = np.maximum(1e-6, h0 * 1e-3)[tiny]
    return np.minimum(100 * h0, h1)


def wsum(K, w):
    """``np.einsum('snf,s->nf', K, w)`` in NumPy's own summation order.

    In ``rk_step`` the stage array ``K`` is ``self.K[..., indices]`` (a fancy-
    indexed copy laid out column-major in ``f``).  With ``n > 1`` variables the
    iterator keeps ``s`` as the outer loop, so the sum is sequential in ``s``
    (the ray problem: n = 5; pinned by the trajectory fixtures).  With ONE
    variable ``s`` becomes the inner loop and einsum runs its SIMD dot product
    (SSE2 baseline of this NumPy build: 2 lanes): even and odd terms are summed
    separately and added at the end (pinned by the stepper KAT fixtures).
    """
    x = [K[j] * w[j] for j in range(len(w))]
    if K.shape[1] == 1:
        even, odd = np.zeros_like(K[0]), np.zeros_like(K[0])
        for j in range(len(w)):
            if j % 2 == 0:
                even = even + x[j]
            else:
                odd = odd + x[j]
        return even + odd
    acc = np.zeros_like(K[0])
    for j in range(len(w)):
        acc = acc + x[j]
    return acc


def dp54_attempt(fun, t, y, f, h):
    """``rk_step`` (rkf45.py:259-321): returns ``(y_new, K[7, n, N])``."""
    K = np.empty((7,) + y.shape)
    K[0] = f
    for s in range(1, 6):
        K[s] = fun(t + DP_C[s] * h, y + wsum(K[:s], DP_A[s, :s]) * h)
    y_new = y + h * wsum(K[:6], DP_B)
    K[6] = fun(t + h, y_new)
    return y_new, K


def error_norm(K, h, y, y_new, rtol, atol):
    """``_estimate_error_norm`` with ``scale`` (rkf45.py:368-373,442-446)."""
    acc = wsum(K, DP_E)
    scale = atol + np.maximum(np.abs(y), np.abs(y_new)) * rtol
    en = norm5(h[None, :] * acc / scale)
    en[np.isnan(en)] = 0
    return en


class SolverFailed(Exception):
    """rkf45.py:423-425: every still-retrying column has a NaN step."""


class DP54:
    """Per-column adaptive DP5(4) stepper with the reference's step semantics.

    ``RungeKutta.__init__`` / ``OdeSolver.step`` / ``_step_impl``
    (rkf45.py:185-253,335-514), one column per ray.
    """

    def __init__(self, fun, t0, y0, t_bound, rtol, atol, min_step, autonomous=True):
        self.fun = fun
        self.rtol = max(rtol, 100 * np.finfo(np.float64).eps)          # validate_tol
        self.atol = atol
        self.y = np.array(y0, dtype=np.float64)
        n = self.y.shape[-1]
        self.t = t0 * np.ones(n)
        self.f = fun(self.t, self.y)
        self.h_abs = initial_step(fun, self.t, self.y, self.f, self.rtol, self.atol)
        self.min_step = min(min_step, (t_bound - t0) * 0.001)          # rkf45.py:362
        self.autonomous = autonomous
        self.nacc = np.zeros(n, np.int64)
        self.nrej = np.zeros(n, np.int64)

    def advance_to(self, t_bound):
        """Repeat ``solver.step()`` until every column reaches ``t_bound``."""
        while not np.all(self.t == t_bound):
            self._step(t_bound)
            if np.all(self.t - t_bound >= 0):
                break

    def _step(self, tb):
        t, y = self.t, self.y
        if not self.autonomous:
            self.f = self.fun(t, y)        # rkf45.py:378 (== FSAL K6 when autonomous)
        f = self.f
        hs = np.maximum(self.h_abs, self.min_step)
        frozen = np.isnan(np.mean(y, axis=0))                          # rkf45.py:400-402
        t[frozen] = tb
        todo = ~frozen & (t != tb)
        rejected = np.zeros(t.shape, bool)
        t_new, y_new, f_new = t.copy(), y.copy(), f.copy()
        while todo.any():
            idx = np.where(todo)[0]
            if np.isnan(hs[idx]).all():
                raise SolverFailed()
            h = hs[idx] * 1.0
            tn = t[idx] + h
            tn[tn - tb > 0] = tb
            h = tn - t[idx]
            ha = np.abs(h)
            yn, K = dp54_attempt(self.fun, t[idx], y[:, idx], f[:, idx], h)
            en = error_norm(K, h, y[:, idx], yn, self.rtol, self.atol)
            ok = en < 1
            with np.errstate(divide="ignore"):
                grow = np.minimum(MAX_FACTOR, SAFETY * LIBM.power(en, ERR_EXP))
                grow[en == 0] = MAX_FACTOR
                grow = np.where(rejected[idx], np.minimum(1.0, grow), grow)
                shrink = np.maximum(MIN_FACTOR, SAFETY * LIBM.power(en, ERR_EXP))
            ha = np.where(ok, ha * grow, ha * shrink)
            hs[idx] = ha
            acc_i, rej_i = idx[ok], idx[~ok]
            t_new[acc_i] = tn[ok]
            y_new[:, acc_i] = yn[:, ok]
            f_new[:, acc_i] = K[6][:, ok]
            self.nacc[acc_i] += 1
            self.nrej[rej_i] += 1
            rejected[rej_i] = True
            todo[acc_i] = False
        t_new[np.isnan(t_new)] = tb
        self.t, self.y, self.f, self.h_abs = t_new, y_new, f_new, hs


# ----------------------------------------------------------------------------
# the interval loop (WR.core_ray_run_rk45)
# ----------------------------------------------------------------------------
def cal_dis(lon_c, lat_c, lon_p, lat_p):
    """wr.py:97-112 (haversine)."""
    a = LIBM.sin((lat_c - lat_p) / 2.0) ** 2 \
        + LIBM.cos(lat_p) * LIBM.cos(lat_c) * LIBM.sin((lon_c - lon_p) / 2.0) ** 2
    return np.abs(2 * np.arctan2(np.sqrt(a), np.sqrt(1.0 - a)))


def ray_run(bg, y0, nt, tstep, rtol=1e-6, atol=1e-6, msf=1e-3, cut_off=0.1,
            ttotal=None, row0=None, fsal=True, columns=None):
    """Integrate rays ``y0[5, nray]`` -> history ``hist[7, nt, nray]`` (rows 1.. filled).

    Row 0 of ``hist`` is ``row0[7, nray]`` when given (the ``ray_initial`` rows),
    else ``y0`` with NaN ``ug, vg``.  Returns ``(hist, nacc, nrej, status)``;
    ``status`` is 0, or -1 when the solver failed (remaining rows NaN,
    wr.py:886-887).

    ``fsal=False`` runs the reference's own loop shape: ``f = fun(t, y)``
    recomputed for EVERY column at each step start (rkf45.py:378, frozen and
    finished columns included) besides the rejected subsets' re-runs
    (rkf45.py:410-502) -- the same values (the RHS is autonomous: f is K6 bit
    for bit), about twice the RHS columns; bench.py times it as the
    reference-structured CPU baseline.  ``columns`` (a one-element list, if
    given) accumulates the RHS columns evaluated.
    """
    def fun(t, y):
        if columns is not None:
            columns[0] += y.shape[-1]
        return rhs(bg, y, t)[0]
    nray = y0.shape[1]
    hist = np.full((7, nt, nray), np.nan)
    if row0 is not None:
        hist[:, 0] = row0
    else:
        hist[:5, 0] = y0
    t_eval = np.arange(nt) * tstep
    if ttotal is not None and t_eval[-1] > ttotal:
        t_eval[-1] = ttotal
    cut = cut_off * tstep / 3600.0                                     # wr.py:170
    try:
        sol = DP54(fun, 0, y0, tstep, rtol, atol, msf * tstep, autonomous=fsal)
    except SolverFailed:
        return hist, np.zeros(nray, np.int64), np.zeros(nray, np.int64), -1
    for i in range(1, nt):
        try:
            sol.advance_to(t_eval[i])
        except SolverFailed:
            return hist, sol.nacc, sol.nrej, -1
        y = sol.y
        y[:, np.abs(y[1]) >= 0.5 * PI] = np.nan                         # wr.py:838-843
        y[:, np.abs(cal_dis(y[0], y[1], hist[0, i - 1], hist[1, i - 1])) >= cut] = np.nan
        if np.isnan(y[0]).all() or (np.abs(y[1]) > 0.5 * PI).all():     # wr.py:853-855
            break
        M = mercator_point(bg, y[0], y[1], np.full(nray, t_eval[i]))   # at the row time
        ug, vg = ugvg_extent(M[0], M[1], M[6], M[7], y[2], y[3])
        hist[:5, i] = y
        hist[5, i], hist[6, i] = ug, vg
    return hist, sol.nacc, sol.nrej, 0


# ----------------------------------------------------------------------------
# initial rays (host prerequisite)
# ----------------------------------------------------------------------------
def _order_roots(m, n):
    """``change_roots_order`` (bs.py:942-982) on one 3-vector; returns reversed."""
    m = list(m)
    if n == 3:
        best = 1
        for i in (1, 2):
            if m[i] >= 0. and m[i] < m[best]:
                m[i], m[best] = m[best], m[i]
                best = i
        if m[0] < 0:
            m[0], m[1] = m[1], m[0]
        if (m[1] < 0 and m[2] < 0 and m[1] < m[2]) or (m[1] > 0 and m[2] < 0.):
            m[1], m[2] = m[2], m[1]
    elif n == 2:
        if not (not np.isnan(m[0]) and m[0] > 0):
            m[0], m[1] = m[1], m[0]
    elif n == 1:
        for i in range(3):
            if (not np.isnan(m[i])) and m[i] >= 0 and i != 0:
                m[i], m[0] = m[0], m[i]
            elif (not np.isnan(m[i])) and m[i] <= 0. and i != 2:
                m[i], m[1] = m[1], m[i]
    for i in range(3):
        if (not np.isnan(m[i])) and abs(m[i]) > 100.:
            m[i] = np.nan
    return np.array(m[::-1])


def meridional_roots(fu, fv, fqx, fqy, freq, k):
    """``cal_ky_numpy`` (bs.py:985-1040) -> ``(nsource, 3)``."""
    out = np.full((len(fu), 3), np.nan)
    if k == 0:
        return out
    ps = freq / k * R_EARTH
    coef = np.stack([k ** 3 * (fu - ps - fqy / k ** 2), k ** 2 * fv + fqx,
                     k * (fu - ps), fv], axis=-1)
    for i in range(coef.shape[0]):
        c = coef[i]
        deg = 3
        while deg > 0 and abs(c[deg]) == 0:
            deg -= 1
        if deg < 1:
            continue
        r = np.roots(c[:deg + 1][::-1] + 0j)
        real = [z.real for z in r if abs(z.imag) < DELT]
        m = np.array(real[:3] + [np.nan] * (3 - len(real)))
        out[i] = _order_roots(m, len(real))
    return out


def ugvg_init(fu, fv, fqx, fqy, k, m):
    """``cal_ugvg_numpy`` (wn.py:209-259) -- the t = 0 group velocity."""
    if k == 0:
        return np.zeros(m.shape), np.zeros(m.shape)
    nans = np.einsum("ij,j->ij", m * 0, fu * fqx * fqy * 0) + 1
    nans[np.isnan(nans)] = 0
    a = k * k - m * m
    b = 2 * k * m
    c = k * k + m * m
    ug = (fu + (a * fqy - b * fqx) / c ** 2) * nans
    vg = (fv + (a * fqx + b * fqy) / c ** 2) * nans
    return ug, vg


def ray_initial(bg, src_lon, src_lat, zwn, freq):
    """``WR.ray_initial_numpy`` (wr.py:344-395) -> 7 arrays ``(3, nsource, nzwn)``."""
    ns, nz = len(src_lon), len(zwn)
    shape = (3, ns, nz)
    lon = np.ones(shape) * src_lon[None, :, None]
    lat = np.ones(shape) * src_lat[None, :, None]
    M = mercator_point(bg, src_lon, src_lat)
    fmu, fmv, fmqx, fmqy = M[0], M[1], M[6], M[7]
    kx = np.ones(shape) * zwn[None, None, :]
    ky, amp, ug, vg = (np.full(shape, np.nan) for _ in range(4))
    freq = np.array([freq], dtype=np.float64)
    for iz in range(nz):
        m = meridional_roots(fmu, fmv, fmqx, fmqy, freq, zwn[iz]).T
        ky[:, :, iz] = m
        a = np.ones(m.shape)
        a[np.isnan(m)] = np.nan
        amp[:, :, iz] = a
        ug[:, :, iz], vg[:, :, iz] = ugvg_init(fmu, fmv, fmqx, fmqy, zwn[iz], m)
    return lon, lat, kx, ky, amp, ug, vg


def source_matrix(SW_lon, SW_lat, dlon, dlat, nnx, nny):
    """``WR.set_source_matrix`` (wr.py:236-258): radians, index ``iy*nnx + ix``."""
    if SW_lat + (nny - 1) * dlat > 89.0:
        raise ValueError("source latitude out of -90~90 range!")
    deg2rad = PI / 180.0
    SW_lon = SW_lon % 360.0
    lon = np.empty(nnx * nny)
    lat = np.empty(nnx * nny)
    for iy in range(nny):
        for ix in range(nnx):
            lon[iy * nnx + ix] = ((SW_lon + ix * dlon) % 360.0) * deg2rad
            lat[iy * nnx + ix] = (SW_lat + iy * dlat) * deg2rad
    return lon, lat


def run_config(bg, cfg, nt=None, **kw):
    """End-to-end oracle of ``real2d_hnf`` for a ``synthetic.SeedConfig``."""
    slon, slat = source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = ray_initial(bg, slon, slat, cfg.zwn, cfg.freq)
    tstep = cfg.tstep * HOUR
    if nt is None:
        nt = int(cfg.ttotal * DAY / tstep) + 1
    y0 = np.array(rows[:5]).reshape(5, -1)
    row0 = np.array(rows).reshape(7, -1)
    return ray_run(bg, y0, nt, tstep, cfg.rtol, cfg.atol, cfg.MinStepFactor,
                   ttotal=cfg.ttotal * DAY, row0=row0, **kw)


# ----------------------------------------------------------------------------
# fixed-step RK4 (the reference's default integrator, inte_method='')
# ----------------------------------------------------------------------------
def rhs7(bg, y):
    """``diffun_numpy`` with all 7 outputs: (dlon, dlat, dk, dl, damp, ug/R, vg).

    ``core_diffun`` (wr.py:68-81) aliases ``dlon = ug`` and divides it in place,
    so the returned ``dug`` is ``ug / R`` while ``dvg`` is ``vg`` itself.
    Returns ``(d[7, N], bad[N])``.
    """
    d5, bad = rhs(bg, y[:5])
    lat, ky, kx = y[1], y[3].copy(), y[2]
    ky[bad] = np.nan
    M = mercator_point(bg, y[0].reshape(-1), lat.reshape(-1))
    ug, vg = ugvg_extent(M[0], M[1], M[6], M[7], kx, ky)
    d = np.concatenate([d5, (ug / R_EARTH)[None], vg[None]], axis=0)
    d[5:, bad] = np.nan
    return d, bad


def ray_run_rk4(bg, y0, nt, tstep, cut_off=0.1, row0=None):
    """``core_ray_run_numpy`` (wr.py:702-765) with ``rk4_step_numpy`` (wr.py:583-622).

    Rays where any of the four stage inputs is masked (|lat| >= pi/2 or
    |l| >= 100) keep their state for that step (wr.py:609-618); NaN states
    are not masked and propagate.  Returns ``(hist[7, nt, nray], status)``.
    """
    nray = y0.shape[1]
    hist = np.full((7, nt, nray), np.nan)
    if row0 is not None:
        hist[:, 0] = row0
    else:
        hist[:5, 0] = y0
    dt = np.array([tstep], dtype=np.float64)
    cut = cut_off * dt / 3600.0
    y = np.array(hist[:, 0])
    for it in range(nt - 1):
        k1, m1 = rhs7(bg, y)
        y_next = y.copy()
        valid1 = ~m1
        if np.any(valid1):
            k2, m2 = rhs7(bg, y + 0.5 * dt * k1)
            k3, m3 = rhs7(bg, y + 0.5 * dt * k2)
            k4, m4 = rhs7(bg, y + dt * k3)
            ok = valid1 & ~m2 & ~m3 & ~m4
            ks = (dt / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)          # core_rk4_step wr.py:89-95
            prop = y.copy()
            prop[0:5] = y[0:5] + ks[0:5]
            prop[5:] = ks[5:] / dt
            y_next[:, ok] = prop[:, ok]
        yn = y_next
        yn[:5, np.abs(yn[1]) >= 0.5 * PI] = np.nan                     # wr.py:721-726
        yn[:5, np.abs(cal_dis(yn[0], yn[1], hist[0, it], hist[1, it])) >= cut] = np.nan
        if np.isnan(yn[0]).all() or (np.abs(yn[1]) > 0.5 * PI).all():  # wr.py:735-736
            break
        M = mercator_point(bg, yn[0], yn[1])
        ug, vg = ugvg_extent(M[0], M[1], M[6], M[7], yn[2], yn[3])
        hist[:5, it + 1] = yn[:5]
        hist[5, it + 1], hist[6, it + 1] = ug, vg
        y = np.array(hist[:, it + 1])
    return hist, 0


def run_config_rk4(bg, cfg, nt=None):
    slon, slat = source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = ray_initial(bg, slon, slat, cfg.zwn, cfg.freq)
    tstep = cfg.tstep * HOUR
    if nt is None:
        nt = int(cfg.ttotal * DAY / tstep) + 1
    row0 = np.array(rows).reshape(7, -1)
    return ray_run_rk4(bg, row0[:5].copy(), nt, tstep, row0=row0)


def ray_run_timed(args):
    """``(bg_kwargs, y0, nt, tstep)`` -> (accepted steps, seconds in ray_run):
    one process of bench.py's multi-core CPU baseline (picklable, imports
    nothing beyond this module)."""
    import time
    bg_kwargs, y0, nt, tstep = args[:4]
    fsal = args[4] if len(args) > 4 else True
    bg = Background(**bg_kwargs)
    t0 = time.perf_counter()
    with np.errstate(all="ignore"):
        _, nacc, _, _ = ray_run(bg, y0, nt, tstep, fsal=fsal)
    return int(nacc.sum()), time.perf_counter() - t0
