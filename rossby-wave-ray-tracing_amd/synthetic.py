"""Synthetic basic states and seed grids for the BASELINE configurations.

The reference ships no input data: ``main_wr.py:23`` points
``inputuv`` at a placeholder path.  Every background used by the tests, the
golden fixtures and ``bench.py`` is therefore synthesised here, exactly as
SURVEY.md §8(d) specifies:

* grid: 2.5 deg, ``lat = arange(-90, 90+, 2.5)`` float32 ascending (73),
  ``lon = arange(0, 360, 2.5)`` float32 (144);
* ``U(phi) = [45 exp(-((phi-32)/10)^2) + 28 exp(-((phi+45)/12)^2)
  - 5 exp(-(phi/10)^2)] cos(phi)`` m/s (DJF-like 300 hPa jets), ``V = 0``;
* non-zonal variant: ``U (1 + 0.3 cos(lambda - 140 deg))`` and
  ``V = 4 sin(3 lambda) cos^2(phi)``.

Arrays are returned the way ``BS.loadbs_ncfile`` (``bs.py:202-262``) reads
them from netCDF: ``u, v`` float32 ``(nlat, nlon)``, ``lat, lon`` float32.
"""
import numpy as np

__all__ = ["background", "background_level", "SeedConfig", "CONFIGS", "config"]


def background(kind="zonal", res=2.5):
    """Return ``dict(u, v, lat, lon)`` for a deterministic synthetic basic state."""
    lat = np.arange(-90.0, 90.0 + res / 2, res).astype(np.float32)
    lon = np.arange(0.0, 360.0, res).astype(np.float32)
    phi = lat.astype(np.float64)[:, None]
    lam = lon.astype(np.float64)[None, :]
    jets = (45.0 * np.exp(-((phi - 32.0) / 10.0) ** 2)
            + 28.0 * np.exp(-((phi + 45.0) / 12.0) ** 2)
            - 5.0 * np.exp(-(phi / 10.0) ** 2))
    coslat = np.cos(np.deg2rad(phi))
    u = jets * coslat * np.ones_like(lam)
    v = np.zeros_like(u)
    if kind == "superrotation":
        # solid-body super-rotation U = U0 cos(phi), V = 0 (U0 = 15 m/s): the
        # docs' Great-Circle example (Hoskins & Karoly 1981), whose
        # stationary rays follow great circles
        u = 15.0 * coslat * np.ones_like(lam)
    elif kind == "nonzonal":
        u = u * (1.0 + 0.3 * np.cos(np.deg2rad(lam - 140.0)))
        v = 4.0 * np.sin(3.0 * np.deg2rad(lam)) * coslat ** 2
    elif kind not in ("zonal", "superrotation"):
        raise ValueError(f"unknown background kind {kind!r}")
    return dict(u=u.astype(np.float32), v=v.astype(np.float32), lat=lat, lon=lon)


def _jets(phi_deg):
    return (45.0 * np.exp(-((phi_deg - 32.0) / 10.0) ** 2)
            + 28.0 * np.exp(-((phi_deg + 45.0) / 12.0) ** 2)
            - 5.0 * np.exp(-(phi_deg / 10.0) ** 2))


def background_level(j, res=2.5, dt_hours=6.0, seed=0, nlev_max=4096):
    """Level ``j`` (valid at ``j * dt_hours``) of the time-varying C5 background
    (SURVEY.md §8(d)): the non-zonal jet of ``background('nonzonal')`` plus a
    travelling wave-4 that moves east at 10 deg/day with a random-walk phase
    (``numpy.random.default_rng(seed)``), and a westward-drifting wave-3 in V.
    Returns ``dict(u, v, lat, lon)`` like ``background``."""
    lat = np.arange(-90.0, 90.0 + res / 2, res).astype(np.float32)
    lon = np.arange(0.0, 360.0, res).astype(np.float32)
    phi = lat.astype(np.float64)[:, None]
    lam = np.deg2rad(lon.astype(np.float64))[None, :]
    t_days = j * dt_hours / 24.0
    phase = np.cumsum(np.random.default_rng(seed).normal(0.0, 0.08, size=nlev_max))[j]
    coslat = np.cos(np.deg2rad(phi))
    wave4 = np.cos(4.0 * (lam - np.deg2rad(10.0) * t_days) + phase)
    u = _jets(phi) * coslat * (1.0 + 0.3 * np.cos(lam - np.deg2rad(140.0)) + 0.15 * wave4)
    v = (4.0 * np.sin(3.0 * lam + np.deg2rad(5.0) * t_days)
         + 2.0 * np.sin(4.0 * (lam - np.deg2rad(10.0) * t_days) + phase)) * coslat ** 2
    return dict(u=u.astype(np.float32), v=v.astype(np.float32), lat=lat, lon=lon)


class SeedConfig:
    """One ray-seed configuration (the ``parameters`` keys of ``main_wr.py:5-30``)."""

    def __init__(self, name, SW_lon, SW_lat, dlon, dlat, nnx, nny, zwn,
                 freq=0.0, tstep=2.0, ttotal=90.0, rtol=1e-6, atol=1e-6,
                 MinStepFactor=1e-3, bg="zonal"):
        self.name = name
        self.SW_lon, self.SW_lat = SW_lon, SW_lat
        self.dlon, self.dlat = dlon, dlat
        self.nnx, self.nny = nnx, nny
        self.zwn = np.asarray(zwn, dtype=np.float64)
        self.freq = freq
        self.tstep, self.ttotal = tstep, ttotal
        self.rtol, self.atol, self.MinStepFactor = rtol, atol, MinStepFactor
        self.bg = bg

    @property
    def nsource(self):
        return self.nnx * self.nny

    @property
    def nzwn(self):
        return len(self.zwn)

    @property
    def nray(self):
        return 3 * self.nsource * self.nzwn

    def parameters(self, **over):
        """``main_wr.py``-style parameter dict for this configuration."""
        p = dict(freq=self.freq, mm=None, nn=None, SW_lon=self.SW_lon,
                 SW_lat=self.SW_lat, dlon=self.dlon, dlat=self.dlat,
                 nnx=self.nnx, nny=self.nny, zwn=self.zwn.copy(),
                 nzwn=self.nzwn, tstep=self.tstep, ttotal=self.ttotal,
                 mode="hip", root_method="numpy", inte_method="rk45",
                 xcyclic=True, cal_dtype="float64", read_dtype="float32",
                 rtol=self.rtol, atol=self.atol,
                 MinStepFactor=self.MinStepFactor)
        p.update(over)
        return p


DAY = 86400.0

# SURVEY.md §8(d) "Seeds / rays".  C3's five periods are separate runs of the
# reference (freq is a scalar per WR); ``config('C3', period=...)`` picks one.
CONFIGS = {
    "C1": dict(SW_lon=120.0, SW_lat=30.0, dlon=4, dlat=2, nnx=1, nny=1,
               zwn=[5.0]),
    "C2": dict(SW_lon=90.0, SW_lat=10.0, dlon=4, dlat=2, nnx=16, nny=16,
               zwn=[3.0, 4.0, 5.0, 6.0]),
    "C3": dict(SW_lon=0.0, SW_lat=-88.0, dlon=2, dlat=2, nnx=180, nny=89,
               zwn=[float(k) for k in range(1, 11)]),
    # C5 (BASELINE configs[4]): 1-degree global seeds x k = 1..10 on the 0.25-degree
    # time-varying background; x the 5 C3 periods = 9.67 M ray slots (~4 M live)
    "C5": dict(SW_lon=0.0, SW_lat=-89.0, dlon=1, dlat=1, nnx=360, nny=179,
               zwn=[float(k) for k in range(1, 11)]),
}

C5_PERIODS_DAYS = [None, 10.0]

C3_PERIODS_DAYS = [None, 50.0, 30.0, 20.0, 10.0]   # None = stationary (freq 0)


def c3_freq(period_days):
    """``freq = -2 pi / (P day)`` (the ``main_wr.py:64`` sign)."""
    if period_days is None:
        return 0.0
    return -2.0 * np.pi / (period_days * DAY)


def config(name, **over):
    kw = dict(CONFIGS[name])
    period = over.pop("period", None)
    if name == "C3" and "freq" not in over:
        kw["freq"] = c3_freq(period)
    kw.update(over)
    return SeedConfig(name, **kw)
