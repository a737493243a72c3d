"""Time-varying basic states on the GPU (BASELINE configs[4]).

The reference integrates rays through ONE basic state (``fun`` ignores ``t``,
wr.py:784-789).  ``Levels`` holds a sequence of basic states -- snapshots of
``u, v`` valid at ``t0 + j*dt`` seconds of ray time -- as packed records
``[nlev][nlon+1][nlat][12]`` in HBM, each built on the device by
``rwrt_bs_ready`` (the reference's ``BS.ready``: vorticity, finite
differences, ``smth9``; bit-identical to the host ``BS.fields``).  Storage is
fp64, or fp32 (half the gather bytes; every operation stays fp64).  The ray
kernels interpolate each level in space exactly like the static state and
then linearly in time (include/rwrt.h ``rwrt_background``).

A one-level ``Levels`` is never integrated through the time-varying kernels:
``RayEngine.from_levels`` routes it to the reference's static path.
"""
import numpy as np
import torch

import _hip as H
from bs import BS


def trig_table(lat):
    """``[3, nlat]``: ``np.cos(lat)`` (for ``u cos(lat)``) and, at ``1..nlat-2``,
    ``np.cos``/``np.sin`` of ``lat[1:-1]`` -- the arrays ``calc_absolute_vorticity``
    evaluates (bs.py:264-279), from the host libm."""
    lat = np.asarray(lat, np.float64)
    t = np.zeros((3, len(lat)))
    t[0] = np.cos(lat[None, :])[0]
    t[1, 1:-1] = np.cos(lat[1:-1])
    t[2, 1:-1] = np.sin(lat[1:-1])
    return t


class Levels:
    """``nlev`` basic states on one GPU, packed for the ray kernels."""

    def __init__(self, lat_deg, lon_deg, nlev, t0=0.0, dt=6 * 3600.0, fp32=False, device=None,
                 arith32=False):
        """Axes in degrees (float32, as read from a file); level ``j`` is valid
        at ``t0 + j*dt`` s of ray time (the initial rays use level 0: t0 = 0).
        ``arith32`` (fp32 levels only): the RHS computes in fp32 as well
        (rwrt_background.fp32 = 2; not the reference's arithmetic)."""
        if arith32 and not fp32:
            raise ValueError("arith32 needs fp32 levels")
        self.arith32 = bool(arith32)
        H.require_gpu()
        H.load()
        lat_deg = np.asarray(lat_deg, np.float32)
        lon_deg = np.asarray(lon_deg, np.float32)
        if not (lat_deg[0] < lat_deg[-1]):
            raise ValueError("Levels needs an ascending latitude axis (flip u, v, lat first)")
        self.nlat, self.nlon = len(lat_deg), len(lon_deg)
        # the axes exactly as BS.loadbs_ncfile builds them (float32 arithmetic)
        b = BS(self.nlon, self.nlat)
        b.load_arrays(np.zeros((self.nlat, self.nlon), np.float32),
                      np.zeros((self.nlat, self.nlon), np.float32), lat_deg, lon_deg)
        self.lat, self.lon = b.lat.copy(), b.lon.copy()
        self.dx, self.dy = float(b.dx[0]), float(b.dy[0])
        self.device = torch.device(device or "cuda")
        self.nlev, self.t0, self.dt, self.fp32 = int(nlev), float(t0), float(dt), bool(fp32)
        dtype = torch.float32 if fp32 else torch.float64
        self.packed = torch.empty((self.nlev, self.nlon + 1, self.nlat, H.NFIELD_PACK), dtype=dtype,
                                  device=self.device)
        # the t = 0 state in fp64 for the initial rays (rwrt_ray_initial reads fp64)
        self.level0_f64 = (torch.empty((self.nlon + 1, self.nlat, H.NFIELD_PACK), dtype=torch.float64,
                                       device=self.device) if fp32 else self.packed[0])
        self.trig = torch.as_tensor(trig_table(self.lat), device=self.device)
        self.scratch = torch.empty(4 * self.nlon * self.nlat, dtype=torch.float64, device=self.device)

    @property
    def grid(self):
        from engine import grid_of
        return grid_of(self.lon, self.lat, self.nlon + 1)

    def set_level(self, j, u, v):
        """Build level ``j`` from ``u, v[nlat, nlon]`` (float32, file layout; host
        arrays or device tensors) with ``rwrt_bs_ready`` (asynchronous)."""
        u = torch.as_tensor(u, dtype=torch.float32).to(self.device).contiguous()
        v = torch.as_tensor(v, dtype=torch.float32).to(self.device).contiguous()
        if u.shape != (self.nlat, self.nlon) or v.shape != (self.nlat, self.nlon):
            raise ValueError(f"u, v must be [{self.nlat}, {self.nlon}]")
        H.check(H.load().rwrt_bs_ready(self.nlon, self.nlat, H.dptr(u), H.dptr(v),
                                       H.dptr(self.trig), self.dx, self.dy, H.dptr(self.scratch),
                                       self.packed[j].data_ptr(), int(self.fp32), H.stream(self.device)))
        if j == 0 and self.fp32:
            H.check(H.load().rwrt_bs_ready(self.nlon, self.nlat, H.dptr(u), H.dptr(v),
                                           H.dptr(self.trig), self.dx, self.dy,
                                           H.dptr(self.scratch), self.level0_f64.data_ptr(), 0,
                                           H.stream(self.device)))

    def background(self):
        """The ``rwrt_background`` description of these levels."""
        return H.Background(self.packed.data_ptr(), self.nlev, 2 if self.arith32 else int(self.fp32),
                            self.t0, self.dt)
