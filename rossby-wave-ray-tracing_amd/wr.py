"""Ray tracer object: the reference's ``WR`` (wr.py:114-977) with a HIP ray loop.

Same constructor, attributes (``rlon .. rvg`` of shape ``(nt, 3, nsource,
nzwn)``, NaN-initialised) and methods as the reference.  The ray loop is
selected the same way: ``ray_run(mode, inte_method)`` builds
``mode + '_rk45'`` (wr.py:897-911) and ``core_ray_run`` dispatches it
(wr.py:889-895).  The one integrator this framework provides is
``mode='hip', inte_method='rk45'`` -> ``core_ray_run_hip_rk45``: the fused
MI355X kernel replaces ``core_ray_run_rk45`` (wr.py:767-887) and everything it
calls (RK45 stepper, ``diffun_numpy``, ``cal_bs_mercator_point``,
``cal_ugvg``).  Other modes raise: there is no CPU fallback.
"""
import sys

import numpy as np

from bs import BS, cal_ky
from constants import day, hour, rad2deg, undef, deg2rad
import ncio
from wn import cal_ugvg

SUPPORTED = ("hip_rk45", "hip")      # GPU RK45 (wr.py:767-887) and GPU RK4 (wr.py:702-765)


def progress_bar(current, total, bar_length=50):
    percent = float(current) / total
    arrow = "=" * int(round(percent * bar_length) - 1) + ">"
    sys.stdout.write(f"\rprocess: [{arrow + ' ' * (bar_length - len(arrow))}] "
                     f"{int(round(percent * 100))}%")
    sys.stdout.flush()


class WR:
    """Barotropic Rossby-wave ray tracer (constructor of wr.py:133-171)."""

    def __init__(self, nzwn, nsource, tstep=1. * hour, ttotal=20. * day, freq=0,
                 cal_dtype="float64", read_dtype="float32", rtol=1e-6, atol=1e-6,
                 cut_off=0.1, nx=None, ny=None, ncfile=None, MinStepFactor=1e-3,
                 chunk_rows=None, progress=False):
        if cal_dtype != "float64":
            raise ValueError("cal_dtype must be 'float64' (as in main_wr.py:21)")
        self.all_dtype = cal_dtype
        if nx is None or ny is None:
            if ncfile is None:
                raise ValueError("ncfile is need")
            ny, nx = self.get_defualt_nlon_and_nlat(ncfile)
        self.bs = BS(nx, ny, read_dtype=read_dtype, cal_dtype=cal_dtype)
        self.tstep = np.array([tstep], dtype=cal_dtype)
        self.ttotal = ttotal
        self.freq = np.array([freq], dtype=cal_dtype)
        self.nzwn = nzwn
        self.zwn = np.zeros(nzwn, dtype=cal_dtype)
        self.nsource = nsource
        self.source_lon = np.zeros(nsource, dtype=cal_dtype)
        self.source_lat = np.zeros(nsource, dtype=cal_dtype)
        self.nt = int(self.ttotal / self.tstep[0]) + 1
        shape = (self.nt, 3, nsource, nzwn)
        for name in ("rlon", "rlat", "rzwn", "rmwn", "ramp", "rug", "rvg"):
            setattr(self, name, np.full(shape, undef, dtype=cal_dtype))
        self.rtol, self.atol = rtol, atol
        self.cut_off = cut_off * self.tstep / 3600.
        self.MinStepFactor = MinStepFactor
        self.chunk_rows = chunk_rows
        self.progress = progress
        self.last_run = None       # engine.RunResult of the last ray_run

    def get_defualt_nlon_and_nlat(self, ncfile):
        """(nlat, nlon) from the file's lat/lon (or u's last two dims), wr.py:173-212."""
        d = ncio.read(ncfile)
        lat = next((d[k] for k in ("lat", "latitude", "Lat", "Latitude") if k in d), None)
        lon = next((d[k] for k in ("lon", "longitude", "Lon", "Longitude") if k in d), None)
        if lat is None or lon is None:
            print("!!!WARNING: Using u.shape[-2] and u.shape[-1] as nlat and nlon!!!")
            return d["u"].shape[-2], d["u"].shape[-1]
        return lat.shape[0], lon.shape[0]

    # ----------------------------------------------------------- sources
    def set_zwn(self, zwn_array):
        if len(zwn_array) != self.nzwn:
            raise ValueError("Length of zwn_array must equal nzwn")
        self.zwn[:] = np.array(zwn_array, dtype=self.all_dtype)

    def set_freq(self, freq):
        self.freq = np.array([freq], dtype=self.all_dtype)

    def set_source_array(self, lon_list, lat_list):
        if len(lon_list) != self.nsource or len(lat_list) != self.nsource:
            raise ValueError("Source list length mismatch nsource")
        self.source_lon = np.array(lon_list, dtype=self.all_dtype) * (1.0 * deg2rad)
        self.source_lat = np.array(lat_list, dtype=self.all_dtype) * (1.0 * deg2rad)

    def set_source_matrix(self, SW_lon, SW_lat, dlon, dlat, nnx, nny):
        """Regular source grid, index ``iy*nnx + ix`` (wr.py:236-258)."""
        if nnx * nny != self.nsource:
            raise ValueError("nsource != nnx * nny, matrix size mismatch!")
        if SW_lat + (nny - 1) * dlat > 89.0:
            raise ValueError("source latitude out of -90~90 range!")
        SW_lon = SW_lon % 360.0
        for iy in range(nny):
            for ix in range(nnx):
                idx = iy * nnx + ix
                self.source_lon[idx] = ((SW_lon + ix * dlon) % 360.0) * deg2rad
                self.source_lat[idx] = (SW_lat + iy * dlat) * deg2rad

    def ray_info(self):
        bar = "=" * 78
        lines = [bar, " WNWR Package: Barotropic Horizontal Rossby Wave Ray Tracing Information ",
                 f" Shape of the Basic Flow (nlon x nlat): {self.bs.nlon} x {self.bs.nlat}",
                 f" Initial Zonal Wave Numbers (nzwn): {self.nzwn}",
                 " " * 15 + " ".join(f"{z:.1f}" for z in self.zwn),
                 f" Source Locations (total {self.nsource} points):"]
        lines += [" " * 15 + f"{lo * rad2deg:7.2f}, {la * rad2deg:7.2f}"
                  for lo, la in zip(self.source_lon, self.source_lat)]
        lines += [f" Time Step (s): {self.tstep[0]:.1f}",
                  f" Total Integration Time (day): {self.ttotal / day:.1f}",
                  f" Total Steps (nt): {self.nt}", bar]
        print("\n".join(lines))

    # ------------------------------------------------------ initial rays
    def ray_initial_numpy(self, root_method="numpy"):
        """Initial rows (wr.py:344-395): positions, k, the 3 m roots, amp, ug, vg."""
        rows = initial_rows(self.bs, self.source_lon, self.source_lat, self.zwn, self.freq,
                            root_method)
        for h, r in zip((self.rlon, self.rlat, self.rzwn, self.rmwn, self.ramp, self.rug,
                         self.rvg), rows):
            h[0] = r

    def ray_initial_hip(self):
        """Initial rows on the GPU (``RayEngine.initial_rows``): bit-identical to
        ``ray_initial_numpy`` -- np.roots' companion-matrix eigenvalues restated
        operation for operation on the device (csrc/nproots.h)."""
        rows = self.bs.engine().initial_rows(self.source_lon, self.source_lat, self.zwn,
                                             self.freq).cpu().numpy()
        for h, r in zip((self.rlon, self.rlat, self.rzwn, self.rmwn, self.ramp, self.rug,
                         self.rvg), rows):
            h[0] = r

    def ray_initial(self, mode="numpy", root_method="numpy"):
        """Initial rays (wr.py:417-421): ``mode='numpy'`` is the reference's
        vectorised host initialiser, ``mode='hip'`` the same on the GPU."""
        if mode == "hip":
            self.ray_initial_hip()
        else:
            self.ray_initial_numpy(root_method=root_method)

    # ---------------------------------------------------------- ray loop
    def core_ray_run_hip_rk45(self, group=None):
        """The RK45 ray loop on the GPU (replaces wr.py:767-887)."""
        return self._core_ray_run_hip("rk45", group)

    def core_ray_run_hip(self, group=None):
        """The fixed-step RK4 ray loop on the GPU (replaces wr.py:702-765)."""
        return self._core_ray_run_hip("rk4", group)

    def _core_ray_run_hip(self, method, group=None):
        """Shared driver of the two GPU ray loops.

        With a torch.distributed ``group`` of one process per GPU, the rays are
        sharded over the ranks (shard.py): rank 0's basic state is broadcast,
        every rank integrates its shard, and rank 0 gathers every output row
        into its history arrays (the other ranks' arrays keep only row 0).
        """
        import torch
        import shard
        rank, world = shard.world_info(group) if group is not None else (0, 1)
        multi = group is not None and shard.collective(world)
        if multi:
            self.bs.fields = shard.broadcast_array(self.bs.fields, 0, group)
            self.bs._engine = None
        eng = self.bs.engine()
        nray = 3 * self.nsource * self.nzwn
        y0 = np.array([self.rlon[0], self.rlat[0], self.rzwn[0], self.rmwn[0],
                       self.ramp[0]], dtype=self.all_dtype).reshape(5, nray)
        idx = np.arange(nray)
        if multi:
            idx = shard.shard_indices(~np.isnan(y0.mean(axis=0)), rank, world)
        rows_shape = (3, self.nsource, self.nzwn)
        hist = (self.rlon, self.rlat, self.rzwn, self.rmwn, self.ramp, self.rug, self.rvg)

        if multi:
            # each rank's previous rows (row 0: the initial rows), as bit patterns
            row0 = np.stack([h[0].reshape(-1)[idx] for h in hist], axis=1)
            last = torch.as_tensor(np.ascontiguousarray(row0)).view(torch.int64).to(eng.device)

        def sink(i0, i1, rows):
            # rank 0 receives only the rays whose rows changed; every other
            # ray repeats its previous row (hostio.fill_rows)
            got = shard.gather_changed_rows(rows, torch.as_tensor(idx, device=rows.device), last, 0, group)
            if got is None:
                return
            cols, data = got
            host = data.permute(2, 1, 0).contiguous().cpu().numpy()        # [7][rows][n]
            cols = np.ascontiguousarray(cols.cpu().numpy())
            from hostio import fill_rows
            for v in range(7):
                dst = hist[v][i0:i1].reshape(i1 - i0, nray)
                fill_rows(dst, hist[v][i0 - 1].reshape(nray), host[v], cols if len(cols) else None)
            if self.progress:
                progress_bar(i1 - 1, self.nt)

        chunk = self.chunk_rows or _default_chunk(nray, self.nt)
        grp = group if multi else None
        out, hs = None, None
        if not multi:
            # single GPU: chunks reach the host arrays while the next one is
            # computed (permute on the device, pinned D2H, threaded copies)
            from hostio import HistorySink
            hs = HistorySink(hist, rows_shape, nray, min(chunk, self.nt - 1), eng.device,
                             progress=(lambda i: progress_bar(i, self.nt)) if self.progress else None)
            sink, out = hs, hs.buffers()
        try:
            if method == "rk4":
                res = eng.integrate_rk4(torch.as_tensor(y0[:, idx]), self.nt, float(self.tstep[0]),
                                        chunk=chunk, sink=sink, cut_rad=float(self.cut_off[0]),
                                        group=grp, out=out)
            else:
                res = eng.integrate(torch.as_tensor(y0[:, idx]), self.nt, float(self.tstep[0]),
                                    self.rtol, self.atol, self.MinStepFactor, ttotal=self.ttotal,
                                    chunk=chunk, sink=sink, cut_rad=float(self.cut_off[0]),
                                    group=grp, out=out)
        finally:
            if hs is not None:
                hs.finish()
                # ray-rows shipped over PCIe vs delivered (frozen rays' rows are filled on the host)
                self.last_delivery = {"shipped_ray_rows": hs.shipped, "delivered_ray_rows": hs.delivered,
                                      "host_fill_s": hs.t_fill, "host_wait_s": hs.t_wait}
        if res.break_row is not None:
            for h in hist:
                h[res.break_row:] = np.nan     # rows never stored (wr.py:853-855, 886-887)
        self.last_run = res
        return res

    def core_ray_run(self, mode="hip_rk45", group=None):
        if mode not in SUPPORTED:
            raise NotImplementedError(
                f"ray loop {mode!r} is not provided by this framework; use "
                f"ray_run(mode='hip', inte_method='rk45') (adaptive RK45) or "
                f"ray_run(mode='hip', inte_method='') (fixed-step RK4) on the MI355X")
        if mode == "hip":
            return self.core_ray_run_hip(group=group)
        return self.core_ray_run_hip_rk45(group=group)

    def ray_run(self, mode="hip", inte_method="rk45", root_method="numpy", debug=False,
                debug_file=None, group=None):
        """Initialise and integrate all rays (wr.py:897-911).

        ``group``: optional torch.distributed process group (one rank per GPU)
        to shard the rays across GPUs; results land on rank 0.
        """
        key = mode + "_rk45" if inte_method == "rk45" else mode
        if key not in SUPPORTED:
            self.core_ray_run(key)     # raises before any work
        self.ray_initial(mode=mode, root_method=root_method)   # wr.py:900 (mode 'hip': GPU)
        if debug and debug_file is not None:
            try:
                self.load_init_from_precal_nc(debug_file)
            except Exception:
                pass
        return self.core_ray_run(key, group=group)

    def load_init_from_precal_nc(self, ncfile):
        """Seed row 0 from a previously written ray file (wr.py:398-415)."""
        d = ncio.read(ncfile)
        for name in ("rlon", "rlat", "rzwn", "rmwn", "ramp", "rug", "rvg"):
            t = np.array(d[name], dtype=self.all_dtype)
            if name in ("rlon", "rlat"):
                t = t / 180 * np.pi
            t[1:] = np.nan
            t[t == 999.] = np.nan
            setattr(self, name, t)

    # ------------------------------------------------------------ output
    def output(self, ncfile):
        """Write the trajectories (lon/lat in degrees), wr.py:916-959."""
        dims = {"zwn": self.nzwn, "source": self.nsource, "root": 3, "time": self.nt}
        full = ("time", "root", "source", "zwn")
        v = {"zwn": (("zwn",), self.zwn),
             "source_index": (("source",), np.arange(self.nsource, dtype=np.int32)),
             "time_index": (("time",), np.arange(self.nt, dtype=np.int32)),
             "rlon": (full, self.rlon * rad2deg, "degrees"),
             "rlat": (full, self.rlat * rad2deg, "degrees"),
             "rzwn": (full, self.rzwn, "rad_per_meter*Rearth"),
             "rmwn": (full, self.rmwn), "ramp": (full, self.ramp),
             "rug": (full, self.rug, "m s-1"), "rvg": (full, self.rvg, "m s-1")}
        ncio.write(ncfile, dims, v)

    def clean(self):
        self.bs.clean()
        for a in ("rlon", "rlat", "rzwn", "rmwn", "ramp", "rug", "rvg", "source_lon",
                  "source_lat", "zwn"):
            if hasattr(self, a):
                delattr(self, a)


def initial_rows(bs, source_lon, source_lat, zwn, freq, root_method="numpy"):
    """The seven initial rows ``(3, nsource, nzwn)`` of ``ray_initial_numpy`` (wr.py:344-395).

    Positions = sources; k = zwn; the three meridional roots of the t = 0
    dispersion relation (``cal_ky``); amp = 1 (NaN for a missing root); the
    t = 0 group velocity (``cal_ugvg`` mode 'numpy').  Host NumPy, bit-identical
    to the reference.
    """
    source_lon = np.asarray(source_lon, np.float64)
    source_lat = np.asarray(source_lat, np.float64)
    zwn = np.asarray(zwn, np.float64)
    freq = np.atleast_1d(np.asarray(freq, np.float64))
    shape = (3, len(source_lon), len(zwn))
    lon = np.ones(shape)
    lat = np.ones(shape)
    lon *= source_lon[None, :, None]
    lat *= source_lat[None, :, None]
    res = bs.cal_bs_mercator_point(source_lon, source_lat, mode="numpy")
    fmu, fmv, fmqx, fmqy = res[0], res[1], res[6], res[7]
    k = np.ones(shape)
    k *= zwn[None, None, :]
    m, amp, ug, vg = (np.full(shape, np.nan) for _ in range(4))
    for iz in range(len(zwn)):
        kz = zwn[iz]
        m_list, _ = cal_ky(fmu, fmv, fmqx, fmqy, freq, kz, iz=iz, mode="numpy",
                           root_method=root_method)
        m_val = m_list.T
        m[:, :, iz] = m_val
        a = np.ones(m_val.shape)
        a[np.isnan(m_val)] = np.nan
        amp[:, :, iz] = a
        ug[:, :, iz], vg[:, :, iz] = cal_ugvg(fmu, fmv, fmqx, fmqy, kz, m_val, mode="numpy")
    return lon, lat, k, m, amp, ug, vg


def _default_chunk(nray, nt):
    """Rows per device chunk: keep the device row buffer near 2 GiB."""
    per_row = nray * 8 * 8
    return int(max(1, min(nt - 1, (2 << 30) // max(per_row, 1))))
