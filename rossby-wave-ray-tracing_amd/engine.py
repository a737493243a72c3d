"""Device-side ray engine: the basic state resident in HBM + the HIP entry points.

``RayEngine`` is what ``WR.core_ray_run_hip_rk45`` (wr.py) and ``bench.py``
drive.  It owns the packed field stack on the GPU and wraps every C-ABI call
of ``include/rwrt.h``; ``integrate`` is the whole ray loop of the reference's
``WR.core_ray_run_rk45`` (wr.py:767-887), streamed in time chunks.
"""
import os

import numpy as np
import torch

import _hip as H
from constants import rearth as R_EARTH

F64 = torch.float64


def grid_of(lon, lat, ncol):
    """``rwrt_grid`` from the float32-rounded radian axes (interpolation.py:78-82)."""
    lon = np.asarray(lon, np.float64)
    lat = np.asarray(lat, np.float64)
    return H.Grid(int(ncol), len(lat), float(lon[0]), float(lon[1] - lon[0]),
                  float(lat[0]), float(lat[1] - lat[0]))


def t_eval_of(nt, tstep, ttotal=None):
    """Output times ``arange(nt) * tstep`` clipped to ``ttotal`` (wr.py:798-801)."""
    t = np.arange(nt) * np.float64(tstep)
    if ttotal is not None and t[-1] > ttotal:
        t[-1] = ttotal
    return t


class RunResult:
    """Per-ray counters and the two global outcomes of one integration."""

    def __init__(self, nacc, nrej, nanrow, failed, break_row, n_live):
        self.nacc = nacc            # accepted steps per ray (torch int64, device)
        self.nrej = nrej            # rejected attempts per ray
        self.nanrow = nanrow        # first stored row with NaN lon per ray (nt = never)
        self.failed = failed        # rkf45.py:423-425 -> wr.py:886-887
        self.break_row = break_row  # wr.py:853-855 global early exit (None = no break)
        self.n_live = n_live
        self.bounds = []            # the [it_begin, it_end) row windows launched

    @property
    def ray_steps(self):
        return int(self.nacc.sum().item())


class Tails:
    """The constant row tails of one ray-loop launch (``rwrt_rk45_run_tails``,
    include/rwrt.h): ray j's rows from ``frm[j]`` (int32, in [i0, i1]; i1 = no
    tail) to the launch's end all equal ``row[j]`` (``[nray, 8]``) and are not
    in the launch's row buffer.  A frozen ray (rkf45.py:400-403) repeats one
    row, so 70 % of C3's output rows are never written; ``RayEngine.expand``
    writes them for a consumer that wants the rows dense."""

    def __init__(self, nray, device):
        self.frm = torch.empty(nray, dtype=torch.int32, device=device)
        self.row = torch.empty((nray, H.NOUT), dtype=F64, device=device)

    def take(self, idx):
        t = Tails.__new__(Tails)
        t.frm, t.row = self.frm[idx].contiguous(), self.row[idx].contiguous()
        return t

    def last_row(self, view, i1):
        """Each ray's last row of the launch ``[i0, i1)`` whose rows are ``view``."""
        return torch.where((self.frm < i1)[:, None], self.row, view[:, -1])


class Slots:
    """The row blocks of one ``rwrt_rk45_run_slots`` launch (ABI 4): ray j's
    rows are block ``slot[j]`` of the launch's row buffer, -1 for a ray frozen
    at the launch's start (its rows are its tail).  ``n``: the blocks the first
    launch of a run needs (later launches need no more: a frozen ray stays
    frozen, rkf45.py:400-403)."""

    def __init__(self, nray, device):
        self.slot = torch.empty(nray, dtype=torch.int32, device=device)
        self.n_dev = torch.zeros(1, dtype=torch.int64, device=device)
        self.n = None

    def compute(self, st, stream):
        """Number the rays of ``st`` live now (``rwrt_row_slots``, async)."""
        H.check(H.load().rwrt_row_slots(st["nray"], H.dptr(st["state"]), H.dptr(self.slot, torch.int32),
                                        H.dptr(self.n_dev, torch.int64), stream))
        return self

    def count(self):
        """The number of live rays (waits for ``compute``)."""
        self.n = int(self.n_dev.item())
        return self.n

    def last_row(self, view, tails, i1):
        """Each ray's last row of the launch ``[i0, i1)`` (row blocks ``view``)."""
        blk = view[self.slot.clamp(min=0).to(torch.int64), -1] if view.shape[0] else tails.row
        return torch.where((tails.frm < i1)[:, None], tails.row, blk)

    def dense(self, view, tails, i0, i1, out=None):
        """The launch's rows ``[nray, i1-i0, 8]`` made dense (``rwrt_expand_slots``)."""
        nray = self.slot.numel()
        if out is None or out.numel() < nray * (i1 - i0) * H.NOUT:
            out = torch.empty((nray, i1 - i0, H.NOUT), dtype=F64, device=self.slot.device)
        d = out.reshape(-1)[: nray * (i1 - i0) * H.NOUT].view(nray, i1 - i0, H.NOUT)
        H.check(H.load().rwrt_expand_slots(nray, int(i0), int(i1), H.dptr(self.slot, torch.int32),
                                           H.dptr(tails.frm, torch.int32), H.dptr(tails.row, F64),
                                           H.dptr(view, F64), H.dptr(d, F64), H.stream(self.slot.device)))
        return d


def deliver(eng, sink, i0, i1, view, tails, slots=None):
    """Hand a launch's rows to ``sink``: with its tails when the sink takes
    them (``sink.takes_tails``), else dense (the tails expanded into ``view``);
    row blocks (``slots``) go only to a sink that takes them."""
    if slots is not None:
        return sink(i0, i1, view, tails, slots)
    if tails is not None and getattr(sink, "takes_tails", False):
        return sink(i0, i1, view, tails)
    if tails is not None:
        eng.expand(view, tails, i0, i1)
    return sink(i0, i1, view)


class RayEngine:
    """The basic state on one GPU and the fused RK45 kernels that read it."""

    # constant row tails (rwrt_rk45_run_tails): frozen rays' rows are stored
    # once per launch and expanded only for sinks that want dense rows; False:
    # every row written by the launch itself (rwrt_rk45_run; A/B and tests)
    use_tails = os.environ.get("RWRT_TAILS", "1") != "0"
    # rays per wave of the fp64 time-varying loops (rwrt_ctx_set_tv_lanes: 32
    # caches both bracketing levels per ray, no HBM gathers while a ray stays
    # in its cell and level pair; 64 caches the lower level only).  Schedule
    # only.  32: C5 1.17 -> 1.24e9 on one GPU, 8 shards 1.42 -> 0.78 s
    # (with the split set's long launches, bench.c5_rows_per_launch)
    tv_lanes = int(os.environ.get("RWRT_TV_LANES", "32"))
    # row blocks for the live rays only (rwrt_rk45_run_slots, ABI 4): a launch
    # whose rows go to a sink that takes them (``sink.takes_slots``), or to no
    # one, gets a row buffer of live rays x rows instead of every slot x rows
    # (C3: 49.5 GB instead of 166 GB); other sinks get dense rows as before
    use_slots = os.environ.get("RWRT_SLOTS", "1") != "0"
    # drain-time hand-off of the static ray loop (rwrt_ctx_set_handoff): a wave
    # with at most this many rays left once the queue is drained continues
    # them in the quad layout (0: off).  Schedule only.
    handoff = int(os.environ.get("RWRT_HANDOFF", "16"))

    def __init__(self, fields, lon, lat, device=None):
        """``fields``: the reference stack ``[nlon(+1), nlat, 18]`` (numpy or tensor);
        ``lon, lat``: the BS radian axes (``bs.lon``, ``bs.lat``)."""
        H.require_gpu()
        H.load()
        self.device = torch.device(device or "cuda")
        f = torch.as_tensor(np.ascontiguousarray(fields, dtype=np.float64)) \
            if not torch.is_tensor(fields) else fields.to(F64)
        if f.ndim != 3 or f.shape[-1] != H.NFIELD_REF:
            raise ValueError(f"fields must be [ncol, nrow, {H.NFIELD_REF}], got {tuple(f.shape)}")
        f = f.to(self.device).contiguous()
        self.grid = grid_of(lon, lat, f.shape[0])
        self.packed = torch.empty((f.shape[0], f.shape[1], H.NFIELD_PACK), dtype=F64,
                                  device=self.device)
        H.check(H.load().rwrt_pack_fields(self.grid, H.dptr(f), H.dptr(self.packed), self._stream()))
        self.work = torch.zeros(4, dtype=torch.int32, device=self.device)

    bg = None   # rwrt_background of a time-varying state (None: the reference's static state)
    split_rho = None   # the last advance()'s rank correlation of its leading launches (split="auto")
    launch_log = ()    # the last advance()'s launches: rows and latency-mode decision
    rows_bytes = 0     # the last advance()'s row buffers (device bytes)
    launch_handoffs = ()   # the last advance()'s rays handed off per launch (device; handoffs())

    def handoffs(self):
        """Rays the drain-time hand-off moved to the quad layout, per launch of
        the last ``advance`` (waits for them)."""
        return [int(h.item()) for h in self.launch_handoffs]
    keep_launch_work = False   # diagnostics: launch_work = [(attempts per ray, latency set)] per launch
    _ctx = None

    @property
    def ctx(self):
        """This engine's ``rwrt_ctx`` (the ray-loop scratch), created on first use."""
        if self._ctx is None:
            self._ctx = H.Context(self.device)
        return self._ctx

    def _stream(self):
        """The current stream of the engine's device (not torch's current device)."""
        return H.stream(self.device)

    def _event_pair(self):
        s = torch.cuda.current_stream(self.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        return e0, e1, s

    @classmethod
    def from_bs(cls, bs, device=None):
        return cls(bs.fields, bs.lon, bs.lat, device)

    @classmethod
    def from_levels(cls, levels, time_varying=None):
        """Engine over a ``levels.Levels`` basic state.  One fp64 level is the
        reference's static state (same kernels, same bits); otherwise the
        time-varying kernels (``rwrt_rk45_*_tv``) run.  ``time_varying=True``
        sends one fp64 level through the time-varying kernels too (the test
        that they reduce to the reference: tests/test_gpu_ref90.py)."""
        self = cls.__new__(cls)
        self.device = levels.device
        self.grid = levels.grid
        self.levels = levels
        self.work = torch.zeros(4, dtype=torch.int32, device=self.device)
        if levels.nlev == 1 and not levels.fp32 and not time_varying:
            self.packed = levels.packed[0]
            self.bg = None
        else:
            self.packed = None
            self.bg = levels.background()
        return self

    @classmethod
    def from_packed(cls, packed, lon, lat):
        """Engine over an already packed ``[nlon+1, nlat, 12]`` fp64 state (e.g.
        from ``rwrt_bs_ready``)."""
        self = cls.__new__(cls)
        self.device = packed.device
        self.grid = grid_of(lon, lat, packed.shape[0])
        self.packed = packed.contiguous()
        self.work = torch.zeros(4, dtype=torch.int32, device=self.device)
        return self

    def rhs_t(self, t, y):
        """The time-varying RHS at per-point times ``t[n]`` for ``y[5, n]``."""
        if self.bg is None:
            return self.rhs(y)
        y = torch.as_tensor(y, dtype=F64, device=self.device).contiguous()
        t = torch.as_tensor(t, dtype=F64, device=self.device).contiguous()
        out = torch.empty_like(y)
        H.check(H.load().rwrt_rhs_tv(self.grid, ctypes_ref(self.bg), y.shape[1], H.dptr(t),
                                     H.dptr(y), H.dptr(out), self._stream()))
        return out

    # ------------------------------------------------------------------ T0/T1
    def mercator_point(self, lon, lat):
        """``cal_bs_mercator_point`` on the GPU: ``(12, n)`` (fmu .. fmqyy)."""
        lon = torch.as_tensor(lon, dtype=F64, device=self.device).contiguous()
        lat = torch.as_tensor(lat, dtype=F64, device=self.device).contiguous()
        n = lon.numel()
        out = torch.empty((H.NMERC, n), dtype=F64, device=self.device)
        H.check(H.load().rwrt_mercator_point(self.grid, H.dptr(self.packed), n, H.dptr(lon),
                                             H.dptr(lat), H.dptr(out), self._stream()))
        return out

    def rhs(self, y):
        """``diffun_numpy(y)[0][0:5]`` on the GPU for ``y[5, n]``."""
        y = torch.as_tensor(y, dtype=F64, device=self.device).contiguous()
        n = y.shape[1]
        out = torch.empty_like(y)
        H.check(H.load().rwrt_rhs(self.grid, H.dptr(self.packed), n, H.dptr(y), H.dptr(out),
                                  self._stream()))
        return out

    def attempt(self, y, f, h, rtol=1e-6, atol=1e-6):
        """One DP5(4) attempt (``rk_step`` + error norm): ``(K[7,5,n], y_new, err)``."""
        y = torch.as_tensor(y, dtype=F64, device=self.device).contiguous()
        f = torch.as_tensor(f, dtype=F64, device=self.device).contiguous()
        h = torch.as_tensor(h, dtype=F64, device=self.device).contiguous()
        n = y.shape[1]
        K = torch.empty((7, 5, n), dtype=F64, device=self.device)
        yn = torch.empty_like(y)
        err = torch.empty(n, dtype=F64, device=self.device)
        H.check(H.load().rwrt_dp54_attempt(self.grid, H.dptr(self.packed), n, H.dptr(y),
                                           H.dptr(f), H.dptr(h), rtol, atol, H.dptr(K),
                                           H.dptr(yn), H.dptr(err), self._stream()))
        return K, yn, err

    # ------------------------------------------------------- initial rays
    @staticmethod
    def zwn_constants(zwn, freq):
        """``{k, k**2, k**3, freq/k*R}`` per zonal wavenumber, evaluated by NumPy
        exactly as ``cal_ky_numpy`` does (bs.py:1005-1012): ``[4, nzwn]``."""
        freq = np.atleast_1d(np.asarray(freq, np.float64))
        zc = np.zeros((4, len(zwn)))
        for iz, kz in enumerate(np.asarray(zwn, np.float64)):
            zc[0, iz] = kz
            zc[1, iz] = kz ** 2
            zc[2, iz] = kz ** 3
            with np.errstate(all="ignore"):
                zc[3, iz] = (freq / kz * R_EARTH)[0]
        return zc

    def sources(self, source_lon, source_lat):
        """Device inputs of rwrt_ray_initial for a source list: lon, lat and the
        host-libm ``np.cos(lat)`` (``[3, nsource]``)."""
        slat = np.ascontiguousarray(source_lat, dtype=np.float64)
        s = np.stack([np.ascontiguousarray(source_lon, dtype=np.float64), slat, np.cos(slat)])
        return torch.as_tensor(s, dtype=F64).to(self.device)

    def zwn_tensor(self, zwn, freq):
        return torch.as_tensor(self.zwn_constants(zwn, freq), dtype=F64).to(self.device)

    def initial_rows_dev(self, src, zc, rows=None, info=None):
        """Launch rwrt_ray_initial on resident inputs (``sources``, ``zwn_tensor``);
        returns ``(rows[7, 3, nsource, nzwn], info[1])`` without synchronising."""
        ns, nz = src.shape[1], zc.shape[1]
        if rows is None:
            rows = torch.empty((7, 3, ns, nz), dtype=F64, device=self.device)
        if info is None:
            info = torch.zeros(1, dtype=torch.int32, device=self.device)
        packed = self.packed if self.bg is None else self.levels.level0_f64   # the t = 0 state
        H.check(H.load().rwrt_ray_initial(self.grid, H.dptr(packed), ns, H.dptr(src[0]),
                                          H.dptr(src[1]), H.dptr(src[2]), nz, H.dptr(zc),
                                          H.dptr(rows), H.dptr(info), self._stream()))
        return rows, info

    def initial_rows(self, source_lon, source_lat, zwn, freq, check=True):
        """``WR.ray_initial_numpy`` (wr.py:344-395) on the GPU: the device tensor
        ``rows[7, 3, nsource, nzwn]`` = lon lat k l amp ug vg.  Bit-identical
        to the host path (np.roots restated in csrc/nproots.h); the source
        ``cos(lat)`` comes from the host libm, as in the reference.  With
        ``check`` (default), non-finite dispersion coefficients raise like
        ``np.linalg.eigvals`` does in the reference."""
        src = self.sources(source_lon, source_lat)
        rows, info = self.initial_rows_dev(src, self.zwn_tensor(zwn, freq))
        if check and int(info.item()) != 0:
            raise np.linalg.LinAlgError(
                f"Array must not contain infs or NaNs ({int(info.item())} dispersion "
                f"polynomials with non-finite coefficients; np.roots raises here too)")
        return rows

    # ------------------------------------------------------------ ray loop
    @staticmethod
    def params(nt, tstep, rtol=1e-6, atol=1e-6, msf=1e-3, cut_off=0.1, cut_rad=None):
        """``rwrt_params`` exactly as WR / RK45 derive them."""
        rtol = max(rtol, 100 * np.finfo(np.float64).eps)          # rkf45.py:21-26
        tstep = float(tstep)
        min_step = min(msf * tstep, (tstep - 0) * 0.001)          # rkf45.py:362, wr.py:792-794
        cut = cut_off * tstep / 3600.0 if cut_rad is None else float(cut_rad)   # wr.py:170
        return H.Params(rtol, atol, min_step, cut, int(nt), 0, tstep)

    def init(self, y0, p):
        """Solver construction on the GPU; returns the per-ray state tensors."""
        y0 = torch.as_tensor(y0, dtype=F64, device=self.device).contiguous()
        nray = y0.shape[1]
        st = dict(
            state=torch.empty((H.NSTATE, nray), dtype=F64, device=self.device),
            count=torch.empty((nray, 2), dtype=torch.int64, device=self.device),
            nanrow=torch.empty(nray, dtype=torch.int32, device=self.device),
            live=torch.empty(nray, dtype=torch.int32, device=self.device),
            summary=torch.zeros(2, dtype=torch.int64, device=self.device),
            nray=nray)
        lib = H.load()
        if self.bg is None:
            fn, bg = lib.rwrt_rk45_init, H.dptr(self.packed)
        else:
            fn, bg = lib.rwrt_rk45_init_tv, ctypes_ref(self.bg)
        H.check(fn(self.grid, bg, nray, H.dptr(y0), ctypes_ref(p), H.dptr(st["state"]),
                   H.dptr(st["count"]), H.dptr(st["nanrow"]), H.dptr(st["live"]),
                   H.dptr(st["summary"]), self._stream()))
        return st

    @staticmethod
    def live_first_order(st):
        """Queue order: live rays first, frozen (NaN-root) slots last (stable)."""
        dead = (st["live"] == 0).to(torch.int8)
        return torch.sort(dead, stable=True).indices.to(torch.int64).contiguous()

    @staticmethod
    def cost_order(st, work):
        """Longest-first queue order for the next chunk.

        ``work`` = attempts each ray made in the previous chunk (a good predictor
        of the next one: step sizes change slowly).  Frozen rays (NaN mean; one
        row computation each) go last, where they fill the tail of the launch.
        """
        y = st["state"][:5]
        frozen = torch.isnan(y.sum(0))
        key = torch.where(frozen, torch.full_like(work, -1), work)
        return torch.sort(key, descending=True, stable=True).indices.to(torch.int64).contiguous()

    CELL_PER_OCTAVE = int(os.environ.get("RWRT_CELL_PER_OCTAVE", "2"))   # (env: A/B only)

    def cost_cell_order(self, st, work, per_octave=None, head=0):
        """``cost_order`` with spatial locality: rays in coarse cost classes
        (``per_octave`` classes per doubling of the previous launch's work,
        heaviest class first) and, within a class, in Morton order of their
        current grid cell, so that the 64 rays a wave starts with share cache
        lines and L2 / MALL sets in their first lookups (the 0.25-degree
        time-varying state of C5 is gathered from HBM: 100 MB per fp64
        level).  Frozen rays last.  ``head``: the ``head`` heaviest live rays
        by ``work`` go first, longest first (the latency mode takes its rays
        from the order's head; a cost class alone does not rank them)."""
        per_octave = self.CELL_PER_OCTAVE if per_octave is None else per_octave
        y = st["state"][:5]
        frozen = torch.isnan(y.sum(0))
        w = torch.where(frozen, torch.zeros_like(work), work).to(F64)
        cls = torch.floor(torch.log2(w + 1.0) * per_octave).to(torch.int64)
        g = self.grid
        lon = torch.remainder(y[0], 2 * np.pi)
        ix = torch.floor((lon - g.lon0) / g.dlon).nan_to_num(0).clamp(0, g.ncol - 1).to(torch.int64)
        iy = torch.floor((y[1] - g.lat0) / g.dlat).nan_to_num(0).clamp(0, g.nrow - 1).to(torch.int64)
        key = cls * (1 << 32) + ((1 << 32) - 1 - morton2(ix, iy))
        key = torch.where(frozen, torch.full_like(key, -1), key)
        order = torch.sort(key, descending=True, stable=True).indices.to(torch.int64)
        if head:
            kw = torch.where(frozen, torch.full_like(work, -1), work)
            top = torch.topk(kw, min(int(head), kw.numel())).indices
            top = top[kw[top] >= 0]
            first = torch.zeros(kw.numel(), dtype=torch.bool, device=kw.device)
            first[top] = True
            order = torch.cat([top.to(torch.int64), order[~first[order]]])
        return order.contiguous()

    # a heavy ray's attempt in latency mode / in a loaded rk45_run_kernel wave
    # (round 2, tools/team_latency.py on the heaviest C3 rays: 10.2 us alone in
    # its wave, 11.5 us at 16 rays per wave, 13.3-13.7 us in the run kernel;
    # round 4, like rays dealt to a wave together: ~9.5-10 us at 16 per wave
    # against ~13.5, profiles/r4/sched/latency_xcd.txt)
    QUAD_RATIO_1 = 0.76
    QUAD_RATIO_16 = 0.85   # (0.72 picks the same sizes on C3 split 2/4/8 ways: r4mm)
    QUAD_MIN_GAIN = 0.10   # (one C3 GPU: predicted 6-9 %, measured -1 %)
    # rays per wave the auto rule considers: sparser waves measured SLOWER per
    # heavy ray in a full run (tools/team_latency.py --density, 90 d: 16 / 64
    # / 256 heaviest rays 0.20 / 0.21 / 0.21 s at 16 per wave, 0.51 / 0.55 /
    # 0.56 s at 1 per wave, 256 rays 0.27 s at 4 per wave), so only 16
    # (RWRT_QUAD_DENSITIES=4,16 lets the rule consider others: A/B only)
    QUAD_DENSITIES = tuple(int(x) for x in os.environ.get("RWRT_QUAD_DENSITIES", "16").split(","))
    # the time-varying latency waves (one ray per wave, BlockVaryingBG): a heavy
    # C5 ray's attempt there against a loaded run-kernel lane's
    TV_RATIO = float(os.environ.get("RWRT_TV_RATIO", "0.77"))

    def team_capacity_tv(self):
        """Rays the time-varying latency mode takes at most (4 per CU, half the CUs)."""
        return (torch.cuda.get_device_properties(self.device).multi_processor_count // 2) * 4

    def team_capacity(self):
        """Rays the latency mode takes at most (64 per CU, half the CUs)."""
        return (torch.cuda.get_device_properties(self.device).multi_processor_count // 2) * 64

    def team_size(self, team, st, work, order, rows):
        """How many of the first rays of ``order`` (live at the launch start)
        go to the latency mode, and how many of them share a wave: ``(n,
        rays_per_wave)``.  An int asks for that many (16 per wave), a pair
        ``(n, rays_per_wave)`` for both; "auto"
        picks the pair that minimises the launch's predicted makespan from each
        ray's previous-launch work (below)."""
        if order is None or (self.bg is not None and self.bg.fp32 == 2):   # (none for fp32 arithmetic)
            return 0, 16
        live = ~torch.isnan(st["state"][:5].sum(0))
        n_live = int(live.sum().item())
        ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
        if team != "auto":
            n, q = (int(team[0]), int(team[1])) if isinstance(team, (tuple, list)) else (int(team), 16)
            # (time-varying: one ray per latency wave, 4 per CU)
            n = min(n, (ncu // 2) * 4 * (1 if self.bg is not None else q), n_live)
            # the first n entries of the order must be live rays
            return (n if n == 0 or bool(live[order[:n]].all()) else 0), q
        if work is None or n_live < 1:
            return 0, 16
        # predicted makespan for n heavy rays in latency mode at q rays per
        # wave (4q per block, each block taking a CU from the run kernel's
        # persistent grid), in run-kernel attempt times:
        #   max(heaviest ray x QUAD_RATIO(q),                 (latency mode)
        #       ray n+1, remaining work / remaining lanes)     (run kernel)
        # minimised over (n, q) (the smallest n, then the densest q, on ties)
        w = torch.where(live, work, torch.zeros_like(work))[order].to(torch.float64)
        cum = torch.cumsum(w, 0)
        best = None
        tv = self.bg is not None   # (time-varying: one ray per latency wave; 32 or 64 run lanes per wave)
        # (fp64 levels run tv_lanes rays per wave -- rwrt_ctx_set_tv_lanes sets
        # half only for VaryingBG<double>; fp32-storage levels run 64)
        lanes_cu = (4.0 * self.tv_lanes) if (tv and self.bg.fp32 == 0) else 256.0
        for q in ((1,) if tv else self.QUAD_DENSITIES):
            cap = min((ncu // 2) * 4 * q, n_live)
            n = torch.arange(0, cap + 1, 4 * q, device=w.device)
            n = torch.unique(torch.cat([n, torch.tensor([cap], device=w.device)]))
            rest = cum[-1] - torch.where(n > 0, cum[(n - 1).clamp(min=0)], torch.zeros_like(cum[:1]))
            lanes = lanes_cu * (ncu - (n + 4 * q - 1) // (4 * q)).clamp(min=1)
            nxt = torch.where(n < w.numel(), w[n.clamp(max=w.numel() - 1)], torch.zeros_like(rest))
            ratio = self.TV_RATIO if tv else \
                self.QUAD_RATIO_1 + (self.QUAD_RATIO_16 - self.QUAD_RATIO_1) * (q - 1) / 15.0
            t = torch.maximum(torch.maximum(nxt, rest / lanes),
                              torch.where(n > 0, w[0] * ratio, torch.zeros_like(rest)))
            k = int(torch.argmin(t).item())
            cand = (float(t[k]), int(n[k].item()), q, float(t[0]))
            if best is None or cand[0] < best[0] - 1e-9 * best[0]:
                best = cand
        t_best, n_best, q_best, t_none = best
        # (the prediction ignores what the split costs beyond the CUs: take the
        # latency mode only for a predicted gain of QUAD_MIN_GAIN or more)
        if n_best == 0 or t_best > (1.0 - self.QUAD_MIN_GAIN) * t_none:
            return 0, 16
        return n_best, q_best

    def run(self, st, p, tbound, it_begin, it_end, out, order=None, n_heavy=0, rays_per_wave=16, tails=None,
            slots=None):
        """Rows ``[it_begin, it_end)`` into ``out[nray, it_end-it_begin, 8]`` (async);
        with ``tails`` (a ``Tails``) the frozen rays' constant rows go there instead;
        with ``slots`` (a ``Slots`` computed on ``st``) ``out`` holds the live
        rays' row blocks only."""
        lib = H.load()
        ctx = self.ctx
        if self.bg is not None:
            ctx.set_tv_lanes(self.tv_lanes)
        if n_heavy:
            ctx.set_latency_density(rays_per_wave)
        ctx.set_handoff(self.handoff)
        if slots is not None and tails is None:
            raise ValueError("row slots need tails")
        if self.bg is None:
            fn, bg = (lib.rwrt_rk45_run if tails is None else lib.rwrt_rk45_run_tails if slots is None
                      else lib.rwrt_rk45_run_slots), H.dptr(self.packed)
        else:
            fn, bg = (lib.rwrt_rk45_run_tv if tails is None else lib.rwrt_rk45_run_tv_tails if slots is None
                      else lib.rwrt_rk45_run_tv_slots), ctypes_ref(self.bg)
        args = [ctx.handle, self.grid, bg, st["nray"], ctypes_ref(p), H.dptr(tbound, F64),
                int(it_begin), int(it_end), H.dptr(order, torch.int64), int(n_heavy),
                H.dptr(st["state"]), H.dptr(st["count"]), H.dptr(st["nanrow"]), H.dptr(out, F64)]
        if slots is not None:
            args += [H.dptr(slots.slot, torch.int32)]
        if tails is not None:
            args += [H.dptr(tails.frm, torch.int32), H.dptr(tails.row, F64)]
        H.check(fn(*args, H.dptr(self.work), self._stream()))

    def tails(self, nray):
        """A ``Tails`` for ``nray`` rays, or None when the engine writes dense rows."""
        return Tails(nray, self.device) if self.use_tails else None

    def expand(self, view, tails, i0, i1):
        """The rows ``[i0, i1)`` of a tails launch made dense: ``view[nray, i1-i0, 8]``
        receives every ray's tail (rwrt_expand_tails; async)."""
        H.check(H.load().rwrt_expand_tails(view.shape[0], int(i0), int(i1), H.dptr(tails.frm, torch.int32),
                                           H.dptr(tails.row, F64), H.dptr(view, F64), self._stream()))

    def integrate_rk4(self, y0, nt, tstep, cut_off=0.1, chunk=None, sink=None, out=None,
                      cut_rad=None, events=None, group=None):
        """The fixed-step RK4 ray loop (wr.py:702-765) for ``y0[5, nray]``.

        Same chunked ``sink`` protocol as ``integrate``; the nacc column and
        ``RunResult.nacc`` count RK4 steps taken, ``nrej`` steps held because a
        stage input was masked (the ray keeps its state, wr.py:609-618; a masked
        first stage holds it for every remaining step, each counted).
        """
        if self.bg is not None:
            raise NotImplementedError("the RK4 loop runs on the reference's static basic state")
        p = self.params(nt, tstep, cut_off=cut_off, cut_rad=cut_rad)
        y0 = torch.as_tensor(y0, dtype=F64, device=self.device).contiguous()
        nray = y0.shape[1]
        st = dict(state=torch.empty((H.NSTATE, nray), dtype=F64, device=self.device),
                  count=torch.zeros((nray, 2), dtype=torch.int64, device=self.device),
                  nanrow=torch.full((nray,), int(nt), dtype=torch.int32, device=self.device),
                  nray=nray)
        st["state"][:5] = y0
        live = ~torch.isnan(y0.sum(0))
        order = torch.sort((~live).to(torch.int8), stable=True).indices.to(torch.int64).contiguous()
        chunk = chunk or (nt - 1)
        rows_max = min(chunk, nt - 1)
        bufs = _row_buffers(out, nray, rows_max, self.device)
        for k, i0 in enumerate(range(1, nt, chunk)):
            i1 = min(i0 + chunk, nt)
            flat = bufs[k % len(bufs)].reshape(-1)
            view = flat[: nray * (i1 - i0) * H.NOUT].view(nray, i1 - i0, H.NOUT)
            if events is not None:
                e0, e1, es = self._event_pair()
            H.check(H.load().rwrt_rk4_run(
                self.ctx.handle, self.grid, H.dptr(self.packed), nray, ctypes_ref(p), int(i0), int(i1),
                H.dptr(order, torch.int64), H.dptr(st["state"]), H.dptr(st["count"]),
                H.dptr(st["nanrow"]), H.dptr(view, F64), H.dptr(self.work), self._stream()))
            if events is not None:
                e1.record(es)
                events.append((e0, e1))
            if sink is not None:
                sink(i0, i1, view)
        mx = int(st["nanrow"].max().item()) if nray else 0
        if group is not None:
            from shard import reduce_max
            mx = reduce_max(mx, group)
        cnt = st["count"]
        return RunResult(cnt[:, 0], cnt[:, 1], st["nanrow"], False, mx if mx < nt else None,
                         int(live.sum().item()))

    def integrate(self, y0, nt, tstep, rtol=1e-6, atol=1e-6, msf=1e-3, cut_off=0.1,
                  ttotal=None, chunk=None, sink=None, out=None, cut_rad=None, events=None,
                  group=None, order_policy="priority", first_chunk=None, team=0, stop_row=None):
        """The whole ray loop for ``y0[5, nray]``; rows 1..nt-1 go to ``sink``.

        ``sink(i0, i1, rows)`` receives each time chunk as a device tensor
        ``rows[nray, i1-i0, 8]`` (lon lat k l amp ug vg nacc) before the next
        chunk overwrites it.  ``first_chunk`` (int or list) sets short leading
        chunks whose measured per-ray work orders the next one.  ``stop_row``
        ends the run before that row (``RunResult.state`` then holds the
        solver state for ``checkpoint`` / ``resume``).  ``team``: rays
        integrated in latency mode per launch (rk45_team_kernel: each ray's
        RHS over the four SIMDs of a CU) -- an int (the heaviest rays by the
        previous launch's work, or the first live ones before any) or "auto"
        (``team_size``).  ``events`` (a list) collects a pair of timing
        events around every ray-loop launch.  With a process ``group`` (rays
        sharded over ranks, shard.py) the two global outcomes -- solver
        failure and the all-NaN early exit -- are decided over every rank, so a
        sharded run equals the single-GPU run.  Returns a ``RunResult``.
        """
        p = self.params(nt, tstep, rtol, atol, msf, cut_off, cut_rad)
        y0 = torch.as_tensor(y0, dtype=F64, device=self.device).contiguous()
        nray = y0.shape[1]
        tb = torch.as_tensor(t_eval_of(nt, tstep, ttotal), dtype=F64, device=self.device)
        st = self.init(y0, p)
        summary = st["summary"]
        n_live_local = int(summary[0].item())   # this rank's shard (the queue bound)
        if group is not None:
            from shard import reduce_summary
            summary = reduce_summary(summary, group)
        summary = summary.cpu()
        n_live, n_finite = int(summary[0]), int(summary[1])
        cnt = st["count"]
        if n_live > 0 and n_finite == 0:
            # rkf45.py:423-425: at the first step every live column has a NaN
            # h_abs -> status -1 -> wr.py:886-887 breaks before storing row 1.
            return RunResult(cnt[:, 0], cnt[:, 1], st["nanrow"], True, 1, n_live)
        return self.advance(st, p, tb, 1, chunk=chunk, sink=sink, out=out, events=events,
                            group=group, order_policy=order_policy, first_chunk=first_chunk,
                            n_live=n_live, n_live_local=n_live_local, team=team, stop_row=stop_row)

    # Adaptive split of the long launch after the leading ones (split="auto"):
    # a launch is list scheduling of its rays on the lanes in the queue order,
    # so its makespan is as good as the previous launch's per-ray work
    # predicts this one's.  When the two leading launches' per-ray work
    # correlates weakly (rank correlation below SPLIT_RHO: the non-zonal C3,
    # ~0.5, against ~0.8 on the zonal jets), the rest is split once after
    # SPLIT_ROWS rows and re-ordered by the work so far there
    # (round 3, profiles/r3/sched/: the non-zonal last launch
    # runs 1.66x its throughput bound in the predicted order, 1.00x in the
    # actual one; one split: +5 %).
    SPLIT_RHO = 0.7
    SPLIT_ROWS = 300

    @classmethod
    def parse_split(cls, split):
        """``split`` -> (auto?, cut lengths in rows): "auto" (one cut after
        SPLIT_ROWS), "auto:a,b,.." (cuts after a, a+b, ..; an A/B knob,
        profiles/r4/sched/nonzonal_split.txt), anything else: no cut.  Every
        piece is ordered by all the work so far."""
        auto = isinstance(split, str) and split.split(":")[0] == "auto"
        spec = split.split(":", 1)[1] if auto and ":" in split else ""
        rows = [int(x) for x in spec.split(",")] if spec else [cls.SPLIT_ROWS]
        if any(n <= 0 for n in rows):
            raise ValueError(f"split {split!r}: every piece needs a positive row count")
        return auto, rows

    @staticmethod
    def cut_bounds(i0, i1, rows):
        """Rows [i0, i1) cut after rows[0], rows[0] + rows[1], .. (cuts at or past
        i1 dropped): the launches that replace one long launch."""
        cuts = [i0]
        for n in rows:
            if cuts[-1] + n < i1:
                cuts.append(cuts[-1] + n)
        cuts.append(i1)
        return list(zip(cuts[:-1], cuts[1:]))

    @staticmethod
    def rank_corr(a, b, mask):
        """Spearman rank correlation of ``a`` and ``b`` over ``mask`` (device)."""
        a, b = a[mask].to(F64), b[mask].to(F64)
        n = a.numel()
        if n < 3:
            return 1.0
        ar = torch.arange(n, dtype=F64, device=a.device)
        ra, rb = torch.empty_like(a), torch.empty_like(b)
        ra[torch.argsort(a, stable=True)] = ar
        rb[torch.argsort(b, stable=True)] = ar
        ra, rb = ra - ra.mean(), rb - rb.mean()
        den = torch.sqrt((ra * ra).sum() * (rb * rb).sum())
        return float(((ra * rb).sum() / den).item()) if den > 0 else 1.0

    def advance(self, st, p, tb, start, chunk=None, sink=None, out=None, events=None, group=None,
                order_policy="priority", first_chunk=None, n_live=None, n_live_local=None,
                prev_work=None, team=0, stop_row=None, split=None):
        """Rows ``[start, nt)`` of the ray loop for an initialised state ``st``
        (``init``, or a shard of one: ``take``), in time chunks; the body of
        ``integrate``.  ``prev_work`` (each ray's attempt count, accepted +
        rejected, at the start of an earlier launch) orders the first launch
        longest-first by the attempts since; otherwise live rays go first.
        ``split`` ("auto", see SPLIT_RHO) may split the launch after the
        leading ones once more."""
        nt = int(p.nt)
        end = nt if stop_row is None else max(int(start), min(int(stop_row), nt))
        nray = st["nray"]
        cnt = st["count"]
        if n_live_local is None:
            n_live_local = int((~torch.isnan(st["state"][:5].sum(0))).sum().item())
        if n_live is None:
            n_live = n_live_local
        chunk = chunk or (nt - 1)
        bounds = []
        i0 = start
        # short leading chunks measure the per-ray cost that orders the next one
        lead = [first_chunk] if isinstance(first_chunk, int) else list(first_chunk or [])
        if order_policy in ("cost", "priority", "cell", "total"):
            for n in lead:
                if 0 < n < chunk and i0 < end:
                    bounds.append((i0, min(i0 + n, end)))
                    i0 = bounds[-1][1]
        n_lead = len(bounds)
        while i0 < end:
            bounds.append((i0, min(i0 + chunk, end)))
            i0 = bounds[-1][1]
        rows_max = max([b - a for a, b in bounds] or [1])
        use_slots = (self.use_slots and self.use_tails and nray > 0
                     and (getattr(sink, "takes_slots", False) or (sink is None and out is None)))
        sbufs = None
        nblk = nray   # row blocks per buffer
        if use_slots:
            # the first launch's live rays: the most any launch of the run has
            first = Slots(nray, self.device).compute(st, self._stream())
            nblk = max(1, first.count())
        bufs = _row_buffers(out, nblk, rows_max, self.device)
        self.rows_bytes = sum(b.numel() for b in bufs) * 8
        tbufs = [self.tails(nray) for _ in bufs]   # (alternating with the row buffers)
        if use_slots:
            sbufs = [first] + [Slots(nray, self.device) for _ in bufs[1:]]
        order = None
        if prev_work is None or order_policy not in ("cost", "priority", "cell", "total"):
            order = self.live_first_order_of(st)
        works = []          # per-ray attempts of the launches so far (the last two)
        self.split_rho = None
        auto_split, split_rows = self.parse_split(split)   # (cuts of the long launch)
        self.launch_log = []   # per launch: rows, rays in latency mode (diagnostics)
        self.launch_handoffs = []   # per launch: rays handed off at the drain (device int32)
        self.launch_work = []
        k = 0
        while k < len(bounds):
            i0, i1 = bounds[k]
            if (auto_split and k == n_lead and len(works) == 2 and i1 - i0 > 2 * split_rows[0]
                    and order_policy in ("cost", "priority", "total")):
                live = ~torch.isnan(st["state"][:5].sum(0))
                rho = self.rank_corr(works[0], works[1], live)
                self.split_rho = rho
                if rho < self.SPLIT_RHO:
                    bounds[k:k + 1] = self.cut_bounds(i0, i1, split_rows)
                    i1 = bounds[k][1]
                    order_policy = "total"
                if os.environ.get("RWRT_DEBUG_SCHED"):
                    print(f"split: rank correlation {rho:.3f} -> {'split' if rho < self.SPLIT_RHO else 'one launch'}",
                          flush=True)
            flat = bufs[k % len(bufs)].view(-1)
            view = flat[: nblk * (i1 - i0) * H.NOUT].view(nblk, i1 - i0, H.NOUT)
            slots = None
            if sbufs is not None:
                slots = sbufs[k % len(sbufs)]
                if k > 0:   # (the first launch's were computed above)
                    slots.compute(st, self._stream())
            work = None
            if order_policy in ("cost", "priority", "cell", "total") and prev_work is not None:
                # the previous launch's attempts per ray, or ("total") all of them so far
                work = cnt.sum(1) - (0 if order_policy == "total" else prev_work)
            # (a list: one latency-mode size per launch, the last repeated)
            tk = team[min(k, len(team) - 1)] if isinstance(team, list) else team
            if order_policy in ("cost", "priority", "cell", "total") and prev_work is not None:
                head = (self.team_capacity_tv() if self.bg is not None else self.team_capacity()) if tk else 0
                order = (self.cost_cell_order(st, work, head=head)
                         if order_policy == "cell" else self.cost_order(st, work))
            n_heavy, qpw = self.team_size(tk, st, work, order, i1 - i0) if tk else (0, 16)
            self.launch_log.append({"rows": [int(i0), int(i1)], "n_heavy": int(n_heavy), "per_wave": int(qpw)})
            if os.environ.get("RWRT_DEBUG_TEAM"):
                print(f"launch rows [{i0}, {i1}): n_heavy {n_heavy} at {qpw} per wave", flush=True)
            prev_work = cnt.sum(1)
            tails = tbufs[k % len(bufs)]
            if events is not None:
                e0, e1, es = self._event_pair()
                self.run(st, p, tb, i0, i1, view, order, n_heavy, qpw, tails, slots)
                e1.record(es)
                events.append((e0, e1))
            else:
                self.run(st, p, tb, i0, i1, view, order, n_heavy, qpw, tails, slots)
            self.launch_handoffs.append(self.work[0:1].clone())   # (rays handed off, rwrt_ctx_set_handoff)
            if auto_split and k < n_lead:
                works = (works + [cnt.sum(1) - prev_work])[-2:]
            if self.keep_launch_work:   # (diagnostics: each launch's attempts per ray and its latency set)
                self.launch_work.append((cnt.sum(1) - prev_work, order[:n_heavy].clone() if n_heavy else None))
            if sink is not None:
                deliver(self, sink, i0, i1, view, tails, slots)
            elif tails is not None and out is not None:
                self.expand(view, tails, i0, i1)   # (the caller reads its own buffer: dense rows)
            k += 1
        mx = int(st["nanrow"].max().item()) if nray else 0
        if group is not None:
            from shard import reduce_max
            mx = reduce_max(mx, group)
        brk = mx if mx < nt else None
        res = RunResult(cnt[:, 0], cnt[:, 1], st["nanrow"], False, brk, n_live)
        res.bounds = bounds
        res.state, res.next_row = st, end
        res.params = run_params(p, tb)
        return res

    # ------------------------------------------------------ checkpoint / resume
    CHECKPOINT_KEYS = {"state", "count", "nanrow", "next_row", "params", "nray"}

    @staticmethod
    def checkpoint(res):
        """The solver state after the rows a run produced (the
        state is 12 fp64 + 3 integers per ray, so resuming = persisting it at an
        output index): host arrays that ``resume`` continues from bit for bit,
        with the run's parameters (``run_params``: rtol, atol, min step,
        cut-off, nt, tstep, last output time) and ray count, which ``resume``
        checks."""
        st = res.state
        return {"state": st["state"].cpu().numpy(), "count": st["count"].cpu().numpy(),
                "nanrow": st["nanrow"].cpu().numpy(), "next_row": np.int64(res.next_row),
                "params": np.asarray(res.params, np.float64), "nray": np.int64(st["nray"])}

    @staticmethod
    def _ck_path(path):
        p = os.fspath(path)
        return p if p.endswith(".npz") else p + ".npz"   # (np.savez appends .npz)

    @staticmethod
    def save_checkpoint(ck, path):
        np.savez(RayEngine._ck_path(path), **ck)

    @staticmethod
    def load_checkpoint(path):
        path = RayEngine._ck_path(path)
        with np.load(path, allow_pickle=False) as z:
            ck = {k: z[k] for k in z.files}
        if (set(ck) != RayEngine.CHECKPOINT_KEYS or ck["state"].shape[0] != H.NSTATE
                or ck["state"].shape[1] != int(ck["nray"]) or ck["params"].shape != (7,)):
            raise ValueError(f"{path}: not an rwrt checkpoint")
        return ck

    def resume(self, ck, nt, tstep, rtol=1e-6, atol=1e-6, msf=1e-3, cut_off=0.1, ttotal=None,
               chunk=None, sink=None, out=None, cut_rad=None, events=None, group=None,
               order_policy="priority", first_chunk=None, team=0, stop_row=None):
        """Rows ``[ck['next_row'], nt)`` of the run a checkpoint was taken from
        (the same ``nt``, ``tstep`` and tolerances), into ``sink`` as in
        ``integrate``: the rows and counters equal an uninterrupted run's."""
        p = self.params(nt, tstep, rtol, atol, msf, cut_off, cut_rad)
        tb = torch.as_tensor(t_eval_of(nt, tstep, ttotal), dtype=F64, device=self.device)
        nray = int(ck["state"].shape[1])
        want = np.asarray(ck["params"], np.float64)
        got = np.asarray(run_params(p, tb), np.float64)
        if not np.array_equal(want, got) or nray != int(ck["nray"]):
            names = ["rtol", "atol", "min_step", "cut_off", "nt", "tstep", "t_last"]
            diff = {n: (float(a), float(b)) for n, a, b in zip(names, want, got) if a != b}
            raise ValueError(f"checkpoint taken with other run parameters {diff} (checkpoint, resume): "
                             f"the continuation would not equal the uninterrupted run")
        st = dict(state=torch.as_tensor(ck["state"], dtype=F64).to(self.device).contiguous(),
                  count=torch.as_tensor(ck["count"], dtype=torch.int64).to(self.device).contiguous(),
                  nanrow=torch.as_tensor(ck["nanrow"], dtype=torch.int32).to(self.device).contiguous(),
                  nray=nray)
        start = int(ck["next_row"])
        if not 1 <= start <= nt:
            raise ValueError(f"checkpoint row {start} outside [1, {nt}]")
        live = ~torch.isnan(st["state"][:5].sum(0))
        n_live_local = int(live.sum().item())
        return self.advance(st, p, tb, start, chunk=chunk, sink=sink, out=out, events=events,
                            group=group, order_policy=order_policy, first_chunk=first_chunk,
                            n_live=n_live_local, n_live_local=n_live_local, team=team, stop_row=stop_row)

    @staticmethod
    def take(st, idx):
        """The per-ray state of rays ``idx`` (a device index tensor): a shard."""
        return dict(state=st["state"][:, idx].contiguous(), count=st["count"][idx].contiguous(),
                    nanrow=st["nanrow"][idx].contiguous(), nray=int(idx.numel()))

    @staticmethod
    def live_first_order_of(st):
        """Live-first queue order from the state itself (NaN mean = frozen)."""
        dead = torch.isnan(st["state"][:5].sum(0)).to(torch.int8)
        return torch.sort(dead, stable=True).indices.to(torch.int64).contiguous()


def morton2(ix, iy):
    """Morton (Z-order) code of two non-negative int64 tensors below 2^16."""
    def spread(v):
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        return (v | (v << 1)) & 0x55555555
    return spread(ix & 0xFFFF) | (spread(iy & 0xFFFF) << 1)


def run_params(p, tb):
    """The parameters a run's continuation depends on (checkpoints carry them):
    ``[rtol, atol, min_step, cut_off, nt, tstep, last output time]``."""
    return [p.rtol, p.atol, p.min_step, p.cut_off, float(p.nt), p.tstep, float(tb[-1].item())]


def _row_buffers(out, nray, rows_max, device):
    """The device row buffers chunks are written to: ``out`` (one tensor, or a
    list whose buffers alternate so that a consumer can read chunk k while
    chunk k+1 is computed, hostio.HistorySink), each ``[nray][>= rows][8]``;
    allocated when missing or too small."""
    bufs = list(out) if isinstance(out, (list, tuple)) else [out]
    for j, b in enumerate(bufs):
        if b is None or b.numel() < nray * rows_max * H.NOUT:
            bufs[j] = torch.empty((nray, rows_max, H.NOUT), dtype=F64, device=device)
    return bufs


def ctypes_ref(p):
    import ctypes
    return ctypes.byref(p)


def kat_rk45(kind, y0, t_eval, rtol, atol, min_step, device="cuda"):
    """Stepper KAT on the GPU: ``y0[nvar, ncol]`` -> ``ys[nt, nvar, ncol]``."""
    H.require_gpu()
    y0 = torch.as_tensor(y0, dtype=F64, device=device).contiguous()
    te = torch.as_tensor(t_eval, dtype=F64, device=device).contiguous()
    nv, ncol = y0.shape
    out = torch.empty((ncol, len(t_eval), nv), dtype=F64, device=device)
    H.check(H.load().rwrt_kat_rk45(int(kind), ncol, H.dptr(y0), len(t_eval), H.dptr(te),
                                   float(max(rtol, 100 * np.finfo(np.float64).eps)), float(atol),
                                   float(min_step), H.dptr(out), H.stream(y0.device)))
    return out.permute(1, 2, 0)


MATH_KINDS = {"sin": 0, "cos": 1, "tan": 2, "pow": 3, "atan2": 4, "mod": 5, "sqrt": 6,
              "div": 7, "floor": 8, "sincos_sin": 9, "sincos_cos": 10, "div_rearth": 11,
              "fmod": 12, "mod2pi": 13, "mod2pi_twice": 14, "div_hw": 15, "floor_i32": 16,
              "div2_first": 23,
              "div2_second": 24, "nm_sin": 25, "nm_cos": 26, "nm_tan": 27, "nm_pow": 28,
              "nm_rcp14": 29, "k_sin": 30, "k_cos": 31, "k_tan": 32, "k_pow": 33,
              "qdiv": 34, "qdiv_exact_range": 35, "jump_verdict_fast": 36, "jump_verdict_exact": 37}


def selftest_math(name, x, y=None, device="cuda"):
    """Evaluate one device math routine element-wise (``rwrt_selftest_math``)."""
    H.require_gpu()
    x = torch.as_tensor(np.asarray(x, np.float64), device=device).contiguous()
    yt = None if y is None else torch.as_tensor(np.asarray(y, np.float64), device=device).contiguous()
    out = torch.empty_like(x)
    H.check(H.load().rwrt_selftest_math(MATH_KINDS[name], x.numel(), H.dptr(x), H.dptr(yt),
                                        H.dptr(out), H.stream(x.device)))
    return out.cpu().numpy()
