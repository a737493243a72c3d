"""ctypes binding of librwrt.so (the C ABI declared in include/rwrt.h).

PyTorch-ROCm owns every device buffer: callers pass tensors, this module
passes ``data_ptr()`` and the current HIP stream.  There is no CPU fallback:
if the library is missing or no GPU is visible, every entry point raises.
"""
import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first (same SONAME as ours)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RWRT_LIB", os.path.join(_HERE, "librwrt.so"))

NFIELD_REF, NFIELD_PACK, NVAR, NMERC, NOUT, NSTATE = 18, 12, 5, 12, 8, 12
ABI_SYMBOLS = ("rwrt_version", "rwrt_last_error", "rwrt_ctx_create", "rwrt_ctx_destroy",
               "rwrt_ctx_set_latency_density", "rwrt_ctx_set_tv_lanes", "rwrt_ctx_set_handoff",
               "rwrt_ctx_set_trace",
               "rwrt_pack_fields",
               "rwrt_mercator_point", "rwrt_rhs", "rwrt_dp54_attempt",
               "rwrt_ray_initial", "rwrt_rk45_init", "rwrt_rk45_run", "rwrt_rk45_run_tails",
               "rwrt_expand_tails", "rwrt_row_slots", "rwrt_rk45_run_slots", "rwrt_expand_slots",
               "rwrt_rk4_run",
               "rwrt_bs_ready", "rwrt_rk45_init_tv", "rwrt_rk45_run_tv", "rwrt_rk45_run_tv_tails",
               "rwrt_rk45_run_tv_slots", "rwrt_rhs_tv",
               "rwrt_kat_rk45", "rwrt_selftest_math", "rwrt_host_fill_rows")

RWRT_OK, RWRT_ERR_ARG, RWRT_ERR_HIP, RWRT_SOLVER_FAILED = 0, 1, 2, 3


class RwrtError(RuntimeError):
    pass


class SolverFailed(RwrtError):
    """rkf45.py:423-425: every retrying column has a NaN step (status -1)."""


class Grid(ctypes.Structure):
    _fields_ = [("ncol", ctypes.c_int32), ("nrow", ctypes.c_int32),
                ("lon0", ctypes.c_double), ("dlon", ctypes.c_double),
                ("lat0", ctypes.c_double), ("dlat", ctypes.c_double)]


class Params(ctypes.Structure):
    _fields_ = [("rtol", ctypes.c_double), ("atol", ctypes.c_double),
                ("min_step", ctypes.c_double), ("cut_off", ctypes.c_double),
                ("nt", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("tstep", ctypes.c_double)]


class Background(ctypes.Structure):
    _fields_ = [("d_levels", ctypes.c_void_p), ("nlev", ctypes.c_int32), ("fp32", ctypes.c_int32),
                ("t0", ctypes.c_double), ("dt", ctypes.c_double)]


_lib = None
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_D = ctypes.c_double


def load():
    """Load librwrt.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RwrtError(f"HIP library not found at {LIB_PATH}: build it with "
                        f"`make -C rossby-wave-ray-tracing_amd/csrc` (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    lib.rwrt_version.restype = ctypes.c_char_p
    lib.rwrt_last_error.restype = ctypes.c_char_p
    G, Pr, B = ctypes.POINTER(Grid), ctypes.POINTER(Params), ctypes.POINTER(Background)
    sig = {
        "rwrt_pack_fields": [G, _P, _P, _P],
        "rwrt_mercator_point": [G, _P, _I64, _P, _P, _P, _P],
        "rwrt_rhs": [G, _P, _I64, _P, _P, _P],
        "rwrt_dp54_attempt": [G, _P, _I64, _P, _P, _P, _D, _D, _P, _P, _P, _P],
        "rwrt_ray_initial": [G, _P, _I64, _P, _P, _P, _I32, _P, _P, _P, _P],
        "rwrt_rk45_init": [G, _P, _I64, _P, Pr, _P, _P, _P, _P, _P, _P],
        "rwrt_rk45_run": [_P, G, _P, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P],
        "rwrt_rk45_run_tails": [_P, G, _P, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P,
                                _P],
        "rwrt_expand_tails": [_I64, _I32, _I32, _P, _P, _P, _P],
        "rwrt_row_slots": [_I64, _P, _P, _P, _P],
        "rwrt_rk45_run_slots": [_P, G, _P, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P],
        "rwrt_expand_slots": [_I64, _I32, _I32, _P, _P, _P, _P, _P, _P],
        "rwrt_rk4_run": [_P, G, _P, _I64, Pr, _I32, _I32, _P, _P, _P, _P, _P, _P, _P],
        "rwrt_bs_ready": [_I32, _I32, _P, _P, _P, _D, _D, _P, _P, _I32, _P],
        "rwrt_rk45_init_tv": [G, B, _I64, _P, Pr, _P, _P, _P, _P, _P, _P],
        "rwrt_rk45_run_tv": [_P, G, B, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P],
        "rwrt_rk45_run_tv_tails": [_P, G, B, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P,
                                   _P],
        "rwrt_rk45_run_tv_slots": [_P, G, B, _I64, Pr, _P, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P,
                                   _P, _P],
        "rwrt_ctx_create": [_I32, ctypes.POINTER(_P)],
        "rwrt_ctx_destroy": [_P],
        "rwrt_ctx_set_latency_density": [_P, _I32],
        "rwrt_ctx_set_tv_lanes": [_P, _I32],
        "rwrt_ctx_set_handoff": [_P, _I32],
        "rwrt_ctx_set_trace": [_P, _P, _I64],
        "rwrt_rhs_tv": [G, B, _I64, _P, _P, _P, _P],
        "rwrt_kat_rk45": [_I32, _I64, _P, _I32, _P, _D, _D, _D, _P, _P],
        "rwrt_selftest_math": [_I32, _I64, _P, _P, _P, _P],
        "rwrt_host_fill_rows": [_P, _I64, _I64, _I64, _P, _P, _I64, _I64, _P],
    }
    for name, args in sig.items():
        fn = getattr(lib, name, None)
        if fn is None:     # (an older A/B build: bench.py --lib; tests/test_abi.py checks ours)
            continue
        fn.argtypes = args
        fn.restype = ctypes.c_int
    _lib = lib
    return lib


def version():
    return load().rwrt_version().decode()


def check(status):
    if status != RWRT_OK:
        msg = load().rwrt_last_error().decode()
        raise RwrtError(f"rwrt status {status}: {msg}")


def require_gpu():
    if not torch.cuda.is_available():
        raise RwrtError("no HIP device visible: the ray integrator runs only on the GPU "
                        "(there is no CPU fallback)")


def dptr(t, dtype=None, what="tensor"):
    """Device pointer of a contiguous tensor (checked)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RwrtError(f"{what} must be a device tensor")
    if dtype is not None and t.dtype != dtype:
        raise RwrtError(f"{what} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise RwrtError(f"{what} must be contiguous")
    return t.data_ptr()


def stream(device=None):
    """The current HIP stream of ``device`` (default: torch's current device)."""
    return torch.cuda.current_stream(device).cuda_stream


class Context:
    """An ``rwrt_ctx`` (include/rwrt.h): the scratch of the ray-loop entry points
    on one device.  Engines own one each; distinct contexts are independent."""

    def __init__(self, device):
        require_gpu()
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        h = _P()
        check(load().rwrt_ctx_create(int(idx), ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def set_latency_density(self, rays_per_wave):
        """Rays per wave in the latency mode (1..16): rwrt_ctx_set_latency_density."""
        if getattr(self, "_qpw", 16) != int(rays_per_wave):
            check(load().rwrt_ctx_set_latency_density(self._h, int(rays_per_wave)))
            self._qpw = int(rays_per_wave)

    def set_tv_lanes(self, lanes):
        """Rays per wave of the fp64 time-varying loops, 64 or 32 (rwrt_ctx_set_tv_lanes)."""
        if getattr(self, "_tvl", 64) != int(lanes):
            check(load().rwrt_ctx_set_tv_lanes(self._h, int(lanes)))
            self._tvl = int(lanes)

    def set_handoff(self, max_rays):
        """Drain-time hand-off threshold, 0..16 rays per wave (rwrt_ctx_set_handoff)."""
        if getattr(self, "_hof", 16) != int(max_rays):
            check(load().rwrt_ctx_set_handoff(self._h, int(max_rays)))
            self._hof = int(max_rays)

    def set_trace(self, trace=None):
        """Diagnostic ray trace (rwrt_ctx_set_trace): ``trace`` an int64 device
        tensor ``[cap, 10]`` (None: off)."""
        if trace is None:
            check(load().rwrt_ctx_set_trace(self._h, None, 0))
        else:
            check(load().rwrt_ctx_set_trace(self._h, ctypes.c_void_p(trace.data_ptr()), int(trace.shape[0])))
        self._trace = trace

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h is not None and h.value and _lib is not None:
            _lib.rwrt_ctx_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:   # interpreter shutdown
            pass
