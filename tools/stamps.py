"""Where a lone ray's attempt spends its cycles (diagnostic build).

    make -C rossby-wave-ray-tracing_amd/csrc variant NAME=stamps DEFS=-DRWRT_DIAG_STAMPS=1
    python tools/stamps.py [--slot 2190591] [--days 90]

Integrates ONE C3 ray (default: the heaviest of the zonal set) with
librwrt_stamps.so, whose RWRT_STAMP(k) points charge s_memtime cycles to the
sections of ray_rhs / dp54_attempt / Lane::iterate / the post-processing,
and prints cycles per attempt per section.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("RWRT_LIB", os.path.join(ROOT, "rossby-wave-ray-tracing_amd", "librwrt_stamps.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import _hip as H  # noqa: E402
import bench  # noqa: E402
from engine import RayEngine  # noqa: E402

NAMES = ["stage input + loop (to RHS start)", "lookup_begin (cell, refill issue)", "sin/cos/tan",
         "lookup_end (LDS reads, blend)", "mercator12", "ugvg + core_diffun (divisions)",
         "error norm", "pow + step control", "(iterate return)", "post-processing (masks, ugvg_at, row)",
         "refill issue (24 LDS-DMA)", "(refills, count)", "LDS-DMA wait"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slot", type=int, default=2190591)
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--bg", default="zonal")
    ap.add_argument("--team", type=int, default=0)
    ap.add_argument("--batch", action="store_true",
                    help="the whole C3 set instead of one ray (per-wave section fractions)")
    a = ap.parse_args()
    lib = H.load()
    fn = lib.rwrt_diag_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = (ctypes.c_ulonglong * 16)()
    bs, _ = bench.make_bs(a.bg)
    y0 = bench.c3_initial_state(bs)
    y0 = torch.as_tensor(y0 if a.batch else y0[:, [a.slot]], device="cuda")
    eng = RayEngine.from_bs(bs)
    nt = int(a.days * 12) + 1
    eng.integrate(y0, nt, 7200.0, chunk=nt - 1, team=a.team)
    torch.cuda.synchronize()
    H.check(fn(buf))
    r = eng.integrate(y0, nt, 7200.0, chunk=nt - 1, team=a.team)
    torch.cuda.synchronize()
    H.check(fn(buf))
    att = int((r.nacc + r.nrej).sum().item())
    cyc = np.array(list(buf), dtype=np.float64)
    tot = cyc.sum()
    refills = cyc[11]
    cyc[11] = 0.0
    tot = cyc.sum()
    out = {"slot": None if a.batch else a.slot, "attempts": att, "team": a.team, "cycles_per_attempt": tot / att,
           "refills_per_attempt": refills / att,
           "sections": {NAMES[k]: {"cycles_per_attempt": cyc[k] / att, "frac": cyc[k] / tot}
                        for k in range(len(NAMES))}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
