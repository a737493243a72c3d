"""Drop-in rate: ``WR.ray_run(mode='hip', inte_method='rk45')`` on one C3
period (2-degree global seeds x k = 1..10, stationary, 90 days), the
reference's own call surface with the full history delivered into the WR
host arrays (PCIe + host copies included), against the kernel-only time of
the same rays.

    python tools/dropin_rate.py [--days 90] [--chunk ROWS]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import synthetic as S  # noqa: E402
from wr import WR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=90.0)
    ap.add_argument("--chunk", type=int, default=0)
    a = ap.parse_args()
    bs, _ = bench.make_bs("zonal")
    cfg = S.config("C3")
    nt = int(round(a.days * 12)) + 1
    w = WR(cfg.nzwn, cfg.nsource, 7200.0, (nt - 1) * 7200.0, 0.0, nx=bs.nlon, ny=bs.nlat,
           chunk_rows=a.chunk or None)
    w.bs = bs
    w.set_zwn(cfg.zwn)
    w.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        w.ray_run(mode="hip", inte_method="rk45")          # warm-up (GPU init, library load)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w.ray_run(mode="hip", inte_method="rk45")
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    res = w.last_run
    steps = int(res.nacc.sum().item())
    nbytes = sum(getattr(w, n).nbytes for n in ("rlon", "rlat", "rzwn", "rmwn", "ramp", "rug", "rvg"))
    y0 = np.array([w.rlon[0], w.rlat[0], w.rzwn[0], w.rmwn[0], w.ramp[0]]).reshape(5, -1)
    eng = bs.engine()
    y0d = torch.as_tensor(y0, device="cuda")
    out = torch.empty((y0.shape[1], nt - 1, 8), dtype=torch.float64, device="cuda")
    eng.integrate(y0d, nt, 7200.0, ttotal=(nt - 1) * 7200.0, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.integrate(y0d, nt, 7200.0, ttotal=(nt - 1) * 7200.0, out=out)
    torch.cuda.synchronize()
    kern = time.perf_counter() - t0
    print(json.dumps({"workload": f"C3 stationary period, {a.days:g} d, WR.ray_run(mode='hip')",
                      "slots": int(y0.shape[1]), "ray_steps": steps, "history_bytes": int(nbytes),
                      "dropin_s": wall, "dropin_rate": steps / wall,
                      "device_only_s": kern, "device_only_rate": steps / kern,
                      "launch_rows": [b - a_ for a_, b in res.bounds],
                      "delivery": getattr(w, "last_delivery", None)}))


if __name__ == "__main__":
    main()
