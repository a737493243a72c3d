"""RK4 rate: the reference's default integrator (``inte_method=''``,
WR.core_ray_run_numpy, wr.py:702-765) through ``rwrt_rk4_run`` on the C3 ray
set (2.40 M slots, 90 d at 2 h, outputs resident in HBM).

    python tools/rk4_rate.py [--days 90] [--steps 2]

One RK4 step per ray per output interval (4 RHS evaluations); the rate counts
steps taken (the nacc column), as bench.py counts accepted RK45 steps.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from engine import RayEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    bs, _ = bench.make_bs("zonal")
    y0 = torch.as_tensor(bench.c3_initial_state(bs), device="cuda")
    eng = RayEngine.from_bs(bs)
    nt = int(round(a.days * 12)) + 1
    out = torch.empty((y0.shape[1], nt - 1, 8), dtype=torch.float64, device="cuda")
    res = eng.integrate_rk4(y0, nt, 7200.0, out=out)       # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = eng.integrate_rk4(y0, nt, 7200.0, out=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    live = ~torch.isnan(y0.sum(0))      # dead slots (NaN roots) take no counted steps
    steps = int(res.nacc[live].sum().item())
    print(json.dumps({"workload": f"C3 RK4, {a.days:g} d at 2 h", "slots": int(y0.shape[1]),
                      "live": int(live.sum().item()), "rk4_steps": steps, "s_per_run": dt,
                      "rk4_steps_per_s": steps / dt, "rhs_evals_per_s": 4 * steps / dt}))


if __name__ == "__main__":
    main()
