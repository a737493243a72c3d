"""Diagnostic: per-attempt latency of a lone wavefront vs the loaded GPU.

Runs C3 for D days, picks the 64 rays with the most attempts, and re-runs
only those (one wavefront on an otherwise idle GPU).  The lone wave's time per
attempt of its slowest ray is the critical-path latency of the kernel.
    python tools/latency_probe.py [--days 10] [--lib path]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=10)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--n", type=int, default=64)
    a = ap.parse_args()
    if a.lib:
        os.environ["RWRT_LIB"] = os.path.abspath(a.lib)
    import torch
    import bench
    from engine import RayEngine
    bs, bg = bench.make_bs("zonal")
    y0 = bench.c3_initial_state(bs)
    eng = RayEngine.from_bs(bs)
    nt = int(a.days * 12) + 1
    y0d = torch.as_tensor(y0, device="cuda")
    eng.integrate(y0d, nt, 7200.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = eng.integrate(y0d, nt, 7200.0)
    torch.cuda.synchronize()
    full = time.perf_counter() - t0
    att = (res.nacc + res.nrej).cpu().numpy()
    top = np.argsort(-att)[: a.n]
    sub = y0d[:, torch.as_tensor(top, device="cuda")].contiguous()
    eng.integrate(sub, nt, 7200.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r2 = eng.integrate(sub, nt, 7200.0)
    torch.cuda.synchronize()
    solo = time.perf_counter() - t0
    amax = int((r2.nacc + r2.nrej).max())
    print(json.dumps({"days": a.days, "full_s": full, "full_steps": res.ray_steps,
                      "max_attempts_any_ray": int(att.max()), "solo_s": solo,
                      "solo_max_attempts": amax, "solo_us_per_attempt": 1e6 * solo / amax,
                      "full_time_per_max_ray_attempt_us": 1e6 * full / int(att.max())}))


if __name__ == "__main__":
    main()
