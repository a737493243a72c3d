"""The K heaviest C3 rays alone in latency mode (quad_rays) at a given density,
for PMC passes that must see only that launch.

    python tools/latency_only.py --find heavy.npy            # once: the order by work
    python tools/latency_only.py --load heavy.npy --k 256 --density 4 [--run-kernel]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from engine import RayEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--find", default=None)
    ap.add_argument("--load", default=None)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--density", type=int, default=16)
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--run-kernel", action="store_true", help="the same rays through the run kernel instead")
    ap.add_argument("--clone", action="store_true", help="K copies of the heaviest ray instead of the K heaviest")
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    bs, _ = bench.make_bs("zonal")
    y0 = torch.as_tensor(bench.c3_initial_state(bs), device="cuda")
    eng = RayEngine.from_bs(bs)
    nt = int(a.days * 12) + 1
    if a.find:
        full = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, first_chunk=[6, 24, 96])
        work = (full.nacc + full.nrej)
        order = torch.sort(work, descending=True, stable=True).indices
        np.save(a.find, order[:8192].cpu().numpy())
        return
    idx = torch.as_tensor(np.load(a.load)[: a.k], device="cuda")
    if a.clone:
        idx = idx[:1].repeat(a.k)
    yk = y0[:, idx].contiguous()
    out = torch.empty((a.k, nt - 1, 8), dtype=torch.float64, device="cuda")
    team = 0 if a.run_kernel else (a.k, a.density)
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = eng.integrate(yk, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=nt - 1, out=out, team=team)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        att = int((r.nacc + r.nrej).max().item())
        print(f"k {a.k} density {a.density} run_kernel {a.run_kernel} clone {a.clone}: {dt:.4f} s, "
              f"{1e6 * dt / att:.2f} us/attempt", flush=True)


if __name__ == "__main__":
    main()
