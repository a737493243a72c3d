"""Sensitivity of the reference's own ray loop to 1-ulp RHS perturbations (CPU oracle).

The oracle is bit-exact with the reference; here its RHS output is multiplied by
(1 + s * 2^-52), s = +-1 at random per element, on every evaluation -- the size
of a last-bit difference in one transcendental.  The spread between the
perturbed and the clean run is the floor below which no implementation that is
not bit-identical to NumPy's libm/SVML can agree with the reference.

    python tools/noise_floor.py [--kind zonal|nonzonal] [--days 10] [--config C2] [--rk4]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import rwrt_oracle as O  # noqa: E402
import synthetic as S    # noqa: E402


def run(kind, nt, perturb_seed=None, config="C2", rk4=False):
    bg = O.Background(**S.background(kind))
    cfg = S.config(config)
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = np.array(O.ray_initial(bg, slon, slat, cfg.zwn, cfg.freq)).reshape(7, -1)
    orig = O.rhs
    if perturb_seed is not None:
        rng = np.random.default_rng(perturb_seed)

        def rhs(b, y):
            d, bad = orig(b, y)
            return d * (1 + rng.choice([-1.0, 1.0], d.shape) * 2.0 ** -52), bad
        O.rhs = rhs
    try:
        if rk4:
            hist, st = O.ray_run_rk4(bg, rows[:5].copy(), nt, 7200.0, row0=rows)
        else:
            hist, nacc, nrej, st = O.ray_run(bg, rows[:5].copy(), nt, 7200.0, row0=rows)
    finally:
        O.rhs = orig
    return hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="nonzonal")
    ap.add_argument("--days", type=float, default=10.0)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--rk4", action="store_true")
    a = ap.parse_args()
    nt = int(a.days * 12) + 1
    with np.errstate(all="ignore"):
        h0 = run(a.kind, nt, config=a.config, rk4=a.rk4)
        h1 = run(a.kind, nt, perturb_seed=1, config=a.config, rk4=a.rk4)
    live = ~np.isnan(h0[3, 0])
    out = {"kind": a.kind, "config": a.config, "integrator": "rk4" if a.rk4 else "rk45",
           "live_rays": int(live.sum())}
    for row in [1, 12, 24, 60, 120, 360, 1080]:
        if row >= nt:
            continue
        a0, a1 = h0[:2, row, live], h1[:2, row, live]
        ok = ~np.isnan(a0).any(0) & ~np.isnan(a1).any(0)
        d = np.max(np.abs(a0[:, ok] - a1[:, ok]), axis=0)
        out[f"{row / 12:g}d"] = {"p50": float(np.median(d)), "p99": float(np.percentile(d, 99)),
                                 "max": float(d.max()), "frac_gt_1e-6": float(np.mean(d > 1e-6)),
                                 "alive_flips": int(np.sum(np.isnan(a0[0]) != np.isnan(a1[0])))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
