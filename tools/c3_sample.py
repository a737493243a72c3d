"""The C3 test sample and the reference's own noise floor on it (CPU oracle).

Picks a cost-stratified sample of the live C3 rays (BASELINE configs[2]:
2-degree global seeds x k = 1..10 x 5 periods, 2.5-degree zonal DJF jets) and
measures, on that sample, how far the reference's ray loop moves under a
random 1-ulp perturbation of every RHS output -- the spread below which an
implementation that is not bit-identical to NumPy's libm cannot agree with the
reference.

* cost: accepted + rejected attempts per ray over the first day (oracle, all
  live rays, one process per host core);
* sample: the ``--heavy`` most expensive rays, plus an equal number of rays
  drawn at random (seed 0) from each of ``--strata`` cost quantiles of the rest;
* floor: max(|dlon|, |dlat|) between the clean and the perturbed oracle run at
  2 h, 1 d, 4 d and 12 d (p50 / p99 / max / alive flips).

Writes ``tests/golden/c3_sample.npz`` (slot indices into bench.c3_initial_state's
order, 1-day costs) and ``tests/golden/noise_floor_C3_zonal.json``.

    python tools/c3_sample.py [--rays 16384] [--days 12] [--procs 8]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def _run(args):
    bg, y0, nt, seed = args
    import rwrt_oracle as O
    orig = O.rhs
    if seed is not None:
        rng = np.random.default_rng(seed)

        def rhs(b, y, t=None):
            d, bad = orig(b, y, t)
            return d * (1 + rng.choice([-1.0, 1.0], d.shape) * 2.0 ** -52), bad
        O.rhs = rhs
    try:
        with np.errstate(all="ignore"):
            hist, nacc, nrej, st = O.ray_run(O.Background(**bg), y0, nt, 7200.0)
    finally:
        O.rhs = orig
    return hist[:2], nacc + nrej


def run_parallel(bg, y0, nt, procs, seed=None):
    parts = np.array_split(np.arange(y0.shape[1]), procs)
    jobs = [(bg, y0[:, p].copy(), nt, None if seed is None else seed + k) for k, p in enumerate(parts)]
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_run, jobs)
    return np.concatenate([r[0] for r in res], axis=2), np.concatenate([r[1] for r in res])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=16384)
    ap.add_argument("--heavy", type=int, default=512)
    ap.add_argument("--strata", type=int, default=31)
    ap.add_argument("--days", type=float, default=12.0)
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    from bench import c3_initial_state, make_bs
    bs, bg = make_bs("zonal")
    y0 = c3_initial_state(bs)
    live = np.where(~np.isnan(y0.mean(axis=0)))[0]
    _, cost = run_parallel(bg, y0[:, live], 13, a.procs)
    order = np.argsort(-cost, kind="stable")
    heavy = live[order[: a.heavy]]
    rest = order[a.heavy:]
    per = (a.rays - a.heavy) // a.strata
    rng = np.random.default_rng(0)
    picks = [heavy]
    for s in np.array_split(rest, a.strata):
        picks.append(live[rng.choice(s, size=min(per, len(s)), replace=False)])
    idx = np.sort(np.concatenate(picks))
    pos = {int(v): i for i, v in enumerate(live)}
    cost_idx = cost[[pos[int(i)] for i in idx]]
    nt = int(round(a.days * 12)) + 1
    h0, _ = run_parallel(bg, y0[:, idx].copy(), nt, a.procs)
    h1, _ = run_parallel(bg, y0[:, idx].copy(), nt, a.procs, seed=1)
    out = {"config": "C3", "kind": "zonal", "rays": int(len(idx)), "heavy": a.heavy, "strata": a.strata,
           "perturbation": "every RHS output x (1 +- 2^-52), random sign per element",
           "cost_1d": {"min": int(cost.min()), "median": float(np.median(cost)), "max": int(cost.max())}}
    for row in (1, 12, 48, nt - 1):
        p, q = h0[:, row], h1[:, row]
        ok = ~np.isnan(p).any(0) & ~np.isnan(q).any(0)
        d = np.max(np.abs(p[:, ok] - q[:, ok]), axis=0)
        out[f"{row / 12:g}d"] = {"p50": float(np.median(d)), "p99": float(np.percentile(d, 99)),
                                 "max": float(d.max()), "frac_gt_1e-6": float(np.mean(d > 1e-6)),
                                 "alive_flips": int(np.sum(np.isnan(p[0]) != np.isnan(q[0])))}
    gold = os.path.join(ROOT, "tests", "golden")
    np.savez_compressed(os.path.join(gold, "c3_sample.npz"), idx=idx.astype(np.int64),
                        cost_1d=cost_idx.astype(np.int32), nslot=np.int64(y0.shape[1]))
    js = json.dumps(out, indent=1)
    open(os.path.join(gold, "noise_floor_C3_zonal.json"), "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
