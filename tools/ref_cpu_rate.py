"""The reference ITSELF timed on bench.py's CPU-baseline sample (build
container only: it imports /root/reference through tests/golden/refharness.py,
which the GPU box does not have).

bench.py's cpu_baseline times oracle/rwrt_oracle.py in the reference's loop
shape on 8 192 live C3 rays for 12 days (seed 2).  This script runs the same
rays through the reference's own loop -- WR.core_ray_run('numpy_rk45')
(wr.py:767-887) with RK45 from rkf45.py -- times it on one core, and checks
its history against the oracle's bit for bit (NaN == NaN), so the two rates
are for the same work.

    python tools/ref_cpu_rate.py [--rays 8192] [--days 12] [--out profiles/r4/sched/ref_cpu_rate.json]

Phase 1 (a child process: our package's bs / wr / wn module names collide
with the reference's) builds the C3 initial state with the package, picks the
sample exactly as bench.cpu_baseline does and runs the oracle; phase 2 (this
process) runs the reference.
"""
import argparse
import contextlib
import io
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def phase1(path, nrays, days, seed):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
    import bench
    bs, bg = bench.make_bs("zonal")
    y0 = bench.c3_initial_state(bs)
    pick, hist, nacc, dt, nt, nrej, cols = bench.cpu_baseline(bg, y0, nrays, days, seed=seed, fsal=False)
    np.savez(path, y=y0[:, pick], hist=hist, nacc=nacc, dt=dt, nt=nt, nrej=nrej, cols=cols)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=8192)
    ap.add_argument("--days", type=float, default=12)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--phase1", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.phase1:
        phase1(a.phase1, a.rays, a.days, a.seed)
        return
    tmp = os.path.join(tempfile.gettempdir(), "ref_cpu_rate_phase1.npz")
    subprocess.run([sys.executable, __file__, "--phase1", tmp, "--rays", str(a.rays), "--days", str(a.days),
                    "--seed", str(a.seed)], check=True)
    P = np.load(tmp)
    y, nt = P["y"], int(P["nt"])

    sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
    import refharness as H
    import synthetic as S
    R = H.load_reference()
    bg = S.background("zonal")
    cfg = S.config("C3")
    n = y.shape[1]
    nsrc = -(-n // 3)                       # the sample in the three root slots: (3, nsrc, 1)
    H.put_nc("refrate.nc", **bg)
    with contextlib.redirect_stdout(io.StringIO()):
        wr = R.wr.WR(1, nsrc, cfg.tstep * R.constants.hour, (nt - 1) * cfg.tstep * R.constants.hour,
                     S.c3_freq(None), nx=len(bg["lon"]), ny=len(bg["lat"]), rtol=cfg.rtol, atol=cfg.atol,
                     ncfile="refrate.nc", MinStepFactor=cfg.MinStepFactor)
        wr.bs.loadbs_ncfile("refrate.nc")
        wr.bs.ready(xcyclic=True)
    assert wr.nt == nt, (wr.nt, nt)
    slots = np.full((5, 3 * nsrc), np.nan)
    slots[:, :n] = y
    for v, arr in enumerate([wr.rlon, wr.rlat, wr.rzwn, wr.rmwn, wr.ramp]):
        arr[0] = slots[v].reshape(3, nsrc, 1)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()), np.errstate(all="ignore"):
        wr.core_ray_run("numpy_rk45")
    dt = time.perf_counter() - t0
    ref = np.array([wr.rlon, wr.rlat, wr.rzwn, wr.rmwn, wr.ramp]).reshape(5, nt, 3 * nsrc)[:, :, :n]
    ora = P["hist"][:5]
    same = (ref == ora) | (np.isnan(ref) & np.isnan(ora))
    nacc = int(P["nacc"])
    out = {"sample": f"{n} live C3 rays (bench.cpu_baseline's seed-{a.seed} pick) x {a.days:g} d, zonal",
           "accepted_steps": nacc,
           "reference_wr_core_ray_run_rk45": {"seconds": dt, "ray_steps_per_s": nacc / dt, "cores": 1},
           "oracle_reference_loop": {"seconds": float(P["dt"]), "ray_steps_per_s": nacc / float(P["dt"]),
                                     "rhs_columns_per_accepted_step": float(P["cols"]) / nacc, "cores": 1},
           "bitwise_equal_rows_frac": float(same.mean()),
           "note": "the reference's own loop (wr.py:767-887, rkf45.py RK45) run from /root/reference in the "
                   "build container through tests/golden/refharness.py (numba -> identity jit); both timed on "
                   "the same host around the ray loop only"}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
