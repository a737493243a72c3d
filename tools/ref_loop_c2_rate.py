"""The reference-loop oracle timed on the survey's own CPU case (C2: 1 280
live rays, 10 days), to set bench.py's cpu_baseline beside the survey's
measured reference rate (4.97e4 at 10 d, 5.99e4 at 30 d) and
beside the reference itself, timed here in the same process (build container
only: /root/reference through tests/golden/refharness.py, as
tests/golden/make_golden.py runs it), with its accepted-step count checked
against the golden fixture.

    python tools/ref_loop_c2_rate.py [--reps 3]      (CPU only)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd"),
                os.path.join(ROOT, "tests", "golden")]
import rwrt_oracle as O  # noqa: E402
import synthetic as S  # noqa: E402
import refharness as H  # noqa: E402


def reference_c2(kind, nt):
    """The reference's own real2d path for C2 (main_wr.py:66-86 set-up, then
    WR.ray_run(mode='numpy', inte_method='rk45')): seconds in ray_run."""
    import contextlib
    import io
    R = H.load_reference()
    bg = S.background(kind)
    cfg = S.config("C2", bg=kind)
    cfg.ttotal = (nt - 1) * cfg.tstep / 24.0
    H.put_nc("c2rate.nc", **bg)
    with contextlib.redirect_stdout(io.StringIO()):
        wr = R.wr.WR(cfg.nzwn, cfg.nsource, cfg.tstep * R.constants.hour, cfg.ttotal * R.constants.day,
                     cfg.freq, nx=len(bg["lon"]), ny=len(bg["lat"]), rtol=cfg.rtol, atol=cfg.atol,
                     ncfile="c2rate.nc", MinStepFactor=cfg.MinStepFactor)
        wr.bs.loadbs_ncfile("c2rate.nc")
        wr.bs.ready(xcyclic=True)
        wr.set_zwn(cfg.zwn)
        wr.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
        t0 = time.perf_counter()
        with np.errstate(all="ignore"):
            wr.ray_run(mode="numpy", inte_method="rk45", root_method="numpy")
        return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    out = {}
    for kind in ("zonal", "nonzonal"):
        g = np.load(os.path.join(ROOT, "tests", "golden", f"traj_C2_{kind}.npz"))
        bg = O.Background(**S.background(kind))
        nt = int(g["nt"])
        ref_rate = float(g["nacc"].sum()) / min(reference_c2(kind, nt) for _ in range(a.reps))
        best = {}
        for fsal in (False, True):
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                with np.errstate(all="ignore"):
                    hist, nacc, nrej, st = O.run_config(bg, S.config("C2"), nt=nt, fsal=fsal)
                ts.append(time.perf_counter() - t0)
                assert int(nacc.sum()) == int(g["nacc"].sum())
            best["reference_loop" if not fsal else "fsal_port"] = int(nacc.sum()) / min(ts)
        out[kind] = {"case": f"C2 {kind}: 1280 live rays, {nt - 1} rows (10 d)",
                     "accepted_steps": int(g["nacc"].sum()),
                     "reference_itself": ref_rate,
                     "oracle_reference_loop": best["reference_loop"],
                     "oracle_fsal_port": best["fsal_port"],
                     "note": "1 core, best of --reps; both timed around the whole run incl. the initial "
                             "rows (oracle: run_config; reference: WR.ray_run)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
