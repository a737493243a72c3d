"""Which per-ray quantity, known when a launch starts, predicts the ray's work
in that launch best?  (C3, the bench's last launch, rows [190, 1081).)

Runs C3 to row 190 with the bench's leading launches, takes candidate
predictors from the solver state and the rows -- the previous launch's
accepted steps (the bench's order), the last ``--recent`` rows' accepted
steps, 1 / h_abs (the step size the ray will start with) -- then the rest, and
prints each predictor's Spearman correlation with the actual work and the
makespan of the list schedule it induces on 65 536 lanes (tools/sched_sim.py)
against the throughput bound and the oracle order.

    python tools/c3_predictors.py [--bg nonzonal]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg", default="nonzonal")
    ap.add_argument("--recent", default="10,20,40")
    ap.add_argument("--split", type=int, default=190)
    a = ap.parse_args()
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine, t_eval_of
    from sched_sim import makespan, LANES
    from scipy.stats import spearmanr
    nt = 1081
    bs, _ = make_bs(a.bg)
    eng = RayEngine.from_bs(bs)
    src, zcs = c3_sources(eng)
    y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
    last = {}

    def sink(i0, i1, o):
        last["rows"] = (i0, i1, o[:, :, 7].clone())

    r1 = eng.integrate(y0, nt, 7200.0, chunk=nt - 1, first_chunk=[6, 24], sink=sink, stop_row=a.split)
    st = r1.state
    cnt0 = st["count"].clone()
    i0, i1, nrows = last["rows"]
    habs = st["state"][11].clone()
    p = eng.params(nt, 7200.0)
    tb = torch.as_tensor(t_eval_of(nt, 7200.0), dtype=torch.float64, device=eng.device)
    eng.advance(st, p, tb, a.split, chunk=nt - 1)
    work = (st["count"].sum(1) - cnt0.sum(1)).cpu().numpy().astype(np.float64)
    live = work > 0
    cands = {"previous launch (bench)": (nrows[:, -1] - nrows[:, 0]).cpu().numpy(),
             "1 / h_abs": (1.0 / habs).nan_to_num(0.0, 0.0, 0.0).cpu().numpy()}
    for k in [int(x) for x in a.recent.split(",")]:
        cands[f"last {k} rows"] = (nrows[:, -1] - nrows[:, -1 - k]).cpu().numpy()
    lb = max(work.sum() / LANES, work.max())
    print(f"{a.bg}: rows [{a.split}, {nt}), {int(live.sum())} rays, work {work.sum():.0f} attempts, "
          f"max {work.max():.0f}, bound {lb:.0f}")
    print(f"  {'oracle':28s} makespan {makespan(work, np.argsort(-work, kind='stable')) / lb:.3f} x bound")
    for name, v in cands.items():
        v = np.asarray(v, np.float64)
        rho = spearmanr(v[live], work[live])[0]
        m = makespan(work, np.argsort(-v, kind="stable"))
        print(f"  {name:28s} makespan {m / lb:.3f} x bound, spearman {rho:.3f}", flush=True)


if __name__ == "__main__":
    main()
