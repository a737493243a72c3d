"""Diagnostic: distribution of per-ray work (accepted + rejected attempts) on C3.

    python tools/c3_stats.py [--days 90] [--chunk 55]
Prints per-ray totals and per-chunk quantiles (JSON) -- the load-balance input
for the work-queue design.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from engine import RayEngine  # noqa: E402


def q(a):
    a = np.asarray(a)
    return {p: float(np.percentile(a, p)) for p in (0, 10, 50, 90, 99, 99.9, 100)} | {"mean": float(a.mean())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--chunk", type=int, default=55)
    a = ap.parse_args()
    bs, bg = bench.make_bs("zonal")
    y0 = bench.c3_initial_state(bs)
    eng = RayEngine.from_bs(bs)
    nt = int(a.days * 12) + 1
    per_chunk = []
    prev = [None]

    def sink(i0, i1, rows):
        pass

    live = ~np.isnan(y0.mean(0))
    res = eng.integrate(torch.as_tensor(y0), nt, 7200.0, chunk=a.chunk, sink=sink)
    tot = (res.nacc + res.nrej).cpu().numpy()[live]
    out = {"live": int(live.sum()), "attempts_per_live_ray": q(tot),
           "accepted_per_live_ray": q(res.nacc.cpu().numpy()[live])}
    # per-chunk work: rerun chunk by chunk reading counters
    st = eng.init(torch.as_tensor(y0), eng.params(nt, 7200.0))
    tb = torch.as_tensor(np.arange(nt) * 7200.0, dtype=torch.float64, device="cuda")
    order = eng.live_first_order(st)
    buf = torch.empty((y0.shape[1], a.chunk, 8), dtype=torch.float64, device="cuda")
    p = eng.params(nt, 7200.0)
    chunks = []
    for i0 in range(1, nt, a.chunk):
        i1 = min(i0 + a.chunk, nt)
        c0 = st["count"].sum(1).clone()
        view = buf[:, : i1 - i0] if i1 - i0 == a.chunk else torch.empty((y0.shape[1], i1 - i0, 8), dtype=torch.float64, device="cuda")
        eng.run(st, p, tb, i0, i1, view, order)
        w = (st["count"].sum(1) - c0).cpu().numpy()[live]
        chunks.append({"rows": [i0, i1], "work": q(w), "max_over_mean": float(w.max() / max(w.mean(), 1e-9))})
    out["chunks_first_last"] = [chunks[0], chunks[len(chunks) // 2], chunks[-1]]
    out["max_over_mean_all_chunks"] = [round(c["max_over_mean"], 1) for c in chunks]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
