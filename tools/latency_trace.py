"""Where and how long the heaviest C3 rays run (rwrt_ctx_set_trace, diagnostic).

    python tools/latency_trace.py [--cases full:0,full:64,alone:16:16,alone:16:1] [--out f.json]

Cases:
  full:T          the whole zonal C3 set, bench schedule (probe, 24, 160, rest),
                  T rays per launch in latency mode (16 per wave): the last
                  launch's traced rays (its heaviest 256 queue positions)
  alone:K:Q       the K heaviest rays alone, one launch over 90 days, all in
                  latency mode at Q rays per wave (16-256
                  rays at one per wave took 0.51-0.56 s, one ray 0.21 s)
For each case: the launch time (HIP events), per traced ray its attempts,
duration (s_memrealtime, 100 MHz), us per attempt, and hardware placement
(XCC, SE, CU, SIMD, wave slot from HW_REG_HW_ID) -- summarised: how many
traced rays share an XCC / CU / SIMD, and the slowest rays.
"""
import argparse
import json
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def decode(tr, n):
    """Trace rows -> list of dicts (HW_ID fields per the gfx9 layout)."""
    out = []
    for w in range(n):
        ray, hw, xcc, t0, t1, att, lat, blk, c0, c1 = (int(x) for x in tr[w])
        if att <= 0 or t1 <= 0:
            continue
        out.append({"pos": w, "ray": ray, "xcc": xcc & 0xF, "se": (hw >> 13) & 7, "cu": (hw >> 8) & 0xF,
                    "sh": (hw >> 12) & 1, "simd": (hw >> 4) & 3, "wave": hw & 0xF, "block": blk,
                    "latency_mode": bool(lat), "attempts": att, "t0": t0, "t1": t1,
                    "s": (t1 - t0) / 1e8, "us_per_attempt": 1e6 * (t1 - t0) / 1e8 / att,
                    "clock_GHz": (c1 - c0) / ((t1 - t0) / 1e8) / 1e9 if t1 > t0 else None,
                    "kcycles_per_attempt": (c1 - c0) / att / 1e3})
    return out


def summary(rays):
    if not rays:
        return {}
    s = sorted(rays, key=lambda r: -r["s"])
    cu = Counter((r["xcc"], r["se"], r["sh"], r["cu"]) for r in rays)
    simd = Counter((r["xcc"], r["se"], r["sh"], r["cu"], r["simd"]) for r in rays)
    return {"traced": len(rays), "slowest": s[:5],
            "max_s": s[0]["s"], "median_us_per_attempt": float(np.median([r["us_per_attempt"] for r in rays])),
            "xccs": dict(Counter(r["xcc"] for r in rays)), "max_rays_per_cu": max(cu.values()),
            "clock_GHz_by_xcc": {x: float(np.median([r["clock_GHz"] for r in rays if r["xcc"] == x]))
                                 for x in sorted({r["xcc"] for r in rays})},
            "us_per_attempt_by_xcc": {x: float(np.median([r["us_per_attempt"] for r in rays if r["xcc"] == x]))
                                      for x in sorted({r["xcc"] for r in rays})},
            "kcycles_per_attempt_median": float(np.median([r["kcycles_per_attempt"] for r in rays])),
            "max_rays_per_simd": max(simd.values()), "cus": len(cu)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="full:0,full:64,alone:16:16,alone:16:1,alone:1:1")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    from shard import run_sharded
    nt = 1081
    bs, _ = make_bs("zonal")
    eng = RayEngine.from_bs(bs)
    src, zcs = c3_sources(eng)
    y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
    cap = 256
    trace = torch.zeros((cap, 10), dtype=torch.int64, device=eng.device)
    res = {}
    work = None
    for case in a.cases.split(","):
        kind, *par = case.split(":")
        trace.zero_()
        eng.ctx.set_trace(trace)
        ev = []
        if kind == "full":
            r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=6, lead=[24, 160], chunk=nt - 1,
                            events=ev, ttotal=(nt - 1) * 7200.0, team=int(par[0]))
            torch.cuda.synchronize()
            work = r.counts.sum(1)
            launch_s = [x.elapsed_time(y) / 1e3 for x, y in ev]
        else:
            k, q = int(par[0]), int(par[1])
            if work is None:
                r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=6, lead=[24, 160], chunk=nt - 1)
                work = r.counts.sum(1)
            idx = torch.sort(work, descending=True, stable=True).indices[:k]
            yk = y0[:, idx].contiguous()
            trace.zero_()
            r = eng.integrate(yk, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=nt - 1, team=(k, q), events=ev)
            torch.cuda.synchronize()
            launch_s = [x.elapsed_time(y) / 1e3 for x, y in ev]
        rays = decode(trace.cpu().numpy(), cap)
        res[case] = {"launch_s": launch_s, **summary(rays)}
        print(json.dumps({"case": case, "launch_s": launch_s, **{k2: v for k2, v in summary(rays).items()
                                                                if k2 != "slowest"}}), flush=True)
        print("  slowest:", json.dumps(res[case].get("slowest", [])[:3]), flush=True)
    eng.ctx.set_trace(None)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
