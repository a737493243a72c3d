"""When every ray of a C3 launch runs (rwrt_ctx_set_trace on all queue positions).

    python tools/tail_trace.py [--bg nonzonal zonal] [--team N] [--out DIR]

Runs the bench's C3 schedule on one GPU (probe, the 24- and 160-row launches,
the adaptive split, the rest) and traces every queue position of the LAST
launch: ray, start and end (s_memrealtime, 100 MHz), attempts.  Prints the
launch times, how many rays are still running at each tenth of the last
launch, and the rays that end last (their queue position, attempts, and the
attempts the order predicted them by); writes DIR/tail_<bg>.npz (position,
start, end in microseconds from the launch's first start, attempts, predicted
attempts).  (The scheduling-phase runs of round 3 used the reverted
rwrt_rk45_run_budget: profiles/r3/phases/.)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg", nargs="+", default=["nonzonal", "zonal"])
    ap.add_argument("--team", type=int, default=0)
    ap.add_argument("--split", default="auto")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    from shard import run_sharded
    nt = 1081
    for kind in a.bg:
        bs, _ = make_bs(kind)
        eng = RayEngine.from_bs(bs)
        src, zcs = c3_sources(eng)
        y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
        nray = y0.shape[1]
        trace = torch.zeros((nray, 10), dtype=torch.int64, device=eng.device)
        launches = []
        saved = torch.zeros_like(trace)

        def sink(i0, i1, rows, idx):
            # stream-ordered after launch [i0, i1): keep its trace, clear for the next
            launches.append((int(i0), int(i1)))
            saved.copy_(trace)
            trace.zero_()
        ev = []
        eng.ctx.set_trace(trace)
        r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=6, lead=[24, 160], chunk=nt - 1,
                        sink=sink, events=ev, ttotal=(nt - 1) * 7200.0, team=a.team, split=a.split)
        torch.cuda.synchronize()
        eng.ctx.set_trace(None)
        trace = saved
        launch_s = [x.elapsed_time(y) / 1e3 for x, y in ev]
        tr = trace.cpu().numpy()
        ok = (tr[:, 5] > 0) & (tr[:, 4] > 0)
        pos = np.nonzero(ok)[0]
        t0 = tr[ok, 3].astype(np.float64)
        t1 = tr[ok, 4].astype(np.float64)
        base = t0.min()
        t0 = (t0 - base) / 100.0   # us
        t1 = (t1 - base) / 100.0
        att = tr[ok, 5]
        T = t1.max()
        prof = [int(((t0 <= f * T) & (t1 > f * T)).sum()) for f in np.linspace(0, 1, 11)[:-1]]
        last = np.argsort(-t1)[:20]
        info = {"bg": kind, "team": a.team, "launches": launches, "launch_s": launch_s,
                "step_s": sum(launch_s), "traced": int(ok.sum()), "last_launch_us": float(T),
                "rays_running_at_tenths": prof,
                "median_end_us": float(np.median(t1)), "p99_end_us": float(np.percentile(t1, 99)),
                "ends_last": [{"pos": int(pos[i]), "start_us": round(float(t0[i])), "end_us": round(float(t1[i])),
                               "attempts": int(att[i]), "us_per_attempt": round(float((t1[i] - t0[i]) / att[i]), 2)}
                              for i in last[:10]]}
        print(json.dumps(info), flush=True)
        if a.out:
            os.makedirs(a.out, exist_ok=True)
            np.savez_compressed(os.path.join(a.out, f"tail_{kind}_t{a.team}.npz"), pos=pos.astype(np.int32),
                                t0=t0.astype(np.float32), t1=t1.astype(np.float32), att=att.astype(np.int32),
                                launch_s=np.array(launch_s))
        del eng, r, y0, trace
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
