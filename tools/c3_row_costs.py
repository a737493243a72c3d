"""Per-ray cost profile of the C3 bench schedule (GPU): accepted steps per ray at
every ``--every``-th row of every launch, to study how well one launch's
per-ray work predicts the next (the work-queue order of rk45_run_kernel).

Runs the bench's path (shard.run_sharded on one GPU: probe, 24- and
160-row re-ordering launches, the rest) and writes
``<out>/c3_rowcost_<bg>.npz``: ``rows`` (row indices sampled), ``nacc``
``[nslot, len(rows)]`` int32 (running accepted steps, the rows' 8th column),
``att`` ``[nslot]`` final accepted + rejected attempts, and the launch bounds.

    python tools/c3_row_costs.py [--bg nonzonal zonal] [--every 10]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg", nargs="+", default=["nonzonal", "zonal"])
    ap.add_argument("--every", type=int, default=10)
    ap.add_argument("--out", default="/tmp/rwrt_rowcost")
    ap.add_argument("--features", default=None, help="directory for the compact per-live-ray feature file")
    ap.add_argument("--compact", default=None,
                    help="directory for c3_rowsub_<bg>.npz: a random 1/--sub of the live rays, "
                         "running accepted steps as int16 (small enough for gpurun_out/)")
    ap.add_argument("--sub", type=int, default=8)
    ap.add_argument("--skip-full", action="store_true", help="only the --compact file")
    a = ap.parse_args()
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    from shard import run_sharded
    os.makedirs(a.out, exist_ok=True)
    nt = 1081
    for kind in a.bg:
        bs, _ = make_bs(kind)
        eng = RayEngine.from_bs(bs)
        src, zcs = c3_sources(eng)
        y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
        cols, rows, ends = [], [], {}

        def sink(i0, i1, o, idx):
            take = [r for r in range(i0, i1) if r % a.every == 0 or r == i1 - 1]
            cols.append(o[:, [r - i0 for r in take], 7].to(torch.int32).cpu())
            rows.extend(take)
            ends[i1 - 1] = o[:, -1, :7].to(torch.float32).cpu()   # the launch's last row

        r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=6, lead=[24, 160], chunk=nt - 1,
                        sink=sink, ttotal=(nt - 1) * 7200.0, team="auto")
        nacc = torch.cat(cols, dim=1).numpy()
        att = r.counts.sum(1).to(torch.int32).cpu().numpy()
        bounds = np.array([[1, 7]] + [list(b) for b in r.res.bounds])
        if not a.skip_full:
            np.savez_compressed(os.path.join(a.out, f"c3_rowcost_{kind}.npz"), rows=np.array(rows), nacc=nacc,
                                att=att, bounds=bounds)
        if a.compact:
            os.makedirs(a.compact, exist_ok=True)
            live = np.nonzero(att > 0)[0]
            sub = np.sort(np.random.default_rng(1).choice(live, size=len(live) // a.sub, replace=False))
            np.savez_compressed(os.path.join(a.compact, f"c3_rowsub_{kind}.npz"), rows=np.array(rows),
                                nacc=np.minimum(nacc[sub], 32767).astype(np.int16), att=att[sub],
                                slot=sub.astype(np.int32), n_live=len(live), sub=a.sub, bounds=bounds)
        if a.features:
            # a compact per-live-ray feature set for studying cost predictors
            live = np.nonzero(att > 0)[0]
            live = np.sort(np.random.default_rng(0).choice(live, size=min(len(live), 250000), replace=False))
            feat = {f"row{r}": ends[r].numpy()[live][:, :4] for r in sorted(ends) if r < nt - 1}
            np.savez_compressed(os.path.join(a.features, f"c3_features_{kind}.npz"), slot=live.astype(np.int32),
                                att=att[live], rows=np.array(rows),
                                nacc=nacc[live][:, [k for k, r in enumerate(rows) if r % 90 == 0 or r in ends]],
                                nacc_rows=np.array([r for r in rows if r % 90 == 0 or r in ends]), **feat)
        print(kind, nacc.shape, int(att.sum()), flush=True)
        del eng, r, y0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
