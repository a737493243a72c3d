"""C4 on one MI355X: every rank's shard of the cost-balanced split, timed alone.

    python tools/c4_rehearsal.py [--days 90] [--worlds 1,2,4,8] [--out f.json]
    python tools/c4_rehearsal.py --config C5 --fields fp64|fp32 [...]

``--config C5`` splits BASELINE configs[4] instead (bench.py --config C5: the
0.25-degree time-varying background, 361 levels, 9.67 M slots / 4.03 M live
rays, the cell-ordered queue, rows per launch from
``bench.c5_rows_per_launch``), the way ``bench.py --config C5 --gpus W``
splits it.

For each world size W the C3 set is split exactly as ``bench.py --gpus W``
splits it (shard.run_sharded: probe launch over every ray, snake deal by probe
cost); each rank's integration is then run alone on this GPU (no collectives).
The slowest rank's time is the W-GPU makespan of the ray loop without the
RCCL broadcast and gather (which bench.py times: ~1 MB and ~55 MB).  Also
times the single heaviest ray alone -- the critical path no split can beat.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from engine import RayEngine  # noqa: E402
from shard import run_sharded  # noqa: E402


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best, r


def c5_setup(a, nt):
    """bench.main_c5's engine and initial rays (one GPU, all 361 levels)."""
    import synthetic as S
    from levels import Levels
    res, dt_bg = 0.25, 6 * 3600.0
    nlev = int(np.ceil((nt - 1) * 7200.0 / dt_bg)) + 1
    b0 = S.background_level(0, res=res)
    lv = Levels(b0["lat"], b0["lon"], nlev, t0=0.0, dt=dt_bg, fp32=(a.fields == "fp32"))
    for j in range(nlev):
        bj = b0 if j == 0 else S.background_level(j, res=res)
        lv.set_level(j, bj["u"], bj["v"])
    eng = RayEngine.from_levels(lv)
    cfg = S.config("C5")
    deg2rad = np.pi / 180.0
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
    src = eng.sources(lon, lat)
    y0 = torch.cat([eng.initial_rows_dev(src, eng.zwn_tensor(cfg.zwn, S.c3_freq(P)))[0][:5].reshape(5, -1)
                    for P in S.C3_PERIODS_DAYS], dim=1)
    return eng, y0.contiguous(), bench.c5_rows_per_launch(lv.fp32, 1, nt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--out", default=None)
    ap.add_argument("--bg", default="zonal", choices=["zonal", "nonzonal"])
    ap.add_argument("--team", default="auto", help="latency-mode rays per launch (int or 'auto')")
    ap.add_argument("--lead", default="24,96", help="rows of the re-ordering launches after the probe (bench.py default for N > 1)")
    ap.add_argument("--config", default="C3", choices=["C3", "C5"])
    ap.add_argument("--fields", default="fp64", choices=["fp64", "fp32"], help="C5: level storage")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=0, help="C5: rows per launch (default: bench.c5_rows_per_launch)")
    ap.add_argument("--shard-probe", type=int, default=1, choices=[0, 1],
                    help="each rank probes 1/W of the rays, costs all-gathered (bench.py's default)")
    a = ap.parse_args()
    # 'auto', an int (rays per launch at 16 per wave) or n:q (n rays at q per wave)
    team = a.team if a.team == "auto" else (tuple(int(x) for x in a.team.split(":")) if ":" in a.team
                                             else int(a.team))
    lead = [int(x) for x in a.lead.split(",") if x]
    nt = int(a.days * 12) + 1
    kw = {}
    if a.config == "C5":
        eng, y0, _ = c5_setup(a, nt)
        kw = dict(order_policy="cell", ttotal=(nt - 1) * 7200.0)
        team = 0 if a.team == "auto" else team   # (C5: sparse-wave latency mode only when asked)
    else:
        bs, bg = bench.make_bs(a.bg)
        y0 = torch.as_tensor(bench.c3_initial_state(bs), device="cuda")
        eng = RayEngine.from_bs(bs)
    out = {"config": a.config, "chunk": a.chunk or None, "tv_lanes": getattr(eng, "tv_lanes", None), "days": a.days, "bg": a.bg if a.config == "C3" else "C5 time-varying",
           "fields": a.fields if a.config == "C5" else "fp64", "team": a.team, "lead": a.lead,
           "nslot": int(y0.shape[1]), "live": int((~torch.isnan(y0.sum(0))).sum().item()), "worlds": {}}
    for w in [int(x) for x in a.worlds.split(",")]:
        ranks = []
        kw_w = dict(kw)
        if a.config == "C5":   # bench.py main_c5's rows per launch, capped by the row buffer's memory
            torch.cuda.empty_cache()
            n_local = -(-out["live"] // w) + 2   # (row blocks for live rays only, ABI 4)
            cap = max(1, int(0.8 * torch.cuda.mem_get_info()[0]) // (n_local * 64))
            kw_w["chunk"] = min(a.chunk or bench.c5_rows_per_launch(a.fields == "fp32", w, nt), cap)
        if w > 1 and a.shard_probe:   # every share's probe, untimed (the all-gather's result)
            from engine import t_eval_of
            from shard import probe_costs
            p = eng.params(nt, 7200.0)
            st0 = eng.init(y0, p)
            tb = torch.as_tensor(t_eval_of(nt, 7200.0, kw.get("ttotal")), dtype=torch.float64, device=eng.device)
            kw_w["costs"] = probe_costs(eng, st0, p, tb, 6, 0, w)
            del st0
        for r in range(w):
            torch.cuda.empty_cache()   # (row buffers of another size cached by the allocator)
            dt, res = timed(lambda: run_sharded(eng, y0, nt, rank=r, world=w, gather=False,
                                                       team=team, lead=lead, **kw_w), reps=a.reps)
            ev = []
            del res
            torch.cuda.empty_cache()
            eng.keep_launch_work = True
            res = run_sharded(eng, y0, nt, rank=r, world=w, gather=False, team=team, lead=lead, events=ev, **kw_w)
            torch.cuda.synchronize()
            eng.keep_launch_work = False
            # the last launch's heaviest rays: attempts there, and whether the
            # latency set (chosen from the previous launch's work) held them
            lw, lset = eng.launch_work[-1]
            top = torch.topk(lw, 8)
            inset = (torch.isin(top.indices, lset).tolist() if lset is not None else [False] * 8)
            last_top = [[int(a_), bool(b_)] for a_, b_ in zip(top.values.tolist(), inset)]
            launches = [dict(d, ms=a_.elapsed_time(b_)) for d, (a_, b_) in
                        zip([{"rows": [1, 1 + 6], "n_heavy": 0, "per_wave": 16,
                                               "probe": "share + own shard" if "costs" in kw_w else "every ray"}]
                                             + list(eng.launch_log), ev)]
            att = (res.res.nacc + res.res.nrej)
            ranks.append({"rank": r, "s": dt, "rays": int(res.idx.numel()), "ray_steps": res.steps_local,
                          "max_attempts": int(att.max().item()),
                          "top_attempts": [int(x) for x in torch.topk(att, min(8, att.numel())).values.tolist()],
                          "last_launch_top": last_top,
                          "launches": launches})
        steps = sum(x["ray_steps"] for x in ranks)
        mk = max(x["s"] for x in ranks)
        out["worlds"][str(w)] = {"makespan_s": mk, "rate": steps / mk, "ray_steps": steps,
                                 "rows_per_launch": kw_w.get("chunk"), "ranks": ranks,
                                 "shard_probe": bool(w > 1 and a.shard_probe)}
        print(json.dumps({"world": w, "makespan_s": mk, "rate": steps / mk}), flush=True)
    one1 = out["worlds"].get("1")
    if one1:
        for k, v in out["worlds"].items():
            v["speedup_vs_1"] = one1["makespan_s"] / v["makespan_s"]
            v["makespan_frac_of_1"] = v["makespan_s"] / one1["makespan_s"]
    # the heaviest ray alone (its attempts from the 1-rank run), and the
    # heaviest few as one set (C5: its own chunked launches)
    kw_1 = dict(kw)
    if a.config == "C5":   # (capped by the row buffer's memory, as bench.py main_c5 caps it)
        torch.cuda.empty_cache()
        cap = max(1, int(0.8 * torch.cuda.mem_get_info()[0]) // ((out["live"] + 2) * 64))
        kw_1["chunk"] = min(a.chunk or bench.c5_rows_per_launch(a.fields == "fp32", 1, nt), cap)
    full = run_sharded(eng, y0, nt, rank=0, world=1, gather=False, **kw_1)
    work = (full.res.nacc + full.res.nrej)
    ikw = dict(ttotal=(nt - 1) * 7200.0)
    if a.config == "C5":
        ikw.update(order_policy="cell", chunk=kw_1["chunk"], team=team, first_chunk=lead)
    for n in ([1, 8, 64] if a.config == "C5" else [1]):
        top = torch.topk(work, n).indices
        rays = y0[:, full.idx[top]].contiguous()
        dt, r1 = timed(lambda: eng.integrate(rays, nt, 7200.0, **ikw))
        att = (r1.nacc + r1.nrej)
        key = "heaviest_ray" if n == 1 else f"heaviest_{n}"
        out[key] = {"slot": int(full.idx[top[0]].item()), "attempts": int(att.max().item()), "s": dt,
                    "us_per_attempt": 1e6 * dt / max(int(att.max().item()), 1)}
        print(json.dumps({key: out[key]}), flush=True)
    if a.config == "C5":
        js = json.dumps(out)
        print(js)
        if a.out:
            open(a.out, "w").write(js + "\n")
        return
    w = work[work > 0].double()
    q = torch.tensor([0.5, 0.9, 0.99, 0.999, 0.9999], dtype=torch.float64, device=w.device)
    out["attempts_per_live_ray"] = {"mean": float(w.mean()), "max": int(w.max()),
                                    "quantiles": dict(zip(["p50", "p90", "p99", "p999", "p9999"],
                                                          [float(x) for x in torch.quantile(w, q)]))}
    js = json.dumps(out)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
