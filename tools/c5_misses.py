"""Cell-cache refills per attempt of the C5 rays (diagnostic build only).

    make -C rossby-wave-ray-tracing_amd/csrc variant NAME=missdiag DEFS=-DRWRT_TV_MISS_DIAG
    RWRT_LIB=rossby-wave-ray-tracing_amd/librwrt_missdiag.so python tools/c5_misses.py [--days 90]

The diagnostic build adds every lane's LDS-cache refills of the fp64
time-varying loop (CachedVaryingBG64::begin: a new cell or level pair) to
trace[ray].  Runs bench.py --config C5's whole set on one GPU and prints the
refills per attempt over all live rays and for the heaviest ones (the rays
whose chains set the multi-GPU makespan)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd"), os.path.join(ROOT, "tools")]
import torch  # noqa: E402
import c4_rehearsal as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=90)
    ap.add_argument("--fields", default="fp64")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    nt = int(a.days * 12) + 1
    eng, y0, chunk = R.c5_setup(a, nt)
    nray = y0.shape[1]
    tr = torch.zeros(nray, dtype=torch.int64, device=eng.device)
    eng.ctx.set_trace(tr)
    r = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, order_policy="cell", chunk=chunk)
    torch.cuda.synchronize()
    eng.ctx.set_trace(None)
    att = (r.nacc + r.nrej).to(torch.float64)
    live = att > 0
    m = tr.to(torch.float64)
    out = {"days": a.days, "live": int(live.sum()), "refills": float(m[live].sum()),
           "attempts": float(att[live].sum()),
           "refills_per_attempt_all": float(m[live].sum() / att[live].sum()), "heaviest": []}
    top = torch.topk(att, 64).indices
    for k, j in enumerate(top.tolist()):
        if k < 16 or k % 8 == 0:
            out["heaviest"].append({"slot": j, "attempts": int(att[j]), "refills": int(m[j]),
                                    "per_attempt": float(m[j] / att[j])})
    js = json.dumps(out)
    print(js)
    if a.out:
        open(a.out, "w").write(js + "\n")


if __name__ == "__main__":
    main()
