"""VALU wave-instructions of the pieces of an attempt (run under rocprofv3 --pmc).

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace \\
        -d <dir> -o run --output-format csv -- python tools/valu_parts.py
    python tools/valu_parts.py --summarize <dir>

Launches, on C3-like inputs (the live C3 initial states, tiled), the device
kernels that evaluate one piece each: the RHS's sin/cos/tan of the latitude
(math_kernel kind 30), SVML pow (kind 33), the shared-reciprocal division
(kind 34), one RHS (rhs_kernel: plain gathers, no LDS cache), one DP5(4)
attempt (attempt_kernel: six RHS + stage sums + error norm).  Per kernel:
instructions per wave = counter / SQ_WAVES (each wave evaluates 64 points),
so the table reads as instructions per evaluation of a wave.
"""
import csv
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]
N = 1 << 22


def run():
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine, selftest_math
    bs, _ = make_bs("zonal")
    eng = RayEngine.from_bs(bs)
    src, zcs = c3_sources(eng)
    y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
    y0 = y0[:, ~torch.isnan(y0.sum(0))]
    y = y0.repeat(1, -(-N // y0.shape[1]))[:, :N].contiguous()
    lat = y[1].cpu().numpy()
    rng = np.random.default_rng(0)
    for _ in range(2):
        selftest_math("k_sin", lat)
        selftest_math("k_pow", rng.uniform(1e-3, 2.0, N), np.full(N, -0.2))
        selftest_math("qdiv", rng.standard_normal(N), rng.uniform(0.1, 1.0, N))
        f = eng.rhs(y)
        eng.attempt(y, f, torch.full((N,), 600.0, dtype=torch.float64, device=y.device))
    torch.cuda.synchronize()


def summarize(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for fn in files:
        for r in csv.DictReader(open(fn)):
            k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", "").strip()[:40])
            e = per.setdefault(k, {})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the pieces in launch order (math kinds 30, 33, 34; rhs; attempt), the second round
    for (i, k), e in sorted(per.items()):
        w = e.get("SQ_WAVES", 0.0)
        if w < 1000:
            continue
        print(f"{i:4d} {k:40s} " + "  ".join(f"{c[8:]}/wave {e[c] / w:8.1f}" for c in sorted(e) if c != "SQ_WAVES"))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarize":
        summarize(sys.argv[2])
    else:
        run()
