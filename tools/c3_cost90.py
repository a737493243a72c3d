"""Per-ray 90-day cost of the whole C3 set (GPU), to pick the 90-day parity sample.

Runs the full C3 set (BASELINE configs[2]: 2.40 M slots) for 90 days on the
GPU and writes each slot's accepted and rejected attempt counts to
``<out>/c3_cost90_<bg>.npz``.  The GPU's counts are the oracle's (the kernel
is bit-identical to the reference's arithmetic), so the sample chosen from
them (tools/make_c3_ref90.py) is the heaviest rays of the reference's own
90-day run; the expected rows themselves come from the CPU oracle.

    python tools/c3_cost90.py [--bg zonal nonzonal] [--out gpurun_out]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg", nargs="+", default=["zonal", "nonzonal"])
    ap.add_argument("--days", type=float, default=90.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    a = ap.parse_args()
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    os.makedirs(a.out, exist_ok=True)
    nt = int(round(a.days * 12)) + 1
    for kind in a.bg:
        t0 = time.time()
        bs, _ = make_bs(kind)
        eng = RayEngine.from_bs(bs)
        src, zcs = c3_sources(eng)
        y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
        res = eng.integrate(y0, nt, 7200.0, chunk=120, first_chunk=[6, 24])
        torch.cuda.synchronize()
        nacc = res.nacc.cpu().numpy().astype(np.int32)
        nrej = res.nrej.cpu().numpy().astype(np.int32)
        np.savez_compressed(os.path.join(a.out, f"c3_cost90_{kind}.npz"), nacc=nacc, nrej=nrej,
                            nt=np.int64(nt), nslot=np.int64(y0.shape[1]))
        att = nacc.astype(np.int64) + nrej
        print(f"{kind}: {y0.shape[1]} slots, {int(nacc.sum())} accepted, max attempts {int(att.max())} "
              f"(slot {int(att.argmax())}), {time.time() - t0:.1f} s", flush=True)
        del eng, res, y0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
