"""Generate tests/golden/c5_ref10_<storage>.npz: 10-day histories of a C5 sample
(BASELINE configs[4]: 0.25-degree time-varying background, 1-degree global
seeds x k = 1..10 x the 5 C3 periods = 9.67 M slots) computed by the oracle's
TimeVaryingBackground (CPU, NumPy) for fp64 and fp32 level storage.

The reference has no time-varying mode (its ``fun`` ignores t, wr.py:784-789),
so the oracle's restatement of the extension is the check; its building
blocks are the reference's (per-level ``BS.ready``, bilinear ``_cell``,
Mercator, RHS, DP5(4) stepper), pinned by tests/test_oracle_golden.py.  10
days at 2 h cross 41 six-hourly levels (40 level pairs).

The sample: ``--rays`` random live slots (seed 3) of the whole 5-period set.
Each fixture holds the slot indices, per output row the sha256 of the 7
history variables (NaN canonicalised; make_devmath.row_hashes), the last row,
and per-ray accepted / rejected attempt counts.

    python tools/make_c5_ref.py [--days 10] [--rays 4096]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd"),
                os.path.join(ROOT, "tests", "golden")]

TSTEP, DT = 7200.0, 6 * 3600.0


def c5_rows(ob0):
    """Initial rows [7, nslot] of every C5 slot (5 periods) on the t = 0 level."""
    import rwrt_oracle as O
    import synthetic as S
    cfg = S.config("C5")
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    out = []
    for P in S.C3_PERIODS_DAYS:
        with np.errstate(all="ignore"):
            rows = O.ray_initial(ob0, slon, slat, np.asarray(cfg.zwn), S.c3_freq(P))
        out.append(np.array(rows).reshape(7, -1))
    return np.concatenate(out, axis=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--days", type=float, default=10.0)
    ap.add_argument("--rays", type=int, default=4096)
    a = ap.parse_args()
    import rwrt_oracle as O
    import synthetic as S
    from make_devmath import row_hashes
    nt = int(round(a.days * 12)) + 1
    nlev = int(np.ceil((nt - 1) * TSTEP / DT)) + 1
    t0 = time.time()
    levels = []
    for j in range(nlev):
        b = S.background_level(j, res=0.25)
        levels.append(O.Background(**b))
    print(f"{nlev} levels built, {time.time() - t0:.0f} s", flush=True)
    rows0 = c5_rows(levels[0])
    live = np.where(~np.isnan(rows0[:5].mean(axis=0)))[0]
    idx = np.sort(np.random.default_rng(3).choice(live, size=a.rays, replace=False))
    print(f"{rows0.shape[1]} slots, {live.size} live, {time.time() - t0:.0f} s", flush=True)
    for fp32 in (False, True):
        ob = O.TimeVaryingBackground(levels, 0.0, DT, fp32=fp32)
        t1 = time.time()
        with np.errstate(all="ignore"):
            hist, nacc, nrej, st = O.ray_run(ob, rows0[:5, idx].copy(), nt, TSTEP,
                                             ttotal=(nt - 1) * TSTEP, row0=rows0[:, idx])
        assert st == 0
        name = "fp32" if fp32 else "fp64"
        out = os.path.join(ROOT, "tests", "golden", f"c5_ref10_{name}.npz")
        np.savez_compressed(out, idx=idx.astype(np.int64), nt=np.int64(nt), nlev=np.int64(nlev),
                            nslot=np.int64(rows0.shape[1]), row_sha=row_hashes(hist), last=hist[:, -1],
                            nacc=nacc, nrej=nrej, first=hist[:, 1])
        moved = np.nanmax(np.abs(hist[0, -1] - hist[0, 0]))
        print(f"{name}: {idx.size} rays, {int(nacc.sum())} accepted steps, alive at {a.days:g} d: "
              f"{int((~np.isnan(hist[0, -1])).sum())}, max |dlon| {moved:.2f} rad, {time.time() - t1:.0f} s "
              f"-> {os.path.relpath(out, ROOT)}", flush=True)
        del ob


if __name__ == "__main__":
    main()
