"""Generate tests/golden/c3_ref90_<bg>.npz: the reference's 90-day histories of a
C3 sample (BASELINE configs[2]) computed by the oracle (CPU, NumPy: the
reference's arithmetic -- the oracle is pinned bit-exact to the reference by
tests/test_oracle_golden.py).

The sample: the ``--heavy`` rays with the most DP5(4) attempts over 90 days
(the rays whose thousands of accept/reject decisions are where any arithmetic
difference would surface, and which set the makespan), plus ``--strata``
cost quantiles of the other live rays, ``--per`` random rays each (seed 0).
Per-ray 90-day costs come from tools/c3_cost90.py (one GPU run of the whole
set; its counts are the oracle's -- the kernel is bit-identical -- and they
only choose WHICH rays are checked: the expected rows are the oracle's).

Each fixture holds the slot indices (bench.c3_initial_state's order), per
output row the sha256 of the 7 history variables of the sample (``(7, n)``
fp64, NaN canonicalised; tests/golden/make_devmath.row_hashes), the last row
in full, per-ray accepted and rejected attempt counts, and the 90-day costs
used for the pick; and the same rows of the reference's default integrator,
fixed-step RK4 (wr.py:702-765), on the same rays (``rk4_row_sha``,
``rk4_last``).

    python tools/make_c3_ref90.py --costs profiles/r3/c3_cost90 [--bg zonal nonzonal]
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd"),
                os.path.join(ROOT, "tests", "golden")]

NT = 1081          # 90 days at 2 h (main_wr.py:15-16)
TSTEP = 7200.0


def _run(args):
    bg, y0, row0 = args
    import rwrt_oracle as O
    ob = O.Background(**bg)
    with np.errstate(all="ignore"):
        hist, nacc, nrej, st = O.ray_run(ob, y0, NT, TSTEP, row0=row0)
        hist4, st4 = O.ray_run_rk4(ob, y0.copy(), NT, TSTEP, row0=row0)
    assert st == 0 and st4 == 0
    return hist, nacc, nrej, hist4


def pick(cost, heavy, strata, per, seed=0):
    """``heavy`` costliest live slots + ``per`` random slots from each of
    ``strata`` cost quantiles of the other live slots (sorted slot indices)."""
    live = np.where(cost > 0)[0]
    order = live[np.argsort(-cost[live], kind="stable")]
    top, rest = order[:heavy], order[heavy:]
    rng = np.random.default_rng(seed)
    picks = [top] + [rng.choice(s, size=min(per, len(s)), replace=False)
                     for s in np.array_split(rest, strata)]
    return np.sort(np.concatenate(picks))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--costs", default=os.path.join(ROOT, "profiles", "r3", "c3_cost90"))
    ap.add_argument("--bg", nargs="+", default=["zonal", "nonzonal"])
    ap.add_argument("--heavy", type=int, default=512)
    ap.add_argument("--strata", type=int, default=32)
    ap.add_argument("--per", type=int, default=48)
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    from bench import c3_initial_state, make_bs
    from make_devmath import row_hashes
    for kind in a.bg:
        z = np.load(os.path.join(a.costs, f"c3_cost90_{kind}.npz"))
        cost = z["nacc"].astype(np.int64) + z["nrej"]
        bs, bg = make_bs(kind)
        rows0 = c3_initial_rows(bs)
        assert rows0.shape[1] == cost.size
        idx = pick(cost, a.heavy, a.strata, a.per)
        # heavy rays dealt over the processes (each process's makespan is its heaviest ray)
        parts = [idx[k::a.procs] for k in range(a.procs)]
        jobs = [(bg, rows0[:5, p].copy(), rows0[:, p].copy()) for p in parts]
        t0 = time.time()
        with mp.get_context("spawn").Pool(a.procs) as pool:
            res = pool.map(_run, jobs)
        hist = np.empty((7, NT, idx.size))
        hist4 = np.empty((7, NT, idx.size))
        nacc = np.empty(idx.size, np.int64)
        nrej = np.empty(idx.size, np.int64)
        for k, (h, na, nr, h4) in enumerate(res):
            sel = np.arange(k, idx.size, a.procs)
            hist[:, :, sel], nacc[sel], nrej[sel], hist4[:, :, sel] = h, na, nr, h4
        assert np.array_equal(nacc + nrej, cost[idx]), "GPU cost survey disagrees with the oracle"
        out = os.path.join(ROOT, "tests", "golden", f"c3_ref90_{kind}.npz")
        np.savez_compressed(out, idx=idx.astype(np.int64), nt=np.int64(NT), nslot=np.int64(cost.size),
                            row_sha=row_hashes(hist), last=hist[:, -1], nacc=nacc, nrej=nrej,
                            cost90=cost[idx].astype(np.int32), heavy=np.int64(a.heavy),
                            rk4_row_sha=row_hashes(hist4), rk4_last=hist4[:, -1])
        print(f"{kind}: {idx.size} rays ({a.heavy} heaviest: {int(cost[idx].max())} attempts max), "
              f"{int(nacc.sum())} accepted steps, alive at 90 d: {int((~np.isnan(hist[0, -1])).sum())}, "
              f"{time.time() - t0:.0f} s -> {os.path.relpath(out, ROOT)}", flush=True)


def c3_initial_rows(bs):
    """The 7 initial rows (lon lat k l amp ug vg) of every C3 slot, all periods."""
    from bench import c3_rows
    return c3_rows(bs)


if __name__ == "__main__":
    main()
