"""Generate tests/golden/ref90_C2_*.npz: the reference's 90-day C2 histories,
computed by the oracle with NumPy's own transcendentals (the reference's
arithmetic: the oracle is pinned bit-exact to the reference by
tests/test_oracle_golden.py).

    python tests/golden/make_devmath.py

The GPU must reproduce these histories bit for bit, every row of 90 days
(tests/test_gpu_devmath.py): its sin/cos/tan/pow are NumPy's, restated
(csrc/np_math.h), and every other operation is the reference's in the
reference's order.  The inputs are the reference's own C2 initial rows
(init_C2_<kind>.npz).

Each fixture holds, per output row, the sha256 of the 7 history variables
(``(7, nray)`` fp64, NaN canonicalised), the last row in full and the
per-ray accepted-step counts (RK45).  Runs in a few minutes on one core.
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rossby-wave-ray-tracing_amd")]

import rwrt_oracle as O   # noqa: E402
import synthetic as S     # noqa: E402

NT = 1081          # 90 days at 2 h (main_wr.py:15-16)
TSTEP = 7200.0


def row_hashes(hist):
    """sha256 per output row of ``hist[7, nt, nray]`` (NaN canonicalised)."""
    h = np.array(hist, np.float64, copy=True)
    h[np.isnan(h)] = np.nan
    return np.array([hashlib.sha256(np.ascontiguousarray(h[:, i]).tobytes()).hexdigest()
                     for i in range(h.shape[1])])


def main():
    for kind in ("zonal", "nonzonal"):
        g = np.load(os.path.join(HERE, f"init_C2_{kind}.npz"))
        rows = g["rows"].reshape(7, -1)
        ob = O.Background(**S.background(kind))
        t0 = time.time()
        with np.errstate(all="ignore"):
            hist, nacc, nrej, st = O.ray_run(ob, rows[:5].copy(), NT, TSTEP, row0=rows)
            hist4, st4 = O.ray_run_rk4(ob, rows[:5].copy(), NT, TSTEP, row0=rows)
        assert st == 0 and st4 == 0
        np.savez_compressed(os.path.join(HERE, f"ref90_C2_{kind}.npz"),
                            nt=NT, row_sha=row_hashes(hist), last=hist[:, -1], nacc=nacc,
                            nrej=nrej, rk4_row_sha=row_hashes(hist4), rk4_last=hist4[:, -1])
        print(kind, f"{time.time() - t0:.0f} s", int(nacc.sum()), "accepted steps")


if __name__ == "__main__":
    main()
