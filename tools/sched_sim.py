"""Work-queue order vs makespan of the C3 ray loop's last launch (CPU model).

    python tools/sched_sim.py gpurun_out/rowcost/c3_rowcost_nonzonal.npz

rk45_run_kernel's lanes pull rays from a queue in the host's order and each
integrates its ray to the end of the launch, so a launch is list scheduling
on 65 536 lanes (1 024 one-wave SIMDs x 64; a wave iterates while any of its
lanes has work, and a lane refills at once).  Given every ray's actual work
in the launch (accepted steps from the rows' running count:
tools/c3_row_costs.py), this compares the makespan of several queue orders
with the throughput bound (total work / lanes) and the serial bound (the
heaviest ray): how much of the launch is lost to the order.
"""
import heapq
import sys

import numpy as np

LANES = 65536


def makespan(work, order, lanes=LANES):
    """Greedy list scheduling: rays in ``order`` to the earliest-free lane."""
    free = [0.0] * lanes
    heapq.heapify(free)
    end = 0.0
    for i in order:
        w = float(work[i])
        if w <= 0:
            continue
        t = heapq.heappop(free) + w
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def main():
    z = np.load(sys.argv[1])
    rows, nacc = z["rows"], z["nacc"].astype(np.int64)
    bounds = z["bounds"]
    col = {int(r): k for k, r in enumerate(rows)}

    def at(r):
        return nacc[:, col[int(r)]]

    last = bounds[-1]
    prev = bounds[-2]
    w_last = at(last[1] - 1) - at(last[0] - 1)           # work of the last launch
    w_prev = at(prev[1] - 1) - at(prev[0] - 1)           # of the one before (the queue key)
    w_sofar = at(prev[1] - 1)                            # everything before the last launch
    live = w_last > 0
    tot = w_last.sum()
    lb = max(tot / LANES, w_last.max())
    print(f"last launch rows {list(last)}: {int(live.sum())} rays working, total {tot}, "
          f"max ray {w_last.max()}, throughput bound {tot / LANES:.0f}")
    orders = {
        "previous launch's work (bench)": np.argsort(-w_prev, kind="stable"),
        "work so far / rows so far": np.argsort(-(w_sofar / (prev[1] - 1)), kind="stable"),
        "oracle: actual work": np.argsort(-w_last, kind="stable"),
        "random": np.random.default_rng(0).permutation(len(w_last)),
    }
    for name, o in orders.items():
        m = makespan(w_last, o)
        print(f"  {name:34s} makespan {m:8.0f}  = {m / lb:.3f} x bound")
    # how good is the predictor: rank correlation of predicted vs actual among working rays
    from scipy.stats import spearmanr
    print("  spearman(prev launch, last launch) =", float(spearmanr(w_prev[live], w_last[live])[0]))


if __name__ == "__main__":
    main()
