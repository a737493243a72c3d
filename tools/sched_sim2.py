"""In-launch scheduling policies for the C3 ray loop (CPU model).

    python tools/sched_sim2.py gpurun_out/r3i/c3_rowsub_nonzonal.npz [--slices 10,20,40]

Input: tools/c3_row_costs.py --compact (a random 1/sub of the live rays, the
running accepted steps every 10th row).  A ray's work in rows [r0, r1) is its
accepted steps there scaled by its attempts / accepted steps; lanes are
independent (65 536 / sub of them) and a ray pulled from a queue costs
``--pull`` attempts of overhead (state load, cold cell cache).

Policies (rows after the probe launch):
  launches   the bench's schedule: one launch per `bounds` row range, each a
             greedy list in the order of the previous launch's work (longest
             first), a barrier between launches
  sliced     one launch over rows [r0, nt): slices of S rows, work items
             (ray, slice) claimed in round order (slice 0 of every ray in the
             static order, then slice 1, ...); an item whose ray has not
             finished the previous slice waits on its lane
  dynamic    idealised: a freed lane takes the ready item with the lowest
             slice index, heaviest previous slice first (upper bound of what
             a device priority queue could do)
Makespans are in attempts per lane, against the throughput bound.
"""
import argparse
import heapq

import numpy as np


def load(path):
    z = np.load(path)
    rows = z["rows"].astype(np.int64)
    nacc = z["nacc"].astype(np.int64)
    att = z["att"].astype(np.float64)
    scale = att / np.maximum(nacc[:, -1], 1)
    return rows, nacc, scale, z["bounds"], int(z["sub"])


def work_fn(rows, nacc, scale):
    col = {int(r): k for k, r in enumerate(rows)}
    sampled = np.array(sorted(col))

    def at(r):  # running accepted steps after row r (nearest sampled row <= r)
        if r < sampled[0]:
            return np.zeros(nacc.shape[0])
        k = sampled[np.searchsorted(sampled, r, side="right") - 1]
        return nacc[:, col[int(k)]].astype(np.float64)

    def work(r0, r1):  # rows [r0, r1)
        return (at(r1 - 1) - at(r0 - 1)) * scale
    return work


def list_schedule(w, order, lanes, t0=0.0, pull=0.0):
    free = [t0] * lanes
    end = t0
    for i in order:
        if w[i] <= 0:
            continue
        t = heapq.heappop(free) + w[i] + pull
        end = max(end, t)
        heapq.heappush(free, t)
    return end


def launches(work, bounds, lanes, pull):
    t = 0.0
    prev = None
    for r0, r1 in bounds[1:]:
        w = work(r0, r1)
        order = np.argsort(-prev, kind="stable") if prev is not None else np.arange(len(w))
        t = list_schedule(w, order, lanes, t, pull)
        prev = w
    return t


def slice_bounds(r0, nt, S):
    b = list(range(r0, nt, S)) + [nt]
    return list(zip(b[:-1], b[1:]))


def sliced(work, r0, nt, S, order, lanes, pull, t0=0.0):
    sb = slice_bounds(r0, nt, S)
    W = np.stack([work(a, b) for a, b in sb])           # [K, nray]
    done = np.full(W.shape[1], t0)
    free = [t0] * lanes
    end = t0
    wait = 0.0
    for k in range(len(sb)):
        wk = W[k]
        for i in order:
            if wk[i] <= 0:
                continue
            f = heapq.heappop(free)
            s = max(f, done[i])
            wait += s - f
            e = s + wk[i] + pull
            done[i] = e
            end = max(end, e)
            heapq.heappush(free, e)
    return end, wait / lanes


def dynamic(work, r0, nt, S, prev0, lanes, pull, t0=0.0):
    sb = slice_bounds(r0, nt, S)
    W = np.stack([work(a, b) for a, b in sb])
    K, n = W.shape
    ready = [(0, -prev0[i], i) for i in range(n)]
    heapq.heapify(ready)
    events = []          # (time, ray, next slice, its previous slice's work)
    free_lanes = lanes
    t = t0
    end = t0
    while ready or events:
        while free_lanes and ready:
            k, _, i = heapq.heappop(ready)
            e = t + W[k, i] + (pull if W[k, i] > 0 else 0.0)
            heapq.heappush(events, (e, i, k + 1, W[k, i]))
            free_lanes -= 1
        e, i, k, wprev = heapq.heappop(events)
        t = e
        end = max(end, e)
        free_lanes += 1
        if k < K:
            heapq.heappush(ready, (k, -wprev, i))
    return end


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--slices", default="10,20,45,90")
    ap.add_argument("--pull", type=float, default=2.0)
    a = ap.parse_args()
    rows, nacc, scale, bounds, sub = load(a.npz)
    lanes = 65536 // sub
    work = work_fn(rows, nacc, scale)
    nt = int(bounds[-1][1])
    total = work(int(bounds[1][0]), nt).sum()
    tb = total / lanes
    print(f"{a.npz}: {nacc.shape[0]} rays (1/{sub}), {lanes} lanes, launches {bounds.tolist()}")
    print(f"throughput bound after the probe: {tb:.0f} attempts/lane; heaviest ray {work(int(bounds[1][0]), nt).max():.0f}")
    m = launches(work, bounds, lanes, a.pull)
    print(f"  launches (bench)                     {m:8.0f} = {m / tb:.3f} x bound")
    probe = work(int(bounds[0][0]), int(bounds[0][1]))
    order_probe = np.argsort(-probe, kind="stable")
    # the bench's leading launches, then one sliced launch for the rest
    r_lead = int(bounds[1][0])
    for S in [int(s) for s in a.slices.split(",")]:
        m, wt = sliced(work, r_lead, nt, S, order_probe, lanes, a.pull)
        print(f"  sliced S={S:3d} from row {r_lead}, probe order {m:8.0f} = {m / tb:.3f} x bound (lane wait {wt:.0f})")
        m = dynamic(work, r_lead, nt, S, probe, lanes, a.pull)
        print(f"  dynamic S={S:3d}                         {m:8.0f} = {m / tb:.3f} x bound")


if __name__ == "__main__":
    main()
