"""Sharding rays across GPUs (one process per GPU, torch.distributed over RCCL).

Rays never interact (``test_sharding_is_bitwise_invisible``),
so a ray set splits across ranks with no exchange during integration.  What
crosses ranks is setup and collection only:

* ``broadcast_array`` -- rank 0's basic-state stack (or initial rays) to every
  rank (RCCL broadcast over xGMI; ~1 MB at 2.5 deg, ~91 MB per 0.25 deg level);
* ``broadcast_levels`` -- a time-varying background (C5): rank 0's u, v
  snapshots (read or synthesised there only, as bs.py:202-262 reads a file
  once) broadcast in blocks, every rank building its packed levels on its own
  GPU (rwrt_bs_ready): 8.3 MB per 0.25-degree level instead of 100 MB packed;
* ``shard_indices``   -- a balanced split: live rays and NaN-root slots are
  dealt round-robin separately, so every rank gets the same number of rays
  that actually integrate;
* ``reduce_summary`` / ``reduce_max`` -- the reference's two global couplings
  (solver failure, rkf45.py:423-425; early exit, wr.py:853-855) evaluated over
  all ranks so that a sharded run equals the single-GPU run exactly;
* ``gather_rows``     -- per-chunk trajectory rows back to rank 0;
* ``gather_changed_rows`` -- the same for the drop-in, but only the rays whose
  rows changed (frozen rays repeat their previous row: ~70 % of C3's slots);
* ``cost_partition`` / ``run_sharded`` -- BASELINE configs[3] (C4): ONE ray set
  split over the ranks by measured cost (a short probe launch over every ray,
  then a longest-first snake deal), each rank integrating its shard, the
  endpoints and step counters gathered to rank 0.

Works with the ``nccl`` (RCCL) backend on device tensors and with ``gloo`` on
CPU tensors (tests/test_shard.py).
"""
import time

import numpy as np
import torch
import torch.distributed as dist


# Collectives run for groups of at least COLLECTIVE_MIN_WORLD ranks: 2 (a
# one-rank group needs none).  A test sets 1 to drive a one-rank RCCL group
# through the very branches an N-rank job takes -- RCCL's broadcast,
# all_gather, gather and all_reduce on device tensors -- on a one-GPU box,
# where RCCL refuses two ranks on one device ("Duplicate GPU detected";
# tests/test_gpu_multirank.py::test_rccl_world1_runs_the_collective_paths).
COLLECTIVE_MIN_WORLD = 2


def collective(world):
    """Whether a group of ``world`` ranks exchanges data (see COLLECTIVE_MIN_WORLD)."""
    return world >= COLLECTIVE_MIN_WORLD


def world_info(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _dev(group=None):
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def shard_indices(live, rank, world):
    """Ray indices of ``rank``: live and dead rays dealt round-robin (sorted)."""
    live = np.asarray(live, bool)
    li, di = np.where(live)[0], np.where(~live)[0]
    return np.sort(np.concatenate([li[rank::world], di[rank::world]]))


def broadcast_array(arr, src=0, group=None):
    """Broadcast a float64/int64 numpy array from ``src``; returns it on every rank."""
    rank, world = world_info(group)
    if not collective(world):
        return np.asarray(arr)
    dev = _dev(group)
    if rank == src:
        a = np.ascontiguousarray(arr)
        meta = torch.tensor([a.ndim, 1 if a.dtype == np.int64 else 0] + list(a.shape) +
                            [0] * (8 - a.ndim), dtype=torch.int64, device=dev)
    else:
        meta = torch.zeros(10, dtype=torch.int64, device=dev)
    dist.broadcast(meta, src, group=group)
    ndim, is_int = int(meta[0]), int(meta[1])
    shape = tuple(int(x) for x in meta[2:2 + ndim])
    dtype = torch.int64 if is_int else torch.float64
    if rank == src:
        t = torch.as_tensor(a, device=dev).to(dtype).contiguous()
    else:
        t = torch.empty(shape, dtype=dtype, device=dev)
    dist.broadcast(t, src, group=group)
    return t.cpu().numpy()


def broadcast_levels(lv, make_uv, group=None, src=0, block=16):
    """Fill ``lv`` (a ``levels.Levels``, one per rank) with the same levels on
    every rank: ``make_uv(j) -> (u, v)`` (float32 ``[nlat, nlon]``, file
    layout) is called on rank ``src`` only; the snapshots travel in blocks of
    ``block`` levels (RCCL broadcast of device tensors, or gloo on CPU
    tensors) and each rank builds its packed records with ``rwrt_bs_ready``.
    Returns ``{"levels", "bytes", "seconds", "collectives"}`` (bytes = what the
    broadcasts carried; 0 collectives on one rank)."""
    rank, world = world_info(group)
    dev = _dev(group) if collective(world) else lv.device
    t0 = time.perf_counter()
    nbytes = ncoll = 0
    for j0 in range(0, lv.nlev, block):
        j1 = min(j0 + block, lv.nlev)
        buf = torch.empty((j1 - j0, 2, lv.nlat, lv.nlon), dtype=torch.float32, device=dev)
        if rank == src:
            for j in range(j0, j1):
                u, v = make_uv(j)
                buf[j - j0, 0].copy_(torch.as_tensor(np.ascontiguousarray(u, np.float32)))
                buf[j - j0, 1].copy_(torch.as_tensor(np.ascontiguousarray(v, np.float32)))
        if collective(world):
            dist.broadcast(buf, src, group=group)
            nbytes += buf.numel() * buf.element_size()
            ncoll += 1
        for j in range(j0, j1):
            lv.set_level(j, buf[j - j0, 0], buf[j - j0, 1])
    torch.cuda.synchronize(lv.device)
    return {"levels": int(lv.nlev), "bytes": int(nbytes), "seconds": time.perf_counter() - t0,
            "collectives": ncoll}


def reduce_summary(summary, group=None):
    """SUM of the per-rank {live rays, live rays with finite h_abs} counters."""
    rank, world = world_info(group)
    if not collective(world):
        return summary
    t = summary.to(_dev(group)).clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.to(summary.device)


def reduce_max(value, group=None):
    rank, world = world_info(group)
    if not collective(world):
        return int(value)
    t = torch.tensor([int(value)], dtype=torch.int64, device=_dev(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def gather_rows(local, idx, nray, dst=0, group=None):
    """Collect ``local[n_local, ...]`` (rows of rays ``idx``) into ``full[nray, ...]`` on ``dst``.

    Shards differ in size by at most one live and one dead ray; they are padded
    to the largest shard for ``dist.gather``.  Returns the full array on
    ``dst`` and ``None`` elsewhere.
    """
    rank, world = world_info(group)
    if not collective(world):
        out = torch.empty((nray,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        out[torch.as_tensor(idx, device=local.device)] = local
        return out
    dev = _dev(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s) for s in sizes]
    m = max(sizes)
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    pad[: local.shape[0]] = local.to(dev)
    ipad = torch.full((m,), -1, dtype=torch.int64, device=dev)
    ipad[: len(idx)] = torch.as_tensor(np.asarray(idx), dtype=torch.int64, device=dev)
    if rank == dst:
        bufs = [torch.empty_like(pad) for _ in range(world)]
        ibufs = [torch.empty_like(ipad) for _ in range(world)]
    else:
        bufs = ibufs = None
    dist.gather(pad, bufs, dst=dst, group=group)
    dist.gather(ipad, ibufs, dst=dst, group=group)
    if rank != dst:
        return None
    out = torch.empty((nray,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    for s, b, ib in zip(sizes, bufs, ibufs):
        out[ib[:s]] = b[:s]
    return out


def gather_changed_rows(local, idx, last, dst=0, group=None):
    """The multi-rank drop-in's per-chunk collection: only rays whose rows changed.

    ``local[n_local, rows, >= 7]`` are this rank's rows of a chunk (rays
    ``idx``, a device or host int64 tensor); ``last[n_local, 7]`` (int64 bit
    patterns, updated in place) each ray's previous row.  A ray is sent when
    any of its 7 delivered values in any row differs bit for bit from its
    previous row -- a frozen ray (rkf45.py:400-403) repeats itself and is
    never sent again.  Returns ``(cols, rows)`` on ``dst`` -- the changed
    rays' global indices, ascending, and their rows ``[n, rows, 7]`` -- and
    ``None`` elsewhere; the receiver copies every other ray's previous row
    (hostio.fill_rows).
    """
    rank, world = world_info(group)
    bits = local[:, :, :7].contiguous().view(torch.int64)
    changed = torch.any((bits != last[:, None, :]).reshape(bits.shape[0], -1), dim=1)
    last.copy_(bits[:, -1, :])
    sel = torch.nonzero(changed).squeeze(1)
    rows = bits.index_select(0, sel)
    gidx = torch.as_tensor(idx, device=local.device)[sel]
    if collective(world):
        dev = _dev(group)
        n = torch.tensor([int(sel.numel())], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sizes, n, group=group)
        sizes = [int(x) for x in sizes]
        m = max(sizes)
        pad = torch.zeros((m,) + tuple(rows.shape[1:]), dtype=torch.int64, device=dev)
        pad[: rows.shape[0]] = rows.to(dev)
        ipad = torch.full((m,), -1, dtype=torch.int64, device=dev)
        ipad[: gidx.numel()] = gidx.to(dev)
        bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        ibufs = [torch.empty_like(ipad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, bufs, dst=dst, group=group)
        dist.gather(ipad, ibufs, dst=dst, group=group)
        if rank != dst:
            return None
        rows = torch.cat([b[:k] for k, b in zip(sizes, bufs)])
        gidx = torch.cat([b[:k] for k, b in zip(sizes, ibufs)])
    order = torch.argsort(gidx)
    return gidx[order], rows[order].view(torch.float64)


def cost_partition(cost, frozen, rank, world):
    """Rays of ``rank`` (sorted device index tensor) in a cost-balanced split.

    Live rays are sorted by ``cost`` (descending, stable: the same order on every
    rank) and dealt in snake order 0, 1, .., w-1, w-1, .., 0, 0, 1, .. so each
    rank receives heavy, middling and light rays alike; frozen rays (NaN state,
    rows written by the fill kernel, no integration) are dealt round-robin.
    Every rank evaluates the same deterministic rule on the same probe counts,
    so the split needs no communication.
    """
    if world == 1:
        return torch.arange(cost.numel(), device=cost.device)
    key = torch.where(frozen, torch.full_like(cost, -1), cost)
    order = torch.sort(key, descending=True, stable=True).indices
    n_live = int((~frozen).sum().item())
    pos = torch.arange(order.numel(), device=cost.device)
    blk, r = pos // world, pos % world
    owner = torch.where(blk % 2 == 0, r, world - 1 - r)
    # frozen rays (the tail of ``order``): plain round-robin
    owner = torch.where(pos >= n_live, (pos - n_live) % world, owner)
    return torch.sort(order[owner == rank]).values


def probe_share(nray, rank, world, device):
    """The rays ``rank`` probes when the probe is sharded: every ``world``-th
    slot from ``rank`` (interleaved, so each share holds every kind of ray)."""
    return torch.arange(rank, nray, world, device=device, dtype=torch.int64)


def probe_costs(eng, st, p, tb, npr, rank, world, group=None):
    """Each ray's probe cost, the probe sharded: this rank runs rows [1, 1 +
    npr) for its ``probe_share`` of the rays (from the initial state ``st``,
    which stays untouched) and the per-ray results are all-gathered -- ONE
    collective of 8 B per ray (RCCL over xGMI: 19 MB for C3, 77 MB for C5) --
    into ``(cost, frozen)`` over every ray, the same on every rank.  Without a
    group (a single-GPU rehearsal of one rank) every share is probed here.
    A ray's probe is the same on any rank (rays are independent), so a ray
    live after the probe has the unsharded probe's cost bit for bit; a ray
    frozen by then gets -1 (the unsharded path keeps its attempt count), and
    ``cost_partition`` keys frozen rays as -1 either way, so the partition is
    the same."""
    nray = st["nray"]
    dev = st["state"].device
    m = -(-nray // world)

    def one(r):
        sh = probe_share(nray, r, world, dev)
        sub = eng.take(st, sh)
        rows = torch.empty((sh.numel(), npr, 8), dtype=torch.float64, device=dev)
        eng.run(sub, p, tb, 1, 1 + npr, rows, eng.live_first_order_of(sub), 0, tails=eng.tails(sh.numel()))
        v = torch.where(torch.isnan(sub["state"][:5].sum(0)), torch.full_like(sub["count"][:, 0], -1),
                        sub["count"].sum(1))
        out = torch.full((m,), -2, dtype=torch.int64, device=dev)
        out[: v.numel()] = v
        return out
    if group is not None and collective(world):
        mine = one(rank)
        cdev = _dev(group)
        parts = [torch.empty(m, dtype=torch.int64, device=cdev) for _ in range(world)]
        dist.all_gather(parts, mine.to(cdev), group=group)
        parts = [x.to(dev) for x in parts]
    else:
        parts = [one(r) for r in range(world)]
    v = torch.empty(nray, dtype=torch.int64, device=dev)
    for r, x in enumerate(parts):
        v[r::world] = x[: len(range(r, nray, world))]
    return v.clamp(min=0), v < 0


class ShardedRun:
    """Outcome of ``run_sharded`` on one rank."""

    def __init__(self, idx, res, steps_local, endpoints=None, counts=None, failed=False):
        self.idx = idx                  # this rank's rays (device index tensor)
        self.res = res                  # engine.RunResult of the shard (None if failed)
        self.steps_local = steps_local  # accepted steps of this rank's rays
        self.endpoints = endpoints      # rank 0: last row [nray, 8] of every ray (an emulated rank: its own, idx order)
        self.counts = counts            # rank 0: [nray, 2] accepted / rejected (likewise)
        self.failed = failed


def run_sharded(eng, y0, nt, tstep=7200.0, group=None, rank=None, world=None, probe=6,
                lead=(24, 96), chunk=None, out=None, sink=None, events=None, gather=True,
                ttotal=None, order_policy="priority", team=0, split=None, shard_probe=False,
                costs=None):
    """One ray set ``y0[5, nray]`` (identical on every rank) integrated across
    the ranks of ``group``.

    Every rank constructs the solver for all rays and runs the first ``probe``
    output rows for all of them (identical, cheap: ~0.5 % of a 90-day run);
    the attempts each ray needed there decide the split (``cost_partition``).
    Each rank then integrates only its own rays to ``nt`` and ``gather`` sends
    their last row and step counters to rank 0 (RCCL ``gather`` on device
    tensors).  ``sink(i0, i1, rows, idx)`` receives this rank's rows.
    ``team`` is ``RayEngine.advance``'s latency-mode size per launch, ``split``
    its adaptive split of the long launch.
    ``shard_probe`` (world > 1): each rank probes only its ``probe_share``
    and the probe costs are all-gathered (``probe_costs``); the rank then
    re-runs the probe rows for its own shard only -- 2/world of the probe's
    work per rank instead of all of it.  ``costs`` (rehearsals): the
    ``(cost, frozen)`` of ``probe_costs`` computed beforehand, so that the
    timed call runs only this rank's share.
    ``rank``/``world`` without a group emulate one rank of a larger job on
    this device (single-GPU rehearsal: no collectives).  Rays are independent
    and both global couplings are decided over every ray, so the union of the
    shards equals the single-GPU run bit for bit.
    """
    from engine import t_eval_of
    if rank is None:
        rank, world = world_info(group)
    p = eng.params(nt, tstep)
    y0 = torch.as_tensor(y0, dtype=torch.float64, device=eng.device).contiguous()
    nray = y0.shape[1]
    tb = torch.as_tensor(t_eval_of(nt, tstep, ttotal), dtype=torch.float64, device=eng.device)
    st = eng.init(y0, p)
    summary = st["summary"].cpu()
    if int(summary[0]) > 0 and int(summary[1]) == 0:      # rkf45.py:423-425 (all rays, every rank)
        return ShardedRun(None, None, 0, failed=True)
    npr = min(probe, nt - 1)
    if events is not None:
        e0, e1, es = eng._event_pair()
    if collective(world) and (shard_probe or costs is not None):
        if costs is None:
            cost, frozen = probe_costs(eng, st, p, tb, npr, rank, world, group=group)
        else:   # (a rehearsal: the other shares were probed beforehand)
            cost, frozen = costs
            sh = probe_share(nray, rank, world, eng.device)
            sub = eng.take(st, sh)
            eng.run(sub, p, tb, 1, 1 + npr, torch.empty((sh.numel(), npr, 8), dtype=torch.float64,
                                                         device=eng.device),
                    eng.live_first_order_of(sub), 0, tails=eng.tails(sh.numel()))
        idx = cost_partition(cost, frozen, rank, world)
        local = eng.take(st, idx)                    # (the initial state: re-probe this shard)
        prow = torch.empty((idx.numel(), npr, 8), dtype=torch.float64, device=eng.device)
        ptails = eng.tails(idx.numel())
        eng.run(local, p, tb, 1, 1 + npr, prow, eng.live_first_order_of(local), 0, tails=ptails)
        prow_local, ptails_local = prow, ptails
        if events is not None:
            e1.record(es)
            events.append((e0, e1))
    else:
        prow = torch.empty((nray, npr, 8), dtype=torch.float64, device=eng.device)
        ptails = eng.tails(nray)
        eng.run(st, p, tb, 1, 1 + npr, prow, eng.live_first_order_of(st), 0, tails=ptails)
        if events is not None:
            e1.record(es)
            events.append((e0, e1))
        cost = st["count"].sum(1)                        # attempts in the probe
        frozen = torch.isnan(st["state"][:5].sum(0))
        idx = cost_partition(cost, frozen, rank, world)
        local = eng.take(st, idx)
        prow_local, ptails_local = prow[idx], None if ptails is None else ptails.take(idx)
    last = {}

    dense = {}

    def keep(i0, i1, rows, tails=None, slots=None):
        # the endpoints need each ray's last row only: a frozen ray's is its tail
        if slots is not None:
            last["row"] = slots.last_row(rows, tails, i1)
        else:
            last["row"] = rows[:, -1] if tails is None else tails.last_row(rows, i1)
        if sink is None:
            return
        if slots is not None:
            if getattr(sink, "takes_slots", False):
                return sink(i0, i1, rows, idx, tails, slots)
            # (a sink that wants dense rows: the row blocks and tails expanded)
            dense["buf"] = slots.dense(rows, tails, i0, i1, dense.get("buf"))
            return sink(i0, i1, dense["buf"], idx)
        if tails is not None and getattr(sink, "takes_tails", False):
            sink(i0, i1, rows, idx, tails)
        else:
            if tails is not None:
                eng.expand(rows, tails, i0, i1)   # (a sink that wants the rows dense)
            sink(i0, i1, rows, idx)
    keep.takes_tails = True
    keep.takes_slots = True

    keep(1, 1 + npr, prow_local, ptails_local)
    n_live_local = int((~frozen[idx]).sum().item())
    res = eng.advance(local, p, tb, 1 + npr, chunk=chunk, sink=keep, out=out, events=events,
                      group=group, order_policy=order_policy, first_chunk=list(lead),
                      n_live=int(summary[0]), n_live_local=n_live_local,
                      prev_work=torch.zeros_like(cost[idx]), team=team, split=split)
    steps_local = int(local["count"][:, 0].sum().item())
    ends = cnts = None
    if gather:
        end_row = last["row"].clone()
        if group is not None and collective(world):
            ends = gather_rows(end_row, idx.cpu().numpy(), nray, group=group)
            cnts = gather_rows(local["count"], idx.cpu().numpy(), nray, group=group)
        else:   # (one rank, or one emulated rank of a larger job: its own rays, in idx order)
            ends, cnts = end_row, local["count"]
    return ShardedRun(idx, res, steps_local, ends, cnts)
