"""Multi-rank plumbing of shard.py on the CPU: world size 2 over gloo (127.0.0.1).

The GPU kernel cannot run here; the per-ray integration is replaced by a
deterministic per-ray function so that the sharded pipeline (split, broadcast,
per-rank work, global reductions, gather) can be checked against the
unsharded result exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_integrate(y0):
    """Stands in for RayEngine.integrate: per-ray rows (nray, 3, 8)."""
    t = torch.as_tensor(y0).T.contiguous()
    rows = torch.stack([t.sum(1), t.prod(1), t[:, 0] * 2, t[:, 1] - 1,
                        t[:, 2], t[:, 3], t[:, 4], torch.zeros(t.shape[0], dtype=t.dtype)], 1)
    return torch.stack([rows, rows * 2, rows * 3], 1)


def _worker(rank, world, port, q, min_world=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ncoll = []
    for name in ("broadcast", "all_reduce", "all_gather", "gather"):
        def counted(*a, _f=getattr(dist, name), **k):
            ncoll.append(1)
            return _f(*a, **k)
        setattr(dist, name, counted)
    try:
        import shard
        shard.COLLECTIVE_MIN_WORLD = min_world
        rng = np.random.default_rng(0)
        nray = 101
        y0 = rng.standard_normal((5, nray)) if rank == 0 else None
        y0 = shard.broadcast_array(y0 if rank == 0 else np.zeros(1), 0)
        y0[:, ::3] = np.nan                                 # dead slots
        live = ~np.isnan(y0.mean(axis=0))
        idx = shard.shard_indices(live, rank, world)
        local = fake_integrate(y0[:, idx])
        full = shard.gather_rows(local, idx, nray, 0)
        summ = shard.reduce_summary(torch.tensor([int(live[idx].sum()), rank], dtype=torch.int64))
        mx = shard.reduce_max(10 + rank)
        if rank == 0:
            q.put(("ok", full.numpy(), fake_integrate(y0).numpy(), summ.tolist(), mx,
                   int(live.sum()), len(ncoll)))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_shard_indices_partition_and_balance():
    import shard
    live = np.random.default_rng(1).random(1000) < 0.3
    parts = [shard.shard_indices(live, r, 4) for r in range(4)]
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(1000))
    nl = [int(live[p].sum()) for p in parts]
    assert max(nl) - min(nl) <= 1


def test_world2_gloo_pipeline_equals_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    _, full, ref, summ, mx, nlive, ncoll = res
    assert np.array_equal(full, ref, equal_nan=True)
    assert summ == [nlive, 1]
    assert mx == 11
    assert ncoll >= 7


@pytest.mark.parametrize("min_world,ncoll", [(2, 0), (1, 7)])
def test_world1_collective_knob(min_world, ncoll):
    """One rank: no collective by default; with shard.COLLECTIVE_MIN_WORLD = 1
    the N-rank branches run (2 broadcasts, all_gather + 2 gathers, 2
    all_reduces) and give the same result (tests/test_gpu_multirank.py drives
    RCCL this way on the one-GPU box)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), q, min_world))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res[0] == "ok", res
    _, full, ref, summ, mx, nlive, n = res
    assert np.array_equal(full, ref, equal_nan=True)
    assert summ == [nlive, 0] and mx == 10
    assert n == ncoll


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_cost_partition_is_a_balanced_split(world):
    """C4's split (shard.cost_partition): disjoint and complete; every rank gets
    the same number of live rays (+-1) and nearly the same total cost; the
    heaviest rays spread over the ranks."""
    import shard
    rng = np.random.default_rng(2)
    n = 100_003
    cost = torch.as_tensor(np.round(rng.lognormal(3.0, 0.8, n)).astype(np.int64))
    frozen = torch.as_tensor(rng.random(n) < 0.7)
    parts = [shard.cost_partition(cost, frozen, r, world) for r in range(world)]
    allidx = torch.sort(torch.cat(parts)).values
    assert torch.equal(allidx, torch.arange(n))
    live_n = [int((~frozen[p]).sum()) for p in parts]
    tot = [int(cost[p][~frozen[p]].sum()) for p in parts]
    assert max(live_n) - min(live_n) <= 1
    assert max(tot) - min(tot) <= int(cost.max())          # within one ray's cost
    top = torch.sort(torch.where(frozen, -1, cost), descending=True).indices[:world]
    owners = {r for r, p in enumerate(parts) for i in top.tolist() if i in set(p.tolist())}
    assert len(owners) == world
    # the same rule on every rank: repeated evaluation is identical
    assert all(torch.equal(shard.cost_partition(cost, frozen, r, world), parts[r]) for r in range(world))


def _delta_worker(rank, world, port, q):
    """Each rank sends only its changed rays per chunk (shard.gather_changed_rows);
    rank 0 rebuilds the full history with hostio.fill_rows."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import shard
        from hostio import fill_rows
        rng = np.random.default_rng(3)
        nray, nt = 203, 25
        full = rng.standard_normal((nray, nt, 8))          # the same on every rank
        freeze = rng.integers(1, nt + 5, nray)
        for i in range(nray):
            if freeze[i] < nt:
                full[i, freeze[i]:] = full[i, freeze[i]]
        full[::5, 4:, 2] = np.nan
        full[:, 12:18] = full[:, 11:12]                     # a chunk where nothing changes
        idx = shard.shard_indices(np.ones(nray, bool), rank, world)
        last = torch.as_tensor(np.ascontiguousarray(full[idx, 0, :7])).view(torch.int64).clone()
        hist = np.full((nt, nray, 7), np.nan)
        hist[0] = full[:, 0, :7]
        sent = 0
        for i0, i1 in [(1, 6), (6, 12), (12, 18), (18, 25)]:
            local = torch.as_tensor(np.ascontiguousarray(full[idx, i0:i1]))
            got = shard.gather_changed_rows(local, torch.as_tensor(idx), last, 0)
            if rank == 0:
                cols, data = got
                sent += cols.numel()
                host = data.permute(2, 1, 0).contiguous().numpy()
                c = np.ascontiguousarray(cols.numpy())
                for v in range(7):
                    blk = np.empty((i1 - i0, nray))
                    fill_rows(blk, np.ascontiguousarray(hist[i0 - 1, :, v]), host[v], c if len(c) else None)
                    hist[i0:i1, :, v] = blk
        if rank == 0:
            q.put(("ok", hist, np.transpose(full[:, :, :7], (1, 0, 2)), sent))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_world2_gloo_changed_rows_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_delta_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    _, hist, want, sent = res
    assert np.array_equal(hist.view(np.int64), want.view(np.int64))   # bit for bit
    assert sent < 4 * 203                                             # frozen rays were not sent
