"""Sharding rays across GPUs (one process per GPU, torch.distributed over RCCL).

Rays never interact (``test_sharding_is_bitwise_invisible``),
so a ray set splits across ranks with no exchange during integration.  What
crosses ranks is setup and collection only:

* ``broadcast_array`` -- rank 0's basic-state stack (or initial rays) to every
  rank (RCCL broadcast over xGMI; ~1 MB at 2.5 deg, ~91 MB per 0.25 deg level);
* ``shard_indices``   -- a balanced split: live rays and NaN-root slots are
  dealt round-robin separately, so every rank gets the same number of rays
  that actually integrate;
* ``reduce_summary`` / ``reduce_max`` -- the reference's two global couplings
  (solver failure, rkf45.py:423-425; early exit, wr.py:853-855) evaluated over
  all ranks so that a sharded run equals the single-GPU run exactly;
* ``gather_rows``     -- per-chunk trajectory rows back to rank 0.

Works with the ``nccl`` (RCCL) backend on device tensors and with ``gloo`` on
CPU tensors (tests/test_shard.py).
"""
import numpy as np
import torch
import torch.distributed as dist


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
    if world == 1:
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


def reduce_summary(summary, group=None):
    """SUM of the per-rank {live rays, live rays with finite h_abs} counters."""
    rank, world = world_info(group)
    if world == 1:
        return summary
    t = summary.to(_dev(group)).clone()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.to(summary.device)


def reduce_max(value, group=None):
    rank, world = world_info(group)
    if world == 1:
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
    if world == 1:
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
