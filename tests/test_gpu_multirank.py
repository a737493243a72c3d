"""Multi-rank drop-in on the GPU box, world size 2.

Two processes share the box's one GPU over ``gloo`` (the nccl/RCCL backend
refuses two ranks on one device; the data path is the same: shard.py moves
tensors to the host for gloo).  ``WR.ray_run(mode='hip', group=WORLD)``
broadcasts rank 0's basic state, integrates each rank's shard and gathers
every row to rank 0, whose history must equal the single-process run bit for
bit (rays are independent).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NT = 61      # 5 days


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_c2(group=None):
    import synthetic as S
    from bs import BS
    from wr import WR
    bg = S.background("nonzonal")
    bs = BS(len(bg["lon"]), len(bg["lat"]))
    bs.load_arrays(**bg)
    bs.ready(xcyclic=True)
    cfg = S.config("C2")
    w = WR(cfg.nzwn, cfg.nsource, 7200.0, (NT - 1) * 7200.0, cfg.freq, nx=bs.nlon, ny=bs.nlat,
           chunk_rows=20)
    w.bs = bs
    w.set_zwn(cfg.zwn)
    w.set_source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    with np.errstate(all="ignore"):
        w.ray_run(mode="hip", inte_method="rk45", group=group)
    return np.array([w.rlon, w.rlat, w.rzwn, w.rmwn, w.ramp, w.rug, w.rvg]).reshape(7, NT, -1)


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "rossby-wave-ray-tracing_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hist = run_c2(dist.group.WORLD)
        if rank == 0:
            q.put(("ok", hist))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_world2_dropin_equals_single_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=110)
    for p in procs:
        p.join(timeout=60)
    assert res[0] == "ok", res
    got = res[1]
    want = run_c2()
    a = np.where(np.isnan(got), np.nan, got)
    b = np.where(np.isnan(want), np.nan, want)
    assert np.array_equal(a.view(np.int64), b.view(np.int64))
