"""Multi-rank drop-in on the GPU box, world size 2.

Two processes share the box's one GPU over ``gloo`` (the nccl/RCCL backend
refuses two ranks on one device; the data path is the same: shard.py moves
tensors to the host for gloo).  ``WR.ray_run(mode='hip', group=WORLD)``
broadcasts rank 0's basic state, integrates each rank's shard and gathers
every row to rank 0, whose history must equal the single-process run bit for
bit (rays are independent).

RCCL itself is driven by a one-rank nccl group with
``shard.COLLECTIVE_MIN_WORLD = 1``: the N-rank branches (RCCL broadcast,
all_gather, gather, all_reduce of device tensors) run on one GPU.
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


# ------------------------------------- RCCL: a one-rank nccl group
def _rccl_worker(port, q):
    import sys
    from collections import Counter
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [os.path.join(root, "rossby-wave-ray-tracing_amd"), root, here]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    calls = Counter()

    def counted(name):
        f = getattr(dist, name)

        def g(*a, **k):
            calls[name] += 1
            return f(*a, **k)
        return g
    for name in ("broadcast", "all_reduce", "all_gather", "gather"):
        setattr(dist, name, counted(name))
    try:
        import shard
        shard.COLLECTIVE_MIN_WORLD = 1     # (the N-rank branches on one rank)
        grp = dist.group.WORLD
        backend = dist.get_backend(grp)
        hist = run_c2(grp)                 # WR drop-in: broadcast_array, gather_changed_rows
        c2_calls = dict(calls)
        calls.clear()
        import synthetic as S
        from bench import c5_rows_per_launch
        from conftest import golden
        from engine import RayEngine
        from levels import Levels
        g = golden("c5_ref10_fp64.npz")
        nt, nlev = int(g["nt"]), int(g["nlev"])
        b0 = S.background_level(0, res=0.25)
        lv = Levels(b0["lat"], b0["lon"], nlev, t0=0.0, dt=6 * 3600.0)

        def make_uv(j):
            b = S.background_level(j, res=0.25)
            return b["u"], b["v"]
        info = shard.broadcast_levels(lv, make_uv, group=grp)
        eng = RayEngine.from_levels(lv)
        cfg = S.config("C5")
        deg2rad = np.pi / 180.0
        ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
        lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
        lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
        src = eng.sources(lon, lat)
        rows0 = torch.cat([eng.initial_rows_dev(src, eng.zwn_tensor(cfg.zwn, S.c3_freq(P)))[0].reshape(7, -1)
                           for P in S.C3_PERIODS_DAYS], dim=1)
        r0 = rows0[:, torch.as_tensor(g["idx"], device=eng.device)]
        parts = []
        r = shard.run_sharded(eng, r0[:5].contiguous(), nt, 7200.0, group=grp, probe=6, lead=[24, 96],
                              chunk=c5_rows_per_launch(False, 1, nt), ttotal=(nt - 1) * 7200.0,
                              order_policy="cell", shard_probe=True,
                              sink=lambda a, b, o, idx: parts.append(o[:, :, :7].cpu()))
        full = shard.gather_rows(torch.cat(parts, dim=1), r.idx.cpu().numpy(), r0.shape[1], group=grp)
        q.put(("ok", backend, hist, c2_calls, dict(calls), info, full.cpu().numpy(), r0.cpu().numpy(),
               r.counts.cpu().numpy()))
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_world1_runs_the_collective_paths():
    """A one-rank RCCL group taken through the N-rank branches of shard.py and
    the WR drop-in (RCCL refuses two ranks on one GPU: "Duplicate GPU
    detected").  The C2 drop-in's history equals the run without a group bit
    for bit; the C5 fixture's 4 096 rays over 41 broadcast levels -- the probe
    all-gathered, the rows gathered -- hash like the oracle's in every row,
    with every ray's attempt counts."""
    import sys
    import torch.multiprocessing as mp
    from conftest import GOLDEN, golden
    sys.path.insert(0, GOLDEN)
    from make_devmath import row_hashes
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "ok", res
    _, backend, hist, c2_calls, c5_calls, info, full, r0, counts = res
    assert backend == "nccl"
    # every collective of the N-rank path ran over RCCL
    assert c2_calls.get("broadcast", 0) >= 2 and c2_calls.get("gather", 0) >= 2, c2_calls
    assert c2_calls.get("all_reduce", 0) >= 1, c2_calls
    assert c5_calls.get("all_gather", 0) >= 1 and c5_calls.get("gather", 0) >= 2, c5_calls
    assert c5_calls.get("broadcast", 0) == info["collectives"] >= 1, (c5_calls, info)
    want = run_c2()
    a = np.where(np.isnan(hist), np.nan, hist)
    b = np.where(np.isnan(want), np.nan, want)
    assert np.array_equal(a.view(np.int64), b.view(np.int64))
    g = golden("c5_ref10_fp64.npz")
    nt = int(g["nt"])
    h = np.full((7, nt, r0.shape[1]), np.nan)
    h[:, 0] = r0
    h[:, 1:] = np.transpose(full, (2, 1, 0))
    got = row_hashes(h)
    assert np.array_equal(got, g["row_sha"]), f"{int((got != g['row_sha']).sum())} of {nt} rows differ"
    assert np.array_equal(counts[:, 0], g["nacc"])
    assert np.array_equal(counts[:, 1], g["nrej"])
