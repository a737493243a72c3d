"""Constant row tails (``rwrt_rk45_run_tails`` / ``rwrt_rk45_run_tv_tails``,
ABI 3) against the dense ray loop (``rwrt_rk45_run``), bit for bit.

A frozen ray (rkf45.py:400-403: a dead root slot, or a ray masked by
wr.py:838-850) repeats one row for the rest of a launch.  With tails the
launch stores that row once per ray (``Tails.row``) with the row it starts
at (``Tails.frm``) and writes nothing into the row buffer from there on; the
bench's endpoints and every dense consumer (after ``RayEngine.expand``) see
exactly the rows the dense launch writes.  Checked per launch:

* rows before a ray's tail are the dense launch's rows, bit for bit;
* rows from the tail on are NOT written (the buffer keeps a sentinel) and the
  tail row equals every one of the dense launch's rows there;
* rays frozen at the launch start have their tail from its first row, every
  other ray none (a ray that freezes inside a launch writes its rows as the
  dense launch does), and the solver state, counters and early-exit rows
  agree;
* the same through the latency mode (quad_rays), the time-varying kernels
  (C5 levels, fp64 and fp32 storage) and ``shard.run_sharded`` (the bench's
  path: its endpoints come from the tails without any expansion).
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu
SENTINEL = 7.25


def bits(t):
    a = t.detach().cpu().numpy().astype(np.float64, copy=True)
    a[np.isnan(a)] = np.nan
    return a.view(np.int64)


class Recorder:
    """A sink that keeps every launch's rows (and tails), then refills the
    row buffer with the sentinel so that the next launch's unwritten rows
    show."""

    def __init__(self, buf, takes_tails):
        self.buf, self.takes_tails, self.chunks = buf, takes_tails, {}

    def __call__(self, i0, i1, view, tails=None):
        self.chunks[i0] = (i1, view.clone(), None if tails is None else (tails.frm.clone(), tails.row.clone()))
        self.buf.fill_(SENTINEL)


def run_both(eng, y0, nt, chunk, **kw):
    out = {}
    for tails in (False, True):
        eng.use_tails = tails
        buf = torch.full((y0.shape[1], chunk, 8), SENTINEL, dtype=torch.float64, device=eng.device)
        rec = Recorder(buf, tails)
        res = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=chunk, out=buf, sink=rec, **kw)
        out[tails] = (rec, res)
    eng.use_tails = True
    return out


def compare(out):
    (dense, rd), (tl, rt) = out[False], out[True]
    assert sorted(dense.chunks) == sorted(tl.chunks)
    n_start = n_mid = 0
    for i0, (i1, dv, _) in dense.chunks.items():
        j1, tv, (frm, row) = tl.chunks[i0]
        assert j1 == i1
        frm = frm.cpu().numpy()
        assert ((frm >= i0) & (frm <= i1)).all()
        r = np.arange(i1 - i0)[None, :]
        tailed = (i0 + r) >= frm[:, None]                   # [nray, rows]
        db, tb = bits(dv), bits(tv)
        assert np.array_equal(db[~tailed], tb[~tailed]), f"launch {i0}: rows before the tails differ"
        sent = np.float64(SENTINEL).view(np.int64)
        assert (tb[tailed] == sent).all(), f"launch {i0}: a tail row was written densely"
        rb = bits(row)
        rep = np.broadcast_to(rb[:, None, :], db.shape)
        assert np.array_equal(db[tailed], rep[tailed]), f"launch {i0}: a tail row differs from the dense rows"
        n_start += int((frm == i0).sum())
        n_mid += int(((frm > i0) & (frm < i1)).sum())
    for name in ("nacc", "nrej", "nanrow"):
        assert torch.equal(getattr(rd, name), getattr(rt, name)), name
    assert rd.break_row == rt.break_row
    assert np.array_equal(bits(rd.state["state"]), bits(rt.state["state"]))
    return n_start, n_mid


def c3_sample_y0(eng, n_dead=2048):
    from bench import c3_sources
    src, zcs = c3_sources(eng)
    y0 = torch.cat([eng.initial_rows_dev(src, zc)[0][:5].reshape(5, -1) for zc in zcs], dim=1)
    g = golden("c3_sample.npz")
    dead = torch.nonzero(torch.isnan(y0.sum(0))).squeeze(1)[:: 397][:n_dead]
    sel = torch.cat([torch.as_tensor(g["idx"], device=eng.device), dead])
    return y0[:, sel].contiguous()


@pytest.mark.parametrize("team", [0, [64, 64, 64]])
def test_c3_tails_equal_dense_rows(team):
    """16 384 cost-stratified live C3 rays + 2 048 dead slots, 12 days in the
    bench's launch shape (probe-sized and re-ordering launches, then 48 rows),
    with and without the latency mode."""
    from bench import make_bs
    from engine import RayEngine
    bs, _ = make_bs("zonal")
    eng = RayEngine.from_bs(bs)
    y0 = c3_sample_y0(eng)
    n_start, n_mid = compare(run_both(eng, y0, 12 * 12 + 1, 48, first_chunk=[6, 24], team=team))
    assert n_start > 2048 and n_mid == 0, (n_start, n_mid)


def test_sharded_endpoints_from_tails():
    """shard.run_sharded (the bench's step) takes each ray's last row from its
    tail: the endpoints and counters equal the dense run's bit for bit."""
    from bench import make_bs
    from engine import RayEngine
    from shard import run_sharded
    bs, _ = make_bs("nonzonal")
    eng = RayEngine.from_bs(bs)
    y0 = c3_sample_y0(eng)
    nt = 12 * 12 + 1
    ends = {}
    for tails in (False, True):
        eng.use_tails = tails
        r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=4, lead=[24, 48], chunk=nt - 1,
                        ttotal=(nt - 1) * 7200.0, team="auto")
        ends[tails] = (bits(r.endpoints), r.counts.cpu().numpy())
    eng.use_tails = True
    assert np.array_equal(ends[False][0], ends[True][0])
    assert np.array_equal(ends[False][1], ends[True][1])


@pytest.mark.parametrize("fp32", [False, True])
def test_time_varying_tails_equal_dense_rows(fp32):
    """The C5 kernels (0.25 degrees, 9 six-hourly levels, 2 days) with tails."""
    import rwrt_oracle as O
    import synthetic as S
    from engine import RayEngine
    from levels import Levels
    dt, nlev, nt = 6 * 3600.0, 9, 25
    bl = [S.background_level(j, res=0.25) for j in range(nlev)]
    lv = Levels(bl[0]["lat"], bl[0]["lon"], nlev, t0=0.0, dt=dt, fp32=fp32)
    for j, b in enumerate(bl):
        lv.set_level(j, b["u"], b["v"])
    eng = RayEngine.from_levels(lv)
    cfg = S.config("C5")
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = eng.initial_rows(slon, slat, cfg.zwn, S.c3_freq(S.C5_PERIODS_DAYS[-1])).cpu().numpy()
    y0 = rows[:5].reshape(5, -1)
    pick = np.sort(np.random.default_rng(5).choice(y0.shape[1], size=8192, replace=False))
    y0 = torch.as_tensor(y0[:, pick].copy(), device=eng.device)
    n_start, _ = compare(run_both(eng, y0, nt, 8))
    assert n_start > 0
