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


# ----------------------------------------------------------------- row slots
# ABI 4 (rwrt_rk45_run_slots): the launch's row buffer holds row blocks for
# the rays live at its start only; rwrt_expand_slots makes them dense.

class SlotRecorder:
    """A sink that takes row blocks: keeps each launch's rows made dense
    (rwrt_expand_slots) and its slot map, then refills the row blocks with the
    sentinel."""
    takes_slots = True

    def __init__(self):
        self.chunks, self.nblk = {}, set()

    def __call__(self, i0, i1, view, tails, slots):
        self.nblk.add(view.shape[0])
        self.chunks[i0] = (i1, slots.dense(view, tails, i0, i1).clone(), slots.slot.clone())
        view.fill_(SENTINEL)


def run_slots(eng, y0, nt, chunk, **kw):
    """The dense run (no tails) and the row-block run of the same rays."""
    eng.use_tails = False
    buf = torch.full((y0.shape[1], chunk, 8), SENTINEL, dtype=torch.float64, device=eng.device)
    dense = Recorder(buf, False)
    rd = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=chunk, out=buf, sink=dense, **kw)
    eng.use_tails = True
    rec = SlotRecorder()
    rs = eng.integrate(y0, nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=chunk, sink=rec, **kw)
    assert sorted(dense.chunks) == sorted(rec.chunks)
    for i0, (i1, dv, _) in dense.chunks.items():
        j1, sv, _ = rec.chunks[i0]
        assert j1 == i1
        assert np.array_equal(bits(dv), bits(sv)), f"launch {i0}: expanded row blocks differ from the dense rows"
    for name in ("nacc", "nrej", "nanrow"):
        assert torch.equal(getattr(rd, name), getattr(rs, name)), name
    assert rd.break_row == rs.break_row
    assert np.array_equal(bits(rd.state["state"]), bits(rs.state["state"]))
    live0 = int((~torch.isnan(y0.sum(0))).sum().item())
    assert rec.nblk == {live0}, (rec.nblk, live0)      # one block per ray live at the start
    return rec, eng.rows_bytes


@pytest.mark.parametrize("n", [1, 4095, 4096, 4097, 3 * 4096 + 17, 100003])
def test_row_slots_number_the_live_rays(n):
    """rwrt_row_slots: the rays with a finite state mean, numbered in ray
    order (an exclusive scan over tiles of 4 096), -1 for the others."""
    from engine import Slots
    rng = np.random.default_rng(n)
    for frac in (0.0, 0.3, 0.97, 1.0):
        s = rng.standard_normal((12, n))
        dead = rng.random(n) < frac
        s[rng.integers(0, 5, n)[dead], np.nonzero(dead)[0]] = np.nan
        if n > 8:
            s[0, 3], s[1, 3] = np.inf, -np.inf        # inf - inf: a NaN mean (frozen)
            s[2, 5] = np.inf                          # inf: live
            dead[3], dead[5] = True, False
            s[:5, 5] = np.where(np.isnan(s[:5, 5]), 1.0, s[:5, 5])
        st = dict(state=torch.as_tensor(s, device="cuda"), nray=n)
        sl = Slots(n, torch.device("cuda")).compute(st, torch.cuda.current_stream().cuda_stream)
        live = ~np.isnan(s[:5].sum(0) / 5.0)
        want = np.where(live, np.cumsum(live) - 1, -1)
        assert sl.count() == int(live.sum())
        assert np.array_equal(sl.slot.cpu().numpy(), want), frac


@pytest.mark.parametrize("team", [0, [64, 64, 64]])
def test_c3_row_slots_equal_dense_rows(team):
    """The C3 sample (16 384 live rays + 2 048 dead slots) in the bench's
    launch shape: the row blocks, expanded, are the dense launch's rows bit for
    bit, with and without the latency mode (quad_rays writes through its ray's
    block too), and the buffer holds the live rays only."""
    from bench import make_bs
    from engine import RayEngine
    bs, _ = make_bs("zonal")
    eng = RayEngine.from_bs(bs)
    y0 = c3_sample_y0(eng)
    _, nbytes = run_slots(eng, y0, 12 * 12 + 1, 48, first_chunk=[6, 24], team=team)
    live0 = int((~torch.isnan(y0.sum(0))).sum().item())
    assert nbytes == live0 * 48 * 64          # one buffer of 48-row blocks (the dense one: 18 432 rays)


@pytest.mark.parametrize("lanes,team", [(32, 0), (64, 0), (32, (64, 1))])
def test_time_varying_row_slots_equal_dense_rows(lanes, team):
    """The time-varying kernels (0.25 degrees, 9 six-hourly fp64 levels, 2
    days; lane pairs, 64 rays per wave, latency waves) through row blocks."""
    import rwrt_oracle as O
    import synthetic as S
    from engine import RayEngine
    from levels import Levels
    dt, nlev, nt = 6 * 3600.0, 9, 25
    bl = [S.background_level(j, res=0.25) for j in range(nlev)]
    lv = Levels(bl[0]["lat"], bl[0]["lon"], nlev, t0=0.0, dt=dt)
    for j, b in enumerate(bl):
        lv.set_level(j, b["u"], b["v"])
    eng = RayEngine.from_levels(lv)
    eng.tv_lanes = lanes
    cfg = S.config("C5")
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = eng.initial_rows(slon, slat, cfg.zwn, S.c3_freq(S.C5_PERIODS_DAYS[-1])).cpu().numpy()
    y0 = rows[:5].reshape(5, -1)
    pick = np.sort(np.random.default_rng(5).choice(y0.shape[1], size=8192, replace=False))
    y0 = torch.as_tensor(y0[:, pick].copy(), device=eng.device)
    kw = dict(order_policy="cell", first_chunk=[4], team=team) if team else {}
    run_slots(eng, y0, nt, 8, **kw)


def test_sharded_row_slots_equal_dense_endpoints():
    """shard.run_sharded -- the bench's step -- with row blocks (its sink
    takes them) against dense rows: endpoints and counters bit for bit; a
    dense user sink behind it receives the dense rows."""
    from bench import make_bs
    from engine import RayEngine
    from shard import run_sharded
    bs, _ = make_bs("nonzonal")
    eng = RayEngine.from_bs(bs)
    y0 = c3_sample_y0(eng)
    nt = 12 * 12 + 1
    ends, rows = {}, {}
    for slots in (False, True):
        eng.use_slots = slots
        got = {}
        r = run_sharded(eng, y0, nt, 7200.0, rank=0, world=1, probe=4, lead=[24, 48], chunk=nt - 1,
                        ttotal=(nt - 1) * 7200.0, team="auto",
                        sink=lambda i0, i1, v, idx: got.__setitem__(i0, bits(v)))
        ends[slots] = (bits(r.endpoints), r.counts.cpu().numpy())
        rows[slots] = got
    eng.use_slots = True
    assert np.array_equal(ends[False][0], ends[True][0])
    assert np.array_equal(ends[False][1], ends[True][1])
    assert sorted(rows[False]) == sorted(rows[True])
    for k in rows[False]:
        assert np.array_equal(rows[False][k], rows[True][k]), k
