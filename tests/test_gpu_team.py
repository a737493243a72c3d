"""Latency mode: quad_rays (csrc/rwrt.hip, in rk45_run_kernel's first blocks; four lanes of a wave per
ray, the RHS's divisions, stage sums and error norm dealt out over the quad
and exchanged by DPP) -- or, in a RWRT_LATENCY_QUAD=0 build, rk45_team_kernel
(each RHS split over the four waves of a block) -- must give the run kernel's
results bit for bit.

* the C3 cost-stratified sample (tests/golden/c3_sample.npz: the 512 rays
  with the most attempts in day 1 plus rays from 31 cost quantiles) integrated
  12 days with the heaviest half of the rays of every launch in latency mode,
  against the oracle (the reference's arithmetic, NumPy's transcendentals
  included): every value of every row, and the accepted-step counts;
* C2 (both backgrounds, 10 days, chunked) with every live ray in latency
  mode (16, 1 and 4 rays per wave) against the run kernel alone: rows and per-ray accepted / rejected
  counts (reference: wr.py:767-887, rkf45.py:375-514).
"""
import numpy as np
import pytest
import torch

from conftest import golden
import synthetic as S

pytestmark = pytest.mark.gpu


def same(a, b):
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    b = np.where(np.isnan(b), np.nan, np.asarray(b, np.float64))
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def rows_of(eng, y0, nt, **kw):
    rows = {}
    res = eng.integrate(torch.as_tensor(y0, device="cuda"), nt, 7200.0,
                        sink=lambda a, b, o: rows.__setitem__(a, o.cpu().numpy()), **kw)
    return np.concatenate([rows[k] for k in sorted(rows)], axis=1), res


@pytest.mark.refhost
def test_team_c3_sample_bitwise_with_reference_arithmetic():
    import rwrt_oracle as O
    from bench import c3_initial_state, make_bs
    from engine import RayEngine
    bs, bg = make_bs("zonal")
    eng = RayEngine.from_bs(bs)
    g = golden("c3_sample.npz")
    y0 = c3_initial_state(bs)[:, g["idx"]]
    nt = 12 * 12 + 1
    n_team = min(8192, eng.team_capacity())
    hist, res = rows_of(eng, y0, nt, chunk=48, first_chunk=[6, 24], team=n_team)
    with np.errstate(all="ignore"):
        ref, rnacc, _, st = O.ray_run(O.Background(**bg), y0.copy(), nt, 7200.0)
    assert st == 0
    got = np.transpose(hist[:, :, :7], (2, 1, 0))
    assert same(got, ref[:, 1:])
    assert np.array_equal(res.nacc.cpu().numpy(), rnacc)


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_team_equals_run_kernel_c2(kind):
    from bench import make_bs
    from engine import RayEngine
    from wr import initial_rows
    bs, _ = make_bs(kind)
    eng = RayEngine.from_bs(bs)
    cfg = S.config("C2")
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * np.pi / 180.0
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * np.pi / 180.0
    with np.errstate(all="ignore"):
        y0 = np.array(initial_rows(bs, lon, lat, cfg.zwn, cfg.freq)[:5]).reshape(5, -1)
    nt = 10 * 12 + 1
    want, rw = rows_of(eng, y0, nt, chunk=40, first_chunk=[7])
    # 16 rays per wave (64 per block), 1 per wave, 4 per wave over a ragged count
    for team in (eng.team_capacity(), (eng.team_capacity(), 1), (333, 4)):
        got, rg = rows_of(eng, y0, nt, chunk=40, first_chunk=[7], team=team)
        assert same(got[:, :, :7], want[:, :, :7]), team
        assert torch.equal(rg.nacc, rw.nacc) and torch.equal(rg.nrej, rw.nrej), team
        assert torch.equal(rg.nanrow, rw.nanrow), team


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_drain_handoff_equals_run_kernel(kind):
    """The drain-time hand-off (rwrt_ctx_set_handoff): once a launch's queue is
    drained, a wave with at most N rays left continues them in the quad layout
    from where each lane stopped, mid-step state included.  C2 (3 072 slots,
    10 days, chunked) and the C3 sample (12 days, the bench's launch shape) at
    N = 16, 4 and 1 against the hand-off off: rows, accepted / rejected counts
    and early-exit rows bit for bit, and rays were handed off."""
    from bench import c3_initial_state, make_bs
    from engine import RayEngine
    from wr import initial_rows
    bs, _ = make_bs(kind)
    eng = RayEngine.from_bs(bs)
    cfg = S.config("C2")
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * np.pi / 180.0
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * np.pi / 180.0
    with np.errstate(all="ignore"):
        c2 = np.array(initial_rows(bs, lon, lat, cfg.zwn, cfg.freq)[:5]).reshape(5, -1)
    c3 = c3_initial_state(bs)[:, golden("c3_sample.npz")["idx"]]
    for y0, nt, kw in ((c2, 10 * 12 + 1, dict(chunk=40, first_chunk=[7])),
                       (c3, 12 * 12 + 1, dict(chunk=48, first_chunk=[6, 24], team=[64, 64, 64]))):
        eng.handoff = 0
        want, rw = rows_of(eng, y0, nt, **kw)
        assert sum(eng.handoffs()) == 0
        for n in (16, 4, 1):
            eng.handoff = n
            got, rg = rows_of(eng, y0, nt, **kw)
            moved = eng.handoffs()
            assert sum(moved) > 0, (n, moved)
            assert same(got[:, :, :7], want[:, :, :7]), n
            assert same(got[:, :, 7], want[:, :, 7]), n
            assert torch.equal(rg.nacc, rw.nacc) and torch.equal(rg.nrej, rw.nrej), n
            assert torch.equal(rg.nanrow, rw.nanrow), n
    eng.handoff = 16
