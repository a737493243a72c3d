"""Edge cases of the ray loop on the GPU, bitwise against the oracle (the
reference's arithmetic: the kernels' sin/cos/tan/pow are NumPy's own).

* empty batches (nray = 0) launch nothing and return empty results;
* ragged batch sizes around the block and fill-tile sizes (1, 127, 129, 300
  rays; 256-lane blocks, 128-ray fill tiles) with live and dead slots mixed,
  integrated in 7-row chunks so that rays also enter later chunks frozen;
* batches where every ray is frozen from the start (dead root slots: finite
  source position, NaN wavenumber) -- only frozen_fill_kernel writes rows;
* an all-NaN batch: the reference's early exit (wr.py:853-855) at row 1.
"""
import numpy as np
import pytest
import torch

from conftest import golden
import synthetic as S

pytestmark = [pytest.mark.gpu, pytest.mark.refhost]
NT = 25


def _bs(kind):
    from bs import BS
    bg = S.background(kind)
    bs = BS(len(bg["lon"]), len(bg["lat"]))
    bs.load_arrays(**bg)
    bs.ready(xcyclic=True)
    return bs, bg


def _engine(kind):
    from engine import RayEngine
    bs, bg = _bs(kind)
    return RayEngine.from_bs(bs), bg


def _gpu_rows(eng, y0, nt, chunk):
    rows = {}
    res = eng.integrate(torch.as_tensor(y0), nt, 7200.0, ttotal=(nt - 1) * 7200.0, chunk=chunk,
                        sink=lambda a, b, o: rows.__setitem__((a, b), o.cpu().numpy().copy()))
    nray = y0.shape[1]
    hist = np.full((nray, nt, 8), np.nan)
    for (i0, i1), r in rows.items():
        hist[:, i0:i1] = r
    return hist, res


def _oracle(bg, y0, nt):
    import rwrt_oracle as O
    with np.errstate(all="ignore"):
        hist, nacc, nrej, status = O.ray_run(O.Background(**bg), y0.copy(), nt, 7200.0)
    return hist, nacc, nrej, status


def _same(a, b):
    a = np.where(np.isnan(a), np.nan, a)
    b = np.where(np.isnan(b), np.nan, b)
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def _check(hist, res, ref, nrow=None):
    h, nacc, nrej, status = ref
    nrow = nrow or h.shape[1]
    g = np.transpose(hist[:, 1:nrow, :7], (2, 1, 0))        # (7, rows 1.., ray)
    assert _same(g, h[:, 1:nrow])
    assert np.array_equal(res.nacc.cpu().numpy(), nacc)
    assert np.array_equal(res.nrej.cpu().numpy(), nrej)


def test_empty_batch():
    eng, _ = _engine("zonal")
    hist, res = _gpu_rows(eng, np.zeros((5, 0)), NT, 7)
    assert hist.shape == (0, NT, 8)
    assert res.nacc.numel() == 0 and res.ray_steps == 0 and res.n_live == 0
    assert not res.failed


@pytest.mark.parametrize("n", [1, 127, 129, 300])
def test_ragged_batches_bitwise(n):
    eng, bg = _engine("nonzonal")
    rows = golden("init_C2_nonzonal.npz")["rows"][:5].reshape(5, -1)
    rng = np.random.default_rng(n)
    live = np.flatnonzero(~np.isnan(rows.sum(0)))
    dead = np.flatnonzero(np.isnan(rows.sum(0)))
    k = max(1, n // 3)                       # a third dead slots, the rest live
    pick = np.concatenate([rng.choice(dead, min(k, n - 1) if n > 1 else 0, replace=False),
                           rng.choice(live, n - (min(k, n - 1) if n > 1 else 0), replace=False)])
    rng.shuffle(pick)
    y0 = np.ascontiguousarray(rows[:, pick])
    hist, res = _gpu_rows(eng, y0, NT, 7)
    _check(hist, res, _oracle(bg, y0, NT))


def test_all_frozen_batch_bitwise():
    eng, bg = _engine("zonal")
    rows = golden("init_C2_zonal.npz")["rows"][:5].reshape(5, -1)
    dead = np.flatnonzero(np.isnan(rows.sum(0)))
    assert len(dead) > 300
    y0 = np.ascontiguousarray(rows[:, dead[:300]])
    assert np.isfinite(y0[:2]).all()         # dead roots keep their source position
    hist, res = _gpu_rows(eng, y0, NT, 7)
    ref = _oracle(bg, y0, NT)
    _check(hist, res, ref)
    assert res.ray_steps == 0 and res.break_row is None
    # every row is the source position with NaN wavenumbers, ug, vg
    assert _same(hist[:, 1:, :2], np.broadcast_to(y0[:2].T[:, None, :], (300, NT - 1, 2)))


def test_all_nan_batch_breaks_at_row_1():
    eng, bg = _engine("zonal")
    y0 = np.full((5, 200), np.nan)
    hist, res = _gpu_rows(eng, y0, NT, 7)
    assert res.break_row == 1 and res.ray_steps == 0
    h, _, _, _ = _oracle(bg, y0, NT)
    assert np.isnan(h[:, 1:]).all()


def test_calls_on_two_streams_equal_one_stream():
    """The library's frozen-ray scratch is per device: calls issued on two
    streams (two engines) wait for each other and give the same rows."""
    rows = golden("init_C2_nonzonal.npz")["rows"][:5].reshape(5, -1)
    y0 = torch.as_tensor(np.ascontiguousarray(rows), device="cuda")
    nray = y0.shape[1]
    ref, _ = _gpu_rows(_engine("nonzonal")[0], rows, NT, 7)
    outs = []
    for _ in range(2):
        eng = _engine("nonzonal")[0]
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out = torch.empty((nray, NT - 1, 8), dtype=torch.float64, device="cuda")
            eng.integrate(y0, NT, 7200.0, ttotal=(NT - 1) * 7200.0, chunk=6, out=[out])
            outs.append(out)
    torch.cuda.synchronize()
    for out in outs:   # the buffer holds the last 6-row chunk (rows 19..24)
        last = out.reshape(-1)[: nray * 6 * 8].reshape(nray, 6, 8).cpu().numpy()
        assert _same(last, ref[:, NT - 6:])


def test_rk4_chunked_runs_equal_one_launch():
    """RK4 rays with a NaN in lon/lat/k/l at a launch start are written by
    rk4_fill_kernel; 40-row chunks (rays dying in one chunk enter the next one
    flagged) equal one launch bit for bit, and the oracle's RK4 rows."""
    import rwrt_oracle as O
    eng, bg = _engine("nonzonal")
    g = golden("init_C2_nonzonal.npz")
    rows7 = g["rows"].reshape(7, -1)
    y0 = torch.as_tensor(np.ascontiguousarray(rows7[:5]), device="cuda")
    nt = 241
    res = {}
    for chunk in (None, 40):
        got = {}
        r = eng.integrate_rk4(y0, nt, 7200.0, chunk=chunk,
                              sink=lambda a, b, o: got.__setitem__((a, b), o.cpu().numpy().copy()))
        h = np.full((y0.shape[1], nt, 8), np.nan)
        for (i0, i1), v in got.items():
            h[:, i0:i1] = v
        res[chunk] = (h, r)
    (h1, r1), (h2, r2) = res[None], res[40]
    assert _same(h1[:, 1:], h2[:, 1:])
    assert torch.equal(r1.nacc, r2.nacc) and torch.equal(r1.nrej, r2.nrej)
    assert torch.equal(r1.nanrow, r2.nanrow)
    with np.errstate(all="ignore"):
        href, _ = O.ray_run_rk4(O.Background(**bg), rows7[:5].copy(), nt, 7200.0, row0=rows7)
    assert _same(np.transpose(h2[:, 1:, :7], (2, 1, 0)), href[:, 1:])
