"""C3 (BASELINE configs[2]) at the reference's horizon: 90 days, bit for bit.

The whole C3 set (2.40 M slots, 0.72 M / 1.03 M live rays on the zonal / non-
zonal background) is integrated 90 days (1 081 rows at 2 h, main_wr.py:15-16;
the loop wr.py:808-887) on the GPU through the benchmark's own path
(shard.run_sharded on one GPU: GPU initial rows, 6-row probe launch, the
24- and 160-row re-ordering launches, the rest in one launch, latency-mode
choice "auto").  A 2 048-ray sample -- the 512 rays with the most DP5(4)
attempts over 90 days (up to 18 738) plus 48 random rays from each of 32 cost
quantiles of the rest (tools/make_c3_ref90.py) -- must reproduce the
oracle's 90-day history (the reference's arithmetic, NumPy's transcendentals
included) in every row: all 7 variables of all 1 081 rows by per-row sha256
(tests/golden/c3_ref90_<bg>.npz, computed on the CPU), and every ray's
accepted and rejected attempt counts.  The fixtures are data: no host NumPy
is involved at test time, so the result does not depend on the GPU box's
libm.  A second zonal run puts the 1 024 heaviest rays of every launch in
latency mode (quad_rays) and must give the same bits.
"""
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from make_devmath import row_hashes  # noqa: E402

pytestmark = pytest.mark.gpu


def run_c3_90d(kind, team="auto", probe=6, split=None, info=None):
    """Rows [7, 1081, n] and (nacc, nrej) of the fixture's sample, from a
    full-set 90-day run with the bench's schedule.  ``info`` (a dict, if given)
    receives the engine's long-launch split decision."""
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    from shard import run_sharded
    g = golden(f"c3_ref90_{kind}.npz")
    nt = int(g["nt"])
    bs, _ = make_bs(kind)
    eng = RayEngine.from_bs(bs)
    src, zcs = c3_sources(eng)
    rows0 = torch.cat([eng.initial_rows_dev(src, zc)[0].reshape(7, -1) for zc in zcs], dim=1)
    assert rows0.shape[1] == int(g["nslot"])
    idx = torch.as_tensor(g["idx"], device=eng.device)
    pos = torch.full((rows0.shape[1],), -1, dtype=torch.int64, device=eng.device)
    pos[idx] = torch.arange(idx.numel(), device=eng.device)
    n = idx.numel()
    hist = np.full((7, nt, n), np.nan)
    hist[:, 0] = rows0[:, idx].cpu().numpy()

    def sink(i0, i1, rows, ridx):
        # this run's rows of its rays ridx (one GPU: every ray); keep the sample's
        p = pos[ridx]
        m = p >= 0
        got = rows[m][:, :, :7].cpu().numpy()          # (k, i1 - i0, 7)
        hist[:, i0:i1, p[m].cpu().numpy()] = np.transpose(got, (2, 1, 0))

    r = run_sharded(eng, rows0[:5].contiguous(), nt, 7200.0, rank=0, world=1, probe=probe, lead=[24, 160],
                    chunk=nt - 1, sink=sink, ttotal=(nt - 1) * 7200.0, team=team, split=split)
    if info is not None:
        info.update(split_rho=eng.split_rho, threshold=eng.SPLIT_RHO, bounds=list(r.res.bounds))
    counts = torch.empty((rows0.shape[1], 2), dtype=torch.int64, device=eng.device)
    counts[r.idx] = r.counts
    counts = counts[idx].cpu().numpy()
    del eng, r
    torch.cuda.empty_cache()
    return g, hist, counts


def check(g, hist, counts):
    want = g["row_sha"]
    got = row_hashes(hist)
    bad = np.nonzero(got != want)[0]
    if bad.size:
        last = g["last"]
        d = ~((hist[:, -1] == last) | (np.isnan(hist[:, -1]) & np.isnan(last)))
        raise AssertionError(f"{bad.size} of {len(want)} rows differ, first row {int(bad[0])}; "
                             f"{int(d.any(0).sum())} of {last.shape[1]} rays differ in the last row")
    assert np.array_equal(counts[:, 0], g["nacc"])
    assert np.array_equal(counts[:, 1], g["nrej"])


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_c3_90d_sample_bitwise_with_reference_arithmetic(kind):
    """The bench's own schedule for a whole set (bench.schedule_defaults: a
    4-row probe, 24 + 160 rows, the adaptive split of the long launch; latency
    mode 64 / 64 / 64 on the zonal jets, none on the non-zonal set, where the
    split must actually happen)."""
    info = {}
    g, hist, counts = run_c3_90d(kind, team=[64, 64, 64] if kind == "zonal" else 0, probe=4, split="auto",
                                 info=info)
    check(g, hist, counts)
    if kind == "nonzonal":
        assert info["split_rho"] is not None and info["split_rho"] < info["threshold"], info
    # the sample is what it claims: the heaviest rays of the set, alive at 90 d
    assert int(g["cost90"].max()) == int(counts.sum(1).max()) and counts.sum(1).max() > 10000
    assert int((~np.isnan(hist[0, -1])).sum()) > hist.shape[2] // 2


@pytest.mark.parametrize("team", [1024, [64, 256, 64]])
def test_c3_90d_sample_latency_mode_bitwise(team):
    """The heaviest rays of every launch in latency mode (quad_rays): 1 024 per
    launch, and the bench's per-launch default (64 / 256 / 64)."""
    g, hist, counts = run_c3_90d("zonal", team=team)
    check(g, hist, counts)


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_c3_90d_sample_rk4_bitwise(kind):
    """The reference's default integrator (fixed-step RK4, wr.py:702-765) on the
    whole C3 set for 90 days: the same 2 048-ray sample's every row equals the
    oracle's RK4 history bit for bit."""
    import torch
    from bench import c3_sources, make_bs
    from engine import RayEngine
    g = golden(f"c3_ref90_{kind}.npz")
    nt = int(g["nt"])
    bs, _ = make_bs(kind)
    eng = RayEngine.from_bs(bs)
    src, zcs = c3_sources(eng)
    rows0 = torch.cat([eng.initial_rows_dev(src, zc)[0].reshape(7, -1) for zc in zcs], dim=1)
    idx = torch.as_tensor(g["idx"], device=eng.device)
    hist = np.full((7, nt, idx.numel()), np.nan)
    hist[:, 0] = rows0[:, idx].cpu().numpy()

    def sink(i0, i1, rows):
        hist[:, i0:i1] = np.transpose(rows[idx][:, :, :7].cpu().numpy(), (2, 1, 0))

    eng.integrate_rk4(rows0[:5].contiguous(), nt, 7200.0, chunk=270, sink=sink)
    del eng
    torch.cuda.empty_cache()
    bad = np.nonzero(row_hashes(hist) != g["rk4_row_sha"])[0]
    assert not bad.size, f"{bad.size} of {nt} RK4 rows differ, first row {int(bad[0])}"
