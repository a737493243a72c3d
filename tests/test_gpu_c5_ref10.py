"""C5 (BASELINE configs[4]) through 41 levels of its time-varying background.

The whole C5 set -- 1-degree global seeds x k = 1..10 x the 5 C3 periods =
9.67 M slots (4.03 M live) on the 0.25-degree synthetic time-varying state,
one level every 6 h built on the GPU by rwrt_bs_ready -- is integrated 10
days (121 rows, 41 levels) through the benchmark's path (shard.run_sharded:
probe, re-ordering launches, the rest in the bench's rows per launch), with
fp64 and with fp32 level storage.  A 4 096-ray random sample must reproduce
the oracle's TimeVaryingBackground history (tests/golden/c5_ref10_<s>.npz,
tools/make_c5_ref.py, CPU) in every row by per-row sha256 -- all 7 variables
-- and every ray's accepted / rejected attempt counts.  The reference has no
time-varying mode (wr.py:784-789 ignores t); the oracle's restatement of the
extension is built from the reference's pinned pieces.
"""
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from make_devmath import row_hashes  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("storage", ["fp64", "fp32"])
def test_c5_10d_41_levels_bitwise_with_oracle(storage):
    import torch
    import synthetic as S
    from engine import RayEngine
    from levels import Levels
    from shard import run_sharded
    g = golden(f"c5_ref10_{storage}.npz")
    nt, nlev = int(g["nt"]), int(g["nlev"])
    b0 = S.background_level(0, res=0.25)
    lv = Levels(b0["lat"], b0["lon"], nlev, t0=0.0, dt=6 * 3600.0, fp32=storage == "fp32")
    for j in range(nlev):
        bj = b0 if j == 0 else S.background_level(j, res=0.25)
        lv.set_level(j, bj["u"], bj["v"])
    eng = RayEngine.from_levels(lv)
    cfg = S.config("C5")
    deg2rad = np.pi / 180.0
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * deg2rad
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * deg2rad
    src = eng.sources(lon, lat)
    rows0 = torch.cat([eng.initial_rows_dev(src, eng.zwn_tensor(cfg.zwn, S.c3_freq(P)))[0].reshape(7, -1)
                       for P in S.C3_PERIODS_DAYS], dim=1)
    assert rows0.shape[1] == int(g["nslot"])
    idx = torch.as_tensor(g["idx"], device=eng.device)
    pos = torch.full((rows0.shape[1],), -1, dtype=torch.int64, device=eng.device)
    pos[idx] = torch.arange(idx.numel(), device=eng.device)
    hist = np.full((7, nt, idx.numel()), np.nan)
    hist[:, 0] = rows0[:, idx].cpu().numpy()

    def sink(i0, i1, rows, ridx):
        p = pos[ridx]
        m = p >= 0
        hist[:, i0:i1, p[m].cpu().numpy()] = np.transpose(rows[m][:, :, :7].cpu().numpy(), (2, 1, 0))

    chunk = 240 if lv.fp32 else 48          # bench.py main_c5's rows per launch
    r = run_sharded(eng, rows0[:5].contiguous(), nt, 7200.0, rank=0, world=1, probe=6, lead=[24, 96],
                    chunk=chunk, sink=sink, ttotal=(nt - 1) * 7200.0,
                    order_policy="cell")   # bench.py's C5 default queue order
    counts = r.counts[idx].cpu().numpy()
    del eng, lv, r
    torch.cuda.empty_cache()
    got = row_hashes(hist)
    bad = np.nonzero(got != g["row_sha"])[0]
    if bad.size:
        last = g["last"]
        d = ~((hist[:, -1] == last) | (np.isnan(hist[:, -1]) & np.isnan(last)))
        raise AssertionError(f"{bad.size} of {nt} rows differ, first row {int(bad[0])}; "
                             f"{int(d.any(0).sum())} of {last.shape[1]} rays differ in the last row")
    assert np.array_equal(counts[:, 0], g["nacc"])
    assert np.array_equal(counts[:, 1], g["nrej"])
    # the sample crosses the level pairs: rays move, many still alive at 10 d
    assert np.nanmax(np.abs(hist[0, -1] - hist[0, 0])) > 0.5
