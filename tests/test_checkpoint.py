"""Checkpoint / resume (the ray state is tiny, so resuming =
persisting it at an output index).

CPU: the checkpoint file format (np.savez, no pickles) round-trips and a
foreign file is refused.  GPU: C2 (non-zonal, 10 days) run to row 37, saved,
resumed by a FRESH engine from the file to row 121 -- rows and per-ray
accepted / rejected counters equal the uninterrupted run bit for bit
(wr.py:767-887 is resumable at any output row: the solver state is y, f, t,
h_abs and the counters).
"""
import os

import numpy as np
import pytest

import synthetic as S


def test_checkpoint_file_roundtrip(tmp_path):
    from engine import RayEngine
    rng = np.random.default_rng(0)
    ck = {"state": rng.standard_normal((12, 7)), "count": rng.integers(0, 9, (7, 2)),
          "nanrow": np.full(7, 121, np.int32), "next_row": np.int64(37),
          "params": np.array([1e-6, 1e-6, 7.2, 0.2, 121.0, 7200.0, 864000.0]), "nray": np.int64(7)}
    for name in ("ck.npz", "ck"):                 # np.savez appends .npz: the same path loads
        path = os.path.join(tmp_path, name)
        RayEngine.save_checkpoint(ck, path)
        got = RayEngine.load_checkpoint(path)
        for k in ck:
            assert np.array_equal(got[k], ck[k]) and got[k].dtype == np.asarray(ck[k]).dtype
    bad = os.path.join(tmp_path, "bad.npz")
    np.savez(bad, state=np.zeros((5, 3)))
    with pytest.raises(ValueError):
        RayEngine.load_checkpoint(bad)
    np.savez(bad, **dict(ck, nray=np.int64(8)))   # ray count and state disagree
    with pytest.raises(ValueError):
        RayEngine.load_checkpoint(bad)


@pytest.mark.gpu
def test_resume_equals_uninterrupted(tmp_path):
    import torch
    from bench import make_bs
    from engine import RayEngine
    from wr import initial_rows
    bs, _ = make_bs("nonzonal")
    cfg = S.config("C2")
    ix, iy = np.meshgrid(np.arange(cfg.nnx), np.arange(cfg.nny))
    lon = ((cfg.SW_lon % 360.0 + ix.ravel() * cfg.dlon) % 360.0) * np.pi / 180.0
    lat = (cfg.SW_lat + iy.ravel() * cfg.dlat) * np.pi / 180.0
    with np.errstate(all="ignore"):
        y0 = np.array(initial_rows(bs, lon, lat, cfg.zwn, cfg.freq)[:5]).reshape(5, -1)
    nt = 10 * 12 + 1

    def collect(rows):
        return lambda a, b, o: rows.__setitem__(a, o[:, :, :8].cpu().numpy())

    full = {}
    eng = RayEngine.from_bs(bs)
    rf = eng.integrate(torch.as_tensor(y0, device="cuda"), nt, 7200.0, chunk=24, sink=collect(full))
    want = np.concatenate([full[k] for k in sorted(full)], axis=1)

    part = {}
    r1 = eng.integrate(torch.as_tensor(y0, device="cuda"), nt, 7200.0, chunk=24, sink=collect(part),
                       stop_row=37)
    assert r1.next_row == 37
    path = os.path.join(tmp_path, "c2.npz")
    RayEngine.save_checkpoint(RayEngine.checkpoint(r1), path)
    eng2 = RayEngine.from_bs(bs)
    r2 = eng2.resume(RayEngine.load_checkpoint(path), nt, 7200.0, chunk=24, sink=collect(part))
    got = np.concatenate([part[k] for k in sorted(part)], axis=1)
    a = np.where(np.isnan(got), np.nan, got)
    b = np.where(np.isnan(want), np.nan, want)
    assert a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))
    assert torch.equal(r2.nacc, rf.nacc) and torch.equal(r2.nrej, rf.nrej)
    assert torch.equal(r2.nanrow, rf.nanrow)
    # a resume with other run parameters is refused, not silently different
    with pytest.raises(ValueError, match="rtol"):
        eng2.resume(RayEngine.load_checkpoint(path), nt, 7200.0, rtol=1e-5, chunk=24)
