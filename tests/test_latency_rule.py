"""The engine's latency-mode sizing (RayEngine.team_size) and the density
setter's argument checks, on the CPU (no kernel runs).

team_size("auto") predicts a launch's makespan from each ray's previous-launch
work -- max(heaviest ray x QUAD_RATIO_16, ray n+1, remaining work / remaining
lanes) -- and takes latency mode only for a predicted gain of QUAD_MIN_GAIN:
one C3 GPU (throughput-bound) gets none, a 1/8 shard (heavy-ray-bound) gets a
multiple of 64 rays, a flat work distribution none.
"""
import numpy as np
import pytest
import torch

import _hip as H
import engine


class _Props:
    multi_processor_count = 256


@pytest.fixture
def eng(monkeypatch):
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda d: _Props())
    e = engine.RayEngine.__new__(engine.RayEngine)
    e.device, e.bg = "cpu", None
    return e


def c3_like_work(nray, seed=0):
    """Attempts per ray shaped like C3 zonal (mean ~1.6 k, a heavy tail to 18.7 k)."""
    rng = np.random.default_rng(seed)
    w = np.minimum(rng.gamma(1.2, 1350.0, nray), 8622.0)   # C3's p99.9
    w[:10] = 18738 - 60 * np.arange(10)
    return torch.tensor(w.astype(np.int64))


def state_of(nray, frozen=0):
    st = torch.zeros(12, nray, dtype=torch.float64)
    st[:, nray - frozen:] = float("nan")
    return {"state": st}


def order_of(w):
    return torch.sort(w, descending=True, stable=True).indices


def test_one_gpu_c3_takes_no_latency_mode(eng):
    w = c3_like_work(716400)
    assert eng.team_size("auto", state_of(716400), w, order_of(w), 954) == (0, 16)


def test_eighth_shard_takes_heavy_rays(eng):
    w = c3_like_work(716400 // 8, seed=1)
    n, q = eng.team_size("auto", state_of(w.numel()), w, order_of(w), 954)
    assert q == 16 and n > 0 and n % 64 == 0
    assert n <= eng.team_capacity()


def test_flat_work_takes_none(eng):
    w = torch.full((90000,), 100, dtype=torch.int64)
    assert eng.team_size("auto", state_of(90000), w, order_of(w), 954) == (0, 16)


def test_explicit_sizes_and_frozen_heads(eng):
    w = c3_like_work(5000)
    st, order = state_of(5000), order_of(w)
    assert eng.team_size(300, st, w, order, 10) == (300, 16)
    assert eng.team_size((300, 4), st, w, order, 10) == (300, 4)
    # capped at 4 x rays-per-wave per CU on half the CUs
    assert eng.team_size((10 ** 6, 1), st, w, order, 10) == (128 * 4, 1)
    # the order's head must be live rays
    st2 = state_of(5000, frozen=5000)
    assert eng.team_size(300, st2, w, order, 10) == (0, 16)
    # no order (live-first launches): none
    assert eng.team_size("auto", st, w, None, 10) == (0, 16)
    # a time-varying background: one ray per latency wave, 4 per CU on half
    # the CUs; none with fp32 arithmetic (rwrt_background.fp32 == 2)
    import types
    eng.bg, eng.tv_lanes = types.SimpleNamespace(fp32=0), 32
    assert eng.team_size((10 ** 6, 1), st, w, order, 10) == (128 * 4, 1)
    assert eng.team_size(300, st, w, order, 10)[0] == 300
    eng.bg = types.SimpleNamespace(fp32=2)
    assert eng.team_size(300, st, w, order, 10) == (0, 16)
    assert eng.team_size("auto", st, w, order, 10) == (0, 16)


def test_density_setter_checks_arguments():
    lib = H.load()
    assert lib.rwrt_ctx_set_latency_density(None, 16) == H.RWRT_ERR_ARG
    assert b"rwrt_ctx" in lib.rwrt_last_error()
