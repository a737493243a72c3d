"""Execution contexts (include/rwrt.h ``rwrt_ctx``).

The library keeps no state of its own between calls: the ray loop's scratch
(frozen-ray flags, side stream, events) belongs to an ``rwrt_ctx``.  Two
engines -- two contexts -- integrating on two streams from two host threads
at the same time must give exactly what each gives alone.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
NT = 49   # 4 days


def _engine_and_rays(kind):
    import rwrt_oracle as O
    import synthetic as S
    from bench import make_bs
    from engine import RayEngine
    bs, bg = make_bs(kind)
    cfg = S.config("C2")
    eng = RayEngine.from_bs(bs)
    slon, slat = O.source_matrix(cfg.SW_lon, cfg.SW_lat, cfg.dlon, cfg.dlat, cfg.nnx, cfg.nny)
    rows = eng.initial_rows(slon, slat, cfg.zwn, cfg.freq).cpu().numpy()
    return eng, rows[:5].reshape(5, -1)


def _run(eng, y0, stream=None, out=None):
    import torch
    rows = {}
    ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
    with ctx:
        res = eng.integrate(torch.as_tensor(y0, device=eng.device), NT, 7200.0, chunk=16,
                            sink=lambda a, b, o: rows.__setitem__(a, o.clone()))
        torch.cuda.current_stream().synchronize()
    hist = torch.cat([rows[k] for k in sorted(rows)], dim=1).cpu().numpy()
    return hist, res.nacc.cpu().numpy(), res.nrej.cpu().numpy()


def _same(a, b):
    a = np.where(np.isnan(a), np.nan, a)
    b = np.where(np.isnan(b), np.nan, b)
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def test_two_contexts_two_streams_concurrently():
    import torch
    from engine import RayEngine
    eng_a, y_a = _engine_and_rays("zonal")
    eng_b0, y_b = _engine_and_rays("nonzonal")
    # a second engine over the same packed state has its own context
    eng_b = RayEngine.from_packed(eng_b0.packed, *_axes("nonzonal"))
    assert eng_a.ctx.handle.value != eng_b.ctx.handle.value
    want_a = _run(eng_a, y_a)
    want_b = _run(eng_b, y_b)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = {}

    def worker(name, eng, y, s):
        got[name] = _run(eng, y, s)

    for _ in range(2):
        th = [threading.Thread(target=worker, args=("a", eng_a, y_a, s1)),
              threading.Thread(target=worker, args=("b", eng_b, y_b, s2))]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=100)
        for name, want in (("a", want_a), ("b", want_b)):
            for g, w in zip(got[name], want):
                assert _same(np.asarray(g, np.float64), np.asarray(w, np.float64)), name


def test_one_context_on_two_streams():
    """The same context on another stream: the second call waits for the first
    on the device before reusing the flags; results unchanged."""
    import torch
    eng, y0 = _engine_and_rays("nonzonal")
    want = _run(eng, y0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = _run(eng, y0, s1)
    b = _run(eng, y0, s2)
    for g1, g2, w in zip(a, b, want):
        assert _same(np.asarray(g1, np.float64), np.asarray(w, np.float64))
        assert _same(np.asarray(g2, np.float64), np.asarray(w, np.float64))


def _axes(kind):
    from bench import make_bs
    bs, _ = make_bs(kind)
    return bs.lon, bs.lat
