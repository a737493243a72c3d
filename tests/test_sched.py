"""Host-side scheduling helpers of the ray loop (CPU): the Morton key of the
cell-ordered queue (C5), the rank correlation behind the adaptive split of
the long launch, and the order they produce."""
import numpy as np
import pytest
import torch

import _hip as H
from engine import RayEngine, morton2


def test_morton2_interleaves_bits():
    ix = torch.tensor([0, 1, 0, 1, 2, 3, 1440])
    iy = torch.tensor([0, 0, 1, 1, 0, 3, 720])
    want = []
    for x, y in zip(ix.tolist(), iy.tolist()):
        z = 0
        for b in range(16):
            z |= ((x >> b) & 1) << (2 * b) | ((y >> b) & 1) << (2 * b + 1)
        want.append(z)
    assert morton2(ix, iy).tolist() == want


def test_rank_corr_is_spearman():
    from scipy.stats import spearmanr
    rng = np.random.default_rng(0)
    a = rng.standard_normal(5000)
    b = a + rng.standard_normal(5000)
    m = torch.ones(5000, dtype=torch.bool)
    m[::7] = False
    got = RayEngine.rank_corr(torch.as_tensor(a), torch.as_tensor(b), m)
    assert abs(got - spearmanr(a[m.numpy()], b[m.numpy()])[0]) < 1e-12
    assert RayEngine.rank_corr(torch.as_tensor(a), torch.as_tensor(a), m) > 1 - 1e-12
    assert RayEngine.rank_corr(torch.as_tensor(a[:2]), torch.as_tensor(b[:2]), m[:2]) == 1.0


def test_cost_cell_order_classes_then_cells():
    eng = RayEngine.__new__(RayEngine)
    eng.grid = H.Grid(1441, 721, 0.0, np.pi / 720, -np.pi / 2, np.pi / 720)
    n = 8
    state = torch.zeros((H.NSTATE, n), dtype=torch.float64)
    state[0] = torch.tensor([3.0, 0.1, 0.2, 5.0, 0.1, 1.0, 2.0, 0.3])    # lon
    state[1] = torch.tensor([0.0, 0.1, 0.1, 0.0, -1.0, 0.5, 0.5, 0.1])   # lat
    state[:5, 3] = float("nan")                                          # frozen: last
    work = torch.tensor([100.0, 100.0, 101.0, 9999.0, 3.0, 100.0, 100.0, 100.0])
    order = eng.cost_cell_order({"state": state}, work).tolist()
    assert order[-1] == 3 and order[-2] == 4                              # frozen last, light next
    heavy = order[:6]
    assert set(heavy) == {0, 1, 2, 5, 6, 7}                               # one cost class (log2 bins)
    g = eng.grid
    ix = np.floor(np.mod(state[0, heavy].numpy(), 2 * np.pi) / g.dlon).astype(int)
    iy = np.floor((state[1, heavy].numpy() - g.lat0) / g.dlat).astype(int)
    keys = morton2(torch.as_tensor(ix), torch.as_tensor(iy)).tolist()
    assert keys == sorted(keys)                                          # Morton order within the class


def test_long_launch_cuts():
    """split='auto[:a,b,..]' (RayEngine.parse_split / cut_bounds): the
    pieces that replace the long launch after the leading ones."""
    from engine import RayEngine as E
    assert E.parse_split("auto") == (True, [E.SPLIT_ROWS])
    assert E.parse_split("auto:300,300") == (True, [300, 300])
    assert E.parse_split(None)[0] is False and E.parse_split("off")[0] is False
    assert E.cut_bounds(189, 1081, [300]) == [(189, 489), (489, 1081)]
    assert E.cut_bounds(189, 1081, [300, 300]) == [(189, 489), (489, 789), (789, 1081)]
    assert E.cut_bounds(189, 1081, [40]) == [(189, 229), (229, 1081)]
    assert E.cut_bounds(0, 100, [60, 60]) == [(0, 60), (60, 100)]        # a cut past the end is dropped
    for bad in ("auto:0", "auto:-5", "auto:300,0"):                     # (empty / backward pieces)
        with pytest.raises(ValueError):
            E.parse_split(bad)
