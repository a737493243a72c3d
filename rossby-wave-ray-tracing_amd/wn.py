"""Group velocity (the reference's wn.py:140-351) on the host.

``cal_ugvg(mode='numpy')`` is the t = 0 formula used for the initial rows
(wn.py:209-259); ``mode='extent'`` is the formula of the ray loop
(wn.py:266-342), which the HIP kernel evaluates on the device -- the host
version here serves the initial-row/diagnostic path only.
"""
import numpy as np


def cal_ugvg_numpy(fu, fv, fqx, fqy, zwn, mwn, min_val=1e-10):
    """``fu..fqy``: ``(points,)``; ``mwn``: ``(3, points)`` -> ``ug, vg`` ``(3, points)``."""
    if zwn == 0:
        return np.zeros(mwn.shape), np.zeros(mwn.shape)
    nans = np.einsum("ij,j->ij", mwn * 0, fu * fqx * fqy * 0) + 1
    nans[np.isnan(nans)] = 0
    a = zwn * zwn - mwn * mwn
    b = 2 * zwn * mwn
    c = zwn * zwn + mwn * mwn
    ug = fu + (a * fqy - b * fqx) / c ** 2
    vg = fv + (a * fqx + b * fqy) / c ** 2
    return ug * nans, vg * nans


def cal_ugvg_extent(fu, fv, fqx, fqy, zwn, mwn, min_val=1e-10):
    """Element-wise Mercator group velocity (core_cal_ugvg_extent)."""
    kap = mwn / zwn
    kap2 = kap * kap
    kap1 = 1.0 + kap2
    denom = zwn * zwn * kap1 * kap1
    ug = fu + (((1. - kap2) * fqy) - (2. * kap * fqx)) / denom
    vg = fv + ((2. * kap * fqy) + ((1. - kap2) * fqx)) / denom
    return ug, vg


def cal_ugvg(fu, fv, fqx, fqy, zwn, mwn, mode="numpy"):
    if mode == "numpy":
        return cal_ugvg_numpy(fu, fv, fqx, fqy, zwn, mwn)
    if mode == "extent":
        return cal_ugvg_extent(fu, fv, fqx, fqy, zwn, mwn)
    raise ValueError(f"mode must be 'numpy' or 'extent', got {mode!r}")
