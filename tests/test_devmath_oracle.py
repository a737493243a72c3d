"""The oracle with the device's transcendentals (CPU side of tests/test_gpu_devmath.py).

* oracle/devmath.cpp builds and its functions are within 1 ulp of NumPy's
  (they restate the device library's algorithms; NumPy uses glibc/SVML);
* ``device_math()`` is a context: outside it the oracle is the pinned
  NumPy restatement again;
* the committed devmath_C2_* fixtures are reproducible: the first day of
  the RK45 and RK4 histories recomputed here has the same per-row sha256.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden

sys.path.insert(0, GOLDEN)
from make_devmath import TSTEP, row_hashes  # noqa: E402

import rwrt_oracle as O  # noqa: E402
import synthetic as S    # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def test_devmath_within_one_ulp_of_numpy():
    rng = np.random.default_rng(3)
    x = rng.uniform(-1.5707963, 1.5707963, 1 << 18)
    with O.device_math() as M:
        for name in ("sin", "cos", "tan"):
            got, ref = getattr(M, name)(x), getattr(np, name)(x)
            assert np.max(np.abs(got - ref) / np.spacing(np.abs(ref))) <= 1.0, name
        en = 10.0 ** rng.uniform(-12, 6, 1 << 18)
        got, ref = M.power(en, -0.2), en ** -0.2
        assert np.max(np.abs(got - ref) / np.spacing(ref)) <= 1.0
    assert O.LIBM.sin is np.sin and O.LIBM.power is np.power


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_devmath_fixture_first_day_reproduces(kind):
    g = golden(f"devmath_C2_{kind}.npz")
    rows = golden(f"init_C2_{kind}.npz")["rows"].reshape(7, -1)
    ob = O.Background(**S.background(kind))
    nt = 13
    with np.errstate(all="ignore"), O.device_math():
        hist, nacc, _, st = O.ray_run(ob, rows[:5].copy(), nt, TSTEP, row0=rows,
                                      ttotal=(int(g["nt"]) - 1) * TSTEP)
        hist4, st4 = O.ray_run_rk4(ob, rows[:5].copy(), nt, TSTEP, row0=rows)
    assert st == 0 and st4 == 0
    assert np.array_equal(row_hashes(hist), g["row_sha"][:nt])
    assert np.array_equal(row_hashes(hist4), g["rk4_row_sha"][:nt])
