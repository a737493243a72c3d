"""The 90-day C2 fixtures of tests/test_gpu_ref90.py (CPU side).

* ``device_math()`` (the kernel's restated transcendentals, oracle/npmath.cpp)
  changes nothing: the oracle computes the same bits inside and outside it;
* the committed ref90_C2_* fixtures are reproducible: the first day of the
  RK45 and RK4 histories recomputed here has the same per-row sha256.
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
from test_np_math import _svml_host  # noqa: E402

pytestmark = pytest.mark.skipif(not _svml_host(), reason="NumPy without SVML: not the reference's arithmetic")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def test_device_math_is_numpy():
    rng = np.random.default_rng(3)
    x = rng.uniform(-1.5707963, 1.5707963, 1 << 18)
    en = 10.0 ** rng.uniform(-12, 6, 1 << 18)
    with O.device_math() as M:
        for name in ("sin", "cos", "tan"):
            assert np.array_equal(getattr(M, name)(x), getattr(np, name)(x)), name
        assert np.array_equal(M.power(en, -0.2), en ** -0.2)
    assert O.LIBM.sin is np.sin and O.LIBM.power is np.power


@pytest.mark.parametrize("kind", ["zonal", "nonzonal"])
def test_ref90_fixture_first_day_reproduces(kind):
    g = golden(f"ref90_C2_{kind}.npz")
    rows = golden(f"init_C2_{kind}.npz")["rows"].reshape(7, -1)
    ob = O.Background(**S.background(kind))
    nt = 13
    for ctx in (None, O.device_math):
        with np.errstate(all="ignore"):
            if ctx is None:
                hist, _, _, st = O.ray_run(ob, rows[:5].copy(), nt, TSTEP, row0=rows,
                                           ttotal=(int(g["nt"]) - 1) * TSTEP)
                hist4, st4 = O.ray_run_rk4(ob, rows[:5].copy(), nt, TSTEP, row0=rows)
            else:
                with ctx():
                    hist, _, _, st = O.ray_run(ob, rows[:5].copy(), nt, TSTEP, row0=rows,
                                               ttotal=(int(g["nt"]) - 1) * TSTEP)
                    hist4, st4 = O.ray_run_rk4(ob, rows[:5].copy(), nt, TSTEP, row0=rows)
        assert st == 0 and st4 == 0
        assert np.array_equal(row_hashes(hist), g["row_sha"][:nt])
        assert np.array_equal(row_hashes(hist4), g["rk4_row_sha"][:nt])
