import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rossby-wave-ray-tracing_amd")
os.environ.setdefault("PYTHONPATH", os.pathsep.join([PKG, os.path.join(ROOT, "oracle"), ROOT]))
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    config.addinivalue_line("markers", "slow: long CPU-oracle runs")
    config.addinivalue_line(
        "markers",
        "refhost: computes the oracle (or NumPy's transcendentals) on this host at test time; "
        "skipped when this host's NumPy is not the reference's arithmetic")


def golden(name):
    import numpy as np
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


_LIBM = {}


def reference_libm():
    """``(ok, why)``: does this host's NumPy compute the reference's
    transcendentals (sin, cos, tan, power, arctan2 -- SVML-dispatched on the
    reference's AVX-512 hosts)?  Compared by fingerprint
    (tools/host_libm_probe.py) with the container that made the golden
    fixtures (tests/golden/host_libm.json)."""
    if "r" not in _LIBM:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import host_libm_probe as P
        want = json.load(open(os.path.join(GOLDEN, "host_libm.json")))
        got = P.fingerprint(want["n"], want["seed"])
        diff = sorted(k for k in want["fingerprint"] if got.get(k) != want["fingerprint"][k])
        _LIBM["r"] = (not diff, "" if not diff else
                      f"this host's NumPy {', '.join(diff)} differ from the reference's (SVML on AVX-512; "
                      f"tools/host_libm_probe.py): an oracle computed here is not the reference's arithmetic, "
                      f"so a mismatch would blame a correct kernel")
    return _LIBM["r"]


def pytest_runtest_setup(item):
    if item.get_closest_marker("refhost"):
        ok, why = reference_libm()
        if not ok:
            pytest.skip(why)
