"""Which lanes of the single-attempt golden vectors differ from the reference
(rwrt_dp54_attempt vs tests/golden/step_<kind>.npz), and at which stage.

    RWRT_LIB=<lib> python tools/diag_attempt.py [zonal|nonzonal]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rossby-wave-ray-tracing_amd"), os.path.join(ROOT, "tests")]


def bits(a):
    a = np.where(np.isnan(a), np.nan, np.asarray(a, np.float64))
    return a.view(np.int64)


def main():
    from conftest import golden
    from test_gpu_parity import engine
    kind = sys.argv[1] if len(sys.argv) > 1 else "zonal"
    g = golden(f"step_{kind}.npz")
    K, yn, err = engine(kind).attempt(g["y"], g["f"], g["h"])
    K, yn, err = K.cpu().numpy(), yn.cpu().numpy(), err.cpu().numpy()
    bad = np.nonzero((bits(K) != bits(g["K"])).any(axis=(0, 1)))[0]
    print(f"{kind}: {bad.size} of {K.shape[2]} lanes differ in K; y_new {int((bits(yn) != bits(g['y_new'])).any(0).sum())};"
          f" err {int((bits(err) != bits(g['err_norm'])).sum())}")
    for i in bad[:12]:
        st = [s for s in range(K.shape[0]) if (bits(K[s, :, i]) != bits(g["K"][s, :, i])).any()]
        print(f"  lane {i}: y {g['y'][:, i]!r} h {g['h'][i]!r} first stage {st[0]} stages {st}")
        s = st[0]
        print(f"    got {K[s, :, i]!r}\n    ref {g['K'][s, :, i]!r}")


if __name__ == "__main__":
    main()
