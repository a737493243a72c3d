"""Physical and numerical constants (values of the reference's constants.py:13-29)."""
import numpy as np

pi = 3.14159265358979323846264338327950288419716939937510
deg2rad = pi / 180.0
rad2deg = 1.0 / deg2rad
rearth = 6.3712e6          # m
omega = 7.2921e-5          # 1/s
one, zero = 1.0, 0.0
hour = 3600.0
day = 24.0 * hour
delt = 1.0e-8              # "numerically equal" threshold (real-root test, bs.py:1030)
undef = np.nan
