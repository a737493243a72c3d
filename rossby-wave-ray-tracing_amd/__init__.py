"""rwrt -- MI355X-native batched Rossby-wave ray integrator.

The modules of this directory mirror the reference's flat layout (``main_wr``,
``wr``, ``bs``, ``wn``, ``constants``) and are imported the same way: put
this directory on ``sys.path`` and ``from wr import WR``.  ``engine`` and
``_hip`` are the device layer (librwrt.so through ctypes).
"""
import os
import sys

_here = os.path.dirname(os.path.abspath(__file__))
if _here not in sys.path:
    sys.path.insert(0, _here)
