"""Re-export of the synthetic scene generator (``samnerf_amd/synth.py``).

The generator is data, not a restatement of the reference: it lives in the
product package so that ``bench.py``'s timed leg builds its weights and camera
without importing ``oracle/``.  Tests, the golden generator and the oracle
keep importing it under its old name from here.
"""
import os
import sys

_PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "segment-anything-nerf_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)

from samnerf_amd.synth import *  # noqa: E402,F401,F403
from samnerf_amd.synth import GridSpec, ModelSpec, gui_camera, make_params, random_rotation, uniform  # noqa: E402,F401
