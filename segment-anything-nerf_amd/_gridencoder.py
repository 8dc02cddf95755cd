"""Drop-in for the reference's `_gridencoder` pybind module
(gridencoder/src/bindings.cpp:6-9): same function names and signatures,
backed by libsamnerf_hip.so (gfx950).  `import _gridencoder as _backend`
(gridencoder/grid.py:9-10) resolves here."""
from samnerf_amd.ops import (grad_total_variation, grad_weight_decay,  # noqa: F401
                             grid_encode_backward, grid_encode_forward)
