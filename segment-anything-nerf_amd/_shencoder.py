"""Drop-in for the reference's `_shencoder` pybind module
(shencoder/src/bindings.cpp:6-7), backed by libsamnerf_hip.so (gfx950)."""
from samnerf_amd.ops import sh_encode_backward, sh_encode_forward  # noqa: F401
