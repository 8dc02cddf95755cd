"""Drop-in for the reference's `_freqencoder` pybind module
(freqencoder/src/bindings.cpp:6-7), backed by libsamnerf_hip.so (gfx950)."""
from samnerf_amd.ops import freq_encode_backward, freq_encode_forward  # noqa: F401
