"""Test infrastructure: `_gridencoder` / `_shencoder`-compatible backends on
the C oracle (oracle/encoders_oracle.c), for CPU tensors.

Swapping them into the mirror modules (gridencoder.grid._backend,
shencoder.sphere_harmonics._backend) gives a CPU twin of the product's
unfused path whose autograd graph is the same torch ops with the oracle's
encoder forward/backward -- the reference's own structure -- so GPU gradients
of a training step can be compared against it.  Never used by the product.
"""
import contextlib

import numpy as np
import torch

from oracle import encoders as enc


class GridBackend:
    @staticmethod
    def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, max_level, S, H,
                            dy_dx, gridtype, align_corners, interpolation):
        assert dy_dx is None and gridtype == 0 and not align_corners and interpolation == 0
        out = enc.grid_encode_forward(inputs.detach().numpy(), embeddings.detach().numpy(),
                                      offsets.numpy(), L, S, H, max_level=max_level)
        outputs.copy_(torch.from_numpy(np.ascontiguousarray(out)))

    @staticmethod
    def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L,
                             max_level, S, H, dy_dx, grad_inputs, gridtype, align_corners,
                             interpolation):
        assert dy_dx is None and grad_inputs is None
        g = enc.grid_encode_backward(grad.detach().numpy(), inputs.detach().numpy(),
                                     embeddings.detach().numpy(), offsets.numpy(), L, S, H,
                                     max_level=max_level)
        grad_embeddings.copy_(torch.from_numpy(np.ascontiguousarray(g)))


class SHBackend:
    @staticmethod
    def sh_encode_forward(inputs, outputs, B, input_dim, degree, dy_dx):
        assert dy_dx is None
        out = enc.sh_encode_forward(inputs.detach().numpy(), degree)
        out = out[0] if isinstance(out, tuple) else out
        outputs.copy_(torch.from_numpy(np.ascontiguousarray(out)))


@contextlib.contextmanager
def oracle_encoders():
    """Route the mirror's GridEncoder / SHEncoder through the C oracle."""
    import gridencoder.grid as g
    import shencoder.sphere_harmonics as s
    old = (g._backend, s._backend)
    g._backend, s._backend = GridBackend, SHBackend
    try:
        yield
    finally:
        g._backend, s._backend = old
