"""SHEncoder on gfx950 -- interface of shencoder/sphere_harmonics.py:14-89.

Real spherical harmonics of degree 1..8 (output degree**2 values) of unit
directions; optional analytic Jacobian for input gradients.  Compute goes to
libsamnerf_hip.so through the `_shencoder` drop-in module.
"""
import torch
import torch.nn as nn
from torch.autograd import Function

import _shencoder as _backend


class _sh_encoder(Function):
    @staticmethod
    def forward(ctx, inputs, degree, calc_grad_inputs=False):
        inputs = inputs.contiguous().float()
        B, input_dim = inputs.shape
        outputs = torch.empty(B, degree ** 2, dtype=inputs.dtype, device=inputs.device)
        dy_dx = (torch.empty(B, input_dim * degree ** 2, dtype=inputs.dtype, device=inputs.device)
                 if calc_grad_inputs else None)
        _backend.sh_encode_forward(inputs, outputs, B, input_dim, degree, dy_dx)
        ctx.save_for_backward(inputs, dy_dx)
        ctx.dims = [B, input_dim, degree]
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, dy_dx = ctx.saved_tensors
        if dy_dx is None:
            return None, None, None
        grad = grad.contiguous()
        B, input_dim, degree = ctx.dims
        grad_inputs = torch.zeros_like(inputs)
        _backend.sh_encode_backward(grad, inputs, B, input_dim, degree, dy_dx, grad_inputs)
        return grad_inputs, None, None


sh_encode = _sh_encoder.apply


class SHEncoder(nn.Module):
    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        assert input_dim == 3, "SH encoder only support input dim == 3"
        assert 0 < degree <= 8, "SH encoder only supports degree in [1, 8]"
        self.input_dim = input_dim
        self.degree = degree
        self.output_dim = degree ** 2

    def __repr__(self):
        return f"SHEncoder: input_dim={self.input_dim} degree={self.degree}"

    def forward(self, inputs, size=1):
        inputs = inputs / size
        inputs = inputs / torch.norm(inputs, dim=-1, keepdim=True)
        prefix = list(inputs.shape[:-1])
        outputs = sh_encode(inputs.reshape(-1, self.input_dim), self.degree, inputs.requires_grad)
        return outputs.reshape(prefix + [self.output_dim])
