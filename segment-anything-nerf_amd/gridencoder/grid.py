"""GridEncoder on gfx950 -- interface of gridencoder/grid.py:24-204.

Same constructor arguments, `embeddings` parameter / `offsets` buffer
(state_dict-compatible with reference checkpoints), same forward contract
([..., 3] in [-bound, bound] -> [..., L*C]) and the same autograd Function
shape (`grid_encode` saves inputs/embeddings/offsets/dy_dx, backward returns
grad_inputs / grad_embeddings).  Compute goes to libsamnerf_hip.so through
the `_gridencoder` drop-in module.
"""
import numpy as np
import torch
import torch.nn as nn
from torch.autograd import Function

import _gridencoder as _backend

_gridtype_to_id = {"hash": 0, "tiled": 1}
_interp_to_id = {"linear": 0, "smoothstep": 1}


class _grid_encode(Function):
    """grid.py:24-96 -- level-major [L,B,C] kernel output, permuted to [B, L*C]."""

    @staticmethod
    def forward(ctx, inputs, embeddings, offsets, per_level_scale, base_resolution,
                calc_grad_inputs=False, gridtype=0, align_corners=False, interpolation=0,
                max_level=None):
        inputs = inputs.contiguous()
        B, D = inputs.shape
        L = offsets.shape[0] - 1
        C = embeddings.shape[1]
        S = np.log2(per_level_scale)
        H = base_resolution
        max_level = L if max_level is None else min(max_level, L)
        outputs = (torch.zeros if max_level < L else torch.empty)(
            L, B, C, device=inputs.device, dtype=embeddings.dtype)
        dy_dx = None
        if calc_grad_inputs:
            dy_dx = (torch.zeros if max_level < L else torch.empty)(
                B, L * D * C, device=inputs.device, dtype=embeddings.dtype)
        _backend.grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, max_level,
                                     S, H, dy_dx, gridtype, align_corners, interpolation)
        outputs = outputs.permute(1, 0, 2).reshape(B, L * C)
        ctx.save_for_backward(inputs, embeddings, offsets, dy_dx)
        ctx.dims = [B, D, C, L, S, H, gridtype, interpolation, max_level]
        ctx.align_corners = align_corners
        return outputs

    @staticmethod
    def backward(ctx, grad):
        inputs, embeddings, offsets, dy_dx = ctx.saved_tensors
        B, D, C, L, S, H, gridtype, interpolation, max_level = ctx.dims
        grad = grad.view(B, L, C).permute(1, 0, 2).contiguous()
        grad_embeddings = torch.zeros_like(embeddings)
        grad_inputs = torch.zeros_like(inputs, dtype=embeddings.dtype) if dy_dx is not None else None
        _backend.grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C,
                                      L, max_level, S, H, dy_dx, grad_inputs, gridtype,
                                      ctx.align_corners, interpolation)
        if grad_inputs is not None:
            grad_inputs = grad_inputs.to(inputs.dtype)
        return grad_inputs, grad_embeddings, None, None, None, None, None, None, None, None


grid_encode = _grid_encode.apply


class GridEncoder(nn.Module):
    def __init__(self, input_dim=3, num_levels=16, level_dim=2, per_level_scale=2,
                 base_resolution=16, log2_hashmap_size=19, desired_resolution=None,
                 gridtype="hash", align_corners=False, interpolation="linear"):
        super().__init__()
        if desired_resolution is not None:      # grid.py:107-108
            per_level_scale = np.exp2(np.log2(desired_resolution / base_resolution) /
                                      (num_levels - 1))
        self.input_dim = input_dim
        self.num_levels = num_levels
        self.level_dim = level_dim
        self.per_level_scale = per_level_scale
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = base_resolution
        self.output_dim = num_levels * level_dim
        self.gridtype = gridtype
        self.gridtype_id = _gridtype_to_id[gridtype]
        self.interpolation = interpolation
        self.interp_id = _interp_to_id[interpolation]
        self.align_corners = align_corners

        # table layout (grid.py:124-135): ceil(base * scale^l) per axis, capped
        # at 2^log2_hashmap_size, rounded up to a multiple of 8 rows
        cap = 2 ** log2_hashmap_size
        sizes = []
        for lvl in range(num_levels):
            res = int(np.ceil(base_resolution * per_level_scale ** lvl))
            sizes.append(int(np.ceil(min(cap, res ** input_dim) / 8) * 8))
        offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
        self.offsets_host = offsets            # host copy for the fused renderer
        self.register_buffer("offsets", torch.from_numpy(offsets.copy()))
        self.max_params = cap
        self.n_params = int(offsets[-1]) * level_dim
        self.embeddings = nn.Parameter(torch.empty(int(offsets[-1]), level_dim))
        self.reset_parameters()

    def reset_parameters(self):
        std = 1e-4
        self.embeddings.data.uniform_(-std, std)

    @property
    def S(self):
        return float(np.log2(self.per_level_scale))

    def __repr__(self):
        top = int(round(self.base_resolution * self.per_level_scale ** (self.num_levels - 1)))
        return (f"GridEncoder: input_dim={self.input_dim} num_levels={self.num_levels} "
                f"level_dim={self.level_dim} resolution={self.base_resolution} -> {top} "
                f"per_level_scale={self.per_level_scale:.4f} params={tuple(self.embeddings.shape)} "
                f"gridtype={self.gridtype} align_corners={self.align_corners} "
                f"interpolation={self.interpolation}")

    def forward(self, inputs, bound=1, max_level=None):
        inputs = (inputs + bound) / (2 * bound)
        prefix = list(inputs.shape[:-1])
        inputs = inputs.view(-1, self.input_dim)
        outputs = grid_encode(inputs, self.embeddings, self.offsets, self.per_level_scale,
                              self.base_resolution, inputs.requires_grad, self.gridtype_id,
                              self.align_corners, self.interp_id, max_level)
        return outputs.view(prefix + [self.output_dim])

    @torch.no_grad()
    def grad_total_variation(self, weight=1e-7, inputs=None, bound=1, B=1000000):
        D, C = self.input_dim, self.embeddings.shape[1]
        L = self.offsets.shape[0] - 1
        if inputs is None:
            inputs = torch.rand(B, D, device=self.embeddings.device)
        else:
            inputs = ((inputs + bound) / (2 * bound)).view(-1, D).contiguous()
            B = inputs.shape[0]
        if self.embeddings.grad is None:
            raise ValueError("grad is None, should be called after loss.backward() and before "
                             "optimizer.step()!")
        _backend.grad_total_variation(inputs, self.embeddings, self.embeddings.grad, self.offsets,
                                      weight, B, D, C, L, self.S, self.base_resolution,
                                      self.gridtype_id, self.align_corners)

    @torch.no_grad()
    def grad_weight_decay(self, weight=0.1):
        B, C = self.embeddings.shape
        L = self.offsets.shape[0] - 1
        if self.embeddings.grad is None:
            raise ValueError("grad is None, should be called after loss.backward() and before "
                             "optimizer.step()!")
        _backend.grad_weight_decay(self.embeddings, self.embeddings.grad, self.offsets, weight, B,
                                   C, L)
