"""Tensor-level wrappers over the C ABI (torch = device memory + streams only).

The encoder functions keep the exact names, argument order and in-place
output convention of the reference's pybind modules
(gridencoder/src/bindings.cpp:6-9, shencoder/src/bindings.cpp:6-7,
freqencoder/src/bindings.cpp:6-7) and raise RuntimeError on the same argument
checks (gridencoder.cu:15-18: CUDA / contiguous / dtype).
"""
import ctypes

import torch

from ._lib import check, lib


def _stream(t=None):
    dev = t.device if t is not None else None
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _cuda(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")


def _contig(t, name):
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")


def _f32(t, name):
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be a float32 tensor (the fp16 path is not supported; "
                           "the reference forces fp16 off, main.py:222)")


def _i32(t, name):
    if t.dtype != torch.int32:
        raise RuntimeError(f"{name} must be an int tensor")


def _aligned(t, name, nbytes=16):
    if t.data_ptr() % nbytes:
        raise RuntimeError(f"{name} must be {nbytes}-byte aligned")


def _float_tensor(t, name, vec=False):
    _cuda(t, name)
    _contig(t, name)
    _f32(t, name)
    if vec:
        _aligned(t, name)


# -------------------------------------------------------------- gridencoder --

def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, max_level, S, H,
                        dy_dx, gridtype, align_corners, interp):
    _float_tensor(inputs, "inputs")
    _float_tensor(embeddings, "embeddings", vec=True)
    _cuda(offsets, "offsets"); _contig(offsets, "offsets"); _i32(offsets, "offsets")
    _float_tensor(outputs, "outputs", vec=True)
    if dy_dx is not None:
        _float_tensor(dy_dx, "dy_dx", vec=True)
    check(lib().samnerf_grid_encode_forward(
        _ptr(inputs), _ptr(embeddings), _ptr(offsets), _ptr(outputs), B, D, C, L, max_level,
        float(S), H, _ptr(dy_dx), gridtype, int(bool(align_corners)), interp, _stream(inputs)),
        "grid_encode_forward")


def grid_encode_backward(grad, inputs, embeddings, offsets, grad_embeddings, B, D, C, L,
                         max_level, S, H, dy_dx, grad_inputs, gridtype, align_corners, interp):
    _float_tensor(grad, "grad")
    _float_tensor(inputs, "inputs")
    _float_tensor(embeddings, "embeddings")
    _cuda(offsets, "offsets"); _contig(offsets, "offsets"); _i32(offsets, "offsets")
    _float_tensor(grad_embeddings, "grad_embeddings")
    check(lib().samnerf_grid_encode_backward(
        _ptr(grad), _ptr(inputs), _ptr(embeddings), _ptr(offsets), _ptr(grad_embeddings), B, D,
        C, L, max_level, float(S), H, _ptr(dy_dx), _ptr(grad_inputs), gridtype,
        int(bool(align_corners)), interp, _stream(grad)), "grid_encode_backward")


def grad_total_variation(inputs, embeddings, grad, offsets, weight, B, D, C, L, S, H, gridtype,
                         align_corners):
    _float_tensor(inputs, "inputs")
    _float_tensor(embeddings, "embeddings", vec=True)
    _float_tensor(grad, "grad")
    _cuda(offsets, "offsets"); _i32(offsets, "offsets")
    check(lib().samnerf_grad_total_variation(
        _ptr(inputs), _ptr(embeddings), _ptr(grad), _ptr(offsets), float(weight), B, D, C, L,
        float(S), H, gridtype, int(bool(align_corners)), _stream(inputs)), "grad_total_variation")


def grad_weight_decay(embeddings, grad, offsets, weight, B, C, L):
    _float_tensor(embeddings, "embeddings")
    _float_tensor(grad, "grad")
    _cuda(offsets, "offsets"); _i32(offsets, "offsets")
    check(lib().samnerf_grad_weight_decay(_ptr(embeddings), _ptr(grad), _ptr(offsets),
                                          float(weight), B, C, L, _stream(embeddings)),
          "grad_weight_decay")


# ---------------------------------------------------------------- shencoder --

def sh_encode_forward(inputs, outputs, B, D, C, dy_dx):
    _float_tensor(inputs, "inputs")
    _float_tensor(outputs, "outputs")
    if dy_dx is not None:
        _float_tensor(dy_dx, "dy_dx")
    check(lib().samnerf_sh_encode_forward(_ptr(inputs), _ptr(outputs), B, D, C, _ptr(dy_dx),
                                          _stream(inputs)), "sh_encode_forward")


def sh_encode_backward(grad, inputs, B, D, C, dy_dx, grad_inputs):
    for t, n in ((grad, "grad"), (inputs, "inputs"), (dy_dx, "dy_dx"), (grad_inputs, "grad_inputs")):
        _float_tensor(t, n)
    check(lib().samnerf_sh_encode_backward(_ptr(grad), _ptr(inputs), B, D, C, _ptr(dy_dx),
                                           _ptr(grad_inputs), _stream(grad)), "sh_encode_backward")


# -------------------------------------------------------------- freqencoder --

def freq_encode_forward(inputs, B, D, deg, C, outputs):
    _float_tensor(inputs, "inputs")
    _float_tensor(outputs, "outputs")
    check(lib().samnerf_freq_encode_forward(_ptr(inputs), B, D, deg, C, _ptr(outputs),
                                            _stream(inputs)), "freq_encode_forward")


def freq_encode_backward(grad, outputs, B, D, deg, C, grad_inputs):
    for t, n in ((grad, "grad"), (outputs, "outputs"), (grad_inputs, "grad_inputs")):
        _float_tensor(t, n)
    check(lib().samnerf_freq_encode_backward(_ptr(grad), _ptr(outputs), B, D, deg, C,
                                             _ptr(grad_inputs), _stream(grad)),
          "freq_encode_backward")


# ------------------------------------------------------------ step kernels --

def get_rays(pose, intrinsics, H, W, device="cuda", row0=0, rows=None):
    """Full-image rays (nerf/utils.py:145-279, N=-1) for pixel rows
    [row0, row0+rows): returns rays_o, rays_d [rows*W, 3] on `device`."""
    import numpy as np
    rows = H - row0 if rows is None else rows
    p = np.ascontiguousarray(np.asarray(pose, np.float32).reshape(4, 4))
    fx, fy, cx, cy = [float(v) for v in np.asarray(intrinsics, np.float32).reshape(4)]
    ro = torch.empty(rows * W, 3, device=device)
    rd = torch.empty(rows * W, 3, device=device)
    check(lib().samnerf_get_rays(p.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), fx, fy, cx,
                                 cy, H, W, row0, rows, _ptr(ro), _ptr(rd), _stream(ro)),
          "get_rays")
    return ro, rd


def near_far(rays_o, rays_d, aabb, min_near):
    N = rays_o.shape[0]
    box = (ctypes.c_float * 6)(*[float(v) for v in aabb])
    n = torch.empty(N, 1, device=rays_o.device)
    f = torch.empty(N, 1, device=rays_o.device)
    ro, rd = rays_o.contiguous(), rays_d.contiguous()      # held until the launch: _ptr keeps no reference
    check(lib().samnerf_near_far(_ptr(ro), _ptr(rd), N, box,
                                 float(min_near), _ptr(n), _ptr(f), _stream(rays_o)), "near_far")
    return n, f


def contract(x):
    x = x.contiguous()
    z = torch.empty_like(x)
    check(lib().samnerf_contract(_ptr(x), _ptr(z), x.numel() // 3, _stream(x)), "contract")
    return z


def sample_pdf(bins, weights, T, return_inds=False):
    bins = bins.contiguous()
    weights = weights.contiguous()
    N, T0 = weights.shape
    out = torch.empty(N, T, device=bins.device)
    inds = torch.empty(N, T, device=bins.device, dtype=torch.int32) if return_inds else None
    check(lib().samnerf_sample_pdf(_ptr(bins), _ptr(weights), N, T0, T, _ptr(out), _ptr(inds),
                                   _stream(bins)), "sample_pdf")
    return (out, inds) if return_inds else out


def composite_weights(real_bins, sigmas):
    real_bins = real_bins.contiguous()
    sigmas = sigmas.contiguous()
    N, T = sigmas.shape
    w = torch.empty(N, T, device=sigmas.device)
    check(lib().samnerf_composite_weights(_ptr(real_bins), _ptr(sigmas), N, T, _ptr(w),
                                          _stream(sigmas)), "composite_weights")
    return w


def linspace_host(start, end, steps):
    buf = (ctypes.c_float * steps)()
    lib().samnerf_linspace_host(float(start), float(end), steps, buf)
    return list(buf)


def tile_words():
    return int(lib().samnerf_tile_words())


def tile_encode(out):
    """Per-ray render outputs (image [N,3], depth [N], weights_sum [N], samvit
    [N,256]) -> transport records [N, tile_words()] int32 (tile_codec.hip)."""
    t = {k: out[k].contiguous() for k in ("image", "depth", "weights_sum", "samvit")}
    for k, v in t.items():
        _f32(v, k)
        _cuda(v, k)
    N = t["depth"].shape[0]
    if t["samvit"].shape != (N, 256) or t["image"].shape != (N, 3) or t["weights_sum"].shape != (N,):
        raise RuntimeError("tile_encode: expected image [N,3], depth [N], weights_sum [N], samvit [N,256]")
    tile = torch.empty(N, tile_words(), dtype=torch.int32, device=t["depth"].device)
    check(lib().samnerf_tile_encode(_ptr(t["image"]), _ptr(t["depth"]), _ptr(t["weights_sum"]),
                                    _ptr(t["samvit"]), N, _ptr(tile), _stream(tile)), "tile_encode")
    return tile


def tile_decode(tile):
    """Inverse of tile_encode: records [N, tile_words()] int32 -> dict of fp32 outputs."""
    _cuda(tile, "tile")
    _contig(tile, "tile")
    if tile.dtype != torch.int32 or tile.dim() != 2 or tile.shape[1] != tile_words():
        raise RuntimeError(f"tile_decode: expected an int32 [N, {tile_words()}] tensor")
    N, dev = tile.shape[0], tile.device
    out = {"image": torch.empty(N, 3, device=dev), "depth": torch.empty(N, device=dev),
           "weights_sum": torch.empty(N, device=dev), "samvit": torch.empty(N, 256, device=dev)}
    check(lib().samnerf_tile_decode(_ptr(tile), N, _ptr(out["image"]), _ptr(out["depth"]),
                                    _ptr(out["weights_sum"]), _ptr(out["samvit"]), _stream(tile)),
          "tile_decode")
    return out
