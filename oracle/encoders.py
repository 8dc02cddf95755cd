"""ctypes binding of oracle/encoders_oracle.c (test infrastructure only).

Each function mirrors the reference's pybind entry point of the same name
(gridencoder/src/gridencoder.h:12-16, shencoder/src/shencoder.h:9-10,
freqencoder/src/freqencoder.h:7-10) but runs on host memory.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsamnerf_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u32 = ctypes.c_uint32


def build():
    """Compile the C oracle (gcc, a few seconds)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_grid_encode_forward.argtypes = [
            _f32p, _f32p, _i32p, _f32p, _u32, _u32, _u32, _u32, _u32,
            ctypes.c_float, _u32, _f32p, _u32, ctypes.c_int, _u32, _u32p]
        L.oracle_grid_encode_backward.argtypes = [
            _f32p, _f32p, _f32p, _i32p, _f32p, _u32, _u32, _u32, _u32, _u32,
            ctypes.c_float, _u32, _f32p, _f32p, _u32, ctypes.c_int, _u32]
        L.oracle_grad_total_variation.argtypes = [
            _f32p, _f32p, _f32p, _i32p, ctypes.c_float, _u32, _u32, _u32, _u32,
            ctypes.c_float, _u32, _u32, ctypes.c_int]
        L.oracle_grad_weight_decay.argtypes = [
            _f32p, _f32p, _i32p, ctypes.c_float, _u32, _u32, _u32]
        L.oracle_sh_encode_forward.argtypes = [_f32p, _f32p, _u32, _u32, _u32, _f32p]
        L.oracle_sh_encode_backward.argtypes = [_f32p, _f32p, _u32, _u32, _u32, _f32p, _f32p]
        L.oracle_freq_encode_forward.argtypes = [_f32p, _u32, _u32, _u32, _u32, _f32p]
        L.oracle_freq_encode_backward.argtypes = [_f32p, _f32p, _u32, _u32, _u32, _u32, _f32p]
        _lib = L
    return _lib


def _c(a, dtype=np.float32):
    a = np.ascontiguousarray(a, dtype=dtype)
    return a


def _p(a, ptype=_f32p):
    if a is None:
        return None
    return a.ctypes.data_as(ptype)


def grid_level_resolutions(L, S, H):
    """Indexing resolutions, float32 formula of gridencoder.cu:133."""
    S32 = np.float32(S)
    return [int(np.ceil(np.float32(np.exp2(np.float32(l) * S32)) * np.float32(H))) for l in range(L)]


def grid_encode_forward(inputs, embeddings, offsets, L, S, H, max_level=None,
                        calc_dy_dx=False, gridtype=0, align_corners=False, interp=0,
                        return_rows=False):
    """inputs [B, D] in [0,1]; returns outputs [L, B, C] (and dy_dx [B, L*D*C],
    corner rows [L, B, 2^D] uint32 when requested)."""
    inputs = _c(inputs)
    embeddings = _c(embeddings)
    offsets = _c(offsets, np.int32)
    B, D = inputs.shape
    C = embeddings.shape[1]
    max_level = L if max_level is None else min(max_level, L)
    out = np.zeros((L, B, C), np.float32)
    dy = np.zeros((B, L * D * C), np.float32) if calc_dy_dx else None
    rows = np.zeros((L, B, 1 << D), np.uint32) if return_rows else None
    lib().oracle_grid_encode_forward(
        _p(inputs), _p(embeddings), _p(offsets, _i32p), _p(out), B, D, C, L, max_level,
        float(np.float32(S)), H, _p(dy), gridtype, int(bool(align_corners)), interp,
        _p(rows, _u32p))
    res = [out]
    if calc_dy_dx:
        res.append(dy)
    if return_rows:
        res.append(rows)
    return res[0] if len(res) == 1 else tuple(res)


def grid_encode_backward(grad_lbc, inputs, embeddings, offsets, L, S, H, max_level=None,
                         dy_dx=None, gridtype=0, align_corners=False, interp=0):
    grad_lbc = _c(grad_lbc)
    inputs = _c(inputs)
    embeddings = _c(embeddings)
    offsets = _c(offsets, np.int32)
    B, D = inputs.shape
    C = embeddings.shape[1]
    max_level = L if max_level is None else min(max_level, L)
    gemb = np.zeros_like(embeddings)
    gin = np.zeros_like(inputs) if dy_dx is not None else None
    if dy_dx is not None:
        dy_dx = _c(dy_dx)
    lib().oracle_grid_encode_backward(
        _p(grad_lbc), _p(inputs), _p(embeddings), _p(offsets, _i32p), _p(gemb), B, D, C, L,
        max_level, float(np.float32(S)), H, _p(dy_dx), _p(gin), gridtype,
        int(bool(align_corners)), interp)
    return (gemb, gin) if dy_dx is not None else gemb


def grad_total_variation(inputs, embeddings, grad, offsets, weight, L, S, H, gridtype=0,
                         align_corners=False):
    inputs = _c(inputs)
    embeddings = _c(embeddings)
    grad = _c(grad).copy()
    offsets = _c(offsets, np.int32)
    B, D = inputs.shape
    C = embeddings.shape[1]
    lib().oracle_grad_total_variation(
        _p(inputs), _p(embeddings), _p(grad), _p(offsets, _i32p), float(weight), B, D, C, L,
        float(np.float32(S)), H, gridtype, int(bool(align_corners)))
    return grad


def grad_weight_decay(embeddings, grad, offsets, weight, L):
    embeddings = _c(embeddings)
    grad = _c(grad).copy()
    offsets = _c(offsets, np.int32)
    rows, C = embeddings.shape
    lib().oracle_grad_weight_decay(_p(embeddings), _p(grad), _p(offsets, _i32p),
                                   float(weight), rows, C, L)
    return grad


def sh_encode_forward(inputs, degree, calc_dy_dx=False):
    inputs = _c(inputs)
    B, D = inputs.shape
    out = np.zeros((B, degree * degree), np.float32)
    dy = np.zeros((B, D * degree * degree), np.float32) if calc_dy_dx else None
    lib().oracle_sh_encode_forward(_p(inputs), _p(out), B, D, degree, _p(dy))
    return (out, dy) if calc_dy_dx else out


def sh_encode_backward(grad, inputs, degree, dy_dx):
    grad = _c(grad)
    inputs = _c(inputs)
    dy_dx = _c(dy_dx)
    B, D = inputs.shape
    gin = np.zeros_like(inputs)
    lib().oracle_sh_encode_backward(_p(grad), _p(inputs), B, D, degree, _p(dy_dx), _p(gin))
    return gin


def freq_encode_forward(inputs, degree):
    inputs = _c(inputs)
    B, D = inputs.shape
    C = D + 2 * D * degree
    out = np.zeros((B, C), np.float32)
    lib().oracle_freq_encode_forward(_p(inputs), B, D, degree, C, _p(out))
    return out


def freq_encode_backward(grad, outputs, degree):
    grad = _c(grad)
    outputs = _c(outputs)
    B, C = outputs.shape
    D = C // (1 + 2 * degree)
    gin = np.zeros((B, D), np.float32)
    lib().oracle_freq_encode_backward(_p(grad), _p(outputs), B, D, degree, C, _p(gin))
    return gin
