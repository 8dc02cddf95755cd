"""numpy restatement of the multi-GPU transport record (tile_codec.hip) --
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference renders a view on one GPU (nerf/renderer.py:185-219) and has no
transport format; the record exists for the all-gather of a ray-sharded view
(SURVEY.md 8e).  Parity for it is against its own stated error bound on the
fp32 outputs: image / depth / weights_sum round-trip exactly, samvit within
s = 2^(E-15) per element where max|samvit| of the ray is in [2^(E-1), 2^E).
"""
import numpy as np

WORDS = 134


def encode(image, depth, wsum, samvit):
    """-> int32 [N, 134]: image[3], depth, wsum, s (fp32 bits), 256 int16."""
    samvit = np.ascontiguousarray(samvit, np.float32)
    N = samvit.shape[0]
    rec = np.zeros((N, WORDS), np.int32)
    rec[:, 0:3] = np.ascontiguousarray(image, np.float32).view(np.int32)
    rec[:, 3] = np.ascontiguousarray(depth, np.float32).view(np.int32)
    rec[:, 4] = np.ascontiguousarray(wsum, np.float32).view(np.int32)
    mag = (samvit.view(np.uint32) & np.uint32(0x7FFFFFFF)).max(axis=1) if N else np.zeros(0, np.uint32)
    bad = mag >= 0x7F800000                                # inf / NaN in the ray
    amax = np.where(bad, 0, mag).astype(np.uint32).view(np.float32)
    _, e = np.frexp(amax)                                  # amax in [2^(e-1), 2^e); 0 -> 0
    e = np.maximum(e, -100).astype(np.int64)
    s = np.ldexp(np.float32(1), (e - 15)).astype(np.float32)
    inv = np.ldexp(np.float32(1), (15 - e)).astype(np.float32)
    s = np.where(bad, np.float32(np.nan), s).astype(np.float32)
    inv = np.where(bad, np.float32(0), inv).astype(np.float32)
    with np.errstate(invalid="ignore"):
        q = np.rint(samvit * inv[:, None])                 # exact power-of-two scaling
        q = np.where(np.isnan(q), -32767.0, np.clip(q, -32767.0, 32767.0))
    rec[:, 5] = s.view(np.int32)
    rec[:, 6:] = q.astype(np.int16).view(np.int32)         # little-endian int16 pairs
    return rec


def decode(rec):
    rec = np.ascontiguousarray(rec, np.int32)
    s = rec[:, 5].copy().view(np.float32)
    q = rec[:, 6:].copy().view(np.int16).astype(np.float32)
    return {"image": rec[:, 0:3].copy().view(np.float32), "depth": rec[:, 3].copy().view(np.float32),
            "weights_sum": rec[:, 4].copy().view(np.float32), "samvit": q * s[:, None]}


def error_bound(samvit):
    """Per-ray bound s = 2^(E-15) on |samvit - decode(encode(samvit))|."""
    samvit = np.asarray(samvit, np.float32)
    amax = np.abs(samvit).max(axis=1)
    _, e = np.frexp(amax)
    return np.ldexp(np.float32(1), np.maximum(e, -100) - 15).astype(np.float32)
