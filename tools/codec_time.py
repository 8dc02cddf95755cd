"""Time the all-gather transport codec (tile_codec.hip) on one 512x512 view's
outputs: encode of one rank's band, decode of the whole view."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "segment-anything-nerf_amd"))
from samnerf_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
N = 512 * 512
out = {"image": torch.rand(N, 3, device=dev), "depth": torch.rand(N, device=dev),
       "weights_sum": torch.rand(N, device=dev), "samvit": torch.randn(N, 256, device=dev)}
res = {}
for n in (N // 8, N // 4, N // 2, N):
    band = {k: v[:n].contiguous() for k, v in out.items()}
    for _ in range(3):
        rec = ops.tile_encode(band)
        ops.tile_decode(rec)
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    reps = 20
    e0.record()
    for _ in range(reps):
        rec = ops.tile_encode(band)
    e1.record()
    for _ in range(reps):
        dec = ops.tile_decode(rec)
    e2.record()
    torch.cuda.synchronize()
    te, td = e0.elapsed_time(e1) / reps, e1.elapsed_time(e2) / reps
    err = (dec["samvit"] - band["samvit"]).abs().max().item()
    res[n] = {"encode_ms": te, "decode_ms": td,
              "encode_GBps": n * (1044 + 536) / te / 1e6, "decode_GBps": n * (1044 + 536) / td / 1e6,
              "max_abs_err": err}
print(json.dumps(res))
