"""Child process of tests/test_gpu_render.py::test_final_forms_deterministic.

usage: python tests/final_forms_child.py SEG HEAD_MODE
Renders one k_final form (SAMNERF_FINAL_S = SEG segments per ray, head_mode)
three times in this fresh process -- the first render of a process is the one
the removed round-4 prefetch form got wrong -- and prints one
"digest <sha256>" line per render over every output (image, depth,
weights_sum, samvit, the head-input rows).  Needs the diagnostic build
(libsamnerf_hip_diag.so), which reads SAMNERF_FINAL_S.
"""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (os.path.join(REPO, "segment-anything-nerf_amd"), REPO, HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def _scene(head_mode, device):
    from helpers import make_net
    from oracle import synth
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec = synth.ModelSpec(with_sam=True)
    net = make_net(spec, synth.make_params(spec, seed=23, emb_scale=0.5, ln_jitter=0.1), device)
    pose, intr = synth.gui_camera(512, 80, rot=synth.random_rotation(11))
    ro, rd = ops.get_rays(pose, intr, 80, 512, device=device)
    return FusedRenderer(net, head_mode=head_mode), ro, rd


def _digest(fr, ro, rd):
    import torch
    from samnerf_amd.fused import ROW
    rows = torch.empty(ro.shape[0], ROW, device=ro.device)
    o = fr.render(ro, rd, rows=rows, view_width=512)
    o["rows"] = rows
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for k in sorted(o):
        h.update(k.encode())
        h.update(o[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def render_digest(seg, head_mode, device, times=1):
    """Digests of `times` renders of the form (diagnostic build, SAMNERF_FINAL_S = seg)."""
    from samnerf_amd._lib import diag_library
    prev = os.environ.get("SAMNERF_FINAL_S")
    os.environ["SAMNERF_FINAL_S"] = str(seg)
    try:
        with diag_library():
            fr, ro, rd = _scene(int(head_mode), device)
            out = [_digest(fr, ro, rd) for _ in range(times)]
    finally:
        if prev is None:
            os.environ.pop("SAMNERF_FINAL_S", None)
        else:
            os.environ["SAMNERF_FINAL_S"] = prev
    return out[0] if times == 1 else out


if __name__ == "__main__":
    import torch
    for d in render_digest(sys.argv[1], int(sys.argv[2]), torch.device("cuda:0"), times=3):
        print("digest", d, flush=True)
