"""The ray-sharded view (BASELINE config 4) with the real fused
renderer: a world-2 gloo group whose ranks share GPU 0 (a one-GPU box's
rehearsal of the multi-GPU bench), each rendering its 64-row band of a
128x512 view through FusedRenderer and ShardedViewPipeline.

Under the fp32 transport the gathered view must equal, bit for bit, the same
bands rendered by one process (the same kernels run at the same launch size);
under q16 each rank's own band is exact and the other band's samvit within
the codec's bound (2^-14 of the ray's max |samvit|, tile_codec.hip).

The RCCL branch of the gather (`nccl` backend: all_gather_into_tensor on
RCCL's stream, asynchronous behind the next view) runs here in a world-1
group on the box's one GPU (two RCCL ranks may not share a device); the 8-GPU
bench runs it at world 8.
"""
import os
import socket

import pytest
import torch

from helpers import make_net
from oracle import synth

pytestmark = pytest.mark.gpu

H, W = 128, 512
KEYS = ("image", "depth", "weights_sum", "samvit")


def _setup():
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=41, emb_scale=0.5, ln_jitter=0.1)
    pose, intr = synth.gui_camera(W, H, rot=synth.random_rotation(6))
    return spec, params, pose, intr


def _worker(rank, world, port, codec, out_path, q, backend="gloo"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from samnerf_amd import ops
        from samnerf_amd.dist import ShardedViewPipeline
        from samnerf_amd.fused import FusedRenderer
        assert dist.get_backend() == backend
        spec, params, pose, intr = _setup()
        fr = FusedRenderer(make_net(spec, params, dev))

        def ray_fn(row0, rows):
            return ops.get_rays(pose, intr, H, W, device=dev, row0=row0, rows=rows)

        pipe = ShardedViewPipeline(fr.render, H, W, codec=codec)
        pipe.submit(ray_fn)               # two views in flight: view 0's gather
        pipe.submit(ray_fn)               # runs behind view 1's kernels
        outs = pipe.flush()
        torch.cuda.synchronize()
        same = all(torch.equal(outs[0][k], outs[1][k]) for k in KEYS)
        if rank == 0:
            torch.save({k: v.cpu() for k, v in outs[1].items()}, out_path)
        q.put((rank, bool(same)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run_world2(codec, path, world=2, backend="gloo"):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, codec, path, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok in res:
        assert ok is True, f"rank {rank}: {ok} (views differ between pipeline slots or the rank failed)"
    return torch.load(path, weights_only=True)


def _single_process_bands(cuda):
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec, params, pose, intr = _setup()
    fr = FusedRenderer(make_net(spec, params, cuda))
    parts = []
    for b in range(2):
        ro, rd = ops.get_rays(pose, intr, H, W, device=cuda, row0=b * (H // 2), rows=H // 2)
        parts.append({k: v.cpu() for k, v in fr.render(ro, rd).items()})
    full = {k: torch.cat([p[k] for p in parts]) for k in KEYS}
    ro, rd = ops.get_rays(pose, intr, H, W, device=cuda)
    whole = {k: v.cpu() for k, v in fr.render(ro, rd).items()}
    return full, whole


@pytest.mark.parametrize("codec", ["fp32", "q16"])
def test_sharded_view_real_renderer_world2(hip_lib, cuda, tmp_path, codec):
    got = _run_world2(codec, str(tmp_path / f"view_{codec}.pt"))
    ref, whole = _single_process_bands(cuda)
    n = H * W // 2
    for k in KEYS:
        assert got[k].shape == ref[k].shape, k
        if codec == "fp32" or k != "samvit":
            assert torch.equal(got[k], ref[k]), (codec, k, (got[k] - ref[k]).abs().max().item())
        else:
            assert torch.equal(got[k][:n], ref[k][:n])               # rank 0's own band
            err = (got[k][n:] - ref[k][n:]).abs().amax(dim=1)
            bound = ref[k][n:].abs().amax(dim=1) * 2.0 ** -14
            assert bool((err <= bound).all()), (err - bound).max().item()
    # one launch over the whole view (other ray-segment form S in k_final):
    # the same values to fp32 rounding
    for k in KEYS:
        tol = 1e-4 * (1 + ref[k].abs().max().item()) if k == "depth" else 1e-4
        assert (whole[k] - ref[k]).abs().max().item() < tol, k


@pytest.mark.parametrize("codec", ["fp32", "q16"])
def test_sharded_view_rccl_branch_world1(hip_lib, cuda, tmp_path, codec):
    """The `nccl` (RCCL) gather path of ShardedViewPipeline on the GPU: a
    world-1 group renders the whole view as its band; the gathered outputs
    equal the one-launch render bit for bit (q16: its own band is restored
    exactly, so also bit for bit)."""
    got = _run_world2(codec, str(tmp_path / f"rccl_{codec}.pt"), world=1, backend="nccl")
    _, whole = _single_process_bands(cuda)
    for k in KEYS:
        assert torch.equal(got[k], whole[k]), (codec, k, (got[k] - whole[k]).abs().max().item())


# ----------------------------------------------------------------- cfg 4 --
# BASELINE config 4: the 512x512 --with_sam view in 8 row bands of 64 rows
# (32,768 rays), one band per rank, each rank rendering straight into its
# slice of the gather buffer (samnerf_render_forward_tile, tile_cols=261).
H4 = W4 = 512
BANDS = 8


def _setup4():
    spec = synth.ModelSpec(with_sam=True)
    params = synth.make_params(spec, seed=44, emb_scale=0.5, ln_jitter=0.1)
    pose, intr = synth.gui_camera(W4, H4, rot=synth.random_rotation(7))
    return spec, params, pose, intr


def _worker4(rank, world, port, out_path, q, backend, rows_total):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from samnerf_amd import ops
        from samnerf_amd.dist import ShardedViewPipeline
        from samnerf_amd.fused import FusedRenderer
        spec, params, pose, intr = _setup4()
        fr = FusedRenderer(make_net(spec, params, dev))

        def ray_fn(row0, rows):
            return ops.get_rays(pose, intr, H4, W4, device=dev, row0=row0, rows=rows)

        def render_fn(ro, rd, out_tile=None):
            return fr.render(ro, rd, view_width=W4, out_tile=out_tile)

        pipe = ShardedViewPipeline(render_fn, rows_total, W4, tile_cols=261)
        pipe.submit(ray_fn)
        pipe.submit(ray_fn)
        outs = pipe.flush()
        torch.cuda.synchronize()
        same = all(torch.equal(outs[0][k], outs[1][k]) for k in KEYS)
        if rank == 0:
            torch.save({k: v.cpu() for k, v in outs[1].items()}, out_path)
        q.put((rank, bool(same)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _run4(path, world, backend, rows_total):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker4, args=(r, world, port, path, q, backend, rows_total))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=115) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok in res:
        assert ok is True, f"rank {rank}: {ok}"
    return torch.load(path, weights_only=True)


def _bands4(cuda, bands):
    """The same bands rendered one after another by one process (the same
    launch size, 32,768 rays, as each rank's), and the whole view in one launch."""
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    spec, params, pose, intr = _setup4()
    fr = FusedRenderer(make_net(spec, params, cuda))
    band = H4 // BANDS
    parts = []
    for b in range(bands):
        ro, rd = ops.get_rays(pose, intr, H4, W4, device=cuda, row0=b * band, rows=band)
        parts.append({k: v.cpu() for k, v in fr.render(ro, rd, view_width=W4).items()})
    ro, rd = ops.get_rays(pose, intr, H4, W4, device=cuda)
    whole = {k: v.cpu() for k, v in fr.render(ro, rd, view_width=W4).items()}
    return {k: torch.cat([p[k] for p in parts]) for k in KEYS}, whole


def test_cfg4_eight_bands_world8_gloo(hip_lib, cuda, tmp_path):
    """BASELINE config 4's layout on the one-GPU box: a world-8 gloo group
    (8 processes on GPU 0), rank r rendering rows [64 r, 64 r + 64) of the
    512x512 view into its slice of the gather buffer.  The gathered view
    equals the 8 bands rendered by one process bit for bit, and the one-launch
    render of the whole view to fp32 rounding (another ray-segment form)."""
    got = _run4(str(tmp_path / "cfg4_gloo.pt"), BANDS, "gloo", H4)
    ref, whole = _bands4(cuda, BANDS)
    for k in KEYS:
        assert got[k].shape == ref[k].shape, k
        assert torch.equal(got[k], ref[k]), (k, (got[k] - ref[k]).abs().max().item())
        tol = 1e-4 * (1 + whole[k].abs().max().item()) if k == "depth" else 1e-4
        assert (whole[k] - ref[k]).abs().max().item() < tol, k


def test_cfg4_band_rccl_world1(hip_lib, cuda, tmp_path):
    """The RCCL path (all_gather_into_tensor in place on the gather buffer) at
    one rank's 32,768-ray band: a world-1 `nccl` group renders rows 0-63 into
    the buffer; bit for bit the one-process render of that band."""
    got = _run4(str(tmp_path / "cfg4_rccl.pt"), 1, "nccl", H4 // BANDS)
    ref, _ = _bands4(cuda, 1)
    for k in KEYS:
        assert torch.equal(got[k], ref[k]), (k, (got[k] - ref[k]).abs().max().item())
