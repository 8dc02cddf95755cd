"""Transport record of the ray-sharded all-gather (tile_codec.hip,
samnerf_amd/dist.py ShardedViewPipeline(codec="q16")).

CPU: the numpy restatement (oracle/tile_codec.py) against its stated bound.
GPU: the HIP encoder / decoder bit-exact against the restatement, the round
trip of a real render within 2^-14 of each ray's max |samvit| (north star
budget 1e-3), and the pipeline's own band kept exact."""
import numpy as np
import pytest
import torch

from oracle import tile_codec as oc


def _cases(n=257, seed=0):
    rng = np.random.default_rng(seed)
    sv = rng.standard_normal((n, 256)).astype(np.float32)
    sv[1] = 0.0                                             # all-zero ray
    sv[2] *= 1e-35                                          # tiny (E clamp region)
    sv[3] *= 3e4                                            # large magnitudes
    sv[4, :] = 0.0
    sv[4, 7] = 1.0 - 2.0 ** -24                             # rounds to the clamp at 32767
    sv[4, 8] = -(1.0 - 2.0 ** -24)
    sv[5, 3] = np.nan                                       # NaN ray
    sv[6, 9] = np.inf
    sv[7, :] = 2.0 ** np.arange(-8, 8, 1.0 / 16)[:256].astype(np.float32)
    img = rng.random((n, 3), dtype=np.float32)
    depth = rng.random(n, dtype=np.float32) * 10
    ws = rng.random(n, dtype=np.float32)
    return img, depth, ws, sv


def test_oracle_round_trip_within_bound():
    img, depth, ws, sv = _cases()
    rec = oc.encode(img, depth, ws, sv)
    assert rec.shape == (257, 134) and rec.dtype == np.int32
    out = oc.decode(rec)
    assert np.array_equal(out["image"], img) and np.array_equal(out["depth"], depth)
    assert np.array_equal(out["weights_sum"], ws)
    fin = np.isfinite(sv).all(axis=1)
    err = np.abs(out["samvit"][fin] - sv[fin]).max(axis=1)
    assert (err <= oc.error_bound(sv[fin])).all()
    amax = np.abs(sv[fin]).max(axis=1)
    big = amax >= 2.0 ** -100                               # below that E is clamped (error < 2^-115)
    assert (oc.error_bound(sv[fin])[big] <= amax[big] * 2.0 ** -14).all()
    assert (err[~big] <= 2.0 ** -115).all()
    assert np.isnan(out["samvit"][~fin]).all()
    assert np.array_equal(out["samvit"][1], np.zeros(256, np.float32))
    # 536 B per ray against 1,044 B of fp32 outputs
    assert rec.itemsize * rec.shape[1] == 536


def test_oracle_empty():
    rec = oc.encode(np.zeros((0, 3)), np.zeros(0), np.zeros(0), np.zeros((0, 256)))
    assert rec.shape == (0, 134)


@pytest.mark.gpu
def test_hip_codec_bit_exact_vs_oracle(hip_lib, cuda):
    from samnerf_amd import ops
    img, depth, ws, sv = _cases(1027, seed=1)
    dev = cuda
    out = {"image": torch.from_numpy(img).to(dev), "depth": torch.from_numpy(depth).to(dev),
           "weights_sum": torch.from_numpy(ws).to(dev), "samvit": torch.from_numpy(sv).to(dev)}
    assert ops.tile_words() == oc.WORDS
    rec = ops.tile_encode(out)
    torch.cuda.synchronize()
    assert np.array_equal(rec.cpu().numpy(), oc.encode(img, depth, ws, sv))
    dec = ops.tile_decode(rec)
    ref = oc.decode(oc.encode(img, depth, ws, sv))
    for k in ref:
        np.testing.assert_array_equal(dec[k].cpu().numpy(), ref[k])
    empty = {k: v[:0] for k, v in out.items()}
    assert ops.tile_encode(empty).shape == (0, 134)


@pytest.mark.gpu
def test_hip_codec_round_trip_of_a_render(hip_lib, cuda):
    from samnerf_amd import ops
    from samnerf_amd.fused import FusedRenderer
    from helpers import make_net
    from oracle import synth
    spec = synth.ModelSpec(with_sam=True, grid_log2=14, s_grid_log2=14, prop_log2=12)
    params = synth.make_params(spec, seed=8, emb_scale=0.5, ln_jitter=0.1)
    net = make_net(spec, params, cuda)
    pose, intr = synth.gui_camera(64, 64, rot=synth.random_rotation(2))
    ro, rd = ops.get_rays(pose, intr, 64, 64, device=cuda)
    out = FusedRenderer(net).render(ro, rd)
    dec = ops.tile_decode(ops.tile_encode(out))
    for k in ("image", "depth", "weights_sum"):
        assert torch.equal(dec[k], out[k])
    sv = out["samvit"]
    err = (dec["samvit"] - sv).abs().amax(dim=1)
    assert (err <= sv.abs().amax(dim=1) * 2.0 ** -14).all()
    assert err.max().item() < 1e-3                         # the north star's feature budget


@pytest.mark.gpu
def test_pipeline_q16_keeps_own_band_exact(hip_lib, cuda, tmp_path):
    """World size 1 over gloo with CUDA tensors (staged through the host, as in
    the single-GPU rehearsal of the multi-rank bench): the whole view is the
    rank's own band, so the decoded result must equal the render exactly; the
    encode -> gather -> decode path runs all the same."""
    import torch.distributed as dist
    from samnerf_amd.dist import ShardedViewPipeline
    g = torch.Generator(device="cpu").manual_seed(3)
    H, W = 8, 16
    made = []

    def render_fn(ro, rd):
        n = ro.shape[0]
        o = {"image": torch.rand(n, 3, generator=g), "depth": torch.rand(n, generator=g),
             "weights_sum": torch.rand(n, generator=g), "samvit": torch.randn(n, 256, generator=g)}
        o = {k: v.to(cuda) for k, v in o.items()}
        made.append(o)
        return o

    def ray_fn(row0, rows):
        return torch.zeros(rows * W, 3, device=cuda), torch.zeros(rows * W, 3, device=cuda)

    dist.init_process_group("gloo", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1)
    try:
        pipe = ShardedViewPipeline(render_fn, H, W, codec="q16")
        pipe.submit(ray_fn)
        pipe.submit(ray_fn)
        outs = pipe.flush()
        assert len(outs) == 2
        for res, ref in zip(outs, made):
            for k in ref:
                assert torch.equal(res[k], ref[k]), k
        with pytest.raises(ValueError):
            ShardedViewPipeline(render_fn, H, W, codec="fp16")
    finally:
        dist.destroy_process_group()


def _q16_worker(rank, world, port, q):
    """One rank of a world-2 gloo group on GPU 0 (both ranks share the card,
    as in the single-GPU rehearsal of the multi-rank bench)."""
    import os
    import sys
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "segment-anything-nerf_amd"))
        from samnerf_amd.dist import ShardedViewPipeline
        dev = torch.device("cuda", 0)
        H, W = 8, 12

        def band(r, n):                      # rank r's outputs, reproducible on every rank
            g = torch.Generator().manual_seed(100 + r)
            return {"image": torch.rand(n, 3, generator=g), "depth": torch.rand(n, generator=g),
                    "weights_sum": torch.rand(n, generator=g),
                    "samvit": torch.randn(n, 256, generator=g) * (1 + 3 * r)}

        def render_fn(ro, rd):
            return {k: v.to(dev) for k, v in band(rank, ro.shape[0]).items()}

        def ray_fn(row0, rows):
            return torch.zeros(rows * W, 3, device=dev), torch.zeros(rows * W, 3, device=dev)

        pipe = ShardedViewPipeline(render_fn, H, W, codec="q16")
        pipe.submit(ray_fn)
        (res,) = pipe.flush()
        n = H * W // world
        ok = True
        for r in range(world):
            ref = band(r, n)
            got = {k: v[r * n:(r + 1) * n].cpu() for k, v in res.items()}
            for k in ("image", "depth", "weights_sum"):
                ok &= torch.equal(got[k], ref[k])
            if r == rank:
                ok &= torch.equal(got["samvit"], ref["samvit"])        # own band exact
            else:
                err = (got["samvit"] - ref["samvit"]).abs().amax(dim=1)
                ok &= bool((err <= ref["samvit"].abs().amax(dim=1) * 2.0 ** -14).all())
                ok &= not torch.equal(got["samvit"], ref["samvit"])    # it did go through q16
        q.put((rank, bool(ok)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_pipeline_q16_world2_gloo_on_one_gpu(hip_lib, cuda):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_q16_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok in res:
        assert ok is True, f"rank {rank}: {ok}"
