"""Training steps of the reference's Trainer on this package's kernels.

`rgb_train_step` is Trainer.train_step's RGB branch (nerf/utils.py:897-937):
render with perturbed sampling through the reference's op sequence with the
HIP drop-in encoders (forward and backward kernels: grid, SH), MSE + the
proposal (mip-NeRF 360 inter-level) and distortion losses, optional entropy
regulariser, and the adaptive ray-count update.  `sam_train_step` is its
SAM-distillation branch (utils.py:1072-1106) on the fused forward and the HIP
s_grid scatter (BASELINE config 5).  Optimisation (Adam over
NeRFNetwork.get_params-style groups, main.py:296) is the caller's.
"""
import torch
import torch.nn.functional as F


def update_proposal_now(global_step, with_sam=False):
    """utils.py:912-913: proposal nets train every step for the first 3000,
    then every 5th."""
    return (not with_sam) and (global_step <= 3000 or global_step % 5 == 0)


def rgb_train_step(model, rays_o, rays_d, gt_rgb, global_step, bg_color=None,
                   cam_near_far=None, perturb=True):
    """Returns (pred_rgb, loss, outputs).  gt_rgb [N,3] (or [N,4] with alpha,
    composited on bg as utils.py:903-906).  Updates model.opt.num_rays like
    the reference when adaptive_num_rays is on."""
    opt = model.opt
    if bg_color is None:
        bg_color = 1
    if gt_rgb.shape[-1] == 4:
        gt_rgb = gt_rgb[..., :3] * gt_rgb[..., 3:] + bg_color * (1 - gt_rgb[..., 3:])
    update_proposal = update_proposal_now(global_step, opt.with_sam)
    outputs = model.render(rays_o, rays_d, staged=False, bg_color=bg_color, perturb=perturb,
                           cam_near_far=cam_near_far, update_proposal=update_proposal,
                           return_feats=0)
    pred_rgb = outputs["image"]
    loss = F.mse_loss(pred_rgb, gt_rgb, reduction="none").mean()
    if "proposal_loss" in outputs and opt.lambda_proposal > 0:
        loss = loss + opt.lambda_proposal * outputs["proposal_loss"]
    if "distort_loss" in outputs and opt.lambda_distort > 0:
        loss = loss + opt.lambda_distort * outputs["distort_loss"]
    if opt.lambda_entropy > 0:
        w = outputs["weights_sum"].clamp(1e-5, 1 - 1e-5)
        entropy = -w * torch.log2(w) - (1 - w) * torch.log2(1 - w)
        loss = loss + opt.lambda_entropy * entropy.mean()
    if opt.adaptive_num_rays and "num_points" in outputs:
        opt.num_rays = int(round((opt.num_points / outputs["num_points"]) * opt.num_rays))
    return pred_rgb, loss, outputs


def rgb_train_step_fused(model, rays_o, rays_d, gt_rgb, global_step, bg_color=None,
                         cam_near_far=None, perturb=True):
    """rgb_train_step on the HIP training kernels (samnerf_rgb_train_step,
    csrc/rgb_train.hip): one C call renders the rays (the reference's perturbed
    sampling, drawn with torch's generator in its order), forms the loss of
    utils.py:917-931 and writes every trained tensor's gradient into .grad --
    what loss.backward() leaves there (the proposal tensors' .grad is None on
    the steps the reference does not update them, utils.py:912-913).  Returns
    (pred_rgb, loss, outputs) like rgb_train_step; loss is a detached 0-d
    tensor, outputs holds image / depth / weights_sum / num_points and the
    unweighted loss terms.  Gradients accumulate into an existing .grad as
    loss.backward() does (proposal tensors: not touched on the steps they do
    not train)."""
    import ctypes

    from ._lib import SamnerfRgbGrads, SamnerfRgbTrainOpts, check, lib
    from .fused import FusedRenderer, perturbed_positions, rgb_train_params
    from .ops import _ptr, _stream

    opt = model.opt
    if bg_color is None:
        bg_color = 1
    if gt_rgb.shape[-1] == 4:
        gt_rgb = gt_rgb[..., :3] * gt_rgb[..., 3:] + bg_color * (1 - gt_rgb[..., 3:])
    if torch.is_tensor(bg_color):
        if bg_color.numel() != 1:
            raise NotImplementedError("fused RGB step: per-ray background colours")
        bg_color = float(bg_color)
    update_proposal = update_proposal_now(global_step, opt.with_sam)
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    gt = gt_rgb.reshape(-1, 3).contiguous().float()
    N = rays_o.shape[0]
    dev = rays_o.device
    fr = getattr(model, "_fused_train", None)
    if fr is None or fr.net is not model:
        fr = model._fused_train = FusedRenderer(model, head_mode=1)
    m = fr.model()
    m.view_width = 0
    m.with_mask = 0
    pert = None
    if isinstance(perturb, (tuple, list)) or perturb:
        pert = tuple(perturb) if isinstance(perturb, (tuple, list)) else \
            perturbed_positions(N, list(m.num_steps), dev)
        pert = tuple(t.contiguous().float() for t in pert)
    for i in range(3):
        m.perturb[i] = ctypes.c_void_p(pert[i].data_ptr()) if pert is not None else None
    o = SamnerfRgbTrainOpts()
    o.lambda_proposal = float(getattr(opt, "lambda_proposal", 0.0))
    o.lambda_distort = float(getattr(opt, "lambda_distort", 0.0))
    o.lambda_entropy = float(getattr(opt, "lambda_entropy", 0.0))
    o.update_proposal = int(bool(update_proposal))
    o.bg_color = float(bg_color)
    with_prop = bool(update_proposal) and o.lambda_proposal > 0
    every = rgb_train_params(model, True)
    main, prop = every[:7], every[7:]
    trained = main + (prop if with_prop else [])
    # the kernels OVERWRITE their gradient buffers: they write into fresh
    # buffers, which become .grad where it is None and are added into an
    # existing .grad otherwise (loss.backward()'s accumulation)
    for p in trained:
        if p.grad is not None and (p.grad.dtype != torch.float32 or p.grad.device != p.device
                                   or p.grad.shape != p.shape):
            raise RuntimeError("rgb_train_step_fused: existing .grad must be float32, on the "
                               "parameter's device and of its shape")
    scratch = [torch.empty_like(p, memory_format=torch.contiguous_format) for p in trained]
    g = SamnerfRgbGrads()
    g.grid = scratch[0].data_ptr()
    for i in range(3):
        g.grid_mlp[i] = scratch[1 + i].data_ptr()
        g.view_mlp[i] = scratch[4 + i].data_ptr()
    if with_prop:
        g.prop[0], g.prop[1] = scratch[7].data_ptr(), scratch[8].data_ptr()
        for q in range(2):
            for i in range(2):
                g.prop_mlp[q][i] = scratch[9 + 2 * q + i].data_ptr()
    need = lib().samnerf_rgb_train_workspace_size(ctypes.byref(m), N)
    ws = getattr(fr, "_rt_ws", None)
    if ws is None or ws.device != dev or ws.numel() < need:
        ws = fr._rt_ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
    cnf, n_cnf = None, 0
    if cam_near_far is not None:
        cnf = cam_near_far.contiguous().float()
        n_cnf = cnf.shape[0]
    image = torch.empty(N, 3, device=dev)
    depth = torch.empty(N, device=dev)
    wsum = torch.empty(N, device=dev)
    loss = torch.empty(5, device=dev)
    try:
        check(lib().samnerf_rgb_train_step(
            ctypes.byref(m), _ptr(rays_o), _ptr(rays_d), N, _ptr(cnf), n_cnf, _ptr(gt),
            ctypes.byref(o), _ptr(image), _ptr(depth), _ptr(wsum), _ptr(loss), ctypes.byref(g),
            _ptr(ws), need, _stream(rays_o)), "rgb_train_step")
    finally:
        for i in range(3):
            m.perturb[i] = None
    for p, t in zip(trained, scratch):
        if p.grad is None:
            p.grad = t
        else:
            p.grad.add_(t)
    outputs = {"image": image, "depth": depth, "weights_sum": wsum, "num_points": N * int(m.num_steps[2]),
               "mse": loss[0], "proposal_loss": loss[1], "distort_loss": loss[2], "entropy": loss[3]}
    if opt.adaptive_num_rays:
        opt.num_rays = int(round((opt.num_points / outputs["num_points"]) * opt.num_rays))
    return image, loss[4], outputs


def sam_train_step(renderer, rays_o_lr, rays_d_lr, h, w, gt_samvit, cam_near_far=None):
    """utils.py:1091-1106 on the fused path: 64x64 feature rays, bilinear
    resize to the target, MSE.  Returns (pred [1,256,h',w'], loss)."""
    from .fused import render_sam_train
    out = render_sam_train(renderer, rays_o_lr, rays_d_lr, cam_near_far=cam_near_far)
    pred = out["samvit"].reshape(1, h, w, 256).permute(0, 3, 1, 2).contiguous()
    pred = F.interpolate(pred, gt_samvit.shape[2:], mode="bilinear")
    return pred, F.mse_loss(pred, gt_samvit, reduction="none").mean()


def mask_train_step(model, rays_o, rays_d, gt_mask, num_rays=None, cam_near_far=None):
    """Trainer.train_step's --with_mask branch (nerf/utils.py:941-977, 1026):
    render the instance logits (perturb off, proposal nets frozen, white
    background), softmax over instances, clamp to [epsilon, 1 - epsilon], and
    the mean negative log-likelihood of the labels of the first `num_rays`
    rays (the global rays of mixed sampling; no loss if no pixel is labelled,
    label -1 = unlabelled; like the reference, a -1 among the rays that enter
    the gather is an error -- raised here before it can become a device-side
    assert).  The error-map EMA, incoherent-region
    re-weighting, label regularisation and RGB-similarity terms
    (utils.py:978-1065) are options of the data pipeline and are not
    reproduced.  gt_mask: int64 [N] (or [B, N]).  Returns (pred_ids, loss)."""
    opt = model.opt
    gt = gt_mask.reshape(-1).long()
    n = gt.shape[0] if num_rays is None else num_rays
    outputs = model.render(rays_o, rays_d, staged=False, bg_color=1, perturb=False,
                           cam_near_far=cam_near_far, update_proposal=False, return_feats=0,
                           return_mask=1)
    inst = torch.softmax(outputs["instance_mask_logits"], dim=-1)
    pred = inst.view(-1, opt.n_inst)
    pred = torch.clamp(pred, min=opt.epsilon, max=1 - opt.epsilon)
    labeled = gt != -1
    if labeled.sum() > 0:
        if bool((gt[:n] < 0).any()):
            raise RuntimeError("mask_train_step: label -1 inside the gathered rays "
                               "(utils.py:973 gathers with it: index out of bounds)")
        loss = -torch.log(torch.gather(pred[:n], -1, gt[:n, None]))
    else:
        loss = torch.zeros((), dtype=pred.dtype, device=pred.device)
    return pred.argmax(dim=-1), loss.mean()
