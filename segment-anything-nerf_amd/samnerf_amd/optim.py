"""Adam as one HIP pass over every parameter (samnerf_adam_step,
train_optim.hip): the optimiser of the SAM-distillation step
(nerf/utils.py:1831; Adam(lr=1e-2, eps=1e-15) over get_params groups,
main.py:296).

Drop-in for torch.optim.Adam (amsgrad / maximize / capturable off): the same
constructor arguments, parameter groups, state keys ('step', 'exp_avg',
'exp_avg_sq') and state_dict layout, so checkpoints move between the two.
"""
import ctypes

import torch
from torch.autograd.graph import increment_version

from ._lib import SamnerfAdamTensor, check, lib


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0 or eps < 0 or weight_decay < 0:
            raise ValueError("FusedAdam: lr, eps and weight_decay must be >= 0")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"FusedAdam: invalid betas {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                        and p.grad.is_contiguous() and not p.grad.is_sparse):
                    raise RuntimeError("FusedAdam: parameters and grads must be contiguous float32 "
                                       "CUDA tensors")
                st = self.state[p]
                if not st:
                    st["step"] = torch.zeros((), dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            b1, b2 = group["betas"]
            for t, ps in by_step.items():
                tab = (SamnerfAdamTensor * len(ps))()
                for j, p in enumerate(ps):
                    st = self.state[p]
                    tab[j] = SamnerfAdamTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                               st["exp_avg_sq"].data_ptr(), p.numel())
                stream = ctypes.c_void_p(torch.cuda.current_stream(ps[0].device).cuda_stream)
                check(lib().samnerf_adam_step(ctypes.byref(tab), len(ps), float(group["lr"]), float(b1),
                                              float(b2), float(group["eps"]),
                                              float(group["weight_decay"]), t, stream), "adam_step")
                # the kernel writes through raw pointers: bump each parameter's
                # version counter as torch's in-place update would (autograd's
                # saved-tensor checks, FusedRenderer's packed-weight reuse)
                for p in ps:
                    increment_version(p)
        return loss
