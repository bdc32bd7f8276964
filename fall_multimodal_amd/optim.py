"""Optimizer with the reference's semantics on the fused HIP kernel.

Reference: build_optimizer(model, config) -> (RMSprop(model.parameters(), lr), scheduler)
(Multimodal_Fall3/model/optimizer.py:8-35). Only the RMSprop branch is on the hot path;
the sgd/adam/adamw branches delegate to torch.optim (PyTorch's own fused HIP kernels).
"""
from __future__ import annotations

import torch

from ._lib import check, lib, ptr, require_device, stream_handle


class RMSprop(torch.optim.Optimizer):
    """torch.optim.RMSprop(lr, alpha=0.99, eps=1e-8) — no momentum, not centred, no
    weight decay — as one f3_rmsprop_step launch per parameter tensor (or one launch
    over a flat buffer via `step_flat`)."""

    def __init__(self, params, lr=1e-2, alpha=0.99, eps=1e-8):
        super().__init__(params, dict(lr=lr, alpha=alpha, eps=eps))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        L = lib()
        st = stream_handle()
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                require_device(p, "parameter")
                state = self.state[p]
                if "square_avg" not in state:
                    state["step"] = torch.zeros((), dtype=torch.float32)
                    state["square_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["step"] += 1
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if not p.is_contiguous():
                    raise RuntimeError("fall3 RMSprop needs contiguous parameters")
                check(L.f3_rmsprop_step(ptr(p), ptr(state["square_avg"]), ptr(g), p.numel(), group["lr"],
                                        group["alpha"], group["eps"], 1.0, st), "rmsprop")
        return loss


def build_optimizer(model, config):
    t = config.OPTIM.TYPE
    if t == "rmsprop":
        opt = RMSprop(model.parameters(), lr=config.OPTIM.LR)
    elif t == "sgd":
        opt = torch.optim.SGD(model.parameters(), lr=config.OPTIM.LR, momentum=config.OPTIM.MOMENTUM,
                              weight_decay=config.OPTIM.WEIGHT_DECAY)
    elif t == "adam":
        opt = torch.optim.Adam(model.parameters(), lr=config.OPTIM.LR, betas=config.OPTIM.BETAS,
                               eps=config.OPTIM.EPS, weight_decay=config.OPTIM.WEIGHT_DECAY)
    elif t == "adamw":
        opt = torch.optim.AdamW(model.parameters(), lr=config.OPTIM.LR, betas=config.OPTIM.BETAS,
                                eps=config.OPTIM.EPS, weight_decay=config.OPTIM.WEIGHT_DECAY)
    else:
        raise RuntimeError(f"Optimizer type [{t}] is not implemented.")
    if config.LR_SCHEDULER.TYPE is None:
        return opt, None
    if config.LR_SCHEDULER.TYPE == "cosine":
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=config.LR_SCHEDULER.T_INITIAL,
                                                           eta_min=config.LR_SCHEDULER.LR_MIN)
        return opt, sched
    raise RuntimeError(f"LR Scheduler type [{config.LR_SCHEDULER.TYPE}] is not implemented.")
