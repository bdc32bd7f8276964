"""Optimizer with the reference's semantics on the fused HIP kernel.

Reference: build_optimizer(model, config) -> (RMSprop(model.parameters(), lr), scheduler)
(Multimodal_Fall3/model/optimizer.py:8-35). Only the RMSprop branch is on the hot path;
the sgd/adam/adamw branches delegate to torch.optim (PyTorch's own fused HIP kernels).
"""
from __future__ import annotations

import math

import torch

from . import ops  # noqa: F401  (registers fall3::rmsprop_)
from ._lib import require_device


def _flat_view(t, start, n):
    """1-D view of n elements of t's storage from element `start`."""
    return torch.empty(0, dtype=t.dtype, device=t.device).set_(t.untyped_storage(), start, (n,))


class RMSprop(torch.optim.Optimizer):
    """torch.optim.RMSprop(lr, alpha=0.99, eps=1e-8) — no momentum, not centred, no
    weight decay — as fall3::rmsprop_ custom ops (f3_rmsprop_step).

    Flat path: the fall3 modules keep their parameters as views of ONE flat buffer and
    loss.backward() hands back their gradients as views of ONE flat gradient buffer in the
    same layout (ops.py `_split_grads`). When a group's parameters, gradients and square_avg
    states are laid out that way, step() is one launch over the whole range (the 16-B
    alignment pads between tensors carry zero gradients, so they stay unchanged), and the
    group shares one `step` counter tensor. Anything else (a user-built group, states loaded
    from a state_dict, gradients that autograd copied) takes the per-tensor path."""

    def __init__(self, params, lr=1e-2, alpha=0.99, eps=1e-8):
        super().__init__(params, dict(lr=lr, alpha=alpha, eps=eps))

    def _flat(self, group):
        """(params, square_avg, grads) flat views covering the group, or None. The full layout check
        below is ~7 us of Python per parameter; once it has passed, the group remembers the layout
        and later steps only check that the gradients are still views of one buffer at the same
        relative offsets (the parameters and the flat square_avg do not move between steps)."""
        ps = group["params"]
        if not ps or any(p.grad is None for p in ps):
            return None
        caches = self.__dict__.setdefault("_f3_flat", {})  # per group (not in param_groups: state_dict)
        cache = caches.get(id(group))
        if cache is not None:
            hit = self._flat_cached(ps, cache)
            if hit is not None:
                return hit
            del caches[id(group)]
        flat = self._flat_full(ps)
        if flat is not None:
            p0 = min(ps, key=lambda t: t.storage_offset())
            caches[id(group)] = (tuple(map(id, ps)), [p.storage_offset() - p0.storage_offset() for p in ps], flat[0],
                                 flat[1], self.state[p0]["square_avg"], p0)
        return flat

    def _flat_cached(self, ps, cache):
        """The remembered layout still holds when every gradient is contiguous and sits at its
        parameter's relative offset from the first gradient, and that gradient's storage spans the
        whole range: the gradients then ARE the range of one buffer. (Addresses, not `_base`: the
        autograd engine hands parameters detached gradients, which share the buffer but are not
        views of it, so a `_base` test failed on every step and sent it to the full ~7 us/parameter
        check.)"""
        ids, rel, flat_p, flat_sq, sq0, p0 = cache
        if tuple(map(id, ps)) != ids or self.state[p0].get("square_avg") is not sq0:
            return None
        g0 = p0.grad
        if g0.dtype != torch.float32 or g0.device != p0.device:
            return None
        n = flat_p.numel()
        gbase = g0.storage_offset()
        if (gbase + n) * 4 > g0.untyped_storage().nbytes():
            return None
        a0 = g0.data_ptr()
        for p, r in zip(ps, rel):
            g = p.grad
            if g is None or g.data_ptr() - a0 != 4 * r or not g.is_contiguous() or g.dtype != torch.float32:
                return None
        return flat_p, flat_sq, _flat_view(g0, gbase, n)

    def _flat_full(self, ps):
        ps = sorted(ps, key=lambda t: t.storage_offset())  # module order is not the flat order
        p0, g0 = ps[0], ps[0].grad
        if p0.dtype != torch.float32 or g0.dtype != torch.float32:
            return None
        pst, gst = p0.untyped_storage().data_ptr(), g0.untyped_storage().data_ptr()
        pbase, gbase = p0.storage_offset(), g0.storage_offset()
        st0 = self.state[p0]
        sq0 = st0.get("square_avg")
        sst = sq0.untyped_storage().data_ptr() if sq0 is not None else None
        sbase = sq0.storage_offset() if sq0 is not None else 0
        end = pbase
        for i, p in enumerate(ps):
            g = p.grad
            # every tensor starts exactly at the previous one's end rounded up to 16 B: a larger gap
            # could hold a tensor outside this group (another param_group, a frozen parameter), which
            # one launch over [first, last] would update with this group's lr
            if (p.untyped_storage().data_ptr() != pst or g.untyped_storage().data_ptr() != gst
                    or not p.is_contiguous() or not g.is_contiguous() or g.shape != p.shape
                    or (i > 0 and p.storage_offset() != (end + 3) // 4 * 4)
                    or g.storage_offset() - gbase != p.storage_offset() - pbase):
                return None
            s = self.state[p].get("square_avg")
            if (s is None) != (sq0 is None) or (s is not None and (
                    s.untyped_storage().data_ptr() != sst or s.storage_offset() - sbase != p.storage_offset() - pbase)):
                return None
            end = p.storage_offset() + p.numel()
        n = end - pbase
        if sq0 is None:  # first step: one flat square_avg, per-tensor views as the states
            flat_sq = torch.zeros(n, dtype=torch.float32, device=p0.device)
            step = torch.zeros((), dtype=torch.float32)
            for p in ps:
                o = p.storage_offset() - pbase
                self.state[p]["square_avg"] = flat_sq[o:o + p.numel()].view_as(p)
                self.state[p]["step"] = step
        else:
            flat_sq = _flat_view(sq0, sbase, n)
        return _flat_view(p0, pbase, n), flat_sq, _flat_view(g0, gbase, n)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            flat = self._flat(group)
            if flat is not None:
                require_device(flat[0], "parameter")
                self.state[group["params"][0]]["step"] += 1  # one counter shared by the group
                torch.ops.fall3.rmsprop_(flat[0], flat[1], flat[2], group["lr"], group["alpha"], group["eps"], 1.0)
                continue
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
                torch.ops.fall3.rmsprop_(p, state["square_avg"], g, group["lr"], group["alpha"], group["eps"], 1.0)
        return loss


class CosineLRScheduler:
    """timm.scheduler.CosineLRScheduler as the reference builds it (model/optimizer.py:31; timm is
    not installed here, so its published schedule is restated): cycle_mul 1, decay_rate 1,
    cycle_limit 1, k_decay 1, warmup_prefix False, no noise.
      t <  warmup_t : lr = warmup_lr_init + t * (base_lr - warmup_lr_init) / warmup_t
      t <  t_initial: lr = lr_min + (base_lr - lr_min) * (1 + cos(pi * t / t_initial)) / 2
      otherwise     : lr = lr_min
    The warm-up value is applied at construction (so epoch 0 trains at warmup_lr_init) and
    step(epoch) sets the value for `epoch` (t_in_epochs; step_update(num_updates) otherwise)."""

    def __init__(self, optimizer, t_initial, lr_min=0.0, t_in_epochs=True, warmup_t=0, warmup_lr_init=0.0):
        self.optimizer = optimizer
        self.t_initial, self.lr_min, self.t_in_epochs = t_initial, lr_min, t_in_epochs
        self.warmup_t, self.warmup_lr_init = warmup_t, warmup_lr_init
        for g in optimizer.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self.base_values = [g["initial_lr"] for g in optimizer.param_groups]
        self.warmup_steps = [(v - warmup_lr_init) / warmup_t for v in self.base_values] if warmup_t else []
        if warmup_t:
            self._set([warmup_lr_init] * len(self.base_values))

    def _get_lr(self, t):
        if t < self.warmup_t:
            return [self.warmup_lr_init + t * s for s in self.warmup_steps]
        if t < self.t_initial:
            return [self.lr_min + 0.5 * (v - self.lr_min) * (1 + math.cos(math.pi * t / self.t_initial))
                    for v in self.base_values]
        return [self.lr_min for _ in self.base_values]

    def _set(self, values):
        for g, v in zip(self.optimizer.param_groups, values):
            g["lr"] = v

    def step(self, epoch, metric=None):
        if self.t_in_epochs:
            self._set(self._get_lr(epoch))

    def step_update(self, num_updates, metric=None):
        if not self.t_in_epochs:
            self._set(self._get_lr(num_updates))

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, state):
        self.__dict__.update(state)


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
        c = config.LR_SCHEDULER
        return opt, CosineLRScheduler(opt, t_initial=c.T_INITIAL, lr_min=c.LR_MIN, t_in_epochs=c.T_IN_EPOCHS,
                                      warmup_t=c.WARMUP_T, warmup_lr_init=c.WARMUP_LR_INIT)
    raise RuntimeError(f"LR Scheduler type [{config.LR_SCHEDULER.TYPE}] is not implemented.")
