"""Fused training step: forward -> soft-target CE -> backward -> (all-reduce) -> RMSprop.

This is the reference's inner loop body (Multimodal_Fall3/model/main.py:97-132; notebook
GSTCAN_HAR_conv_10kfold.ipynb:1103-1116) as native calls on one HIP stream with every
buffer preallocated, so it can be captured into HIP graphs and replayed per batch.

Data parallel: one process per GPU. Gradients live in ONE flat fp32 buffer whose layout
puts the parameters the first backward phase finalises (head, sensor branch, skeleton
layers 4-6; f3_net_grad_split) first. Phase 1 returns without joining its private queues:
the head bucket's all-reduce (RCCL, sum) is issued from a side stream that waits on phase
1's per-queue events (f3_net_wait_phase1), so phase 2's critical path (layers 0-3, data_bn)
starts at once while phase 1's weight gradients drain and the all-reduce runs; the remainder
follows phase 2. 1/world is applied inside the RMSprop kernel. BatchNorm statistics stay
per-rank (the reference's per-device batch semantics).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.distributed as dist

from ._lib import check, lib, ptr, stream_handle


class GradSync:
    """Two-bucket gradient all-reduce over a flat buffer: `head` = grads[:split] (final after
    backward phase 1), `tail` = grads[split:]. Both are issued async; `finish()` orders the
    caller's stream after them. `wait_phase1(stream_handle)` (optional) makes a stream wait for
    the phase-1 gradients: the head bucket is then issued from a side stream ordered after them
    rather than after everything on the caller's stream."""

    def __init__(self, grads: torch.Tensor, split: int, group=None, wait_phase1=None, force=False):
        self.grads, self.split, self.group = grads, int(split), group
        self.world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
        self.wait_phase1 = wait_phase1
        # force: issue both buckets even at world 1 (a world-1 sum is the identity), so the collective
        # path runs on a one-GPU box (tests/test_gpu_rccl.py); needs an initialised process group
        self.active = self.world > 1 or bool(force)
        # high priority: ROCm draws high-priority streams from their own hardware-queue pool, so the head
        # bucket's wait + all-reduce never queue behind main-chain kernels on a shared normal-priority
        # queue (the step's four native queues already fill GPU_MAX_HW_QUEUES = 4)
        self._side = (torch.cuda.Stream(device=grads.device, priority=-1) if (self.active and grads.is_cuda)
                      else None)
        self._work = []

    def _reduce(self, t):
        if t.numel():
            self._work.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def start_head(self, after_current=False):
        """after_current: order the bucket after everything on the caller's stream (a replayed
        graph, whose phase 1 joined its queues) instead of after phase 1's per-queue events."""
        if not self.active:
            return
        if after_current and self._side is not None:
            self._side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self._side):
                self._reduce(self.grads[:self.split])
            return
        if self.wait_phase1 is None or self._side is None:
            self._reduce(self.grads[:self.split])
            return
        self.wait_phase1(ctypes.c_void_p(self._side.cuda_stream))
        with torch.cuda.stream(self._side):
            self._reduce(self.grads[:self.split])

    def start_tail(self):
        if self.active:
            self._reduce(self.grads[self.split:])

    def finish(self):
        for w in self._work:
            w.wait()
        self._work = []

    def all(self):
        self.start_head()
        self.start_tail()
        self.finish()


def rccl_options():
    """ProcessGroupNCCL options for the gradient all-reduce: RCCL's internal stream high priority, for
    the same reason as GradSync's side stream (pass as init_process_group("nccl", pg_options=...))."""
    o = dist.ProcessGroupNCCL.Options()
    o.is_high_priority_stream = True
    return o


class TrainStep:
    """`optimizer` (optional, e.g. fall3 RMSprop driven by a CosineLRScheduler): its
    param_groups[0] lr / alpha / eps are read at every step, so a scheduler's step(epoch) takes
    effect as with the reference's optimizer.step() (model/main.py:127, 321-322)."""

    def __init__(self, model, batch, lr=1e-3, alpha=0.99, eps=1e-8, process_group=None, optimizer=None,
                 phased=None, force_sync=False):
        self.model = model
        self.N = batch
        self.lr, self.alpha, self.eps = lr, alpha, eps
        self.optimizer = optimizer
        dev = model.flat_parameters().device
        nat = model._native
        self.grads = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.square_avg = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.ws = torch.empty(nat.workspace_bytes(batch), dtype=torch.uint8, device=dev)
        self.out = torch.empty(batch, model.spec.num_class, dtype=torch.float32, device=dev)
        self.dout = torch.empty_like(self.out)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.pg = process_group
        h = nat.h
        self.sync = GradSync(self.grads, lib().f3_net_grad_split(h), process_group,
                             wait_phase1=lambda st: check(lib().f3_net_wait_phase1(h, st), "wait phase 1"),
                             force=force_sync)
        self.world = self.sync.world
        # phased=True runs the two-phase backward even on one rank (times its cost against phase 0);
        # force_sync=True (tests) also issues the two all-reduce buckets at world 1
        self.phased = (self.world > 1 or force_sync) if phased is None else bool(phased)
        # expose the flat gradient through the usual .grad attributes
        for (name, shape, off), p in zip(model.param_views(), model.parameters()):
            p.grad = self.grads[off:off + int(np.prod(shape))].view(shape)
        self.graph = None
        self._static = None
        # world 1: the RMSprop update per layer inside the backward (F3_FUSED_OPT=0: one launch after it)
        self.fused_optimizer = not self.sync.active and os.environ.get("F3_FUSED_OPT", "1") != "0"

    # -- the pieces ------------------------------------------------------------
    def prepare(self, skel, sensor, label):
        """Validate a batch against the step's preallocated buffers (batch N, contiguous fp32 on the
        device) and turn 1-D class-index labels into one-hot targets as model/main.py:104-109 does."""
        m = self.model
        m.check_inputs(skel, sensor)
        for t, what in ((skel, "skel"), (sensor, "sensor")):
            if t is None:
                continue
            if t.shape[0] != self.N:
                raise ValueError(f"TrainStep was built for batch {self.N}, got {what} with batch {t.shape[0]}")
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"TrainStep: {what} must be contiguous fp32")
        dev = m.flat_parameters().device
        if label.dim() == 1:
            label = torch.nn.functional.one_hot(label.to(dev).long(), num_classes=m.spec.num_class).float()
        if tuple(label.shape) != (self.N, m.spec.num_class):
            raise ValueError(f"TrainStep: label must be [{self.N},{m.spec.num_class}] (or [{self.N}] class indices), "
                             f"got {tuple(label.shape)}")
        if label.device != dev or label.dtype != torch.float32 or not label.is_contiguous():
            label = label.to(device=dev, dtype=torch.float32).contiguous()
        return label

    def forward_loss(self, skel, sensor, label):
        L = lib()
        st = stream_handle()
        m = self.model
        m.native_forward(skel, sensor, self.out, self.ws, True, st)
        check(L.f3_net_loss(m._native.h, self.N, ptr(self.out), ptr(label), ptr(self.loss), ptr(self.dout), st),
              "fall3 loss")

    def backward_phase(self, phase):
        m = self.model
        check(lib().f3_net_backward_phase(m._native.h, self.N, ptr(m.flat_parameters()), ptr(self.dout),
                                          ptr(self.grads), ptr(self.ws), phase, stream_handle()),
              f"fall3 backward phase {phase}")

    def forward_backward(self, skel, sensor, label):
        self.forward_loss(skel, sensor, label)
        self.backward_phase(0)

    def optimizer_step(self):
        if self.optimizer is not None:
            g = self.optimizer.param_groups[0]
            self.lr, self.alpha, self.eps = g["lr"], g.get("alpha", self.alpha), g.get("eps", self.eps)
        scale = 1.0 / self.world
        check(lib().f3_rmsprop_step(ptr(self.model.flat_parameters()), ptr(self.square_avg), ptr(self.grads),
                                    self.grads.numel(), self.lr, self.alpha, self.eps, scale, stream_handle()),
              "rmsprop")

    def backward_optimizer_step(self):
        """loss.backward() + optimizer.step() in one native call (world 1): each skeleton layer's
        RMSprop update starts on the queue that finishes its gradients (f3_net_backward_rmsprop);
        self.grads holds the gradients afterwards as with backward_phase(0)."""
        if self.optimizer is not None:
            g = self.optimizer.param_groups[0]
            self.lr, self.alpha, self.eps = g["lr"], g.get("alpha", self.alpha), g.get("eps", self.eps)
        m = self.model
        check(lib().f3_net_backward_rmsprop(m._native.h, self.N, ptr(m.flat_parameters()), ptr(self.dout),
                                            ptr(self.grads), ptr(self.square_avg), ptr(self.ws), self.lr, self.alpha,
                                            self.eps, stream_handle()), "fall3 backward + rmsprop")

    def allreduce(self):
        self.sync.all()

    # -- one step ----------------------------------------------------------------
    def _eager(self, skel, sensor, label):
        self.forward_loss(skel, sensor, label)
        if self.phased:
            self.backward_phase(1)
            self.sync.start_head()       # after phase 1's queues, concurrent with phase 2
            self.backward_phase(2)
            self.sync.start_tail()
            self.sync.finish()
        elif self.fused_optimizer:
            self.backward_optimizer_step()
            return
        else:
            self.backward_phase(0)
        self.optimizer_step()

    def __call__(self, skel, sensor, label):
        label = self.prepare(skel, sensor, label)
        if self.graph is None:
            self._eager(skel, sensor, label)
            return self.loss
        s = self._static
        if skel is not None and skel.data_ptr() != s[0].data_ptr():
            s[0].copy_(skel)
        if sensor is not None and sensor.data_ptr() != s[1].data_ptr():
            s[1].copy_(sensor)
        if label.data_ptr() != s[2].data_ptr():
            s[2].copy_(label)
        g_head, g_tail, g_opt = self.graph
        g_head.replay()
        if g_tail is not None:
            # the captured phase 1 joined its queues into the capturing stream (net.cpp
            # mark_phase1), so the head bucket is ordered after the replay itself
            self.sync.start_head(after_current=True)  # RCCL on the comm stream, concurrent with phase 2
            g_tail.replay()
            self.sync.start_tail()
            self.sync.finish()
        g_opt.replay()
        return self.loss

    def capture(self, skel, sensor, label, warmup=2):
        """Capture the step into HIP graphs; the given tensors become the static inputs
        (later calls copy new batches into them). world == 1: [fwd+loss+bwd], [RMSprop].
        world > 1: [fwd+loss+bwd phase 1], [bwd phase 2], [RMSprop], with the two all-reduce
        buckets issued between replays."""
        self._static = (skel, sensor, label)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.forward_backward(skel, sensor, label)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g_head = torch.cuda.CUDAGraph()
        g_tail = None
        if self.phased:
            with torch.cuda.graph(g_head):
                self.forward_loss(skel, sensor, label)
                self.backward_phase(1)
            g_tail = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_tail):
                self.backward_phase(2)
        else:
            with torch.cuda.graph(g_head):
                self.forward_backward(skel, sensor, label)
        g_opt = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_opt):
            self.optimizer_step()
        self.graph = (g_head, g_tail, g_opt)
