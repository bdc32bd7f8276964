"""Fused training step: forward -> soft-target CE -> backward -> (all-reduce) -> RMSprop.

This is the reference's inner loop body (Multimodal_Fall3/model/main.py:97-132; notebook
GSTCAN_HAR_conv_10kfold.ipynb:1103-1116) as four native calls on one HIP stream with every
buffer preallocated, so it can be captured once into a HIP graph and replayed per batch.

Data parallel: one process per GPU; gradients live in ONE flat fp32 buffer, all-reduced
(sum) over RCCL and scaled by 1/world inside the RMSprop kernel. BatchNorm statistics stay
per-rank (the reference's per-device batch semantics).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ._lib import check, lib, ptr, stream_handle


class TrainStep:
    def __init__(self, model, batch, lr=1e-3, alpha=0.99, eps=1e-8, process_group=None, bucket_mb=None):
        self.model = model
        self.N = batch
        self.lr, self.alpha, self.eps = lr, alpha, eps
        dev = model.flat_parameters().device
        nat = model._native
        self.grads = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.square_avg = torch.zeros(nat.nparam, dtype=torch.float32, device=dev)
        self.ws = torch.empty(nat.workspace_bytes(batch), dtype=torch.uint8, device=dev)
        self.out = torch.empty(batch, model.spec.num_class, dtype=torch.float32, device=dev)
        self.dout = torch.empty_like(self.out)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if (dist.is_available() and dist.is_initialized()) else 1
        # expose the flat gradient through the usual .grad attributes
        for (name, shape, off), p in zip(model.param_views(), model.parameters()):
            p.grad = self.grads[off:off + int(np.prod(shape))].view(shape)
        self.graph = None
        self._static = None

    # one step, eager
    def forward_backward(self, skel, sensor, label):
        L = lib()
        st = stream_handle()
        m = self.model
        m.native_forward(skel, sensor, self.out, self.ws, True, st)
        check(L.f3_net_loss(m._native.h, self.N, ptr(self.out), ptr(label), ptr(self.loss), ptr(self.dout), st),
              "fall3 loss")
        m.native_backward(self.N, self.dout, self.grads, self.ws, st)

    def optimizer_step(self):
        scale = 1.0 / self.world
        check(lib().f3_rmsprop_step(ptr(self.model.flat_parameters()), ptr(self.square_avg), ptr(self.grads),
                                    self.grads.numel(), self.lr, self.alpha, self.eps, scale, stream_handle()),
              "rmsprop")

    def allreduce(self):
        if self.world > 1:
            dist.all_reduce(self.grads, op=dist.ReduceOp.SUM, group=self.pg)

    def __call__(self, skel, sensor, label):
        if self.graph is not None:
            s = self._static
            if skel is not None and skel.data_ptr() != s[0].data_ptr():
                s[0].copy_(skel)
            if sensor is not None and sensor.data_ptr() != s[1].data_ptr():
                s[1].copy_(sensor)
            if label.data_ptr() != s[2].data_ptr():
                s[2].copy_(label)
            self.graph[0].replay()
            self.allreduce()
            if self.graph[1] is not None:
                self.graph[1].replay()
            else:
                self.optimizer_step()
            return self.loss
        self.forward_backward(skel, sensor, label)
        self.allreduce()
        self.optimizer_step()
        return self.loss

    def capture(self, skel, sensor, label, warmup=2):
        """Capture forward+loss+backward (and the optimizer) into HIP graphs; the given
        tensors become the static inputs (later calls copy new batches into them)."""
        self._static = (skel, sensor, label)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.forward_backward(skel, sensor, label)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            self.forward_backward(skel, sensor, label)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            self.optimizer_step()
        self.graph = (g1, g2)
