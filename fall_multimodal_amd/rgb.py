"""RGB spatial-conv branch — BUILD-DEFINED (the north star names an "RGB spatial-conv branch"; the
reference has RGB frames only in preprocessing, 3_stream/har_create3.py:36-42,101-158, and no RGB
model arithmetic, so this branch's parity is unpinned; SURVEY.md section 8a row R-RGB).

    RGBSpatialConv   Conv2d(3, 64, 8, stride 8) over each 224x224 frame -> ReLU -> mean over the
                     frames and the 28x28 patches -> feat [B, 64]   (HIP: csrc/rgb.hip)
    RGBBranch        RGBSpatialConv + Linear(64, num_class): the branch's late-fusion logits
    Fall3WithRGB     the reference 3-stream model plus the RGB branch, fused by adding logits
    Fall3RGBStep     the north-star workload as ONE fused training step (skeleton + IMU + RGB): the
                     RGB branch on its own HIP stream, concurrent with the skeleton / sensor queues

Frames are channels-last bf16 [B, T, 224, 224, 3]. The conv runs as `fall3::rgb_forward` /
`fall3::rgb_backward` custom ops (no input gradient: the frames are data)."""
from __future__ import annotations

import math
from typing import Optional

import torch
from torch import Tensor, nn

from ._lib import check, lib, ptr, require_device, stream_handle


def _pack(w: Tensor) -> Tensor:  # [64, 3, 8, 8] -> bf16 [64, 192], k = (dy*8 + dx)*3 + ch
    return w.detach().permute(0, 2, 3, 1).reshape(w.shape[0], -1).to(torch.bfloat16).contiguous()


def _check_frames(frames: Tensor, weight: Tensor, bias: Tensor, dfeat: Optional[Tensor] = None):
    """Validation shared by both custom ops (they hand raw pointers to the kernels)."""
    require_device(frames, "frames")
    if frames.dim() != 5 or frames.dtype != torch.bfloat16 or tuple(frames.shape[2:]) != (224, 224, 3) \
            or not frames.is_contiguous():
        raise ValueError("fall3 rgb: frames must be contiguous bf16 [B, T, 224, 224, 3]")
    if tuple(weight.shape) != (64, 3, 8, 8) or tuple(bias.shape) != (64,):
        raise ValueError("fall3 rgb: weight must be [64, 3, 8, 8] and bias [64]")
    tensors = [weight, bias] + ([] if dfeat is None else [dfeat])
    if any(t.device != frames.device for t in tensors):
        raise ValueError("fall3 rgb: frames, weight, bias (and dfeat) must be on one device")
    if dfeat is not None and tuple(dfeat.shape) != (frames.shape[0], 64):
        raise ValueError(f"fall3 rgb: dfeat must be [{frames.shape[0]}, 64], got {tuple(dfeat.shape)}")


@torch.library.custom_op("fall3::rgb_forward", mutates_args=())
def rgb_forward(frames: Tensor, weight: Tensor, bias: Tensor) -> Tensor:
    _check_frames(frames, weight, bias)
    B, T = frames.shape[:2]
    feat = torch.empty(B, 64, dtype=torch.float32, device=frames.device)
    wp, b = _pack(weight), bias.detach().float().contiguous()
    check(lib().f3_rgb_forward(ptr(frames), ptr(wp), ptr(b), ptr(feat), B, T, stream_handle()), "rgb forward")
    return feat


@rgb_forward.register_fake
def _(frames, weight, bias):
    return frames.new_empty(frames.shape[0], 64, dtype=torch.float32)


@torch.library.custom_op("fall3::rgb_backward", mutates_args=())
def rgb_backward(frames: Tensor, weight: Tensor, bias: Tensor, dfeat: Tensor) -> tuple[Tensor, Tensor]:
    _check_frames(frames, weight, bias, dfeat)
    B, T = frames.shape[:2]
    L = lib()
    scratch = torch.empty(int(L.f3_rgb_scratch_floats(B, T)), dtype=torch.float32, device=frames.device)
    dwp = torch.empty(64, 192, dtype=torch.float32, device=frames.device)
    db = torch.empty(64, dtype=torch.float32, device=frames.device)
    wp, b, d = _pack(weight), bias.detach().float().contiguous(), dfeat.float().contiguous()
    check(L.f3_rgb_backward(ptr(frames), ptr(wp), ptr(b), ptr(d), ptr(dwp), ptr(db), ptr(scratch), scratch.numel(),
                            B, T, stream_handle()), "rgb backward")
    return dwp.reshape(64, 8, 8, 3).permute(0, 3, 1, 2).contiguous(), db


@rgb_backward.register_fake
def _(frames, weight, bias, dfeat):
    return weight.new_empty(weight.shape, dtype=torch.float32), bias.new_empty(bias.shape, dtype=torch.float32)


def _rgb_setup(ctx, inputs, output):
    frames, weight, bias = inputs
    ctx.save_for_backward(frames, weight, bias)


def _rgb_bwd(ctx, dfeat):
    frames, weight, bias = ctx.saved_tensors
    dw, db = torch.ops.fall3.rgb_backward(frames, weight, bias, dfeat)
    return None, dw.to(weight.dtype), db.to(bias.dtype)


rgb_forward.register_autograd(_rgb_bwd, setup_context=_rgb_setup)


class RGBSpatialConv(nn.Module):
    """Conv2d(3, 64, 8, stride 8) -> ReLU -> mean over frames and patches (nn.Conv2d's default init)."""

    def __init__(self, device=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(64, 3, 8, 8, device=device))
        self.bias = nn.Parameter(torch.empty(64, device=device))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(3 * 8 * 8)
        nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, frames: Tensor) -> Tensor:
        return torch.ops.fall3.rgb_forward(frames, self.weight, self.bias)


class RGBBranch(nn.Module):
    """The branch's late-fusion logits: RGBSpatialConv -> Linear(64, num_class)."""

    def __init__(self, num_class: int, device=None):
        super().__init__()
        self.conv = RGBSpatialConv(device=device)
        self.fc = nn.Linear(64, num_class, device=device)

    def forward(self, frames: Tensor) -> Tensor:
        return self.fc(self.conv(frames))


class Fall3WithRGB(nn.Module):
    """The reference's 3-stream model (unchanged, its own state_dict keys under `fall3.`) plus the
    build-defined RGB branch; logits = fall3(skel, sensor) + rgb(frames)."""

    def __init__(self, fall3: nn.Module, num_class: int, device=None):
        super().__init__()
        self.fall3 = fall3
        self.rgb = RGBBranch(num_class, device=device)

    def forward(self, skel: Tensor, sensor: Optional[Tensor], frames: Tensor) -> Tensor:
        return self.fall3(skel, sensor) + self.rgb(frames)


class Fall3RGBStep:
    """North-star training step with the RGB branch (BASELINE.json: "B=256, T=30, J=17 skeleton +
    6-axis IMU + 224^2 RGB" as ONE step): logits = fall3(skel, sensor) + fc(rgb_conv(frames)), soft-target
    CE, backward of both branches, RMSprop over both parameter sets (torch.optim.RMSprop semantics).

    Queues: the fall3 model runs exactly as TrainStep runs it (the caller's stream plus its private
    branch queues); the RGB forward (conv, fc), and after the loss its backward (fc gradients, dfeat,
    conv backward), run on one extra HIP stream, so the frames' two HBM passes overlap the skeleton
    streams. The RGB parameters are views into one flat buffer (16-B aligned entries) so the update is
    one f3_rmsprop_step launch, like the fall3 flat range. The reference has no RGB model arithmetic:
    this branch's parity is unpinned (oracle/rgb_cpu.py restates the build's definition)."""

    def __init__(self, model: Fall3WithRGB, batch, lr=1e-3, alpha=0.99, eps=1e-8, optimizer=None):
        from .train import TrainStep
        self.model, self.N = model, batch
        self.inner = TrainStep(model.fall3, batch, lr=lr, alpha=alpha, eps=eps, optimizer=optimizer)
        if self.inner.world > 1:
            # this step has no gradient all-reduce (neither the skeleton's phased buckets nor the RGB
            # range): under torchrun it would update each rank from its own shard only
            raise NotImplementedError("Fall3RGBStep is single-GPU (world 1); use TrainStep for data parallelism")
        dev = model.fall3.flat_parameters().device
        params = [model.rgb.conv.weight, model.rgb.conv.bias, model.rgb.fc.weight, model.rgb.fc.bias]
        offs, off = [], 0
        for p in params:
            offs.append(off)
            off += (p.numel() + 3) // 4 * 4
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grads = torch.zeros_like(self.flat)
        self.square_avg = torch.zeros_like(self.flat)
        with torch.no_grad():
            for p, o in zip(params, offs):
                v = self.flat[o:o + p.numel()].view(p.shape)
                v.copy_(p.detach())
                p.data = v
                p.grad = self.grads[o:o + p.numel()].view(p.shape)
        self.params = params
        C = model.fall3.spec.num_class
        self.feat = torch.empty(batch, 64, dtype=torch.float32, device=dev)
        self.rlog = torch.empty(batch, C, dtype=torch.float32, device=dev)
        self.total = torch.empty(batch, C, dtype=torch.float32, device=dev)
        self.stream = torch.cuda.Stream(device=dev)

    @property
    def loss(self):
        return self.inner.loss

    @property
    def out(self):
        return self.total

    def __call__(self, skel, sensor, frames, label):
        inner, m = self.inner, self.model.fall3
        label = inner.prepare(skel, sensor, label)
        _check_frames(frames, self.params[0], self.params[1])
        if frames.shape[0] != self.N:
            raise ValueError(f"Fall3RGBStep was built for batch {self.N}, got frames with batch {frames.shape[0]}")
        cw, cb, fw, fb = self.params
        cur = torch.cuda.current_stream()
        s = self.stream
        s.wait_stream(cur)  # frames and the previous step's parameter update
        with torch.cuda.stream(s):
            self.feat.copy_(torch.ops.fall3.rgb_forward(frames, cw.detach(), cb.detach()))
            torch.addmm(fb.detach(), self.feat, fw.detach().t(), out=self.rlog)
        st = stream_handle()
        m.native_forward(skel, sensor, inner.out, inner.ws, True, st)
        cur.wait_stream(s)
        torch.add(inner.out, self.rlog, out=self.total)
        check(lib().f3_net_loss(m._native.h, self.N, ptr(self.total), ptr(label), ptr(inner.loss), ptr(inner.dout),
                                st), "fall3 loss")
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            dout = inner.dout
            torch.mm(dout.t(), self.feat, out=fw.grad)
            torch.sum(dout, 0, out=fb.grad)
            dfeat = dout @ fw.detach()
            dw, db = torch.ops.fall3.rgb_backward(frames, cw.detach(), cb.detach(), dfeat)
            cw.grad.copy_(dw)
            cb.grad.copy_(db)
        inner.backward_phase(0)
        cur.wait_stream(s)
        inner.optimizer_step()
        check(lib().f3_rmsprop_step(ptr(self.flat), ptr(self.square_avg), ptr(self.grads), self.grads.numel(),
                                    inner.lr, inner.alpha, inner.eps, 1.0, stream_handle()), "rgb rmsprop")
        for t in (frames, dout, dfeat):
            t.record_stream(s)
        return inner.loss
