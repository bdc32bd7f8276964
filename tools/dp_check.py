#!/usr/bin/env python3
"""Data-parallel invariant check of the native training step (run under torchrun):

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/dp_check.py [--backend gloo] [--same-device]

Each rank trains its own shard of synthetic clips (B per rank) through TrainStep with the
two-bucket gradient all-reduce overlapping backward phase 2. Checks:
* the first data-parallel step's reduced gradient equals the MEAN of the per-shard gradients,
  each shard's gradient computed alone (single-rank backward, no collective) and all-gathered —
  within 10x the backward's own run-to-run floor (fp32 atomics reassociate; BatchNorm at small
  per-rank batch amplifies it), cosine >= 0.9999 — and the update is RMSprop on it (1/world scale);
* after K steps every rank holds bit-identical parameters (replicas stay in sync) that moved. --same-device puts every rank on
cuda:0 (a one-GPU box); gloo reduces device tensors through the host, RCCL ("nccl") is the
production backend.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if a.backend == "nccl":
        from fall_multimodal_amd.train import rccl_options
        dist.init_process_group(a.backend, pg_options=rccl_options())
    else:
        dist.init_process_group(a.backend)
    dev = torch.device("cuda", local)
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    torch.manual_seed(0)  # identical init on every rank
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                      precision=a.precision)
    p0 = model.flat_parameters().clone()
    step = f3.TrainStep(model, a.batch, lr=1e-3)
    assert step.world == world
    # (1) the per-shard gradients alone (twice: the run-to-run floor of the backward's fp32 atomics,
    # amplified by BatchNorm at small batch), their mean over the shards
    batch0 = [torch.from_numpy(x).to(dev) for x in synthetic_batch(a.batch, 18, 11, 6, 1000 * rank)]
    lab0 = step.prepare(*batch0)
    step.forward_backward(batch0[0], batch0[1], lab0)
    g_own = step.grads.clone()
    step.forward_backward(batch0[0], batch0[1], lab0)
    floor = torch.tensor([float((step.grads - g_own).abs().max()) / max(float(g_own.abs().max()), 1e-30)], device=dev)
    dist.all_reduce(floor, op=dist.ReduceOp.MAX)
    gs = [torch.empty_like(g_own) for _ in range(world)]
    dist.all_gather(gs, g_own)
    g_mean = torch.stack(gs).double().mean(0)
    gmax = float(g_mean.abs().max())
    lr, alpha, eps = 1e-3, 0.99, 1e-8
    step1 = None
    for i in range(a.steps):
        batch = [torch.from_numpy(x).to(dev) for x in synthetic_batch(a.batch, 18, 11, 6, 1000 * rank + i)]
        step(*batch)
        if i == 0:
            torch.cuda.synchronize()
            g_dp = step.grads.double() / world   # the all-reduced sum the update used, scaled as RMSprop does
            err = float((g_dp - g_mean).abs().max()) / gmax
            cos = float((g_dp * g_mean).sum() / (g_dp.norm() * g_mean.norm()))
            upd = p0.double() - lr * g_dp / (torch.sqrt((1 - alpha) * g_dp * g_dp) + eps)
            step1 = {"reduced_vs_mean_of_shard_grads_rel": err, "cosine": cos,
                     "run_to_run_floor_rel": float(floor.item()),
                     "update_vs_rmsprop_of_reduced_max_abs": float((model.flat_parameters().double() - upd).abs().max())}
            step1["ok"] = bool(err <= max(10 * float(floor.item()), 1e-4) and cos >= 0.9999
                               and step1["update_vs_rmsprop_of_reduced_max_abs"] < 1e-6)
    torch.cuda.synchronize()
    p = model.flat_parameters()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p.contiguous())
    same = all(torch.equal(gathered[0], g) for g in gathered[1:])
    moved = float((p - p0).abs().max())
    if rank == 0:
        print(json.dumps({"world": world, "replicas_identical": same, "max_param_change": moved,
                          "backend": a.backend, "first_step_vs_mean_of_shard_grads": step1}), flush=True)
    dist.destroy_process_group()
    if not same or moved == 0.0 or not step1["ok"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
