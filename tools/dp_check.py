#!/usr/bin/env python3
"""Data-parallel invariant check of the native training step (run under torchrun):

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/dp_check.py [--backend gloo] [--same-device]

Each rank trains its own shard of synthetic clips (B per rank) through TrainStep with the
two-bucket gradient all-reduce overlapping backward phase 2; after K steps every rank must
hold bit-identical parameters (replicas stay in sync: each rank applied the same summed
gradients with the 1/world scale) that moved from the initial ones. --same-device puts every rank on
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
    ap.add_argument("--batch", type=int, default=16)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if a.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group(a.backend)
    dev = torch.device("cuda", local)
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    torch.manual_seed(0)  # identical init on every rank
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                      precision="bf16")
    p0 = model.flat_parameters().clone()
    step = f3.TrainStep(model, a.batch, lr=1e-3)
    assert step.world == world
    for i in range(a.steps):
        batch = [torch.from_numpy(x).to(dev) for x in synthetic_batch(a.batch, 18, 11, 6, 1000 * rank + i)]
        step(*batch)
    torch.cuda.synchronize()
    p = model.flat_parameters()
    gathered = [torch.empty_like(p) for _ in range(world)]
    dist.all_gather(gathered, p.contiguous())
    same = all(torch.equal(gathered[0], g) for g in gathered[1:])
    moved = float((p - p0).abs().max())
    if rank == 0:
        print(json.dumps({"world": world, "replicas_identical": same, "max_param_change": moved,
                          "backend": a.backend}), flush=True)
    dist.destroy_process_group()
    if not same or moved == 0.0:
        sys.exit(1)


if __name__ == "__main__":
    main()
