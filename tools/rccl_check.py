#!/usr/bin/env python3
"""First contact of the RCCL gradient path on a one-GPU box (run under torchrun, ONE rank):

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port P \
        tools/rccl_check.py [--steps 3] [--precision bf16x3]

The rank creates the production process group, init_process_group("nccl", pg_options=rccl_options())
(RCCL with its internal stream at high priority), and trains K phased TrainSteps with GradSync forced
to issue both all-reduce buckets at world 1: the head bucket from GradSync's high-priority side
stream after f3_net_wait_phase1 (phase 1's per-queue events), the tail bucket after phase 2. A world-1
sum is the identity, so the parameters must equal, bit for bit, those of the same phased steps
without any collective (the bf16x3 step is bit-deterministic: tests/test_gpu_determinism.py).
Prints one JSON line; exit 1 on a mismatch. The 8-GPU run of this path is the driver's scaling bench.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def train(dev, precision, steps, batch, force_sync):
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    torch.manual_seed(0)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                      precision=precision)
    step = f3.TrainStep(model, batch, lr=1e-3, phased=True, force_sync=force_sync)
    for i in range(steps):
        step(*[torch.from_numpy(x).to(dev) for x in synthetic_batch(batch, 18, 11, 6, 500 + i)])
    torch.cuda.synchronize()
    return model.flat_parameters().clone(), step.grads.clone(), step.sync


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--precision", default="bf16x3")
    a = ap.parse_args()
    assert int(os.environ["WORLD_SIZE"]) == 1, "one rank: the one-GPU first contact"
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from fall_multimodal_amd.train import rccl_options
    dist.init_process_group("nccl", pg_options=rccl_options())
    backend = dist.get_backend()
    p_dp, g_dp, sync = train(dev, a.precision, a.steps, a.batch, True)
    p_ref, g_ref, _ = train(dev, a.precision, a.steps, a.batch, False)
    # a plain RCCL all-reduce of a known vector at world 1 (identity), on torch's current stream
    v = torch.arange(1024, dtype=torch.float32, device=dev)
    dist.all_reduce(v)
    torch.cuda.synchronize()
    res = {"backend": backend, "world": dist.get_world_size(), "steps": a.steps, "precision": a.precision,
           "grad_sync_active": sync.active, "side_stream_priority": sync._side.priority if sync._side else None,
           "params_bit_identical": bool(torch.equal(p_dp, p_ref)), "grads_bit_identical": bool(torch.equal(g_dp, g_ref)),
           "params_moved": float((p_ref - p_ref.new_zeros(())).abs().max()) > 0,
           "plain_allreduce_identity": bool(torch.equal(v, torch.arange(1024, dtype=torch.float32, device=dev)))}
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()
    ok = res["params_bit_identical"] and res["grads_bit_identical"] and res["plain_allreduce_identity"] and \
        res["grad_sync_active"] and backend == "nccl"
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
