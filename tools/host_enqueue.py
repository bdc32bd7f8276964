#!/usr/bin/env python3
"""Host-side enqueue cost of the training step (is the GPU ever starved by the launcher?).

    python tools/host_enqueue.py [--steps 30]

Times each host call of TrainStep's eager step (forward+loss, backward, RMSprop) without
synchronising, over back-to-back steps, and the GPU step time; prints one JSON line."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--no-single", action="store_true")
    a = ap.parse_args()
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                      precision="bf16")
    step = f3.TrainStep(model, a.batch, lr=1e-3)
    sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(a.batch, 18, 11, 6, 1))
    for _ in range(5):
        step(sk, se, lb)
    torch.cuda.synchronize()
    host = {"forward_loss": 0.0, "backward": 0.0, "rmsprop": 0.0}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t = time.perf_counter()
        step.forward_loss(sk, se, lb)
        t1 = time.perf_counter()
        step.backward_phase(0)
        t2 = time.perf_counter()
        step.optimizer_step()
        t3 = time.perf_counter()
        host["forward_loss"] += t1 - t
        host["backward"] += t2 - t1
        host["rmsprop"] += t3 - t2
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    res = {k: round(v / a.steps * 1e3, 3) for k, v in host.items()}
    res.update({"host_ms_per_step": round(t_enq / a.steps * 1e3, 3), "gpu_ms_per_step": round(t_all / a.steps * 1e3, 3)})
    if a.no_single:
        print(json.dumps(res), flush=True)
        return
    # a single step from idle: enqueue vs completion
    torch.cuda.synchronize()
    t = time.perf_counter()
    step(sk, se, lb)
    te = time.perf_counter()
    torch.cuda.synchronize()
    res.update({"single_enqueue_ms": round((te - t) * 1e3, 3), "single_total_ms": round((time.perf_counter() - t) * 1e3, 3)})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
