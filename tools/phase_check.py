#!/usr/bin/env python3
"""One rank: gradients of the two-phase backward (the DP path) vs the one-pass backward, and two
one-pass runs against each other (the run-to-run floor), for fp32 and bf16."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    dev = torch.device("cuda")
    res = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=dev,
                                          precision=prec)
        B = int(os.environ.get("B", "16"))
        step = f3.TrainStep(model, B, lr=1e-3)
        sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(B, 18, 11, 6, 5))
        lb = step.prepare(sk, se, lb)
        runs = {}
        for name, phased in (("p0a", False), ("p0b", False), ("ph", True)):
            step.forward_loss(sk, se, lb)
            if phased:
                step.backward_phase(1)
                step.backward_phase(2)
            else:
                step.backward_phase(0)
            torch.cuda.synchronize()
            runs[name] = step.grads.double().clone()
        gmax = float(runs["p0a"].abs().max())
        split = step.sync.split
        res[prec] = {"p0_vs_p0": float((runs["p0a"] - runs["p0b"]).abs().max()) / gmax,
                     "phased_vs_p0": float((runs["ph"] - runs["p0a"]).abs().max()) / gmax,
                     "phased_vs_p0_head": float((runs["ph"] - runs["p0a"])[:split].abs().max()) / gmax,
                     "phased_vs_p0_tail": float((runs["ph"] - runs["p0a"])[split:].abs().max()) / gmax}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
