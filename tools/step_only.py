"""The bench's 3-stream training step alone (B=256, V=18, S=6, eager; precision from F3_STEP_PREC,
default bf16x3, the headline mode), for kernel traces:
    rocprofv3 --kernel-trace -d gpurun_out/step -o run -- python tools/step_only.py [steps] [autograd]
    python tools/timeline.py gpurun_out/step/run_results.db --list
With `autograd` the step is the reference loop body through the custom ops instead of TrainStep
(opt.zero_grad(); CrossEntropyLoss()(model(x, s), y).backward(); f3.RMSprop.step(), model/main.py:112-127)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda")
    B, V, S, C = 256, 18, 6, 11
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, C, S, device=dev,
                                      precision=os.environ.get("F3_STEP_PREC", "bf16x3"))
    sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(B, V, C, S, 100))
    if len(sys.argv) > 2 and sys.argv[2] == "autograd":
        opt = f3.RMSprop(model.parameters(), lr=1e-3)
        loss_fn = torch.nn.CrossEntropyLoss()

        def step(sk, se, lb):
            opt.zero_grad()
            loss_fn(model(sk, se), lb).backward()
            opt.step()
    else:
        step = f3.TrainStep(model, B, lr=1e-3)
    for _ in range(3):
        step(sk, se, lb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(sk, se, lb)
    t1 = time.perf_counter()  # host submission done (no per-step sync in the loop)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{(t2 - t0) / steps * 1e3:.3f} ms/step (host submit {(t1 - t0) / steps * 1e3:.3f} ms/step)")


if __name__ == "__main__":
    main()
