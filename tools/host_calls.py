"""Host-side duration of each TrainStep call in a back-to-back loop (no sync between calls):
shows whether the host runs ahead of the GPU or is held back every step.
    python tools/host_calls.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import fall_multimodal_amd as f3
    from oracle.prng import synthetic_batch
    dev = torch.device("cuda")
    B, V, S, C = 256, 18, 6, 11
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, C, S, device=dev,
                                      precision="bf16")
    step = f3.TrainStep(model, B, lr=1e-3)
    sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(B, V, C, S, 100))
    for _ in range(3):
        step(sk, se, lb)
    torch.cuda.synchronize()
    ts = []
    t0 = time.perf_counter()
    for _ in range(12):
        a = time.perf_counter()
        step(sk, se, lb)
        ts.append((time.perf_counter() - a) * 1e3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("host ms per call:", " ".join(f"{t:.2f}" for t in ts))
    print(f"loop {(t1 - t0) * 1e3 / 12:.3f} ms/step on the host, {(t2 - t0) * 1e3 / 12:.3f} ms/step incl. the drain")
    # the same with the forward / backward / optimizer pieces timed separately on the host
    torch.cuda.synchronize()
    label = step.prepare(sk, se, lb)
    for name, fn in (("forward_loss", lambda: step.forward_loss(sk, se, label)),
                     ("backward", lambda: step.backward_phase(0)), ("rmsprop", step.optimizer_step)):
        torch.cuda.synchronize()
        a = time.perf_counter()
        fn()
        b = time.perf_counter()
        torch.cuda.synchronize()
        print(f"{name}: host {(b - a) * 1e3:.3f} ms, with the GPU {(time.perf_counter() - a) * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
