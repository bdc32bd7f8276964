"""Host cost of the reference loop body through the custom ops (model(x) -> CE -> backward ->
f3.RMSprop.step), piece by piece, against the GPU time of the same step.
    python tools/autograd_host.py"""
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
    sk, se, lb = (torch.from_numpy(x).to(dev) for x in synthetic_batch(B, V, C, S, 100))
    opt = f3.RMSprop(model.parameters(), lr=1e-3)
    loss_fn = torch.nn.CrossEntropyLoss()
    for _ in range(3):
        opt.zero_grad()
        loss_fn(model(sk, se), lb).backward()
        opt.step()
    torch.cuda.synchronize()
    acc = {"zero_grad": 0.0, "forward": 0.0, "loss": 0.0, "backward": 0.0, "step": 0.0}
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter(); opt.zero_grad(); b = time.perf_counter(); acc["zero_grad"] += b - a
        out = model(sk, se); c = time.perf_counter(); acc["forward"] += c - b
        loss = loss_fn(out, lb); d = time.perf_counter(); acc["loss"] += d - c
        loss.backward(); e = time.perf_counter(); acc["backward"] += e - d
        opt.step(); f = time.perf_counter(); acc["step"] += f - e
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(" ".join(f"{k} {v / n * 1e3:.3f}" for k, v in acc.items()), "ms host per step")
    print(f"host loop {(t1 - t0) / n * 1e3:.3f} ms/step, with the drain {(t2 - t0) / n * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
