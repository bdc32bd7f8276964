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
    # the same pieces from an idle device (synchronised before each step): pure host cost, no throttling
    acc = {k: 0.0 for k in acc}
    for _ in range(n):
        torch.cuda.synchronize()
        a = time.perf_counter(); opt.zero_grad(); b = time.perf_counter(); acc["zero_grad"] += b - a
        out = model(sk, se); c = time.perf_counter(); acc["forward"] += c - b
        loss = loss_fn(out, lb); d = time.perf_counter(); acc["loss"] += d - c
        loss.backward(); e = time.perf_counter(); acc["backward"] += e - d
        opt.step(); f = time.perf_counter(); acc["step"] += f - e
    torch.cuda.synchronize()
    print("from idle:", " ".join(f"{k} {v / n * 1e3:.3f}" for k, v in acc.items()), "ms host per step")
    # where the forward / backward / step host time goes (cProfile over 5 steps from idle)
    import cProfile
    import io
    import pstats
    pr = cProfile.Profile()
    for _ in range(5):
        torch.cuda.synchronize()
        pr.enable()
        opt.zero_grad()
        loss_fn(model(sk, se), lb).backward()
        opt.step()
        pr.disable()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
    print(buf.getvalue())
    # the fused TrainStep's single call, from idle and back to back
    step = f3.TrainStep(model, sk.shape[0], lr=1e-3)
    for _ in range(3):
        step(sk, se, lb)
    torch.cuda.synchronize()
    hi = 0.0
    for _ in range(n):
        torch.cuda.synchronize()
        a = time.perf_counter(); step(sk, se, lb); hi += time.perf_counter() - a
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step(sk, se, lb)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"TrainStep: from idle {hi / n * 1e3:.3f} ms host; back to back host {(t1 - t0) / n * 1e3:.3f}, "
          f"with the drain {(t2 - t0) / n * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
