"""Repeat the musa golden-case backward a few times on the GPU and report, per run, the tensors
furthest from the fp64 oracle and the run-to-run spread (is a gradient gap a bug or ordering noise?).
GPU only: python tools/musa_repeat.py [--runs 4]"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import musa_cpu as mu  # noqa: E402
from tests.golden_util import GOLDEN  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    a = ap.parse_args()
    import fall_multimodal_amd as f3
    d = torch.device("cuda")
    torch.set_num_threads(16)
    z = np.load(os.path.join(GOLDEN, "musa_b4.npz"))
    g = {k: z[k] for k in z.files}
    st = mu.init_state(int(g["seed"][0]))
    st64 = {k: (v.double() if v.dtype == torch.float32 else v.clone()) for k, v in st.items()}
    _, _, ref = mu.train_step(st64, torch.from_numpy(g["x"]).double(), torch.from_numpy(g["label"]).double(),
                              draws=None)
    names = [k for k in ref if float(ref[k].abs().max()) > 1e-12]
    runs = []
    for r in range(a.runs):
        m = f3.musa.Model(11, 14, 300, f3.musa.adjGraph("coco_cut", "uniform"), True, True, 41, device=d,
                          dropblock=False)
        m.load_state_dict(st, strict=True)
        m.train()
        out = m(torch.from_numpy(g["x"]).to(d))
        torch.nn.CrossEntropyLoss()(out, torch.from_numpy(g["label"]).to(d)).backward()
        ours = {n: p.grad.detach().cpu().numpy() for n, p in m.named_parameters() if p.grad is not None}
        rel = {k: float(np.abs(ours[k] - ref[k].numpy()).max() / max(float(ref[k].abs().max()), 1e-2))
               for k in names if k in ours}
        top = sorted(rel.items(), key=lambda t: -t[1])[:5]
        print(f"run {r}: " + ", ".join(f"{k} {v:.2e}" for k, v in top), flush=True)
        runs.append(ours)
    for r in range(1, len(runs)):
        diff = {k: float(np.abs(runs[r][k] - runs[0][k]).max() / max(float(np.abs(runs[0][k]).max()), 1e-2))
                for k in runs[0]}
        top = sorted(diff.items(), key=lambda t: -t[1])[:3]
        print(f"run {r} vs run 0: " + ", ".join(f"{k} {v:.2e}" for k, v in top), flush=True)
    k = "stream_mot.3.sep11.seq.3.weight"
    if k in runs[0]:
        e = np.abs(runs[0][k] - ref[k].numpy())
        i = np.unravel_index(int(e.argmax()), e.shape)
        print(k, "shape", e.shape, "worst at", i, "ours", runs[0][k][i], "ref", float(ref[k].numpy()[i]),
              "n>1e-4:", int((e > 1e-4).sum()), "max|ref|", float(ref[k].abs().max()))


if __name__ == "__main__":
    main()
