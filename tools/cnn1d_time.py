"""Sensor CNN1D time in the B=256 CNN_BiLSTM training step (bench.py cnn1d_stage_times), for the
cooperative form and the per-layer launches (F3_CNN1D_COOP=0), interleaved over rounds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import fall_multimodal_amd as f3  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
m = f3.CNN_BiLSTM(device=dev)
x = torch.randn(256, 30, 4, generator=g).to(dev)
lab = torch.softmax(torch.randn(256, m.spec.num_class, generator=g), 1).to(dev)
step = f3.TrainStep(m, 256, lr=1e-3)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for coop in ("1", "0"):
        os.environ["F3_CNN1D_COOP"] = coop
        res = bench.cnn1d_stage_times(m, step, x, lab, 256, 4)
        print(json.dumps({"round": r, "coop": coop, "forward_us": res["forward"]["us"],
                          "backward_us": res["backward"]["us"], "total_us": res["total_us"]}), flush=True)
