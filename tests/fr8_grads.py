"""Helper of tests/test_gpu_bnbwd_fr8.py (not a test module): one forward + backward of the B=32
3-stream step in the precision given on the command line, gradients and logits saved to an .npz.
Run in a child process so that its environment (F3_BNBWD_FR, read once per process) applies."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model_cpu as oc  # noqa: E402
from oracle.prng import synthetic_batch  # noqa: E402


def run(precision, out_path):
    import fall_multimodal_amd as f3
    d = torch.device("cuda")
    spec = oc.Spec(model="two_stgcan_bilstm", layout="coco_mmpose", num_class=11, sensor_dim=6)
    model = f3.TwoStreamSTGCAN_BiLSTM(3, {"layout": "coco_mmpose", "strategy": "spatial"}, 11, 6, device=d,
                                      precision=precision)
    model.load_state_dict(oc.init_state(spec, 21))
    B = 32
    step = f3.TrainStep(model, B, lr=0.0)
    sk, se, lb = (torch.from_numpy(x).to(d) for x in synthetic_batch(B, 18, 11, 6, 8))
    step.forward_backward(sk, se, step.prepare(sk, se, lb))
    torch.cuda.synchronize()
    np.savez(out_path, grads=step.grads.cpu().numpy(), logits=step.out.cpu().numpy())


if __name__ == "__main__":
    run(sys.argv[1], sys.argv[2])
