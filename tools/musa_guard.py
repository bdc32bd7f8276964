"""Out-of-region write hunt for the musa_model step: with F3_MU_GUARD set, the workspace plan puts a
guard band after every region; the workspace is filled with a byte pattern, one training step
(forward + backward, DropBlock on) runs, and every guard band that changed is reported with its
index (the region before it, in plan order) and the changed byte range. GPU only:
    F3_MU_GUARD=65536 python tools/musa_guard.py [--batch 4]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--dropblock", type=int, default=1)
    a = ap.parse_args()
    gb = int(os.environ.get("F3_MU_GUARD", "0"))
    assert gb > 0, "set F3_MU_GUARD"
    import fall_multimodal_amd as f3
    import fall_multimodal_amd._lib as L
    from oracle import musa_cpu as mu
    from oracle.prng import synthetic_batch
    d = torch.device("cuda")
    st = mu.init_state(77)
    m = f3.musa.Model(11, 14, 300, f3.musa.adjGraph("coco_cut", "uniform"), True, True, 41, device=d,
                      dropblock=bool(a.dropblock))
    m.load_state_dict(st, strict=True)
    B = a.batch
    step = f3.musa.MusaStep(m, B)
    offs = (ctypes.c_int64 * 512)()
    n = L.lib().f3_musa_guards(m._native.h, B, offs, 512)
    print("guards", n, "workspace bytes", step.ws.numel(), flush=True)
    pat = 0x5A
    step.ws.fill_(pat)
    x, _, lab = synthetic_batch(B, 14, 11, 1, 5)
    step.forward_backward(torch.from_numpy(x).to(d), torch.from_numpy(lab).to(d), seed=7)
    torch.cuda.synchronize()
    ws = step.ws.cpu().numpy()
    bad = 0
    for i in range(n):
        g = ws[offs[i]:offs[i] + gb]
        idx = np.nonzero(g != pat)[0]
        if idx.size:
            bad += 1
            print(f"guard {i} (after region {i}) at {offs[i]}: {idx.size} bytes changed, first +{idx[0]} last +{idx[-1]}",
                  flush=True)
    print("changed guards:", bad, flush=True)


if __name__ == "__main__":
    main()
