#!/usr/bin/env python3
"""Top-1 accuracy at convergence of the ORACLE (CPU restatement of the reference, pinned to its
golden vectors) on the separable synthetic task, for tests/test_gpu_parity.py::
test_top1_at_convergence ("train identical seeds for N epochs; compare accuracy to
±0.5 %"). The HIP fp32 and bf16 paths train the same recipe on the GPU and are compared with the
numbers this script records:

    python tools/gen_convergence.py > tests/golden/convergence.json     (~15 min on 8 cores)

Recipe (fixed here, read back by the test): 3-stream coco_mmpose model, V=18, S=6, 11 classes,
init seed 123; STEPS steps of RMSprop (alpha 0.99, eps 1e-8) at B=32 on fresh synthetic batches
(seed 10000 + step, separation 1.8, spread 0.15) with a cosine learning rate from 1e-3 to 0 over the
run (the reference's CosineLRScheduler, t_initial = STEPS, no warm-up, per step); held-out top-1 on
1024 clips (seed 999, same generator) in eval mode (BN running statistics, the reference's
valid/test protocol) and with batch statistics."""
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import model_cpu as oc  # noqa: E402
from oracle.prng import synthetic_batch  # noqa: E402

RECIPE = {"model": "two_stgcan_bilstm", "layout": "coco_mmpose", "V": 18, "S": 6, "classes": 11, "init_seed": 123,
          "steps": 400, "batch": 32, "batch_seed0": 10000, "lr0": 1e-3, "separation": 1.8, "spread": 0.15,
          "heldout": 1024, "heldout_seed": 999, "checkpoints": [100, 200, 300, 400]}


def lr_at(step, r=RECIPE):
    return 0.5 * r["lr0"] * (1 + math.cos(math.pi * step / r["steps"]))


def main():
    r = RECIPE
    torch.set_num_threads(int(os.environ.get("THREADS", os.cpu_count() or 1)))
    spec = oc.Spec(model=r["model"], layout=r["layout"], num_class=r["classes"], sensor_dim=r["S"])
    st = oc.init_state(spec, r["init_seed"])
    kw = dict(separation=r["separation"], spread=r["spread"])
    tsk, tse, tlb = (torch.from_numpy(x) for x in synthetic_batch(r["heldout"], r["V"], r["classes"], r["S"],
                                                                  r["heldout_seed"], **kw))
    truth = tlb.argmax(1).numpy()
    sq = {k: torch.zeros_like(v) for k, v in st.items() if not oc.is_buffer(k)}
    out = {"recipe": r, "oracle": {}, "losses": []}
    t0 = time.time()
    for i in range(r["steps"]):
        b = [torch.from_numpy(x) for x in synthetic_batch(r["batch"], r["V"], r["classes"], r["S"],
                                                          r["batch_seed0"] + i, **kw)]
        _, loss, _ = oc.train_step(st, spec, *b, sq=sq, lr=lr_at(i))
        out["losses"].append(round(float(loss), 6))
        if i + 1 in r["checkpoints"]:
            with torch.no_grad():
                ev = oc.forward(st, spec, tsk, tse, training=False)
                sc = {k: (v.clone() if oc.is_buffer(k) else v) for k, v in st.items()}
                bt = oc.forward(sc, spec, tsk, tse, training=True)
            out["oracle"][str(i + 1)] = {"eval": float((ev.argmax(1).numpy() == truth).mean()),
                                         "batch": float((bt.argmax(1).numpy() == truth).mean())}
            print(f"step {i + 1}: {out['oracle'][str(i + 1)]} ({time.time() - t0:.0f} s)", file=sys.stderr, flush=True)
    out["threads"] = torch.get_num_threads()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
