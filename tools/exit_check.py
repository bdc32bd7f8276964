#!/usr/bin/env python3
"""Clean process exit after the library's stateful models have run.

Runs two training steps each of the sensor-only CNN_BiLSTM (the cooperative CNN1D: group barriers,
the device status ring of status_ring.h) and of TARGCN in bf16 (the node-partitioned GRU: its status
ring and pinned host words), then leaves the handles to be released by normal interpreter teardown
and returns from main: the exit status must be 0. Round 5 recorded SIGSEGVs inside exit handlers,
after rocprofv3's finalisation, of `python tools/cnn1d_time.py` while the CNN1D was launched with
hipLaunchCooperativeKernel (gpurun_out/c27-c30.log). Run plainly by
tests/test_gpu_exit.py and under `rocprofv3 --kernel-trace` by tools/gpu_session.sh `exit_prof`.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(what):
    """what: "both" (default), "cnn" (CNN_BiLSTM only), "targcn" (TARGCN only), "torch" (a torch op only,
    the library not loaded), "lib" (the library loaded, no kernel launched)."""
    dev = torch.device("cuda", 0)
    if what == "torch":
        x = torch.randn(1024, device=dev)
        print("exit_check: torch op", float((x * 2).sum()) * 0 + 1, flush=True)
        print("exit_check: steps done, exiting", flush=True)
        return 0
    import fall_multimodal_amd as f3
    from oracle import targcn_cpu as tg
    if what == "lib":
        f3._lib.lib()
        torch.cuda.synchronize()
        print("exit_check: steps done, exiting", flush=True)
        return 0
    if what in ("both", "cnn"):
        g = torch.Generator().manual_seed(0)
        m = f3.CNN_BiLSTM(device=dev)
        x = torch.randn(256, 30, 4, generator=g).to(dev)
        lab = torch.softmax(torch.randn(256, m.spec.num_class, generator=g), 1).to(dev)
        step = f3.TrainStep(m, 256, lr=1e-3)
        for _ in range(2):
            step(None, x, lab)
        m.device_status(wait=True)
    if what in ("both", "targcn"):
        V, B = 17, 64
        t = f3.TARGCN(num_nodes=V, device=dev, precision="bf16")
        t.load_state_dict(tg.init_state(V, 11))
        src, label = (torch.from_numpy(a).to(dev) for a in tg.synthetic_source(B, V, 11, 5))
        ts = f3.TargcnStep(t, B, lr=1e-5)
        for _ in range(2):
            ts.forward_backward(src, label)
        t.device_status(wait=True)
    torch.cuda.synchronize()
    print("exit_check: steps done, exiting", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "both"))
