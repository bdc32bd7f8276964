"""Data parallel on the device (needs an MI355X): two ranks (torchrun, both on cuda:0, gloo
reducing the device gradients through the host) train their own clip shards through
TrainStep — backward in two phases, the head bucket's all-reduce ordered after phase 1's
per-queue events and overlapping phase 2, RMSprop with the 1/world scale. The first step's
reduced gradient must equal the mean of the per-shard gradients (each computed alone, within
10x the backward's run-to-run floor) and its update RMSprop on it; the replicas must end with
bit-identical parameters (tools/dp_check.py).
The 8-GPU RCCL run is the driver's scaling bench; this checks the same code path on one GPU."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_two_rank_replicas_stay_identical(precision):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "dp_check.py"), "--backend",
           "gloo", "--same-device", "--steps", "3", "--precision", precision]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(lines[-1])
    assert res["world"] == 2 and res["replicas_identical"] and res["max_param_change"] > 0
    s1 = res["first_step_vs_mean_of_shard_grads"]
    print(precision, s1)
    assert s1["ok"], s1
