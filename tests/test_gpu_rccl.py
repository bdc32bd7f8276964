"""Process-level checks on the device (needs an MI355X), each in a fresh child process started before
this process's GPU work can matter to it:

* RCCL first contact: ONE torchrun rank creates the production process group,
  init_process_group("nccl", pg_options=rccl_options()), and trains phased TrainSteps with GradSync
  forced to issue both all-reduce buckets at world 1 (the head bucket on the high-priority side stream
  after f3_net_wait_phase1, the tail after phase 2). A world-1 sum is the identity, so parameters and
  gradients must equal bit for bit those of the same phased steps without a collective
  (tools/rccl_check.py). The 8-rank run of the same code is the driver's scaling bench.
* Clean exit: a CNN_BiLSTM (cooperative CNN1D) and a TARGCN (node-partitioned GRU)
  training run in a child that then exits through normal interpreter teardown: exit status 0
  (tools/exit_check.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _has_gpu():
    import torch
    return torch.cuda.is_available()


def test_rccl_world1_phased_step_matches_step_without_collective():
    if not _has_gpu():
        pytest.skip("no HIP device")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tools", "rccl_check.py"),
           "--steps", "3", "--precision", "bf16x3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, r.stdout[-2000:] + r.stderr[-3000:]
    res = json.loads(lines[-1])
    print(res)
    assert res["backend"] == "nccl" and res["world"] == 1 and res["grad_sync_active"]
    assert res["params_bit_identical"] and res["grads_bit_identical"] and res["plain_allreduce_identity"]


def test_child_process_exits_cleanly_after_cnn1d_and_targcn_steps():
    if not _has_gpu():
        pytest.skip("no HIP device")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "exit_check.py")], capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert "steps done" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
