"""bench.py's multi-GPU launch: `bench.py --gpus N` with no torch.distributed
environment starts N ranks itself and asserts that the launcher's world equals N. Checked on CPU:
the ranks come up and see each other over gloo (--launch-check), and a real run asking for more
GPUs than the node has fails loudly instead of printing an n_gpus: 1 line."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT, env=env)


def test_gpus_2_starts_two_ranks():
    r = _run("--gpus", "2", "--launch-check")
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["world"] == 2 and rec["ranks_seen"] == [0, 1]


def test_gpus_beyond_node_fails_loudly():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    r = _run("--gpus", str(n), "--steps", "1", "--warmup", "0")
    assert r.returncode != 0
    assert "refusing" in (r.stdout + r.stderr)
    assert '"n_gpus"' not in r.stdout


def test_world_mismatch_rejected():
    env_args = ("--gpus", "2", "--launch-check")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *env_args], capture_output=True, text=True,
                       timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "launcher started 1 rank" in (r.stdout + r.stderr)
