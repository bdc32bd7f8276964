"""Data-parallel host logic on CPU with the gloo backend, world_size 2 (the GPU path uses
the same code over RCCL): the two-bucket gradient all-reduce that overlaps backward phase 2
sums every element exactly once, and the 1/world RMSprop scaling gives the averaged-gradient
update the single-process reference would make."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, split, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fall_multimodal_amd.train import GradSync
        g = torch.Generator().manual_seed(rank)
        grads = torch.randn(n, generator=g)
        mine = grads.clone()
        sync = GradSync(grads, split)
        assert sync.world == world
        sync.start_head()
        grads[split:] += 0.0          # "phase 2" compute touching only the tail
        sync.start_tail()
        sync.finish()
        q.put((rank, mine.numpy(), grads.numpy().copy()))  # by value: a shared tensor dies with its sender
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("split", [0, 37, 1000])
def test_gradsync_two_buckets_gloo(split):
    world, n = 2, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, split, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, mine, out = q.get(timeout=120)
        res[r] = (mine, out)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    total = torch.from_numpy(res[0][0] + res[1][0])
    for r in range(world):
        torch.testing.assert_close(torch.from_numpy(res[r][1]), total, rtol=0, atol=1e-6)


def test_rmsprop_grad_scale_is_gradient_average():
    """RMSprop on sum/world (what f3_rmsprop_step(grad_scale=1/world) computes) equals RMSprop
    on the mean gradient: oracle restatement of torch.optim.RMSprop (optimizer.py:20-21)."""
    from oracle.model_cpu import rmsprop_step
    torch.manual_seed(0)
    world = 4
    per_rank = [torch.randn(50) for _ in range(world)]
    p0 = torch.randn(50)
    a, b = {"w": p0.clone()}, {"w": p0.clone()}
    sa, sb = {"w": torch.zeros(50)}, {"w": torch.zeros(50)}
    rmsprop_step(a, {"w": sum(per_rank) * (1.0 / world)}, sa)
    rmsprop_step(b, {"w": torch.stack(per_rank).mean(0)}, sb)
    torch.testing.assert_close(a["w"], b["w"], rtol=0, atol=1e-7)
