"""Fold-to-rank CV driver (fall_multimodal_amd/cv.py) on CPU: world 2 over gloo, the fold function a
stand-in that records its fold (the GPU fold trains a SkeletonTransformer). Checks the reference's fold
construction (Multimodal_Fall3/model/cv_dataloader.py:155-167: KFold(10, shuffle, random_state) over the
unique video names) and that the ranks' folds are disjoint and cover all ten."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from fall_multimodal_amd.cv import cv_table, folds_of_rank, kfold_indices, run_cv


def _videos(n=400, per=7):
    rng = np.random.default_rng(3)
    return [f"vid{int(v):03d}" for v in np.sort(rng.integers(0, n // per, n))]


def _reference_folds(videos, seed=42):
    """cv_dataloader.py:155-167 restated: a window is held out of fold k iff its video is not in
    unique_video_names[train_idx]."""
    from sklearn.model_selection import KFold
    names = np.unique(videos)
    out = []
    for train_idx, _ in KFold(n_splits=10, shuffle=True, random_state=seed).split(names):
        keep = set(names[train_idx])
        out.append([i for i, v in enumerate(videos) if v not in keep])
    return out


def test_kfold_indices_match_reference():
    vids = _videos()
    folds = kfold_indices(vids, seed=42)
    ref = _reference_folds(vids)
    assert len(folds) == 10
    for (tr, held), r in zip(folds, ref):
        assert held.tolist() == r
        assert sorted(tr.tolist() + held.tolist()) == list(range(len(vids)))
    held_all = np.concatenate([h for _, h in folds])
    assert sorted(held_all.tolist()) == list(range(len(vids)))  # every window held out exactly once
    wf = kfold_indices(vids, seed=42, by="window")
    assert sorted(np.concatenate([h for _, h in wf]).tolist()) == list(range(len(vids)))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_folds_of_rank_disjoint_cover(world):
    got = [folds_of_rank(10, r, world) for r in range(world)]
    flat = sorted(k for g in got for k in g)
    assert flat == list(range(10))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vids = _videos()
        folds = kfold_indices(vids, seed=42)

        def fold_fn(k, train_idx, held_idx):
            return {"held": held_idx.tolist(), "ntrain": int(len(train_idx)), "accuracy": 0.5 + k / 100,
                    "precision": 0.1, "recall": 0.2, "f1": 0.3}

        res = run_cv(folds, fold_fn)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_run_cv_two_ranks_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=120)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _reference_folds(_videos())
    assert sorted(res[1]) == [1, 3, 5, 7, 9]              # rank 1 ran only its own folds
    assert sorted(res[0]) == list(range(10))               # rank 0 gathered every fold
    for k, row in res[0].items():
        assert row["rank"] == k % world
        assert row["held"] == ref[k]
    assert cv_table(res[0])["accuracy"] == [0.5 + k / 100 for k in range(10)]
