"""K-fold cross-validation with the folds sharded over ranks (BASELINE config 5: "GSTCAN
skeleton-transformer 10-fold CV, folds sharded across 8 GPUs").

Reference behaviour mirrored here:
  folds by unique video: KFold(n_splits=10, shuffle=True, random_state=seed).split(unique names);
      a window belongs to fold k's training set iff its video is in unique[train_idx], else to the
      held-out set (valid = test)                    Multimodal_Fall3/model/cv_dataloader.py:155-167
  folds by window (the transformer notebook's KFold_load_dataset_v2): KFold(n_splits,
      random_state=42, shuffle=True).split(features)     GSTCAN_HAR_conv_kfold_trans.ipynb cell 6
  per fold: a fresh model and optimizer, EPOCHS of training, evaluation of the held-out windows,
      per-fold precision / recall / F1 / accuracy collected into one table
                                                     Multimodal_Fall3/model/main_cross_validation.py:256-361

The reference runs the folds one after another in one process. The folds are independent, so here
rank r of a world of W runs folds r, r + W, r + 2W, ... with no collective on the data path (each
rank's step is the single-GPU step); only the per-fold result rows are gathered to rank 0 at the end.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def kfold_indices(videos, n_windows: int | None = None, seed: int = 42, n_splits: int = 10, by: str = "video"):
    """[(train_idx, held_idx)] per fold, window indices in file order (int64 arrays).
    by="video": cv_dataloader.py:155-167 (KFold over the sorted unique video names);
    by="window": the notebook's KFold over the windows themselves."""
    from sklearn.model_selection import KFold
    kf = KFold(n_splits=n_splits, shuffle=True, random_state=seed)
    if by == "window":
        n = len(videos) if n_windows is None else n_windows
        return [(np.asarray(tr, np.int64), np.asarray(te, np.int64)) for tr, te in kf.split(np.arange(n))]
    if by != "video":
        raise ValueError(f"by must be 'video' or 'window', got {by!r}")
    vids = np.asarray(videos)
    names = np.unique(vids)
    out = []
    for train_v, _ in kf.split(names):
        tr = np.isin(vids, names[train_v])
        out.append((np.flatnonzero(tr).astype(np.int64), np.flatnonzero(~tr).astype(np.int64)))
    return out


def folds_of_rank(n_folds: int, rank: int, world: int):
    """Folds rank `rank` of `world` runs: rank, rank + world, ... (disjoint, covering all folds)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside a world of {world}")
    return list(range(rank, n_folds, world))


def run_cv(folds, fold_fn, rank: int | None = None, world: int | None = None):
    """Run fold_fn(k, train_idx, held_idx) -> dict for this rank's folds; with torch.distributed
    initialised, the per-fold dicts are gathered to rank 0, which returns {fold: dict} for every
    fold (other ranks return their own). No other communication."""
    on = dist.is_available() and dist.is_initialized()
    if rank is None:
        rank = dist.get_rank() if on else 0
    if world is None:
        world = dist.get_world_size() if on else 1
    mine = {k: dict(fold_fn(k, *folds[k]), rank=rank) for k in folds_of_rank(len(folds), rank, world)}
    if not on or world == 1:
        return mine
    got = [None] * world if rank == 0 else None
    dist.gather_object(mine, got, dst=0)
    if rank != 0:
        return mine
    merged = {}
    for part in got:
        merged.update(part)
    return dict(sorted(merged.items()))


def cv_table(results):
    """The reference's precision_recall_f1.csv columns (main_cross_validation.py:351-357), fold order."""
    keys = ("precision", "recall", "f1", "accuracy")
    return {k: [results[f][k] for f in sorted(results)] for k in keys}


def sktr_fold_fn(x: torch.Tensor, y: torch.Tensor, epochs: int, batch: int, lr: float = 1e-3, seed: int = 0,
                 precision: str = "bf16", device=None):
    """fold_fn training a fresh SkeletonTransformer (skeleton_transformer.py:360-435) on one fold:
    x [N, 3, T, V, M] fp32 and y [N, C] soft labels resident on the device; `epochs` passes over the
    training windows in shuffled full batches (the step's batch is fixed), then one eval-mode pass over
    the held-out windows: top-1 accuracy and macro precision / recall / F1 (evaluate.test's metrics)."""
    from . import evaluate as fe
    from .sktr import SkeletonTransformer, SktrStep

    def fold(k, train_idx, held_idx):
        dev = device or x.device
        torch.manual_seed(seed + k)
        model = SkeletonTransformer(3, x.shape[3], x.shape[2], y.shape[1], persons=x.shape[4], device=dev,
                                    precision=precision, seed=seed + k)
        step = SktrStep(model, batch, lr=lr)
        tr = torch.from_numpy(train_idx).to(dev)
        g = torch.Generator().manual_seed(seed + k)
        nsteps = 0
        for _ in range(epochs):
            order = tr[torch.randperm(len(tr), generator=g).to(dev)]
            for b in range(len(order) // batch):
                idx = order[b * batch:(b + 1) * batch]
                step(x.index_select(0, idx).contiguous(), y.index_select(0, idx).contiguous())
                nsteps += 1
        model.eval()
        outs = []
        held = torch.from_numpy(held_idx).to(dev)
        with torch.no_grad():
            for b in range(0, len(held), batch):
                outs.append(model(x.index_select(0, held[b:b + batch]).contiguous()))
        out = torch.cat(outs)
        lab = y.index_select(0, held)
        m = fe.class_metrics(out.argmax(1).cpu().numpy(), lab.argmax(1).cpu().numpy(), y.shape[1])
        return {"accuracy": fe.cal_top_k_accuracy(out, lab, (1,))[0], "precision": m["precision"],
                "recall": m["recall"], "f1": m["f1"], "train_steps": nsteps, "held_out": int(len(held_idx))}

    return fold
