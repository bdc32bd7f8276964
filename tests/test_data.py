"""Data step and eval-step host logic (CPU): the reference's window format, its video-wise
splits, DataLoader sample order, per-sample layout, and the eval metrics / checkpoint format.

The reference behaviour is restated here from model/dataloader.py:177-247,
model/cv_dataloader.py:155-167, model/dataset.py:12-28 and model/main.py:57-77 (the
reference modules themselves need termcolor / yacs / tensorboard, absent in this image)."""
import os

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader, Dataset

from fall_multimodal_amd import data as fd
from fall_multimodal_amd import evaluate as fe


def make_windows(n_videos=23, per_video=5, T=30, V=18, S=6, C=11, seed=0):
    rng = np.random.default_rng(seed)
    videos = [f"S{v // 4}_A{v % 11}_T{v}" for v in range(n_videos) for _ in range(per_video)]
    n = len(videos)
    cls = rng.integers(0, C, n)
    lab = np.eye(C, dtype=np.float32)[cls] * 0.9 + 0.01
    return fd.Windows(videos, rng.normal(size=(n, T, V, 3)).astype(np.float32),
                      rng.normal(size=(n, T, S)).astype(np.float32), lab.astype(np.float32))


def test_window_file_roundtrip(tmp_path):
    w = make_windows()
    a, b = tmp_path / "a.pkl", tmp_path / "b.pkl"
    fd.save_windows(a, w.subset(np.arange(len(w)) < 40))
    fd.save_windows(b, w.subset(np.arange(len(w)) >= 40))
    r = fd.load_windows([str(a), str(b)])
    assert r.videos == w.videos
    for x, y in ((r.features, w.features), (r.sensors, w.sensors), (r.labels, w.labels)):
        assert x.dtype == np.float32 and np.array_equal(x, y)


def _reference_split(videos, seed):
    """model/dataloader.py:204-220, restated: membership loop over the windows."""
    from sklearn.model_selection import train_test_split
    names = np.unique(videos)
    tr, other = train_test_split(names, test_size=0.4, shuffle=True, random_state=seed)
    va, te = train_test_split(other, test_size=0.5, shuffle=True, random_state=seed)
    out = {"train": [], "valid": [], "test": []}
    for i, v in enumerate(videos):
        out["train" if v in tr else "valid" if v in va else "test"].append(i)
    return out


@pytest.mark.parametrize("seed", [42, 7])
def test_video_split_matches_reference(seed):
    w = make_windows()
    ours = fd.video_split(w, seed)
    ref = _reference_split(w.videos, seed)
    for k in ("train", "valid", "test"):
        assert np.array_equal(ours[k].features, w.features[ref[k]]), k
        assert ours[k].videos == [w.videos[i] for i in ref[k]]
    # no video straddles two splits
    sets = [set(ours[k].videos) for k in ("train", "valid", "test")]
    assert not (sets[0] & sets[1] or sets[0] & sets[2] or sets[1] & sets[2])


def test_video_kfold_matches_reference():
    from sklearn.model_selection import KFold
    w = make_windows()
    folds = fd.video_kfold(w, 42)
    names = np.unique(w.videos)
    ref = list(KFold(n_splits=10, shuffle=True, random_state=42).split(names))
    assert len(folds) == 10
    for f, (tr, _) in zip(folds, ref):
        idx = [i for i, v in enumerate(w.videos) if v in names[tr]]
        assert np.array_equal(f["train"].labels, w.labels[idx])
        assert f["valid"] is f["test"]


def test_dataloader_order_matches_torch():
    """Three loaders sharing one generator (train shuffled + drop_last, valid/test not), as
    model/dataloader.py:232-247 builds them, over three epochs."""
    class Idx(Dataset):
        def __len__(self):
            return 23

        def __getitem__(self, i):
            return i

    g = torch.Generator().manual_seed(42)
    dls = {k: DataLoader(Idx(), batch_size=4, shuffle=k == "train", drop_last=k == "train", generator=g)
           for k in ("train", "valid", "test")}
    g2 = torch.Generator().manual_seed(42)
    for _ in range(3):
        for k in ("train", "valid", "test"):
            ref = torch.cat(list(dls[k])).tolist()
            ours = fd.dataloader_order(23, g2, k == "train").tolist()
            if k == "train":
                ours = ours[:20]
            assert ours == ref, k


class _RefDataset(Dataset):
    """model/dataset.py:12-28 restated: per-item tensors, skeleton.permute(2,0,1)."""

    def __init__(self, w):
        self.w = w

    def __len__(self):
        return len(self.w)

    def __getitem__(self, i):
        return (torch.tensor(self.w.features[i]).permute(2, 0, 1), torch.tensor(self.w.sensors[i]),
                torch.tensor(self.w.labels[i]))


@pytest.mark.parametrize("shuffle,drop_last", [(True, True), (False, False)])
def test_window_loader_batches_match_reference_dataloader(shuffle, drop_last):
    w = make_windows(n_videos=11, per_video=3)
    ref = DataLoader(_RefDataset(w), batch_size=8, shuffle=shuffle, drop_last=drop_last,
                     generator=torch.Generator().manual_seed(3))
    ours = fd.WindowLoader(w, 8, shuffle, drop_last, "cpu", generator=torch.Generator().manual_seed(3))
    assert len(ours) == len(ref)
    for _ in range(2):  # two epochs: the generator advances identically
        for (a, b, c), (x, y, z) in zip(ref, ours):
            assert x.shape[1:] == (3, 30, 18)
            assert torch.equal(a, x) and torch.equal(b, y) and torch.equal(c, z)


def _ref_topk(output, target, top_k):
    """model/main.py:57-77 restated."""
    _, pred = output.topk(max(top_k), dim=1)
    pred = pred.t()
    if target.dim() != 1:
        _, target = target.topk(1, dim=1)
    res = []
    for k in top_k:
        correct = pred[:k].eq(target.view(1, -1).expand_as(pred[:k]))
        res.append(correct.reshape(-1).float().sum(0, keepdim=True).mul_(1 / target.size(0)).item())
    return res


@pytest.mark.parametrize("soft", [True, False])
def test_top_k_accuracy_matches_reference(soft):
    g = torch.Generator().manual_seed(0)
    out = torch.randn(200, 11, generator=g)
    cls = torch.randint(0, 11, (200,), generator=g)
    tgt = torch.nn.functional.one_hot(cls, 11).float() * 0.8 + 0.01 if soft else cls
    assert fe.cal_top_k_accuracy(out, tgt, (1, 5)) == pytest.approx(_ref_topk(out, tgt, (1, 5)), abs=1e-7)


def test_class_metrics():
    from sklearn.metrics import precision_recall_fscore_support
    rng = np.random.default_rng(1)
    true = rng.integers(0, 4, 300)
    pred = np.where(rng.random(300) < 0.7, true, rng.integers(0, 4, 300))
    m = fe.class_metrics(pred, true, 4)
    p, r, f, _ = precision_recall_fscore_support(true, pred, average="macro", zero_division=0)
    assert (m["precision"], m["recall"], m["f1"]) == pytest.approx((p, r, f))
    for c in range(4):  # specificity = TN / (TN + FP)
        tn = np.sum((true != c) & (pred != c))
        fp = np.sum((true != c) & (pred == c))
        assert m["specificity"][c] == pytest.approx(tn / (tn + fp))
    assert "macro avg" in m["report"]


def test_best_model_checkpoint_format(tmp_path):
    """{'model_weight': state_dict} (model/main.py:323-328), loadable with weights_only."""
    m = torch.nn.Linear(4, 3)
    path = os.path.join(tmp_path, "best_model.pt")
    fe.save_best(m, path)
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"model_weight"} and set(ck["model_weight"]) == {"weight", "bias"}
    m2 = fe.load_best(torch.nn.Linear(4, 3), path)
    assert torch.equal(m2.weight, m.weight)
