"""Data step in front of the hot path: the reference's window format,
its video-wise splits, and a batch loader that feeds the training step from pinned host
memory with asynchronous host-to-device copies.

Reference behaviour mirrored here:
  window files   (videos, features f32[N,T,V,3], sensors f32[N,T_s,S], labels f32[N,C])
                 3_stream/har_create4_sensor.py:76-147; read by model/dataloader.py:177-197
  per sample     skeleton.permute(2,0,1) -> [3,T,V]             model/dataset.py:12-28
  train/valid/test split by unique video, 60/20/20, train_test_split(random_state=seed)
                                                                 model/dataloader.py:204-220
  10-fold CV by unique video, KFold(10, shuffle, random_state)   model/cv_dataloader.py:155-167
  DataLoader(shuffle=key=='train', drop_last=key=='train', generator=manual_seed(seed))
                                                                 model/dataloader.py:232-247

Unlike the reference, which keeps every window as a Python tuple and converts it per item,
the loader holds each split as three contiguous pinned tensors ([N,3,T,V] skeleton,
[N,T_s,S] sensor, [N,C] label) and gathers whole batches at once. It is double-buffered: the
next batch's gather and H2D copy (on a dedicated copy stream) overlap the current step, and
the consumer stream waits on an event, so the step never reads a half-copied batch.
"""
from __future__ import annotations

import pickle
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class Windows:
    videos: list
    features: np.ndarray   # f32 [N, T, V, 3]
    sensors: np.ndarray    # f32 [N, T_s, S]
    labels: np.ndarray     # f32 [N, C]

    def __len__(self):
        return len(self.videos)

    def subset(self, mask):
        idx = np.flatnonzero(mask)
        return Windows([self.videos[i] for i in idx], self.features[idx], self.sensors[idx], self.labels[idx])


def save_windows(path, w: Windows):
    """Write windows in the reference's pickle layout (a 4-tuple), e.g. for synthetic data."""
    with open(path, "wb") as f:
        pickle.dump((list(w.videos), w.features, w.sensors, w.labels), f)


def load_windows(paths) -> Windows:
    """Concatenate the reference's window pickles (model/dataloader.py:185-197): videos are
    a list per file, arrays are concatenated, labels cast to float32 (they are stored as an
    object array). These are the user's own data files: pickle executes code from the file,
    so only load files you produced."""
    videos, feats, sens, labs = [], [], [], []
    for p in ([paths] if isinstance(paths, str) else paths):
        with open(p, "rb") as f:
            vid, fts, sr, lbs = pickle.load(f)
        videos += list(vid)
        feats.append(np.asarray(fts, dtype=np.float32))
        sens.append(np.asarray(sr, dtype=np.float32))
        labs.append(np.asarray(lbs).astype(np.float32))
    return Windows(videos, np.concatenate(feats), np.concatenate(sens), np.concatenate(labs))


def video_split(w: Windows, seed: int = 42):
    """Train / valid / test by unique video name, 60 / 20 / 20 (model/dataloader.py:204-220):
    train_test_split(unique, test_size=0.4) then split the rest 50/50, both shuffled with
    random_state=seed. Windows keep their file order inside each split."""
    from sklearn.model_selection import train_test_split
    names = np.unique(w.videos)
    train_v, other_v = train_test_split(names, test_size=0.4, shuffle=True, random_state=seed)
    valid_v, test_v = train_test_split(other_v, test_size=0.5, shuffle=True, random_state=seed)
    vids = np.asarray(w.videos)
    return {"train": w.subset(np.isin(vids, train_v)), "valid": w.subset(np.isin(vids, valid_v)),
            "test": w.subset(~np.isin(vids, train_v) & ~np.isin(vids, valid_v))}


def video_kfold(w: Windows, seed: int = 42, n_splits: int = 10):
    """10-fold cross-validation over unique videos (model/cv_dataloader.py:155-167):
    KFold(n_splits, shuffle=True, random_state=seed).split(unique names); the held-out fold
    is both 'valid' and 'test', as the reference builds it."""
    from sklearn.model_selection import KFold
    names = np.unique(w.videos)
    vids = np.asarray(w.videos)
    folds = []
    for train_idx, _ in KFold(n_splits=n_splits, shuffle=True, random_state=seed).split(names):
        tr = np.isin(vids, names[train_idx])
        held = w.subset(~tr)
        folds.append({"train": w.subset(tr), "valid": held, "test": held})
    return folds


def dataloader_order(n: int, generator: torch.Generator, shuffle: bool):
    """Sample order of torch's DataLoader(shuffle=shuffle, generator=generator) for one epoch
    (single-process iterator), consuming the generator exactly as it does: every iterator
    first draws a base seed (shuffled or not); RandomSampler then draws randperm(n) for the
    epoch and one more randperm(n) for the (empty) remainder slice. tests/test_data.py checks
    the orders of several epochs of three loaders sharing one generator against DataLoader."""
    torch.empty((), dtype=torch.int64).random_(generator=generator)  # _BaseDataLoaderIter base seed
    if not shuffle:
        return torch.arange(n)
    order = torch.randperm(n, generator=generator)
    torch.randperm(n, generator=generator)  # RandomSampler: randperm(n)[:num_samples % n]
    return order


class WindowLoader:
    """Batches of (skel f32[B,3,T,V], sensor f32[B,T_s,S], label f32[B,C]) on `device`.

    shuffle / drop_last / generator follow the reference's DataLoader arguments
    (train: shuffle + drop_last; valid/test: neither). The epoch order is exactly the one
    torch's DataLoader would produce with the same generator (dataloader_order)."""

    def __init__(self, w: Windows, batch_size: int, shuffle: bool, drop_last: bool, device,
                 generator: torch.Generator | None = None, pin_memory: bool = True):
        self.B, self.shuffle, self.drop_last = int(batch_size), shuffle, drop_last
        self.device = torch.device(device)
        self.generator = generator if generator is not None else torch.Generator().manual_seed(0)
        skel = torch.from_numpy(np.ascontiguousarray(w.features, dtype=np.float32)).permute(0, 3, 1, 2).contiguous()
        self.host = [skel, torch.from_numpy(np.ascontiguousarray(w.sensors, dtype=np.float32)),
                     torch.from_numpy(np.ascontiguousarray(w.labels, dtype=np.float32))]
        self.pin = pin_memory and self.device.type == "cuda"
        if self.pin:
            self.host = [t.pin_memory() for t in self.host]
        self.n = len(w)
        self._copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None

    def __len__(self):
        return self.n // self.B if self.drop_last else (self.n + self.B - 1) // self.B

    def _stage(self, idx):
        """Gather one batch into pinned staging buffers and start its H2D copy."""
        if self.device.type != "cuda":
            return [t.index_select(0, idx) for t in self.host], None
        staged = [torch.empty((len(idx),) + t.shape[1:], dtype=t.dtype, pin_memory=self.pin) for t in self.host]
        for dst, src in zip(staged, self.host):
            torch.index_select(src, 0, idx, out=dst)
        with torch.cuda.stream(self._copy_stream):
            dev = [t.to(self.device, non_blocking=True) for t in staged]
            ev = torch.cuda.Event()
            ev.record(self._copy_stream)
        return dev, (ev, staged)  # keep the pinned buffers alive until the copy is done

    def __iter__(self):
        order = dataloader_order(self.n, self.generator, self.shuffle)
        nb = len(self)
        batches = [order[i * self.B:(i + 1) * self.B] for i in range(nb)]
        if not batches:
            return
        nxt = self._stage(batches[0])
        for b in range(nb):
            cur = nxt
            if b + 1 < nb:
                nxt = self._stage(batches[b + 1])  # overlaps the consumer's work on this batch
            tensors, sync = cur
            if sync is not None:
                ev, _ = sync
                torch.cuda.current_stream(self.device).wait_event(ev)
                for t in tensors:
                    t.record_stream(torch.cuda.current_stream(self.device))
            yield tuple(tensors)


def build_dataloaders(w: Windows, batch_size: int, device, seed: int = 42):
    """model/dataloader.py:_build_harup_dataloader: video-wise split, then one loader per
    split with the reference's shuffle / drop_last / generator settings."""
    splits = video_split(w, seed)
    g = torch.Generator().manual_seed(seed)
    return {k: WindowLoader(v, batch_size, shuffle=(k == "train"), drop_last=(k == "train"), device=device,
                            generator=g) for k, v in splits.items()}
