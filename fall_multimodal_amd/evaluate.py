"""Eval step after the hot path: the reference's valid / test loops, its
metrics and its best-model checkpoint format, driving the native model in eval mode (BN
running statistics).

Reference behaviour mirrored here:
  cal_top_k_accuracy(output, target, top_k)    model/main.py:57-77 (soft targets -> argmax)
  valid(...)  eval mode, no_grad, loss per batch, top-k of the concatenated predictions
                                               model/main.py:148-197
  test(...)   + classification_report, argmax of soft labels   model/main.py:199-245
              + macro precision / recall / F1  model/main_cross_validation.py:247
  best model  torch.save({'model_weight': model.state_dict()})  model/main.py:323-328
The notebook 3-stream form adds per-class specificity (TN / (TN + FP)), given here too.
"""
from __future__ import annotations

import numpy as np
import torch


def cal_top_k_accuracy(output: torch.Tensor, target: torch.Tensor, top_k=(1,)):
    """model/main.py:57-77: fraction of rows whose target class is among the top-k outputs;
    a 2-D (soft / one-hot) target is reduced to its argmax (topk(1))."""
    output, target = output.detach().float().cpu(), target.detach().cpu()
    max_k = max(top_k)
    pred = output.topk(max_k, dim=1).indices.t()
    if target.dim() != 1:
        target = target.topk(1, dim=1).indices.view(-1)
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    return [float(correct[:k].reshape(-1).float().sum().item() / target.size(0)) for k in top_k]


def class_metrics(pred: np.ndarray, true: np.ndarray, num_classes: int | None = None):
    """Macro precision / recall / F1 (sklearn precision_recall_fscore_support(average='macro'),
    as main_cross_validation.py:247), per-class specificity from the confusion matrix, and the
    classification_report text the reference logs."""
    from sklearn.metrics import classification_report, confusion_matrix, precision_recall_fscore_support
    labels = np.arange(num_classes) if num_classes else None
    p, r, f, _ = precision_recall_fscore_support(true, pred, average="macro", zero_division=0)
    cm = confusion_matrix(true, pred, labels=labels)
    tp = np.diag(cm)
    fp = cm.sum(0) - tp
    fn = cm.sum(1) - tp
    tn = cm.sum() - tp - fp - fn
    with np.errstate(divide="ignore", invalid="ignore"):
        spec = np.where(tn + fp > 0, tn / np.maximum(tn + fp, 1), 0.0)
    return {"precision": float(p), "recall": float(r), "f1": float(f), "specificity": spec.tolist(),
            "confusion": cm.tolist(),
            "report": classification_report(true, pred, digits=5, zero_division=0)}


@torch.no_grad()
def predict(model, loader):
    """Eval-mode forward over a loader of (skel, sensor, label): concatenated outputs + labels."""
    was_training = model.training
    model.eval()
    outs, labs = [], []
    for skel, sensor, label in loader:
        outs.append(model(skel, sensor))
        labs.append(label)
    if was_training:
        model.train()
    return torch.cat(outs), torch.cat(labs)


def _eval_pass(model, loader, loss_fn=None):
    """One eval-mode pass: concatenated outputs and labels, per-batch losses."""
    was_training = model.training
    model.eval()
    outs, labs, losses = [], [], []
    for skel, sensor, label in loader:
        out = model(skel, sensor)
        if loss_fn is not None:
            losses.append(float(loss_fn(out, label).item()))
        outs.append(out)
        labs.append(label)
    if was_training:
        model.train()
    return torch.cat(outs), torch.cat(labs), losses


@torch.no_grad()
def valid(model, loader, loss_fn=None, top_k=(1, 5)):
    """model/main.py:148-197: mean batch loss and top-k accuracy of the whole split."""
    out, lab, losses = _eval_pass(model, loader, loss_fn)
    return {"loss": float(np.mean(losses)) if losses else None, "top_k": cal_top_k_accuracy(out, lab, top_k)}


@torch.no_grad()
def test(model, loader, loss_fn=None, top_k=(1, 5), num_classes: int | None = None):
    """model/main.py:199-245 (+ main_cross_validation.py:247): loss, top-k and the per-class
    metrics of argmax predictions against argmax labels, from ONE pass over the loader as the
    reference's test() makes (a second pass would also draw an extra shuffle seed)."""
    out, lab, losses = _eval_pass(model, loader, loss_fn)
    res = {"loss": float(np.mean(losses)) if losses else None, "top_k": cal_top_k_accuracy(out, lab, top_k)}
    pred = out.argmax(1).cpu().numpy()
    true = (lab if lab.dim() == 1 else lab.argmax(1)).cpu().numpy()
    res.update(class_metrics(pred, true, num_classes or out.shape[1]))
    return res


def save_best(model, path):
    """Best-model checkpoint in the reference's format (model/main.py:323-328): the keys of
    model.state_dict() are the reference's, so the file loads into either implementation."""
    torch.save({"model_weight": {k: v.detach().cpu() for k, v in model.state_dict().items()}}, path)


def load_best(model, path):
    """Counterpart of model/main.py:344: load_state_dict(torch.load(path)['model_weight'])
    (weights only: no pickled code is executed)."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model_weight"])
    return model
