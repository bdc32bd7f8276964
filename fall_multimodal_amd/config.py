"""Config tree with the reference's keys and defaults (Multimodal_Fall3/model/config.py:3-77).

The reference uses yacs; this is a dependency-free equivalent with the same attribute
access, `merge_from_file(yaml)`, `merge_from_list`, `freeze`, `clone` and `dump`, so
the reference YAMLs (e.g. two_stgcan_bilstm_harup.yaml) load unchanged.
"""
from __future__ import annotations

import copy

import yaml


class CfgNode(dict):
    def __init__(self, init=None):
        super().__init__()
        object.__setattr__(self, "_frozen", False)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        if self._frozen:
            raise AttributeError(f"Attempted to set {k} on a frozen CfgNode")
        self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def freeze(self):
        object.__setattr__(self, "_frozen", True)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.freeze()

    def clone(self):
        return copy.deepcopy(self)

    def merge_from_dict(self, d):
        for k, v in d.items():
            if k not in self:
                raise KeyError(f"Non-existent config key: {k}")
            if isinstance(v, dict):
                self[k].merge_from_dict(v)
            else:
                self[k] = _coerce(v)

    def merge_from_file(self, path):
        with open(path) as f:
            self.merge_from_dict(yaml.safe_load(f) or {})

    def merge_from_list(self, opts):
        for k, v in zip(opts[0::2], opts[1::2]):
            node = self
            *head, leaf = k.split(".")
            for h in head:
                node = node[h]
            node[leaf] = _coerce(yaml.safe_load(v) if isinstance(v, str) else v)

    def dump(self):
        return yaml.safe_dump(_plain(self), sort_keys=False)


def _coerce(v):
    return None if v == "None" else v


def _plain(n):
    return {k: _plain(v) if isinstance(v, CfgNode) else v for k, v in n.items()}


_C = CfgNode({
    "TRAIN": {"EPOCHS": 10, "LABEL_SMOOTHING": 0.0, "USE_SCALER": True, "MAX_NORM": 100, "ACCUM_ITER": 1},
    "DATA": {"BATCH_SIZE": 16, "DATASET": "harup", "SUBSET": "", "IN_CHANNELS": 3, "NUM_CLASSES": 11,
             "SENSOR_DIM": 15},
    "MODEL": {"NAME": "stgcn"},
    "GRAPH": {"LAYOUT": "coco_cut", "STRATEGY": "spatial"},
    "OPTIM": {"TYPE": "rmsprop", "LR": 0.001, "MOMENTUM": 0.99, "WEIGHT_DECAY": 0.01, "BETAS": [0.9, 0.999],
              "EPS": 1.0e-8},
    "LR_SCHEDULER": {"TYPE": None, "T_INITIAL": 500, "LR_MIN": 1.0e-5, "T_IN_EPOCHS": True, "WARMUP_T": 5,
                     "WARMUP_LR_INIT": 1.0e-4},
    "SEED": 42, "DEVICE": "cuda", "SAVE_CHECKPOINT": True, "RESUME_FROM": None, "PRETRAINED_WEIGHT_PATH": None,
    "TEST_ONLY": False, "NUM_WORKERS": 8, "PIN_MEMORY": True, "LOG_DIR": None, "LOGGING_TIMING": 10,
    "TENSORBOARD_LOG": False, "TOP_K": [1],
})


def get_cfg_defaults():
    return _C.clone()
