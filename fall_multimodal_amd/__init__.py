"""fall_multimodal_amd — MI355X-native (gfx950) training path for the 3-stream
fall-detection model of musaru/Fall_Multimodal (skeleton-position ST-GCAN, skeleton-motion
ST-GCAN, IMU BiLSTM; late fusion; soft-target CE; RMSprop).

Public surface mirrors the reference (Multimodal_Fall3/model/):
    build_model(config)          -> model/build_model.py
    build_optimizer(model, cfg)  -> model/optimizer.py
    get_cfg_defaults()           -> model/config.py
plus TrainStep, the fused multi-stream step used by bench.py, the skeleton-only TARGCN model
(BASELINE config 2: TRAGCN.py / EmbGCN.py / GRU.py / TA.py) with its fused TargcnStep, the
SkeletonTransformer (BASELINE config 5: skeleton_transformer.py) with SktrStep, musa.Model (the model
the root Multimodal_Fall3/main.py trains: musa_model.py) with musa.MusaStep, and the steps either side of it
(SURVEY §8f): data (window files, video-wise splits, pinned double-buffered loader) and
evaluate (valid / test loops, top-k, macro P/R/F1, best-model checkpoints).
"""
from .config import CfgNode, get_cfg_defaults
from .graph import Graph
from .model import (BiLSTM, CNN_BiLSTM, Fall3Net, NetSpec, STGCAN, TwoStreamSpatialTemporalGraph, TwoStreamSTGCAN,
                    TwoStreamSTGCAN_BiLSTM, build_model)
from .optim import RMSprop, build_optimizer
from .train import TrainStep
from .targcn import TARGCN, TargcnStep
from .sktr import SkeletonTransformer, SktrStep
from . import musa
from . import data, evaluate

__all__ = ["build_model", "build_optimizer", "get_cfg_defaults", "CfgNode", "Graph", "Fall3Net", "NetSpec",
           "STGCAN", "BiLSTM", "CNN_BiLSTM", "TwoStreamSTGCAN", "TwoStreamSTGCAN_BiLSTM", "TwoStreamSpatialTemporalGraph",
           "RMSprop", "TrainStep", "TARGCN", "TargcnStep", "SkeletonTransformer", "SktrStep", "musa", "data", "evaluate"]
