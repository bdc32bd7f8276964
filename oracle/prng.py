"""ORACLE / TEST INFRASTRUCTURE — portable deterministic weight + input generator.

Only `tests/`, `tools/gen_golden.py`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg use this module. It is never on the product path.

Every parameter tensor is drawn from numpy's PCG64 (`default_rng`), seeded by
(seed, crc32(name)), so a golden fixture only has to store the seed: the same
weights are regenerated bit-for-bit here, in the tests and on the GPU box.
The value range is chosen from the name and rank alone:

* rank >= 2 ``*.weight`` (Conv/Linear)      U(±1/sqrt(fan_in))
* LSTM ``weight_ih/hh``, ``bias_ih/hh``      U(±1/sqrt(H))  (H = rows/4)
* rank 1 ``*.weight`` (BatchNorm gamma)      U(0.5, 1.5)
* rank 1 ``*.bias``                          U(-0.2, 0.2)
* ``edge_importance.*``                      U(0.5, 1.5)    (reference init is ones,
                                              stgcan.py:198-201; randomised so its
                                              gradient path is exercised)
* ``node_embeddings`` (TARGCN)               U(±sqrt 3): unit variance, as the reference's
                                              torch.randn init (TRAGCN.py:194)
"""
from __future__ import annotations

import zlib

import numpy as np


def param_value(name: str, shape, seed: int) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    rng = np.random.default_rng([int(seed), zlib.crc32(name.encode())])
    leaf = name.rsplit(".", 1)[-1]
    if "edge_importance" in name:
        lo, hi = 0.5, 1.5
    elif name.endswith("node_embeddings"):
        lo, hi = -np.sqrt(3.0), np.sqrt(3.0)
    elif leaf.startswith(("weight_ih", "weight_hh", "bias_ih", "bias_hh")):
        h = shape[0] // 4
        b = 1.0 / np.sqrt(h)
        lo, hi = -b, b
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        b = 1.0 / np.sqrt(fan_in)
        lo, hi = -b, b
    elif leaf == "weight":
        lo, hi = 0.5, 1.5
    else:
        lo, hi = -0.2, 0.2
    return rng.uniform(lo, hi, size=shape).astype(np.float32)


def synthetic_batch(batch: int, num_node: int, num_class: int, sensor_dim: int,
                    seed: int, frames: int = 30, sensor_frames: int | None = None,
                    center: int | None = None, separation: float = 0.8, spread: float = 0.5):
    """Synthetic clip batch in the reference's loader format.

    skel  f32[N,3,T,V]: x,y ~ U(-1,1) (post scale_pose range,
          har_create4_sensor.py:36-47), score ~ U(0.3,1); the centre node is the
          mean of joints 1 and 2 (coco_cut, har_create4_sensor.py:125) or of the
          shoulders 5 and 6 (coco_mmpose node 17).
    sensor f32[N,Ts,S]: N(0,0.5^2) + 1.0 on every third axis (gravity).
    label f32[N,C]: smoothed one-hot (eps 0.1) scaled by a score in U(0.5,1) —
          rows do not sum to 1 (har_create4_sensor.py:99-101,128-136).
    A class-conditional shift on joints 0..3 makes the data separable: x of those joints is
    spread * U(-1,1) + (cls/(C-1) - 1/2) * separation (defaults: the bench / parity data;
    the convergence test uses a wider separation so training reaches a plateau quickly).
    """
    rng = np.random.default_rng([int(seed), 0xC11B5])
    ts = frames if sensor_frames is None else sensor_frames
    cls = rng.integers(0, num_class, size=batch)
    skel = np.empty((batch, 3, frames, num_node), np.float32)
    skel[:, :2] = rng.uniform(-1, 1, size=(batch, 2, frames, num_node))
    skel[:, 2] = rng.uniform(0.3, 1.0, size=(batch, frames, num_node))
    shift = (cls[:, None, None].astype(np.float32) / max(num_class - 1, 1) - 0.5) * np.float32(separation)
    skel[:, 0, :, :4] = np.clip(skel[:, 0, :, :4] * np.float32(spread) + shift, -1, 1)
    if center is None:
        center = num_node - 1
    if num_node == 14:
        skel[:, :, :, center] = 0.5 * (skel[:, :, :, 1] + skel[:, :, :, 2])
    elif num_node == 18:
        skel[:, :, :, center] = 0.5 * (skel[:, :, :, 5] + skel[:, :, :, 6])
    sensor = rng.normal(0.0, 0.5, size=(batch, ts, sensor_dim)).astype(np.float32)
    sensor[:, :, ::3] += 1.0
    sensor += (cls[:, None, None].astype(np.float32) / max(num_class, 1)) * 0.5
    eps = 0.1
    onehot = np.eye(num_class, dtype=np.float32)[cls]
    lab = onehot * (1 - eps) + (1 - onehot) * eps / max(num_class - 1, 1)
    lab *= rng.uniform(0.5, 1.0, size=(batch, 1)).astype(np.float32)
    return skel.astype(np.float32), sensor.astype(np.float32), lab.astype(np.float32)
