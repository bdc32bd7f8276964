"""Skeleton graph adjacency A[K,V,V] (reference: Multimodal_Fall3/model/graph.py:20-126).

Layouts: `coco_cut` (14 nodes: COCO minus eyes/ears + centre node 13) and `coco_mmpose`
(17 COCO keypoints + centre node 17). Strategies: uniform (K=1), distance (K=2),
spatial (K=3: root / centripetal / centrifugal partitions). Column-normalised A·D^-1.
Computed once on the host; the result is the `A` buffer of each skeleton stream.
"""
from __future__ import annotations

import numpy as np

LAYOUTS = {
    "coco_cut": (14, 13, ((6, 4), (4, 2), (2, 13), (13, 1), (5, 3), (3, 1), (12, 10), (10, 8),
                          (8, 2), (11, 9), (9, 7), (7, 1), (13, 0))),
    "coco_mmpose": (18, 17, ((0, 1), (1, 3), (0, 2), (2, 4), (17, 0), (17, 6), (6, 8), (8, 10),
                             (17, 5), (5, 7), (7, 9), (17, 12), (12, 14), (14, 16), (17, 11),
                             (11, 13), (13, 15))),
}
STRATEGY_PARTITIONS = {"uniform": 1, "distance": 2, "spatial": 3}


def _hops(num_node, links, max_hop):
    adj = np.eye(num_node)
    for i, j in links:
        adj[i, j] = adj[j, i] = 1.0
    dist = np.full((num_node, num_node), np.inf)
    power = np.eye(num_node)
    reach = [power > 0]
    for _ in range(max_hop):
        power = power @ adj
        reach.append(power > 0)
    for d in range(max_hop, -1, -1):
        dist[reach[d]] = d
    return dist


class Graph:
    def __init__(self, layout="coco_cut", strategy="uniform", max_hop=1, dilation=1):
        if layout not in LAYOUTS:
            raise ValueError("This layout is not supported!")
        self.num_node, self.center, links = LAYOUTS[layout]
        self.hop_dis = _hops(self.num_node, links, max_hop)
        self.A = self._partition(strategy, max_hop, dilation)

    def _partition(self, strategy, max_hop, dilation):
        v, hop = self.num_node, self.hop_dis
        hops = range(0, max_hop + 1, dilation)
        base = np.isin(hop, list(hops)).astype(np.float64)
        deg = base.sum(axis=0)
        norm = base * np.where(deg > 0, 1.0 / np.maximum(deg, 1e-300), 0.0)[None, :]
        if strategy == "uniform":
            return norm[None].copy()
        if strategy == "distance":
            return np.stack([np.where(hop == h, norm, 0.0) for h in hops])
        if strategy != "spatial":
            raise ValueError("This strategy is not supported!")
        to_c = hop[:, self.center]
        parts = []
        for h in hops:
            on = hop == h  # entry [j, i]: node j is h hops from node i
            same = on & (to_c[:, None] == to_c[None, :])
            closer = on & (to_c[:, None] > to_c[None, :])
            farther = on & ~same & ~closer
            root, close, far = (np.where(m, norm, 0.0) for m in (same, closer, farther))
            if h == 0:
                parts.append(root)
            else:
                parts += [root + close, far]
        return np.stack(parts)
