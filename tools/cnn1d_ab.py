#!/usr/bin/env python3
"""The sensor CNN1D stage times of bench.py's sensor leg alone (cfg 1 at B=32 and the B=256 case),
one line per process; run it once per environment setting to A/B the CNN1D forms, e.g.
    F3_CNN_FUSED=0 python tools/cnn1d_ab.py      (round-3 launches)
    F3_CNN_GRID=128 python tools/cnn1d_ab.py     (fused, 128 workgroups)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    s = bench.sensor_bench(torch.device("cuda"))
    env = {k: os.environ[k] for k in ("F3_CNN_FUSED", "F3_CNN_GRID") if k in os.environ}
    out = {"env": env, "cfg1_ms_per_step": s["cfg1_cnn_bilstm"]["ms_per_step"]}
    for key, rec in (("B32", s["cfg1_cnn_bilstm"].get("cnn1d")), ("B256", s.get("cnn1d_B256"))):
        if rec:
            out[key] = {k: (v["us"] if isinstance(v, dict) else v) for k, v in rec.items()
                        if k not in ("note", "batch")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
