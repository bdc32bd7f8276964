"""bench.py's rgb_branch leg alone (the build-defined RGB branch, B=256, T=30): python tools/rgb_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

if __name__ == "__main__":
    import bench
    print(json.dumps(bench.rgb_bench(torch.device("cuda", 0))))
