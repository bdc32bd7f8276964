import json, sys, torch
sys.path.insert(0, '.')
import bench
print(json.dumps(bench.sensor_bench(torch.device('cuda'))))
