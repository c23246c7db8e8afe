import json, sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "celestia-app_amd"))
import torch
import bench, cda
ctx = cda.Context(0)
print(json.dumps(bench.repair_measure(ctx)))
