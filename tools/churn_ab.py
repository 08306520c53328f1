"""bench.py's rpc_pool_extras alone (blb's rpc.GetBuffer pool churn: 16 threads, registered 4 MiB
class buffers, Encode per call, rpc.gc() every 0 / 64 / 8 calls), for an A/B of two libraries run
in turn under BLBRS_LIB_PATH.  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
out = bench.rpc_pool_extras(6, 3, dev)
out["lib"] = os.environ.get("BLBRS_LIB_PATH", "shipped")
print(json.dumps(out))
