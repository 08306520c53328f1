"""bench.py's RS(8,3) (blb's COLD class) rows alone, as one JSON line: for rocprofv3 runs and
A/B checks of the RS(8,3) kernels without the whole default bench."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
print(json.dumps(bench.cold_class_extras(bench.TRACT, dev)), flush=True)
