"""bench.py's recovery_shapes extra alone (blb's RPC and client recovery shapes for every
storage class, shipped path vs tables vs the stream probe), for rocprof runs and A/B boxes.
Knobs as KNOB=value arguments (blbrs_set_tuning), e.g. BLBRS_RTC_WIDE=9; REPS and CLASSES
("k,m,B;k,m,B") from the environment."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

for arg in sys.argv[1:]:
    name, _, value = arg.partition("=")
    rs.set_tuning(name, int(value))
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
classes = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("CLASSES", "6,3,1024;8,3,768;10,3,640;12,5,480").split(";")]
print(json.dumps(bench.recovery_extras(bench.TRACT, dev, reps=int(os.environ.get("REPS", "3")), classes=classes)))
