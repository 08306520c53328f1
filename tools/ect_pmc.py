"""One plain encode and one fused encode+CRC (65532-byte blocks) of RS(k,m), B stripes of
8 MiB, for rocprofv3 --pmc passes (tools/ect_pmc.sh) comparing the two kernels' SQ counters."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--k", type=int, default=12)
p.add_argument("--m", type=int, default=5)
p.add_argument("--batch", type=int, default=512)
a = p.parse_args()
dev = torch.device("cuda:0")
stripes = torch.randint(0, 256, (a.batch, a.k + a.m, 8 << 20), dtype=torch.uint8, device=dev)
enc = rs.New(a.k, a.m)
enc.EncodeBatch(stripes)
enc.EncodeBatchCRC(stripes, 65532)
torch.cuda.synchronize(dev)
