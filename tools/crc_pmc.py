"""Standalone CRC-32C (crc_stream_kernel) traffic and time, for the load-path A/B of DESIGN §4b.

Run under `rocprofv3 --pmc FETCH_SIZE` and `--kernel-trace` by tools/crc_pmc.sh, once per library
(BLBRS_LIB_PATH: the shipped nontemporal coalesced loads, and variants built with
-DBLBRS_CRC_COAL=1 / 0).  Ops, each one warm-up + REPS launches, one dispatch at a time:

  calib_copy     torch copy_ of 8 GiB (FETCH_SIZE scale, as tools/pmc_prod.py)
  parity_65532   ChecksumBatch(st[:, k], 65532): the parity shards of RS(6,3) B=1024 stripes
                 (rows 9 x 8 MiB apart; pmc_prod.py's crc32c_65532)
  rows_65532     ChecksumBatch of 1024 contiguous 8 MiB rows, 65532-byte blocks
  rows_whole     the same rows as one frame each (64 KiB-aligned segments)
Prints the plan as one JSON line (label, launches, algorithmic bytes)."""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blb_amd import _lib, checksum  # noqa: E402

REPS = int(os.environ.get("PMC_REPS", "3"))
k, m, B, S = 6, 3, 1024, 8 << 20
dev = torch.device("cuda:0")
plan = []


def op(label, fn, algo):
    for _ in range(1 + REPS):
        fn()
        torch.cuda.synchronize()
    plan.append({"label": label, "needle": "crc_stream_kernel", "launches": 1 + REPS, "algorithmic_bytes": algo})


src = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
src.fill_(1)
torch.cuda.synchronize()
dst.copy_(src)
torch.cuda.synchronize()
del src, dst
torch.cuda.empty_cache()

st = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device=dev)
op("parity_65532", lambda: checksum.ChecksumBatch(st[:, k], 65532), B * S)
rows = st[:, :k].reshape(B * k, S)[:B]
op("rows_65532", lambda: checksum.ChecksumBatch(rows, 65532), B * S)
op("rows_whole", lambda: checksum.ChecksumBatch(rows, 0), B * S)
lib = _lib.LIB_PATH
print(json.dumps({"lib": lib, "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(), "reps": REPS,
                  "plan": plan}))
