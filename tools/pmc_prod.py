"""PMC driver for the PRODUCTION library (blb_amd/libblbrs.so as bench.py loads it), run under
`rocprofv3 --pmc ...` by tools/pmc_prod.sh.  One dispatch of each hot-path kernel at the
BASELINE size, plus calibration kernels of known traffic in the same process:

  calib_copy      torch copy_ of 8 GiB (reads 8 GiB, writes 8 GiB)
  encode          EncodeBatch, RS(6,3) B=1024 x 8 MiB          (rs_code_kernel, store)
  reconstruct     ReconstructBatch, data shard 1 missing        (rs_code_kernel, 1 row)
  verify          VerifyBatch                                   (rs_code_kernel, verify)
  encode_crc      EncodeBatchCRC(65532)                         (encode_crc_tile_kernel + combine)
  crc32c          ChecksumBatch of parity shard k, 65532 blocks (crc_stream_kernel)
  pack            PackPieces of B 8 MiB pieces from distinct tract sources (pack_kernel)
  then RS(12,5) B=512: EncodeBatch and EncodeBatchCRC(65532) on the compiled bit-plane
  network, and a VerifyBatch of the result

Markers: the dispatch order is fixed; tools/pmc_prod_summary.py matches kernels by name and
order.  Prints the libblbrs.so sha256 it loaded."""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from blb_amd import _lib  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

k, m, B, S = 6, 3, 1024, 8 << 20
dev = torch.device("cuda:0")
src = torch.empty(8 << 30, dtype=torch.uint8, device=dev)
dst = torch.empty_like(src)
src.fill_(1)
torch.cuda.synchronize()
dst.copy_(src)  # calib_copy
torch.cuda.synchronize()
del src, dst
torch.cuda.empty_cache()
st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
g = torch.Generator(device=dev)
g.manual_seed(97531)
st[:, :k].random_(0, 256, generator=g)
enc = rs.New(k, m)
torch.cuda.synchronize()
enc.EncodeBatch(st)
torch.cuda.synchronize()
enc.ReconstructBatch(st, [i != 1 for i in range(k + m)], data_only=True)
torch.cuda.synchronize()
ok = enc.VerifyBatch(st)
torch.cuda.synchronize()
crc = enc.EncodeBatchCRC(st, 65532)
torch.cuda.synchronize()
from blb_amd import checksum  # noqa: E402
crc1 = checksum.ChecksumBatch(st[:, k], 65532)  # crc32c: parity shard k of every stripe
torch.cuda.synchronize()
# PackTracts into data shard 0 of every stripe (B pieces of 8 MiB): tracts of 64 KiB..8 MiB at
# padToLength offsets, every tract its own source bytes (end to end in a shuffled order, so
# no read is served by another tract's cached lines).
import numpy as np  # noqa: E402
from blb_amd import pack  # noqa: E402
prng = np.random.default_rng(17)
plan = []
for b in range(B):
    off = 0
    while True:
        ln = int(prng.integers(64 << 10, (8 << 20) + 1))
        if off + ln > S:
            break
        plan.append((b, off, ln))
        off += pack.padded_length(ln)
slots = [(ln + 16 + 255) // 256 * 256 for _, _, ln in plan]
pool = torch.empty(sum(slots) + 4096, dtype=torch.uint8, device=dev)
pool.random_(0, 256, generator=g)
starts, pos = [0] * len(plan), 0
for i in prng.permutation(len(plan)):
    starts[i] = pos + int(prng.integers(0, 16))
    pos += slots[i]
pack_ext = [(pool[starts[i]:], off, ln, b) for i, (b, off, ln) in enumerate(plan)]
pack_read = sum(ln for _, _, ln in plan)
torch.cuda.synchronize()
pack.PackPieces(st[:, 0], S, pack_ext)
torch.cuda.synchronize()
del pool, pack_ext
# blb's widest class on the compiled bit-plane network: encode, then encode fused
# with the ChecksumFile CRCs
del st, crc, crc1
torch.cuda.empty_cache()
k2, m2, B2 = 12, 5, 512
st = torch.empty((B2, k2 + m2, S), dtype=torch.uint8, device=dev)
st[:, :k2].random_(0, 256, generator=g)
enc2 = rs.New(k2, m2)
torch.cuda.synchronize()
enc2.EncodeBatch(st)
torch.cuda.synchronize()
crc2 = enc2.EncodeBatchCRC(st, 65532)
torch.cuda.synchronize()
ok2 = enc2.VerifyBatch(st)
torch.cuda.synchronize()
lib = _lib.LIB_PATH
print(json.dumps({"lib": lib, "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
                  "verify_ok": bool(ok.all()), "k": k, "m": m, "batch": B, "shard": S,
                  "pack": {"pieces": B, "bytes_read": pack_read, "bytes_written": B * S},
                  "wide": {"k": k2, "m": m2, "batch": B2, "compiled_network": enc2.compiled_network(),
                           "verify_ok": bool(ok2.all())}}))
