"""CRC-32C throughput probe: ChecksumBatch over 3072 x 8 MiB device rows (24 GiB), 65532-byte
blocks (blb's ChecksumFile framing) and whole-row frames.  Median of 5 timed calls."""
import sys

import torch

sys.path.insert(0, '.')
from blb_amd import checksum  # noqa: E402

B, S = 3072, 8 << 20
x = torch.randint(0, 256, (B, S), dtype=torch.uint8, device='cuda')
for blk in (65532, 0):
    checksum.ChecksumBatch(x, blk)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        checksum.ChecksumBatch(x, blk)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = sorted(ts)[2]
    print(f"block={blk} {ms:.2f} ms {B * S / ms / 1e6:.1f} GB/s", flush=True)
