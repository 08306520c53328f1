import sys, torch, time
sys.path.insert(0,'.')
from blb_amd import checksum
B, S = 3072, 8 << 20
x = torch.randint(0, 256, (B, S), dtype=torch.uint8, device='cuda')
for blk in (65532, 0):
    checksum.ChecksumBatch(x, blk); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); checksum.ChecksumBatch(x, blk); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"block={blk} {ms:.2f} ms {B*S/ms/1e6:.1f} GB/s")
