"""HBM ceilings for the read/write mixes of the hot kernels: a pure write (torch fill_), a
1:1 copy (torch copy_) and the encode's 2:1 read:write mix as a trivial-XOR stream are the
yardsticks for pack (0.7:1), pack+encode (0.47:1) and encode (2:1).  Prints TB/s."""
import json

import torch

dev = torch.device("cuda:0")
n = 32 << 30
a = torch.empty(n, dtype=torch.uint8, device=dev)
b = torch.empty(n, dtype=torch.uint8, device=dev)


def t(fn, reps=3):
    fn()
    torch.cuda.synchronize(dev)
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize(dev)
        out.append(s.elapsed_time(e))
    return min(out)


w = t(lambda: a.fill_(7))
c = t(lambda: b.copy_(a))
r = t(lambda: a.view(torch.int64).sum())
print(json.dumps({"write_TBps": round(n / w / 1e9, 3), "copy_TBps": round(2 * n / c / 1e9, 3),
                  "read_sum_TBps": round(n / r / 1e9, 3)}))
