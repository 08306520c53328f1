"""Interleaved timing of the fused encode+CRC kernel variants (BLBRS_EC_FLAGS tuning switches)
against the separate encode and CRC passes, on BASELINE-sized device-resident batches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import checksum  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in evs:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in evs]))


def main():
    flags_list = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "3", "4"])]
    for k, m, B in ((6, 3, 1024), (10, 4, 512)):
        S = 8 << 20
        st = torch.randint(0, 256, (B, k + m, S), dtype=torch.uint8, device="cuda")
        enc = rs.New(k, m)
        algo = B * (k + m) * S
        t_enc = timeit(lambda: enc.EncodeBatch(st))
        views = [st[:, k + j, :] for j in range(m)]
        t_crc = timeit(lambda: [checksum.ChecksumBatch(v, 65532) for v in views])
        print(f"RS({k},{m}) B={B}: encode {t_enc:.3f} ms ({algo / t_enc / 1e6:.0f} GB/s), "
              f"crc65532 {t_crc:.3f} ms, sum {t_enc + t_crc:.3f} ms", flush=True)
        for rep in range(2):
            for fl in flags_list:
                rs.set_tuning("BLBRS_EC_FLAGS", fl)
                for blk in ((65532, 0) if not fl & 8 else (0,)):
                    t = timeit(lambda: enc.EncodeBatchCRC(st, blk))
                    print(f"  rep{rep} flags={fl} block={blk}: {t:.3f} ms ({algo / t / 1e6:.0f} GB/s)", flush=True)
        rs.set_tuning("BLBRS_EC_FLAGS", 0)
        del st, views
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
