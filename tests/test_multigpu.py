"""N>1 path: world_size-2 `gloo` process groups exercise the stripe split and the
max/sum-over-ranks aggregation bench.py uses (one process per GPU; no data-path collective).

* CPU (runs everywhere): each rank encodes its share with the oracle standing in for its GPU;
  the union of the shares must equal the single-process encode of the whole batch.
* GPU (`test_gloo_world2_engine_on_shared_gpu`): the same split through libblbrs itself,
  both ranks on GPU 0, Encode + 2-erasure Reconstruct + Verify per rank, union checked
  against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from blb_amd import multigpu
from blb_amd.hostcopy import to_device, to_numpy


def test_stripe_range_partitions():
    for total in (0, 1, 7, 8, 4096, 4097, 1023):
        for world in (1, 2, 3, 4, 8):
            covered = []
            for r in range(world):
                s, c = multigpu.stripe_range(total, world, r)
                covered.extend(range(s, s + c))
            assert covered == list(range(total))
            counts = [multigpu.stripe_range(total, world, r)[1] for r in range(world)]
            assert max(counts) - min(counts) <= 1
    assert multigpu.stripe_range(4096, 8, 3) == (1536, 512)  # BASELINE config 4 share
    with pytest.raises(ValueError):
        multigpu.stripe_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, root, out_dir):
    import sys
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    k, m, S, total = 10, 4, 4099, 9
    start, count = multigpu.stripe_range(total, world, rank)
    parity = np.zeros((count, m, S), np.uint8)
    for i, b in enumerate(range(start, start + count)):
        rng = np.random.default_rng(97531 * (b + 1))
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        sh = data + [parity[i, j] for j in range(m)]
        O.encode(k, m, sh)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), parity)
    # aggregation exactly as bench.py does it: bytes summed, wall time maxed
    t_local = 1.0 + rank            # rank 1 is the slow one
    assert multigpu.max_over_ranks(t_local) == float(world)
    gibps = multigpu.aggregate_gibps(float(count * k * S), t_local)
    expect = total * k * S / float(1 << 30) / float(world)
    assert abs(gibps - expect) < 1e-12
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_shard_and_aggregate(tmp_path, oracle_lib):
    from conftest import ROOT
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), ROOT, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"rank{r}.npy") for r in range(world)])
    k, m, S, total = 10, 4, 4099, 9
    for b in range(total):
        rng = np.random.default_rng(97531 * (b + 1))
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        sh = data + [np.zeros(S, np.uint8) for _ in range(m)]
        oracle_lib.encode(k, m, sh)
        for j in range(m):
            assert np.array_equal(got[b, j], sh[k + j])


def test_single_process_aggregation_is_identity():
    assert multigpu.max_over_ranks(2.5) == 2.5
    assert multigpu.sum_over_ranks(7.0) == 7.0
    assert multigpu.aggregate_gibps(float(1 << 30), 0.5) == 2.0
    assert torch.distributed.is_available()


def _engine_worker(rank, world, port, root, out_dir):
    """One rank of the N>1 engine path: its stripe_range of the batch through libblbrs on
    its GPU (here both ranks share GPU 0), Encode then a 2-erasure Reconstruct, and the
    bench's max-over-ranks clock."""
    import sys
    import time
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from blb_amd import reedsolomon as rs
    local = rank % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    k, m, S, total = 10, 4, 70001, 9
    start, count = multigpu.stripe_range(total, world, rank)
    host = np.zeros((count, k + m, S), np.uint8)
    for i, b in enumerate(range(start, start + count)):
        rng = np.random.default_rng(97531 * (b + 1))
        for j in range(k):
            host[i, j] = rng.integers(0, 256, S, dtype=np.uint8)
    host[:, k:] = 0xEE  # stale parity buffers
    st = to_device(host, dev)
    enc = rs.New(k, m, devices=[local])
    dist.barrier()
    t0 = time.perf_counter()
    enc.EncodeBatch(st)
    torch.cuda.synchronize(dev)
    t = multigpu.max_over_ranks(time.perf_counter() - t0, dev)
    assert t > 0
    encoded = st.clone()
    st[:, 1].fill_(0)
    st[:, 11].fill_(0)
    enc.ReconstructBatch(st, [i not in (1, 11) for i in range(k + m)])
    torch.cuda.synchronize(dev)
    assert torch.equal(st, encoded), f"rank {rank}: reconstruct differs"
    assert bool(enc.VerifyBatch(st).all())
    np.save(os.path.join(out_dir, f"engine_rank{rank}.npy"), to_numpy(st[:, k:]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gloo_world2_engine_on_shared_gpu(tmp_path, oracle_lib):
    """Two gloo ranks share GPU 0; each encodes and reconstructs its stripe_range through
    libblbrs; the union of their parity equals the oracle's encode of the whole batch."""
    from conftest import ROOT
    world = 2
    mp.spawn(_engine_worker, args=(world, _free_port(), ROOT, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"engine_rank{r}.npy") for r in range(world)])
    k, m, S, total = 10, 4, 70001, 9
    assert got.shape == (total, m, S)
    for b in range(total):
        rng = np.random.default_rng(97531 * (b + 1))
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
        sh = data + [np.zeros(S, np.uint8) for _ in range(m)]
        oracle_lib.encode(k, m, sh)
        for j in range(m):
            assert np.array_equal(got[b, j], sh[k + j]), f"stripe {b} parity {j}"
