"""No library path and no test helper has HIP lock pageable memory in place.

Every GPU memory fault of round 5 whose log survives (r5a, r5i, r5m, r5w, r5y; round 4's r4v2 and
r4i struck at the same point of the suite) was raised by a copy that HIP made by locking the
caller's pageable pages in place: torch's .cuda() (tests/test_rtc.py, r5i,
r5m, r5w) or .cpu() (r5a, r5y) of a 1.4 MB heap array.  HIP takes that path for a pageable copy
larger than 1 MiB (hsa_amd_memory_lock_to_pool over the page-rounded range); AMD_LOG_LEVEL=4 names
it with "HSA Copy Using Pinned resource" (rocblit.cpp), right after "Locking to pool ... memFlags =
0x8h" (profiles/r06/fault/).  1 MiB exactly, and anything smaller, is copied through HIP's own
staging buffer instead.

The product rule is that the engine never gives HIP a pageable range to copy: host calls stage
pageable shards by CPU copies into pinned, device-mapped buffers, and the Python side moves
numpy data through pinned tensors (blb_amd/hostcopy.py).  This test runs the host-memory entry
points on pageable shards of the faulting size, and the helpers, in a child process under
AMD_LOG_LEVEL=4, and counts HIP's in-place-lock copies between markers.  A control copy
(torch.from_numpy(a).cuda()) in the same process must show one, so the detector is live.  The
library of rounds 1-4, which DMA'd pageable shards with hipMemcpyAsync, fails the check."""
import os
import re
import subprocess
import sys

import pytest

from conftest import ROOT

INPLACE = "HSA Copy Using Pinned resource"

CHILD = r'''
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
from blb_amd import checksum, rpc
from blb_amd import reedsolomon as rs
from blb_amd.hostcopy import from_numpy_pinned, to_device, to_numpy
from oracle import rs_numpy as N

def mark(name):
    torch.cuda.synchronize()
    print("=== " + name, file=sys.stderr, flush=True)

S = 1_435_536                      # the faulting copy's size (test_rtc's 3-stripe batch)
k, m = 6, 3
rng = np.random.default_rng(6)
data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
full = data + N.encode(k, m, data)
torch.cuda.init()
enc = rs.New(k, m)
mark("control")
torch.from_numpy(np.full(S, 7, np.uint8)).cuda()
mark("Encode")
sh = [d.copy() for d in data] + [np.empty(S, np.uint8) for _ in range(m)]
enc.Encode(sh)
assert all(np.array_equal(sh[i], full[i]) for i in range(k + m))
mark("Verify")
assert enc.Verify(sh)
mark("ReconstructData")
sh[1] = None
enc.ReconstructData(sh)
assert np.array_equal(sh[1], full[1])
mark("Reconstruct")
sh[0], sh[7] = None, None
enc.Reconstruct(sh)
assert np.array_equal(sh[0], full[0]) and np.array_equal(sh[7], full[7])
mark("ReconstructAndVerify")
sh[2] = None
assert enc.ReconstructAndVerify(sh)
mark("client degraded read")           # k pool replies in, the user's pageable buffer out
reps = [rpc.GetBuffer(S) for _ in range(k)]
for j, i in enumerate([0, 2, 3, 4, 5, 6]):
    reps[j][:] = full[i]
piece = [reps[0], None, reps[1], reps[2], reps[3], reps[4], reps[5], None, None]
out = np.empty(S, np.uint8)
enc.ReconstructData(piece, outs={1: out})
assert np.array_equal(out, full[1])
mark("batched")
b = rs.Batcher(max_batch=8, window_us=0, devices=[0])
enc.SetBatcher(b)
sh = [d.copy() for d in data] + [np.empty(S, np.uint8) for _ in range(m)]
enc.Encode(sh)
enc.SetBatcher(None)
b.close()
assert np.array_equal(sh[8], full[8])
mark("EncodeHostBatch")
stripes = [[d.copy() for d in data] + [np.empty(S, np.uint8) for _ in range(m)] for _ in range(2)]
enc.EncodeHostBatch(stripes)
assert np.array_equal(stripes[1][6], full[6])
mark("EncodeHostBatch copy engines")  # pinned stripes through hipMemcpyAsync (nstreams >= 1)
pin = torch.empty((2, k + m, S), dtype=torch.uint8).pin_memory().numpy()
pin[:, :k] = np.stack(data)
enc.EncodeHostBatch([[pin[b, i] for i in range(k + m)] for b in range(2)], nstreams=3)
assert np.array_equal(pin[1, 7], full[7])
mark("Checksum")
buf = rng.integers(0, 256, 8 * S + 13, dtype=np.uint8)
checksum.Checksum(buf, 65532)
mark("hostcopy helpers")
t = to_device(full[0])
assert np.array_equal(to_numpy(t), full[0])
t.copy_(from_numpy_pinned(full[1]))
assert np.array_equal(to_numpy(t), full[1])
mark("end")
'''


def _count_by_section(log: str) -> dict:
    counts, cur = {}, None
    for line in log.splitlines():
        mk = re.match(r"=== (.+)$", line)
        if mk:
            cur = mk.group(1)
            counts.setdefault(cur, 0)
        elif cur is not None and INPLACE in line:
            counts[cur] += 1
    return counts


def test_section_counter_reads_hip_log_lines():
    """The parser on a fabricated excerpt in HIP's log format (CPU)."""
    log = "\n".join([
        "=== control",
        ":4:rocmemory.cpp :1030: 1 us: [pid:1] Locking to pool 0x1, size 0x15f000, HostPtr = 0x2, memFlags = 0x8h",
        ":4:rocblit.cpp   :673 : 2 us: [pid:1] HSA Copy Using Pinned resource size 1435536",
        "=== Encode",
        ":4:rocblit.cpp   :731 : 3 us: [pid:1] HSA Async Copy staged H2D, Async=0",
        "=== end"])
    assert _count_by_section(log) == {"control": 1, "Encode": 0, "end": 0}


@pytest.mark.gpu
def test_library_and_helpers_make_no_inplace_pinned_copies(tmp_path):
    env = dict(os.environ, AMD_LOG_LEVEL="4", PYTHONUNBUFFERED="1")
    env.pop("GPU_PINNED_MIN_XFER_SIZE", None)   # HIP's default: lock pageable copies > 1 MiB in place
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    r = subprocess.run([sys.executable, str(script), ROOT], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=180)
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "no_inplace_pin_child.log"), "w") as f:   # evidence
        f.write(r.stderr)
    assert r.returncode == 0, r.stderr[-4000:]
    counts = _count_by_section(r.stderr)
    assert "end" in counts, sorted(counts)
    assert counts["control"] >= 1, "HIP did not log an in-place lock for the control copy: detector is blind"
    product = {k: v for k, v in counts.items() if k != "control"}
    assert all(v == 0 for v in product.values()), product
