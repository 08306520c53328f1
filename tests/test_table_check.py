"""The pointer-table check (runtime.hpp TableFault, rs_code.hpp stripe_table_ok) and the lazily
opened run-time compiler (rtc.hip).

Round 4 saw two hipErrorIllegalAddress faults in the GPU suite whose cause inside the runtime was
never pinned.  Two changes answer it:

* every shard-pointer table the library uploads is tagged per upload, and the coding kernel never
  dereferences an entry without its launch's tag -- a stale or foreign entry becomes a named
  error (stripe, slot, entry) instead of a device fault;
* run-time decode networks are off by default and hipRTC is opened with dlopen on first use, so
  blb's tractserver and client processes carry no in-process LLVM unless they opt in.

The GPU tests inject a wrong tag (blbrs_debug_corrupt_next_table: the address stays valid, so the
pre-check logic would have coded the stripe normally) into each path that uploads a table: host
calls on the worker's table (zero-copy and staged), the batcher's lane table, and the caller-stream
*_dev_ptrs table.  Each must leave the stripe untouched, report the slot, and keep the device usable.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from blb_amd import reedsolomon as rs
from blb_amd.hostcopy import to_device, to_numpy
from oracle import rs_numpy as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "blb_amd", "libblbrs.so")


def _maps_after(code: str, torch_first: bool = False) -> str:
    """/proc/self/maps of a fresh interpreter after `code` ran (library loaded as `lib`).  Without
    torch_first the process never imports torch (torch's wheel maps its own hipRTC), so the maps
    show what the library itself brings in."""
    script = ("import ctypes, sys\nsys.path.insert(0, %r)\nfrom blb_amd import _lib\nlib = _lib.load()\n" % ROOT
              + code + "\nprint(open('/proc/self/maps').read())\n")
    env = dict(os.environ)
    if not torch_first:
        env["BLBRS_NO_TORCH"] = "1"
    p = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return p.stdout


def test_library_does_not_link_hiprtc():
    """ldd shows no hipRTC or comgr, and loading the library maps neither."""
    out = subprocess.run(["ldd", LIB], capture_output=True, text=True, check=True).stdout
    assert "hiprtc" not in out and "comgr" not in out, out
    maps = _maps_after("")
    assert "libhiprtc" not in maps


def test_rtc_default_background_for_wide_multirow_passes():
    """Round 6: run-time networks compile in the background by default, for RS(12,5)-wide passes
    of at least 2 rows only (blb's recovery RPC, multi-row ReconstructData); the client's usual
    single-row read and every narrower class stay on tables."""
    assert rs.get_tuning("BLBRS_RTC") == 1
    assert rs.rtc_eligible(12, 5) and rs.rtc_eligible(12, 2)
    assert not rs.rtc_eligible(12, 1) and not rs.rtc_eligible(10, 3) and not rs.rtc_eligible(8, 3)


def test_hiprtc_opened_on_first_compile():
    """A compile request (no device needed) opens hipRTC lazily: mapped afterwards."""
    maps = _maps_after("import numpy as np\nfrom blb_amd import reedsolomon as rs\n"
                       "rs.rtc_compile(np.arange(1, 1 + 2 * 12, dtype=np.uint8).reshape(2, 12), mode=0)")
    assert "libhiprtc" in maps


# ---------------------------------------------------------------- GPU -------------------------

def _torch():
    import torch
    return torch


def _stripe(k, m, S, seed):
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    return data + list(N.encode(k, m, data))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pool", "bounce", "staged"])
def test_gpu_wrong_tag_host_call_names_slot(kind):
    """Host Encode on each host path's table: pool buffers (zero copy, the worker's device table),
    small pageable shards (the worker's pinned bounce buffer, table read over PCIe) and large
    pageable shards (device staging by DMA, per-chunk tables).  An entry with a wrong tag fails
    the call with ErrHIP naming the slot, the parity is not written, and the next call on the
    same encoder is bit-exact."""
    k, m = 6, 3
    S = 3 * 16384 + 100 if kind != "staged" else (1 << 20) + 100   # bounce: <= 512 KiB per call
    pool = kind == "pool"
    truth = _stripe(k, m, S, 11 + len(kind))
    enc = rs.New(k, m)
    for slot in (0, k + 1):
        if pool:
            sh = [rs.GetBuffer(S)[:S] for _ in range(k + m)]
        else:
            sh = [np.empty(S, np.uint8) for _ in range(k + m)]
        for i in range(k):
            sh[i][:] = truth[i]
        for i in range(k, k + m):
            sh[i][:] = 0xA5
        rs.debug_corrupt_next_table(slot)
        with pytest.raises(rs.ErrHIP, match=f"slot {slot} "):
            enc.Encode(sh)
        if kind != "staged":  # in place or bounced: nothing reaches the parity (staged outputs are unspecified)
            for i in range(k, k + m):
                assert (sh[i] == 0xA5).all(), (slot, i)
        enc.Encode(sh)
        for i in range(k, k + m):
            assert np.array_equal(sh[i], truth[i]), (slot, i)
        if pool:
            for b in sh:
                rs.PutBuffer(b)


@pytest.mark.gpu
def test_gpu_wrong_tag_batched_call_names_slot():
    """A batched ReconstructData: the lane's table check fails the group with the slot named;
    the next batched call is bit-exact."""
    k, m, S = 6, 3, 65536
    truth = _stripe(k, m, S, 21)
    enc = rs.New(k, m)
    b = rs.Batcher(max_batch=8, window_us=0)
    enc.SetBatcher(b)
    try:
        for attempt in range(2):
            sh = [truth[i].copy() if i != 2 else None for i in range(k)] + [truth[i].copy() for i in range(k, k + m)]
            if attempt == 0:
                rs.debug_corrupt_next_table(4)
                with pytest.raises(rs.ErrHIP, match="slot 4 "):
                    enc.ReconstructData(sh)
            else:
                enc.ReconstructData(sh)
                assert np.array_equal(sh[2], truth[2])
    finally:
        enc.SetBatcher(None)


@pytest.mark.gpu
def test_gpu_wrong_tag_dev_ptrs_recorded_per_device():
    """Encode of device tensors (blbrs_encode_dev_ptrs, asynchronous on the caller's stream):
    the stripe is skipped and the device record names the slot and both tags; taking the record
    clears it; the device keeps working."""
    torch = _torch()
    k, m, S = 12, 5, 2 * 16384 + 48
    truth = _stripe(k, m, S, 31)
    enc = rs.New(k, m)
    assert rs.table_fault_take(0) is None
    sh = [to_device(truth[i]) if i < k else torch.full((S,), 0xA5, dtype=torch.uint8, device="cuda")
          for i in range(k + m)]
    rs.debug_corrupt_next_table(k + 2)
    enc.Encode(sh)
    torch.cuda.synchronize()
    f = rs.table_fault_take(0)
    assert f is not None and f["slot"] == k + 2 and f["stripe"] == 0, f
    assert f["entry_tag"] != f["launch_tag"] and f["address"] == sh[k + 2].data_ptr()
    assert rs.table_fault_take(0) is None
    for i in range(k, k + m):
        assert bool((sh[i] == 0xA5).all()), i
    enc.Encode(sh)
    torch.cuda.synchronize()
    assert rs.table_fault_take(0) is None
    for i in range(k, k + m):
        assert np.array_equal(to_numpy(sh[i]), truth[i]), i


@pytest.mark.gpu
def test_gpu_default_recovery_compiles_its_network_in_the_background():
    """blb's widest recovery shape (RS(12,5), 5 bad pieces, every absent slot rebuilt) with
    BLBRS_RTC = 0 runs on tables and requests no network; with the default knobs the first call
    runs on tables while its network compiles in the background, and once compiled (rtc_wait)
    the pass loads and runs the network -- the same bytes every time.  (torch's ROCm build maps
    its own libhiprtc, so this torch process cannot show the library leaving hipRTC unmapped:
    test_library_does_not_link_hiprtc checks that without torch.)"""
    code = r'''
import numpy as np, torch
from blb_amd import reedsolomon as rs
from blb_amd.hostcopy import to_device, to_numpy
from oracle import rs_numpy as N
k, m, S = 12, 5, 2 * 16384 + 48
rng = np.random.default_rng(5)
data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
host = np.stack(data + list(N.encode(k, m, data)))[None]
present = [i not in (1, 3, 5, 8, 10) for i in range(k + m)]
enc = rs.New(k, m)
def run():
    st = to_device(host)
    for i in range(k + m):
        if not present[i]:
            st[:, i].fill_(0)
    enc.ReconstructBatch(st, present)
    assert np.array_equal(to_numpy(st), host)
rs.set_tuning("BLBRS_RTC", 0)
run()
assert rs.rtc_stats()["requested"] == 0 and rs.rtc_stats()["loaded"] == 0, rs.rtc_stats()
print("TABLES OK")
rs.set_tuning("BLBRS_RTC", 1)   # the default
run()                            # tables; the network is requested and compiles in the background
assert rs.rtc_stats()["requested"] >= 1, rs.rtc_stats()
assert rs.rtc_wait(120000), rs.rtc_stats()
run()                            # loads and runs the network
assert rs.rtc_stats()["loaded"] >= 1 and rs.rtc_stats()["failed"] == 0, rs.rtc_stats()
print("NETWORK OK", rs.rtc_stats())
'''
    out = _maps_after(code, torch_first=True)
    assert "TABLES OK" in out and "NETWORK OK" in out, out[-2000:]
