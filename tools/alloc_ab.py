"""Does the way a ~77 GB stripe batch is allocated move the coding kernel?  Placement moved the
same kernel by up to 10 % between processes (profiles/r04/rtc_ab/README.md).  In ONE process
this allocates RS(6,3) B=1024 batches (77.3 GB each) three ways -- torch.empty (the caching
allocator's hipMalloc), hipMalloc directly, hipExtMallocWithFlags(hipDeviceMallocContiguous) --
and times the encode (blbrs_encode_dev) on each, interleaved rep by rep.  Prints one JSON line."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import _lib  # noqa: E402
from blb_amd import reedsolomon as rs  # noqa: E402

k, m, B, S = 6, 3, int(os.environ.get("ALLOC_AB_B", "1024")), 8 << 20
n = k + m
size = B * n * S
reps = int(os.environ.get("ALLOC_AB_REPS", "5"))
dev = torch.device("cuda:0")
torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
hip.hipDeviceSynchronize.argtypes = []
lib = _lib.load()
enc = rs.New(k, m)

bufs = {}
t = torch.empty(size, dtype=torch.uint8, device=dev)
bufs["torch_empty"] = t.data_ptr()
for name, fn in (("hipMalloc", lambda p: hip.hipMalloc(ctypes.byref(p), size)),
                 ("contiguous", lambda p: hip.hipExtMallocWithFlags(ctypes.byref(p), size, 0x4))):
    p = ctypes.c_void_p()
    rc = fn(p)
    if rc == 0:
        bufs[name] = p.value
    else:
        print(json.dumps({"alloc_failed": name, "rc": rc}), flush=True)
for name, ptr in bufs.items():
    assert hip.hipMemset(ctypes.c_void_p(ptr), 0x5A, size) == 0
hip.hipDeviceSynchronize()
stream = torch.cuda.current_stream(dev)


def encode(ptr):
    rc = lib.blbrs_encode_dev(enc._h, ctypes.c_void_p(ptr), S, n * S, B, S, ctypes.c_void_p(stream.cuda_stream))
    assert rc == 0, rc


res = {name: [] for name in bufs}
for name, ptr in bufs.items():
    encode(ptr)
torch.cuda.synchronize()
for _ in range(reps):
    for name, ptr in bufs.items():
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(stream)
        encode(ptr)
        e.record(stream)
        torch.cuda.synchronize()
        res[name].append(round(s.elapsed_time(e), 3))
print(json.dumps({"B": B, "GB": round(size / 1e9, 1), "ms": res,
                  "median": {kk: sorted(v)[len(v) // 2] for kk, v in res.items()}}), flush=True)
for name, ptr in bufs.items():
    if name != "torch_empty":
        hip.hipFree(ctypes.c_void_p(ptr))
