"""Is hipRTC compiling on one thread safe while another thread loads a code object
(hipModuleLoadData)?  Both go through comgr (LLVM) inside this process.  The library's
background network compiles overlapped module loads on launching threads (rtc.hip before the
compile/load lock), and runs of tests/cpp/rs_test ended in "LLVM ERROR: Cannot implicitly convert
a scalable size ..." inside hiprtcCompileProgram.

Phase "load": a helper thread compiles distinct networks (blbrs_rtc_compile, real compiles)
while the main thread loads / unloads one precompiled code object in a loop.  Phase "none": the
helper compiles while the main thread only sleeps (control).  One JSON line; a crash ends the
process.  python tools/comgr_race.py load|none [seconds]"""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

phase = sys.argv[1]
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
hip = ctypes.CDLL("libamdhip64.so")
hip.hipModuleLoadData.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
hip.hipModuleUnload.argtypes = [ctypes.c_void_p]
hip.hipSetDevice(0)
rng = np.random.default_rng(3)
code = rs.rtc_compile(rng.integers(1, 256, (5, 12), dtype=np.uint8))
buf = ctypes.create_string_buffer(code, len(code))
stop = threading.Event()
compiled = [0]
errors = []


def helper():
    r = np.random.default_rng(11)
    while not stop.is_set():
        try:
            rs.rtc_compile(r.integers(1, 256, (5, 12), dtype=np.uint8))
            compiled[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))
            return


th = threading.Thread(target=helper)
th.start()
t0 = time.time()
loads = 0
while time.time() - t0 < secs:
    if phase == "load":
        mod = ctypes.c_void_p()
        rc = hip.hipModuleLoadData(ctypes.byref(mod), buf)
        if rc != 0:
            errors.append(f"load rc {rc}")
            break
        hip.hipModuleUnload(mod)
        loads += 1
    else:
        time.sleep(0.05)
stop.set()
th.join()
print(json.dumps({"phase": phase, "seconds": round(time.time() - t0, 1), "compiles": compiled[0], "loads": loads,
                  "errors": errors[:3]}), flush=True)
