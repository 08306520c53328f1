"""Do the GPU's clocks explain the process-to-process spread of the encode (the same
kernel 11.0 ms in one process, 12.2 ms in another)?  Times RS(6,3) B=1024 encodes one by one
while a thread samples the GPU's metrics table through amdsmi (read-only: gfx / memory /
fabric clocks, HBM activity, power, temperatures, throttle status), and prints one JSON line:
launch times and each metric's min / median / max.  Run it in several processes of one call to
compare them.  python tools/clock_probe.py [launches]"""
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

FIELDS = ("average_gfxclk_frequency", "current_gfxclk", "current_uclk", "average_uclk_frequency",
          "current_fclk", "average_fclk_frequency", "current_socclk", "average_umc_activity",
          "average_socket_power", "current_socket_power", "temperature_hotspot", "temperature_mem",
          "throttle_status", "indep_throttle_status", "mem_activity_acc", "average_mm_activity")


def find_handle(amdsmi, bdf):
    for h in amdsmi.amdsmi_get_processor_handles():
        try:
            if amdsmi.amdsmi_get_gpu_device_bdf(h).lower().split(":", 1)[-1] == bdf.lower().split(":", 1)[-1]:
                return h
        except Exception:  # noqa: BLE001
            pass
    return None


def scalar(v):
    if isinstance(v, (list, tuple)):
        v = [x for x in v if isinstance(x, (int, float)) and x != 0xFFFF and x != 0xFFFFFFFF]
        return max(v) if v else None
    return v if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF) else None


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    dev = torch.device("cuda:0")
    k, m, B, S = 6, 3, 1024, 8 << 20
    st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
    st[:, :k].random_(0, 256)
    enc = rs.New(k, m)
    bdf = None
    out = {"pid": os.getpid(), "launches": launches}
    samples, stop = [], threading.Event()
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        if bdf is None:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            buf = ctypes.create_string_buffer(64)
            hip.hipDeviceGetPCIBusId(buf, 64, 0)
            bdf = buf.value.decode()
        h = find_handle(amdsmi, bdf)
        out["bdf"] = bdf

        def sampler():
            while not stop.is_set():
                try:
                    mtr = amdsmi.amdsmi_get_gpu_metrics_info(h)
                    samples.append({f: scalar(mtr.get(f)) for f in FIELDS if f in mtr})
                except Exception as e:  # noqa: BLE001
                    samples.append({"error": repr(e)})
                    return
                time.sleep(0.1)
        th = threading.Thread(target=sampler) if h is not None else None
        if th is None:
            out["amdsmi"] = "no handle for " + str(bdf)
    except Exception as e:  # noqa: BLE001
        out["amdsmi"] = repr(e)
        th = None
    enc.EncodeBatch(st)
    torch.cuda.synchronize()
    def full():
        try:
            return {k_: v_ for k_, v_ in amdsmi.amdsmi_get_gpu_metrics_info(h).items()}
        except Exception as e:  # noqa: BLE001
            return {"error": repr(e)}
    m0 = full() if th is not None else {}
    if th is not None:
        th.start()
    ms = []
    for _ in range(launches):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        enc.EncodeBatch(st)
        e.record()
        torch.cuda.synchronize()
        ms.append(round(s.elapsed_time(e), 3))
    stop.set()
    if th is not None:
        th.join()
        m1 = full()
        # counters that accumulate (residencies, energy, activity): their change over the loop
        deltas = {}
        for key, v1 in m1.items():
            v0 = m0.get(key)
            if isinstance(v1, int) and isinstance(v0, int) and v1 != v0 and v1 < 0xFFFFFFFFFFFFFFFF:
                deltas[key] = v1 - v0
        out["metric_deltas"] = deltas
        out["metrics_after"] = {key: scalar(v) for key, v in m1.items() if scalar(v) is not None}
    srt = sorted(ms)
    out["ms"] = {"min": srt[0], "median": srt[len(srt) // 2], "max": srt[-1], "first5": ms[:5], "last5": ms[-5:]}
    summ = {}
    for f in FIELDS:
        v = sorted(x[f] for x in samples if x.get(f) is not None)
        if v:
            summ[f] = {"min": v[0], "median": v[len(v) // 2], "max": v[-1]}
    out["metrics"] = summ
    out["samples"] = len(samples)
    if samples and "error" in samples[-1]:
        out["sample_error"] = samples[-1]["error"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
