"""Is the RS(6,3) encode power-capped, and does spending less power in the CUs buy bandwidth?
(profiles/r04/clocks: during the encode the socket sits at ~1385 W with the package power
limit (PPT) active most of the time.)  One process, one 77 GB batch, variants interleaved
round by round; each variant runs for about --secs seconds of back-to-back launches while the
GPU's metrics table is read before and after (amdsmi, read-only):
  median launch ms, PPT residency (ppt_residency_acc / accumulation_counter over the run),
  mean socket power from the energy accumulator, gfx clock samples.
Variants are library knobs (rs.tuning): the compiled bit-plane network instead of the v_perm
tables (BLBRS_BITSLICE=2: different VALU work for the same bytes).  The grid caps in
profiles/r04/clocks/power_ab.jsonl used a knob (BLBRS_CODE_GRID, fewer resident waves looping
over the tiles) of the build at commit f5141c9; it was measured 10 % slower and removed, so the
shipped kernel stays the one validated.  Prints one JSON line per variant
per round and a summary."""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--secs", type=float, default=2.0)
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--variants", default="default:;network:BLBRS_BITSLICE=2")
a = p.parse_args()

variants = []
for item in a.variants.split(";"):
    name, _, env = item.partition(":")
    variants.append((name, {kk: int(v) for kk, v in (kv.split("=", 1) for kv in env.split("+") if kv)}))

import amdsmi  # noqa: E402
amdsmi.amdsmi_init()
hip = ctypes.CDLL("libamdhip64.so")
buf = ctypes.create_string_buffer(64)
hip.hipDeviceGetPCIBusId(buf, 64, 0)
bdf = buf.value.decode().lower().split(":", 1)[-1]
h = next(x for x in amdsmi.amdsmi_get_processor_handles()
         if amdsmi.amdsmi_get_gpu_device_bdf(x).lower().split(":", 1)[-1] == bdf)

k, m, B, S = 6, 3, 1024, 8 << 20
dev = torch.device("cuda:0")
st = torch.empty((B, k + m, S), dtype=torch.uint8, device=dev)
st[:, :k].random_(0, 256)
enc = rs.New(k, m)
enc.EncodeBatch(st)
ok = bool(enc.VerifyBatch(st).all())
exact = {}
for name, knobs in variants:   # warm every variant once, on poisoned parity: bit-exactness per variant
    st[:, k:].fill_(0xA5)
    with rs.tuning(**knobs):
        enc.EncodeBatch(st)
    exact[name] = bool(enc.VerifyBatch(st).all())
torch.cuda.synchronize()

ENERGY_J = 15.259e-6  # energy_accumulator unit (J per count)


def run(knobs):
    clocks, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            try:
                clocks.append(amdsmi.amdsmi_get_gpu_metrics_info(h).get("current_gfxclk"))
            except Exception:  # noqa: BLE001
                return
            time.sleep(0.05)
    ms = []
    with rs.tuning(**knobs):
        m0 = amdsmi.amdsmi_get_gpu_metrics_info(h)
        t0 = time.perf_counter()
        th = threading.Thread(target=sampler)
        th.start()
        while time.perf_counter() - t0 < a.secs:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            enc.EncodeBatch(st)
            e.record()
            torch.cuda.synchronize()
            ms.append(s.elapsed_time(e))
        el = time.perf_counter() - t0
        m1 = amdsmi.amdsmi_get_gpu_metrics_info(h)
        stop.set()
        th.join()
    acc = m1["accumulation_counter"] - m0["accumulation_counter"]
    ppt = m1["ppt_residency_acc"] - m0["ppt_residency_acc"]
    energy = (m1["energy_accumulator"] - m0["energy_accumulator"]) * ENERGY_J
    ms.sort()
    clk = sorted(c for c in clocks if isinstance(c, int) and c < 0xFFFF)
    return {"launches": len(ms), "median_ms": round(ms[len(ms) // 2], 3), "min_ms": round(ms[0], 3),
            "ppt_residency": round(ppt / acc, 3) if acc else None,
            "mean_power_W": round(energy / el, 1),
            "gfxclk_median": clk[len(clk) // 2] if clk else None}


res = {}
for r in range(a.rounds):
    for name, knobs in variants:
        x = run(knobs)
        res.setdefault(name, []).append(x)
        print(json.dumps({"round": r, "variant": name, **x}), flush=True)
ok = ok and bool(enc.VerifyBatch(st).all())
summary = {}
for name, xs in res.items():
    med = sorted(x["median_ms"] for x in xs)
    summary[name] = {"median_ms": med[len(med) // 2], "ppt": [x["ppt_residency"] for x in xs],
                     "power_W": [x["mean_power_W"] for x in xs], "gfxclk": [x["gfxclk_median"] for x in xs]}
print(json.dumps({"summary": summary, "verify_ok": ok, "bit_exact": exact}), flush=True)
