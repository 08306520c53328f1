"""Does the NUMA node of pinned host memory matter for the PCIe-inclusive paths?

The GPU box has two sockets (NUMA nodes 0 and 1), four MI355X behind each.  For each node,
pin this process to that node's CPUs, allocate the pinned stripes there (first touch by the
allocating thread), and time: the pinned H2D / D2H copy rate, and the zero-copy RS(6,3)
EncodeHostBatch (BASELINE config 5) of 24 stripes x 8 MiB.  Prints one JSON object.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from blb_amd import reedsolomon as rs  # noqa: E402

GIB = float(1 << 30)


def parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def gpu_numa_node(dev):
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, dev) != 0:
        return None, None
    bus = buf.value.decode().lower()
    try:
        return bus, int(open(f"/sys/bus/pci/devices/{bus}/numa_node").read())
    except OSError:
        return bus, None


def main():
    torch.cuda.init()
    dev = torch.device("cuda:0")
    bus, gnode = gpu_numa_node(0)
    nodes = {}
    for d in sorted(os.listdir("/sys/devices/system/node")):
        if d.startswith("node") and d[4:].isdigit():
            nodes[int(d[4:])] = parse_cpulist(open(f"/sys/devices/system/node/{d}/cpulist").read())
    k, m, S, nb = 6, 3, 8 << 20, 24
    enc = rs.New(k, m, devices=[0])
    out = {"gpu_pci_bus": bus, "gpu_numa_node": gnode, "nodes": len(nodes), "results": {}}
    orig = os.sched_getaffinity(0)
    dsrc = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for node, cpus in nodes.items():
        os.sched_setaffinity(0, cpus)
        res = {}
        for rep in range(2):
            h = torch.empty(512 << 20, dtype=torch.uint8).pin_memory()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(4):
                dsrc.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            res.setdefault("h2d_GBps", []).append(round(4 * h.numel() / (time.perf_counter() - t) / 1e9, 2))
            t = time.perf_counter()
            for _ in range(4):
                h.copy_(dsrc, non_blocking=True)
            torch.cuda.synchronize()
            res.setdefault("d2h_GBps", []).append(round(4 * h.numel() / (time.perf_counter() - t) / 1e9, 2))
            del h
            pinned = torch.empty((nb, k + m, S), dtype=torch.uint8).pin_memory()
            pinned[:, :k].fill_(0x3C + rep)
            host = pinned.numpy()
            lists = [[host[b, i] for i in range(k + m)] for b in range(nb)]
            enc.EncodeHostBatch(lists)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                enc.EncodeHostBatch(lists)
            torch.cuda.synchronize()
            res.setdefault("zero_copy_encode_GiBps_data", []).append(
                round(3 * nb * k * S / GIB / (time.perf_counter() - t), 2))
            del pinned, host, lists
        out["results"][f"node{node}"] = res
    os.sched_setaffinity(0, orig)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
