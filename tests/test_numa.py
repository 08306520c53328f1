"""NUMA placement for 8-GPU hosts (two sockets, four GPUs behind each; SURVEY §5 / BASELINE
config 5): a rank binds its CPUs and host pages to its GPU's node (bench.py via
multigpu.bind_to_node), and the library routes a host call on pool or registered buffers to a
GPU on the node holding them (runtime pick_lane).  On the one-GPU box every lane is
local, so the GPU tests check the recorded nodes, deterministic routing on [0, 0] and bit
exactness; the policy itself is tested on explicit lanes."""
import ctypes
import os
import threading

import numpy as np
import pytest

from blb_amd import multigpu
from blb_amd import reedsolomon as rs

MB = 1 << 20


def test_lane_policy_prefers_local_then_load():
    # lanes 0,1 on node 0, lanes 2,3 on node 1
    nodes = [0, 0, 1, 1]
    assert rs.lane_policy(nodes, [0, 0, 0, 0], 0, 1) == 2          # idle: first local lane from start
    assert rs.lane_policy(nodes, [0, 0, 0, 0], 3, 1) == 3
    assert rs.lane_policy(nodes, [0, 0, 8 * MB, 4 * MB], 0, 1) == 3  # least-loaded local lane
    # a local lane within the 64 MiB slack of the global best still wins
    assert rs.lane_policy(nodes, [0, 0, 60 * MB, 70 * MB], 0, 1) == 2
    # beyond the slack the least-loaded lane overall wins
    assert rs.lane_policy(nodes, [0, 0, 65 * MB, 70 * MB], 0, 1) == 0
    # no preference (pageable memory) or no lane on the node: load only, rotating start
    assert rs.lane_policy(nodes, [5, 1, 1, 9], 0, -1) == 1
    assert rs.lane_policy(nodes, [5, 1, 1, 9], 2, -1) == 2
    assert rs.lane_policy(nodes, [5, 1, 1, 9], 0, 7) == 1
    assert rs.lane_policy([-1, -1], [3, 2], 0, 0) == 1               # unknown device nodes


def test_parse_cpulist():
    assert multigpu.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert multigpu.parse_cpulist("") == set()


def test_bind_to_node_respects_affinity(tmp_path):
    mine = sorted(os.sched_getaffinity(0))
    (tmp_path / "node0").mkdir()
    (tmp_path / "node0" / "cpulist").write_text(f"{mine[0]}-{mine[-1] + 100}\n")
    (tmp_path / "node1").mkdir()
    (tmp_path / "node1" / "cpulist").write_text(f"{mine[-1] + 200}-{mine[-1] + 201}\n")
    try:
        out = multigpu.bind_to_node(1, sysfs=str(tmp_path))   # no CPU of this job on node 1
        assert out["cpus_bound"] == 0 and not out["bound"]
        assert sorted(os.sched_getaffinity(0)) == mine
        out = multigpu.bind_to_node(0, sysfs=str(tmp_path))
        assert out["cpus_bound"] == len(mine)
        assert sorted(os.sched_getaffinity(0)) == mine
        assert multigpu.bind_to_node(-1)["bound"] is False
    finally:
        os.sched_setaffinity(0, mine)
        libc = ctypes.CDLL(None, use_errno=True)
        libc.syscall(238, 0, None, ctypes.c_ulong(0))  # back to MPOL_DEFAULT


# ------------------------------------------------------------------ GPU ------------------------

def _page_node(addr):
    libc = ctypes.CDLL(None, use_errno=True)
    node = ctypes.c_int(-1)
    rc = libc.syscall(239, ctypes.byref(node), None, ctypes.c_ulong(0), ctypes.c_void_p(addr), ctypes.c_ulong(3))
    return node.value if rc == 0 else -1


def _sysfs_gpu_node(dev):
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    assert hip.hipDeviceGetPCIBusId(buf, 64, dev) == 0
    try:
        return int(open(f"/sys/bus/pci/devices/{buf.value.decode().lower()}/numa_node").read())
    except OSError:
        return -1


@pytest.mark.gpu
def test_gpu_recorded_nodes():
    import torch
    torch.cuda.init()
    assert rs.device_numa_node(0) == _sysfs_gpu_node(0)
    b = rs.GetBuffer(4 << 20)
    try:
        addr = b.__array_interface__["data"][0]
        assert rs.host_numa_node(b) == _page_node(addr)
        assert rs.host_numa_node(addr + 123) == rs.host_numa_node(b)   # inside the buffer
    finally:
        rs.PutBuffer(b)
    assert rs.host_numa_node(np.zeros(16, np.uint8)) == -1              # pageable: no record


@pytest.mark.gpu
def test_gpu_numa_routing_on_two_lanes_bit_exact(oracle_lib):
    """[0, 0] with pool buffers: the device's node overridden to the buffers' node (every lane
    local) and to another node (no lane local: load-only routing); 16 concurrent Encodes each
    way, bit-exact, both lanes used, nothing left in flight."""
    import torch
    torch.cuda.init()
    k, m, S = 6, 3, 1 << 20
    threads = 16
    shards = []
    for t in range(threads):
        sh = [rs.GetBuffer(S) for _ in range(k + m)]
        g = np.random.default_rng(t)
        for i in range(k):
            sh[i][:] = g.integers(0, 256, S, dtype=np.uint8)
        shards.append(sh)
    node = rs.host_numa_node(shards[0][0])
    real = rs.device_numa_node(0)
    try:
        for dev_node in (node, node + 1):
            rs.set_device_numa_node(0, dev_node)
            enc = rs.New(k, m, devices=[0, 0])
            before = [enc.LaneStats(i)["calls"] for i in range(2)]

            def work(t):
                for _ in range(4):
                    enc.Encode(shards[t])
            th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            after = [enc.LaneStats(i) for i in range(2)]
            assert all(a["calls"] > b for a, b in zip(after, before)), (dev_node, after)
            assert all(a["inflight_calls"] == 0 for a in after)
            for t in range(0, threads, 5):
                want = [shards[t][i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
                oracle_lib.encode(k, m, want)
                for j in range(k, k + m):
                    assert np.array_equal(shards[t][j], want[j]), (dev_node, t, j)
    finally:
        rs.set_device_numa_node(0, real)
        for sh in shards:
            for x in sh:
                rs.PutBuffer(x)
