"""Decode networks generated per erasure pattern and compiled at run time (rtc.hip).

blb's recovery RPC reads exactly the first k good pieces and rebuilds every absent slot
(internal/curator/reconstruct.go:51-79 -> internal/tractserver/store.go:1062-1102); the
client's degraded read rebuilds the missing data slots (client/blb/reconstruct.go:137-173).
Those passes' rows -- inv(M[valid]) and P * inv(M[valid]) -- depend on the erasure pattern,
so on wide shapes the library generates their bit-plane XOR network and compiles it with
hipRTC.

CPU: the generated network (with and without shared XOR terms) evaluated bit plane by bit
plane equals the oracle's GF(2^8) product for every blb class at 1..m erasures and for
random matrices, and the kernel source compiles for gfx950 (hipRTC needs no device).
GPU: every class at 1..m erasures in the RPC and client shapes, through the device batch
(strided) and the host call (pointer table) and the tractserver mirror with the curator's
indexMap (-1 padding), bit-exact against the oracle, with the network actually loaded.
"""
import os
import re

import numpy as np

import pytest

from blb_amd import reedsolomon as rs
from blb_amd.hostcopy import from_numpy_pinned, to_device, to_numpy
from oracle import rs_numpy as N

CLASSES = [(6, 3), (8, 3), (10, 3), (12, 5)]  # internal/core/StorageClass.go:7-13


def rpc_present(k, m, bad):
    """reconstruct.go:51-53: sources = the first k good pieces in index order."""
    good = [i for i in range(k + m) if i not in bad]
    return [i in good[:k] for i in range(k + m)]


def bad_sets(k, m):
    """1..m bad data pieces spread evenly over the data slots (tools/rpc_shapes.py)."""
    spread = [1 + (i * k) // m for i in range(m)]
    return [spread[:e] for e in range(1, m + 1)]


def pass_rows(k, m, present, data_only):
    """The rows the library's decode plan holds: missing data rows of inv(M[valid]), then (not
    data_only) P[i] * inv(M[valid]) for missing parity i."""
    valid, dec = N.decode_rows(k, m, present)
    mat = N.build_matrix(k, m)
    rows = [dec[i] for i in range(k) if not present[i]]
    if not data_only:
        rows += [N.gf_matmul(mat[i:i + 1], dec)[0] for i in range(k, k + m) if not present[i]]
    return valid, np.array(rows, dtype=np.uint8)


def eval_network(src, k, rows, inputs):
    """Runs the generated device source on the host: planes as 0/1 byte arrays."""
    body = src.split("using blbrs::dev::xor3;")[1].split("#pragma unroll")[0]
    x = [[(inputs[c] >> q) & 1 for q in range(8)] for c in range(k)]
    env = {"x": x, "xor3": lambda a, b, c: a ^ b ^ c, "Z": np.zeros_like(inputs[0])}
    o = [[None] * 8 for _ in range(rows)]
    env["o"] = o
    for stmt in body.split(";"):
        stmt = stmt.strip()
        if not stmt:
            continue
        stmt = re.sub(r"^const uint32_t ", "", stmt).replace("0u", "Z")
        exec(stmt, {"__builtins__": {}}, env)  # noqa: S102 -- our own generated XOR network
    return [sum((o[r][p].astype(np.uint8) << p) for p in range(8)).astype(np.uint8) for r in range(rows)]


def shapes():
    out = []
    for k, m in CLASSES:
        for bad in bad_sets(k, m):
            out.append((k, m, rpc_present(k, m, bad), False))
        out.append((k, m, [i != 1 and i <= k for i in range(k + m)], True))  # client, 1 row
    out.append((10, 4, [i not in (1, 7) for i in range(14)], False))          # BASELINE config 4
    return out


@pytest.mark.parametrize("k,m,present,data_only", shapes())
def test_generated_network_equals_oracle(k, m, present, data_only):
    rng = np.random.default_rng(k * 100 + sum(present))
    valid, rows = pass_rows(k, m, present, data_only)
    inputs = [rng.integers(0, 256, 4096, dtype=np.uint8) for _ in range(k)]
    want = N.code(rows, inputs)
    src, ops = rs.rtc_network_source(rows)
    got = eval_network(src, k, rows.shape[0], inputs)
    for r in range(rows.shape[0]):
        assert np.array_equal(got[r], want[r]), (k, m, r)
    assert ops > 0


def test_generated_network_random_matrices():
    rng = np.random.default_rng(4242)
    for _ in range(12):
        k, r = int(rng.integers(2, 17)), int(rng.integers(1, 9))
        rows = rng.integers(0, 256, (r, k), dtype=np.uint8)
        rows[0, 0] = 0  # zero coefficients and rows are legal
        inputs = [rng.integers(0, 256, 512, dtype=np.uint8) for _ in range(k)]
        src, _ = rs.rtc_network_source(rows)
        got = eval_network(src, k, r, inputs)
        want = N.code(rows, inputs)
        assert all(np.array_equal(a, b) for a, b in zip(got, want)), (k, r)


def test_network_kernel_compiles_for_gfx950():
    """hipRTC compiles rs_code_kernel with a generated network against the embedded headers:
    RS(12,5)'s RPC shape (store, strided), and a store+verify pass on a pointer table."""
    _, rows = pass_rows(12, 5, rpc_present(12, 5, [1]), False)
    rs.rtc_compile(rows, mode=0, strided=True)
    _, rows = pass_rows(10, 4, [i not in (3,) for i in range(14)], False)
    rs.rtc_compile(rows, mode=2, strided=False)
    assert rs.rtc_stats()["compiled"] >= 2


def test_knobs_read_once_and_settable(knob):
    for name in ("BLBRS_BITSLICE", "BLBRS_RTC", "BLBRS_RTC_WIDE", "BLBRS_EC_PERSISTENT", "BLBRS_DONE_WORD"):
        v = rs.get_tuning(name)
        knob(name, v + 1)
        assert rs.get_tuning(name) == v + 1
    with pytest.raises(rs.ErrInvalidArgument):
        rs.set_tuning("BLBRS_NO_SUCH_KNOB", 1)


# ---------------------------------------------------------------- GPU -------------------------

def _torch():
    import torch
    return torch


def _oracle_stripes(k, m, B, S, seed):
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (B, k + m, S), dtype=np.uint8)
    for b in range(B):
        host[b, k:] = np.stack(N.encode(k, m, [host[b, i] for i in range(k)]))
    return host


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", CLASSES)
def test_gpu_rpc_and_client_shapes_with_networks(k, m, knob):
    """Every class, e = 1..m bad data pieces in the RPC shape (all m absent slots rebuilt) and
    the client shape (missing data only), device batch (strided) and host calls (pointer
    table), with the run-time networks compiled by the caller (BLBRS_RTC = 2): bit-exact
    against the oracle; the wide classes must have loaded their networks."""
    torch = _torch()
    knob("BLBRS_RTC", 2)
    knob("BLBRS_RTC_WIDE", 9)   # networks for every wide class (the default takes k + rows > 13)
    S, B = 3 * 16384 + 4 * 1000 + 16, 3          # whole tiles (network) + a ragged tail (tables)
    host = _oracle_stripes(k, m, B, S, 77 * k + m)
    enc = rs.New(k, m)
    before = rs.rtc_stats()
    cases = [(rpc_present(k, m, bad), False) for bad in bad_sets(k, m)]
    cases.append(([i != 1 and i <= k for i in range(k + m)], True))
    miss = bad_sets(k, m)[-1]
    first_k = [j for j in range(k + m) if j not in miss][:k]
    cases.append(([i in first_k for i in range(k + m)], True))
    for ci, (present, data_only) in enumerate(cases):
        print(f"case {ci}: present={[i for i in range(k + m) if present[i]]} data_only={data_only}", flush=True)
        st = to_device(host)
        for i in range(k + m):
            if not present[i]:
                st[:, i].fill_(0xA5)
        torch.cuda.synchronize()   # a fault left by earlier work surfaces here, not after the rebuild
        enc.ReconstructBatch(st, present, data_only=data_only)
        got = to_numpy(st)
        for i in range(k + m):
            if present[i] or (data_only and i >= k):
                continue
            assert np.array_equal(got[:, i], host[:, i]), (k, m, present, i)
        # host call: pointer-table addressing, klauspost slice semantics
        b = 1
        shards = [host[b, i].copy() if present[i] else None for i in range(k + m)]
        (enc.ReconstructData if data_only else enc.Reconstruct)(shards)
        for i in range(k if data_only else k + m):
            assert np.array_equal(shards[i], host[b, i]), (k, m, present, i)
    after = rs.rtc_stats()
    if k + m > 9:
        assert after["loaded"] > before["loaded"], (before, after)
        assert after["failed"] == before["failed"], rs.rtc_stats()


@pytest.mark.gpu
@pytest.mark.parametrize("k,m", [(10, 4), (12, 5)])
def test_gpu_network_verify_modes_flag_corruption(k, m, knob):
    """Networks in the compare modes (opted in, BLBRS_RTC = 2, threshold 9): reconstructAndVerify
    with e < m data pieces missing is ONE store+verify pass (MODE 2: e rows stored, the m - e
    parity pieces the decode did not read compared), on a device batch (strided) and a host call
    (pointer table); a corrupted leftover parity byte inside a whole tile must turn that
    stripe's verdict false and only that one.  The network must have been loaded."""
    torch = _torch()
    knob("BLBRS_RTC", 2)
    knob("BLBRS_RTC_WIDE", 9)
    S, B = 3 * 16384 + 4 * 1000 + 16, 3
    host = _oracle_stripes(k, m, B, S, 500 + k)
    enc = rs.New(k, m)
    before = rs.rtc_stats()
    miss = [1, 4]                          # e = 2 < m: rows = 2 stored + (m - 2) compared
    present = [i not in miss for i in range(k + m)]
    bad = host.copy()
    bad[1, k + m - 1, 5000] ^= 0x40        # a leftover parity piece of stripe 1, inside tile 0
    st = to_device(bad)
    for i in miss:
        st[:, i].fill_(0xA5)
    ok = to_numpy(enc.ReconstructAndVerifyBatch(st, present))
    assert list(ok) == [True, False, True], ok
    got = to_numpy(st)
    for i in miss:
        assert np.array_equal(got[:, i], host[:, i]), i
    for b, want in ((0, True), (1, False)):
        sh = [bad[b, i].copy() if present[i] else None for i in range(k + m)]
        assert enc.ReconstructAndVerify(sh) is want, b
        for i in miss:
            assert np.array_equal(sh[i], host[b, i]), (b, i)
    after = rs.rtc_stats()
    assert after["loaded"] >= before["loaded"] + 2, (before, after)   # strided and pointer-table kernels
    assert after["failed"] == before["failed"]


@pytest.mark.gpu
def test_gpu_network_verify_k_outside_compiled_list(knob):
    """Verify for k = 14 (no compiled encode network): opted in, the parity check runs on a
    run-time network in verify mode (MODE 1); a corrupted parity byte and a corrupted data byte,
    each inside a whole tile of its own stripe, are both flagged."""
    torch = _torch()
    knob("BLBRS_RTC", 2)
    k, m = 14, 4
    S, B = 2 * 16384 + 4 * 1000, 3
    host = _oracle_stripes(k, m, B, S, 1404)
    enc = rs.New(k, m)
    assert enc.compiled_network()["rtc"]
    before = rs.rtc_stats()
    bad = host.copy()
    bad[0, k + 2, 100] ^= 1                # parity
    bad[2, 7, 20000] ^= 0x80               # data
    ok = to_numpy(enc.VerifyBatch(to_device(bad)))
    assert list(ok) == [False, True, False], ok
    assert rs.rtc_stats()["loaded"] > before["loaded"]
    assert rs.rtc_stats()["failed"] == before["failed"]


@pytest.mark.gpu
def test_gpu_network_async_then_loaded(knob):
    """Default mode (BLBRS_RTC = 1): the first calls run the table kernel while the network
    compiles in the background; after rtc_wait() the same pattern runs the network.  Same
    bytes throughout."""
    torch = _torch()
    knob("BLBRS_RTC", 1)
    k, m = 12, 5
    S, B = 2 * 16384 + 48, 2
    host = _oracle_stripes(k, m, B, S, 9)
    enc = rs.New(k, m)
    present = rpc_present(k, m, [2, 9])
    for _ in range(2):
        st = to_device(host)
        for i in range(k + m):
            if not present[i]:
                st[:, i].fill_(0)
        enc.ReconstructBatch(st, present)
        assert np.array_equal(to_numpy(st), host)
        assert rs.rtc_wait(120_000)
    assert rs.rtc_stats()["failed"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,nbad", [(k, m, e) for k, m in CLASSES for e in range(1, m + 1)])
def test_gpu_tractserver_recovery_rpc_with_indexmap_padding(k, m, nbad, knob, oracle_lib):
    """curator.reconstruct_request -> Store.rs_encode for each class and 1..m bad pieces (data
    and parity mixed): the request carries dests padded to m with index -1
    (reconstruct.go:72-79); the tractserver reads the first k good pieces, rebuilds every
    absent slot (networks on wide classes) and writes only the real destinations."""
    from blb_amd import curator
    from blb_amd.blbcore import Error, RSChunkID, TSAddr
    from blb_amd.tractserver import MemTractserverTalker, Store
    knob("BLBRS_RTC", 2)
    knob("BLBRS_RTC_WIDE", 9)
    L = 3 * 16384 + 4096 + 16
    host = _oracle_stripes(k, m, 1, L, 5 * k + m)[0]
    hosts = [TSAddr(10 + i, f"ts{i}") for i in range(k + m)]
    # bad pieces: data slots spread over the stripe, the last one a parity piece when e > 1
    bad = bad_sets(k, m)[nbad - 1][:nbad - 1] + ([k + m - 1] if nbad > 1 else [1 + k // 2])
    req, err = curator.reconstruct_request(RSChunkID(0x80000007, 1000), k, hosts, [10 + i for i in bad],
                                           lambda c: [TSAddr(200 + j, f"new{j}") for j in range(c)], length=L)
    assert err == Error.NoError
    assert req.index_map[k + nbad:] == [-1] * (m - nbad)
    t = MemTractserverTalker()
    for src, idx in zip(req.srcs, req.index_map[:k]):
        t.add_ctl_read_reply(src.host, host[idx], Error.ErrEOF)
    for j in range(nbad):
        t.add_ctl_write_reply(f"new{j}", Error.NoError)
    s = Store(t, encode_increment_size=L)
    assert s.rs_encode(req.chunk_id, L, req.srcs, req.dests, req.index_map) == Error.NoError
    assert sorted(t.ctl_write_calls) == sorted(f"new{j}" for j in range(nbad))
    for j, idx in enumerate(req.index_map[k:k + nbad]):
        got = np.concatenate([b for (_, _, b, _) in t.ctl_write_calls[f"new{j}"]])
        assert np.array_equal(got, host[idx]), (k, m, bad, idx)


@pytest.mark.gpu
def test_gpu_network_loaded_once_by_concurrent_launches(knob):
    """Default mode: the background thread only compiles; the first launches that find the code
    object compiled load it in their own thread (rtc::ready).  Eight threads, each on its own
    stream, race to that first load of one RS(12,5) pattern: exactly one module load, every
    result bit-exact, no failure."""
    import threading
    torch = _torch()
    knob("BLBRS_RTC", 1)
    k, m = 12, 5
    S, B = 2 * 16384 + 48, 2
    host = _oracle_stripes(k, m, B, S, 31)
    enc = rs.New(k, m)
    present = rpc_present(k, m, [0, 4, 11])
    st0 = to_device(host)
    enc.ReconstructBatch(st0, present)           # requests the network; runs the tables
    assert np.array_equal(to_numpy(st0), host)
    assert rs.rtc_wait(120_000)                  # compiled, not yet loaded
    before = rs.rtc_stats()
    bufs = [to_device(host) for _ in range(8)]
    for b in bufs:
        for i in range(k + m):
            if not present[i]:
                b[:, i].fill_(0x3C)
    torch.cuda.synchronize()
    start, errors = threading.Barrier(8), []

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                start.wait()
                enc.ReconstructBatch(bufs[t], present)
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for b in bufs:
        assert np.array_equal(to_numpy(b), host)
    after = rs.rtc_stats()
    assert after["failed"] == before["failed"]
    assert after["loaded"] - before["loaded"] == 1, (before, after)   # one pass, one device


@pytest.mark.gpu
def test_gpu_network_pointer_table_misaligned_and_ragged(knob):
    """A wide decode through the device pointer table (blbrs_reconstruct_dev_ptrs) on its
    run-time network, with one input shard 1 byte off 16-byte alignment and shard lengths that
    end mid-tile: the launch takes the table path for unaligned / partial tiles (rs_code.hpp),
    so every byte must still be the oracle's."""
    torch = _torch()
    knob("BLBRS_RTC", 2)
    k, m = 12, 5
    enc = rs.New(k, m)
    for S, odd in ((3 * 8192 + 4, 2), (4 * 8192, None), (8192 * 2 + 777, 0)):
        host = _oracle_stripes(k, m, 1, S, S)[0]
        bad = [1, 3, 5, 8, 10]
        present = rpc_present(k, m, bad)
        shards = []
        for i in range(k + m):
            if not present[i]:
                shards.append(torch.empty(0, dtype=torch.uint8, device="cuda"))
            elif i == odd:
                t = torch.empty(S + 1, dtype=torch.uint8, device="cuda")[1:]
                t.copy_(from_numpy_pinned(host[i]))
                shards.append(t)
            else:
                shards.append(to_device(host[i]))
        before = rs.rtc_stats()
        enc.Reconstruct(shards)
        torch.cuda.synchronize()
        for i in range(k + m):
            assert np.array_equal(to_numpy(shards[i]), host[i]), (S, odd, i)
        assert rs.rtc_stats()["failed"] == before["failed"]


_EXIT_SCRIPT = r'''
import ctypes, sys, threading, time
sys.path.insert(0, sys.argv[1])
import numpy as np
from blb_amd import _lib
lib = _lib.load()
rng = np.random.default_rng(int(sys.argv[2]))
def loop():
    while True:
        coef = rng.integers(1, 256, 12 * 5, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        lib.blbrs_rtc_compile(12, 5, coef.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 0, 1, None, 0,
                              ctypes.byref(n))
threading.Thread(target=loop, daemon=True).start()
time.sleep(0.6)
print("exiting", flush=True)
'''


@pytest.mark.parametrize("seed", [1, 2])
def test_exit_with_a_compile_in_flight(seed):
    """The library's exit handler (rtc.hip at_exit) waits for its own background compiler only:
    a process that exits while one of ITS threads is inside hipRTC (here a Python daemon thread
    in blbrs_rtc_compile) exits cleanly, neither hanging on that compile nor crashing when the
    thread would return into a finalized interpreter."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # A ctypes-only process (no torch): torch's wheel brings its own comgr, whose static
    # destructors then race a caller-thread compile at exit the same way.
    env = dict(os.environ, BLBRS_NO_TORCH="1")
    p = subprocess.run([sys.executable, "-c", _EXIT_SCRIPT, root, str(seed)], capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode == 0, (p.returncode, p.stdout[-500:], p.stderr[-2000:])
    assert "exiting" in p.stdout
