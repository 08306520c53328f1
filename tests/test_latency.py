"""Single-caller latency of blb's client degraded read (tests/cpp/latency_bench.cpp): blb runs one
client reconstruct at a time (client/blb/reconstruct.go:18-20), so per-call latency is what a reader
sees.  The bench times the drop-in through the C ABI next to the CPU restatement and checks every
GPU result against the CPU's bytes; here it runs short, as a parity test of that call shape (first
call of 132 erasure patterns over blb's four classes, then a steady pattern).  The numbers are in
DESIGN.md §4d."""
import json
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "_build", "latency_bench")


def test_latency_bench_built():
    assert os.path.exists(BIN), "run __graft_entry__.build()"


@pytest.mark.gpu
@pytest.mark.parametrize("size", [4096, 1 << 20])
def test_gpu_degraded_read_latency_bench_bit_exact(size):
    p = subprocess.run([BIN, str(size), "40"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    rows = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    check = [r for r in rows if r["row"] == "check"]
    assert check and check[0]["mismatches"] == 0
    first = [r for r in rows if r["row"] == "first_call_of_pattern" and r["side"] == "gpu"]
    assert first and first[0]["calls"] == 6 * 3 + 8 * 3 + 10 * 3 + 12 * 5
    assert any(r["row"] == "steady_state" and r["side"] == "gpu" and r["calls"] == 40 for r in rows)
