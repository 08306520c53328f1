#!/bin/bash
# Network encode with every load issued before the math (sched_barrier): RS(6,3) and wide
# shapes, tables vs network, plus occupancy caps on the network launches.
set -o pipefail
OUT=gpurun_out/${1:-r3bs5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bitslice.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bitslice_ab.py --shapes "6,3,1024;12,5,512;10,4,512" --reps 3 --ops encode,verify \
  --variants "perm:BLBRS_BITSLICE=0;net:BLBRS_BITSLICE=2;n2:BLBRS_BITSLICE=2+BLBRS_OCC_LDS=65536;n3:BLBRS_BITSLICE=2+BLBRS_OCC_LDS=54000" \
  > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?; cut -c1-1600 "$OUT/ab.jsonl"; exit $rc
