#!/bin/bash
# One GPU A/B step: the GPU tests named in $2 (pytest targets, "-" for none), then an A/B
# driver ($3: a tools/*.py command line), each under its own time limit; output under
# gpurun_out/$1.  Usage: tools/gpu_ab.sh NAME "tests/test_pack.py" "tools/pack_ab.py --reps 3"
set -o pipefail
OUT=gpurun_out/${1:?name}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:--}" != "-" ]; then
  timeout -k 10 400 python -u -m pytest $2 -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$3" ]; then
  timeout -k 10 600 python -u $3 > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
  rc=$?; cut -c1-2000 "$OUT/ab.jsonl"; tail -3 "$OUT/ab.err"; exit $rc
fi
