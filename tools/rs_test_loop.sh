#!/bin/bash
# Runs the C++ mirror's tests (tests/cpp/_build/rs_test) REPS times in a row on the GPU; the
# first failing or aborting run ends the call, with its log (line-buffered: the last "---"
# line names the test before the one that failed).
set -o pipefail
OUT=gpurun_out/${1:-r4loop}
REPS=${2:-10}
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  timeout -k 10 300 tests/cpp/_build/rs_test > "$OUT/rs_test_$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "run $i exit $rc"
    tail -8 "$OUT/rs_test_$i.log"
    exit $rc
  fi
done
echo "all $REPS runs passed"
