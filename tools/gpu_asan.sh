#!/bin/bash
# The C++ mirror's tests on the GPU with the library's and the tests' host code under
# AddressSanitizer (built beforehand by tools/asan_build.sh), REPS times in a row; the first
# report or failing run ends the call.  Device code is not instrumented.
set -o pipefail
OUT=gpurun_out/${1:-r4asan}
REPS=${2:-3}
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  echo "== run $i"
  ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0" \
    timeout -k 10 600 tools/_build/asan/rs_test_asan > "$OUT/rs_test_asan_$i.log" 2>&1
  rc=$?
  grep -E "^(--- FAIL|PASS|FAIL)" "$OUT/rs_test_asan_$i.log" | tail -3
  if [ $rc -ne 0 ]; then
    echo "exit $rc"
    grep -n -A40 "ERROR: AddressSanitizer" "$OUT/rs_test_asan_$i.log" | head -80
    exit $rc
  fi
done
echo "all $REPS runs clean"
