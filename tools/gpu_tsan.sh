#!/bin/bash
# The C++ mirror's tests on the GPU, plain and under ThreadSanitizer (built beforehand by
# tools/tsan_build.sh).  TSan's exit code is forced to 0: the reports are read afterwards
# (tools/tsan_summary.py); a failing test still fails the run.
set -o pipefail
OUT=gpurun_out/${1:-r3tsan}
mkdir -p "$OUT"
echo "== rs_test" && timeout -k 10 300 tests/cpp/_build/rs_test > "$OUT/rs_test.log" 2>&1 \
&& echo "== rs_test_tsan" && TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 exitcode=0" \
   timeout -k 10 900 tools/_build/tsan/rs_test_tsan > "$OUT/rs_test_tsan.log" 2>&1
rc=$?
echo "exit $rc"
grep -E "^(---|PASS|FAIL|    lanes)" "$OUT/rs_test.log" | tail -30
grep -E "^(---|PASS|FAIL|    lanes)" "$OUT/rs_test_tsan.log" | tail -30
grep -c "WARNING: ThreadSanitizer" "$OUT/rs_test_tsan.log"
gzip -f "$OUT/rs_test_tsan.log"
exit $rc
