#!/bin/bash
# GPU suite, then the bit-plane network A/B (tools/bitslice_ab.py) for the library in the tree.
set -o pipefail
OUT=gpurun_out/${1:-r3bs}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"; grep -E "FAIL|Error" "$OUT/pytest_gpu.log" | head -5
[ $rc -eq 0 ] || exit $rc
echo "== bitslice A/B" && timeout -k 10 600 python -u tools/bitslice_ab.py ${AB_ARGS} > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?
cat "$OUT/ab.jsonl" | cut -c1-600; tail -3 "$OUT/ab.err"
exit $rc
