#!/bin/bash
# GPU suite + bench for the library in the tree.
set -o pipefail
OUT=gpurun_out/${1:-r3val3}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "exit $rc"; tail -3 "$OUT/pytest_gpu.log"; grep -E "FAIL|Error" "$OUT/pytest_gpu.log" | head -5; cut -c1-300 "$OUT/bench.json"
exit $rc
