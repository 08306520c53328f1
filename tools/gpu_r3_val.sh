#!/bin/bash
# Round-3 validation on one MI355X: the GPU suite, then the client degraded-read shape with the
# current library and with the round-2 build (tools/_build/libblbrs_r2.so) for before/after.
set -o pipefail
OUT=gpurun_out/${1:-r3val}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& echo "== client shape (current)" && timeout -k 10 300 python -u tools/host_paths.py --client-only > "$OUT/client_shape_after.json" 2> "$OUT/client_after.err" \
&& echo "== client shape (r2 lib)" && BLBRS_LIB_PATH=$PWD/tools/_build/libblbrs_r2.so timeout -k 10 300 python -u tools/host_paths.py --client-only > "$OUT/client_shape_before.json" 2> "$OUT/client_before.err"
rc=$?
echo "exit $rc"; tail -5 "$OUT/pytest_gpu.log"; cat "$OUT"/client_shape_*.json
exit $rc
