#!/bin/bash
# Round-3 validation 2: GPU suite, zero-copy policy sweep, RS(8,3) mix ceilings, bench.
set -o pipefail
OUT=gpurun_out/${1:-r3val2}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& echo "== zc sweep" && timeout -k 10 600 python -u tools/host_paths.py --zc-sweep > "$OUT/zc_sweep.json" 2> "$OUT/zc_sweep.err" \
&& echo "== mix rs83" && timeout -k 10 120 ./tools/_build/mix_probe rs83 > "$OUT/mix_rs83.txt" 2>&1 \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "exit $rc"; tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/mix_rs83.txt"; cat "$OUT/bench.json" | cut -c1-600
exit $rc
