#!/bin/bash
# Round validation on one MI355X: GPU parity suite, smoke(), bench line, rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
OUT=gpurun_out/${1:-val}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "== pytest -m gpu" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& echo "== bench" && timeout -k 10 420 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-extra > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc"; tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/smoke.log"; cat "$OUT/bench.json"
exit $rc
