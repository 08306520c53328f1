#!/bin/bash
# Round-3 artifacts for the library at HEAD: GPU suite, smoke, bench, rocprof kernel stats of
# the bench, PMC traffic of the shipped library (tools/pmc_prod.sh).
set -o pipefail
OUT=gpurun_out/${1:-r3final}
COMMIT=${2:-unknown}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& echo "== smoke" && timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
&& echo "== pmc" && bash tools/pmc_prod.sh "$OUT/pmc" r03 "$COMMIT" > "$OUT/pmc.log" 2>&1 \
&& echo "== bench" && timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& echo "== rocprof" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-extra > "$OUT/prof.log" 2>&1
rc=$?
echo "exit $rc"; tail -3 "$OUT/pytest_gpu.log"; cat "$OUT/smoke.log"; tail -2 "$OUT/pmc.log" | cut -c1-800; cat "$OUT/bench.json" | cut -c1-800
exit $rc
