#!/bin/bash
# One GPU-box session: smoke -> gpu parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== smoke" && timeout -k 10 420 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
&& echo "== pytest -m gpu" && timeout -k 10 1200 python -m pytest tests -m gpu -x -q -rA --durations=15 > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== rocprof" && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o encode -- python bench.py --steps 10 --warmup 2 --no-extra > gpurun_out/prof.log 2>&1
rc=$?
echo "exit $rc"
tail -3 gpurun_out/smoke.log gpurun_out/pytest_gpu.log 2>/dev/null
cat gpurun_out/bench.json 2>/dev/null
exit $rc
