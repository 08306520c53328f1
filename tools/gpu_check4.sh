#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== stride" && timeout -k 10 300 tools/_build/tune stride > gpurun_out/stride.txt 2>&1 \
&& echo "== rocprof" && timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o encode -- python bench.py --steps 10 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?
echo "exit $rc"; tail -2 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json; cat gpurun_out/stride.txt
exit $rc
