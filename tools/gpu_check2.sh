#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf --durations=8 > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== bench" && timeout -k 10 420 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== bench rs104" && timeout -k 10 300 python bench.py --k 10 --m 4 --batch 512 --no-extra --steps 10 > gpurun_out/bench_rs104.json 2>> gpurun_out/bench.err \
&& echo "== bench rs104 B4096 total" && timeout -k 10 300 python bench.py --k 10 --m 4 --total-batch 4096 --no-extra --steps 3 > gpurun_out/bench_rs104_total.json 2>> gpurun_out/bench.err
rc=$?
echo "exit $rc"; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench*.json
exit $rc
