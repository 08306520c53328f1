#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_gpu.log 2>&1 \
&& echo "== tune" && timeout -k 10 400 tools/_build/tune > gpurun_out/tune5.txt 2>&1 \
&& echo "== bench" && timeout -k 10 420 python bench.py --no-extra > gpurun_out/bench.json 2> gpurun_out/bench.err \
&& echo "== bench rs104" && timeout -k 10 300 python bench.py --k 10 --m 4 --batch 512 --no-extra --steps 10 > gpurun_out/bench_rs104.json 2>> gpurun_out/bench.err
rc=$?
echo "exit $rc"; tail -2 gpurun_out/pytest_gpu.log; grep "rep 0" -A 17 gpurun_out/tune5.txt; cat gpurun_out/bench*.json | cut -c1-420
exit $rc
