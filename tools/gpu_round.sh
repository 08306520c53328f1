#!/bin/bash
# The one GPU driver: runs the named steps on one MI355X, each under its own time limit, chained
# so that the first failure ends the call (no GPU step runs after a failed, killed or faulted one).
#
# usage: tools/gpu_round.sh OUT STEPS [TAG] [COMMIT]
#   OUT    directory under gpurun_out/
#   STEPS  comma list, run in order:
#            tests        python -m pytest tests -m gpu (whole GPU suite)
#            tests:PATHS  the GPU tests of PATHS only ("tests/test_rtc.py tests/test_pack.py")
#            smoke        __graft_entry__.smoke()
#            pmc          tools/pmc_prod.sh: FETCH_SIZE / WRITE_SIZE / SQ passes + kernel trace of the
#                         shipped library -> profiles-ready summary (TAG, COMMIT)
#            bench        python bench.py (default flags) -> bench.json
#            rocprof      rocprofv3 --kernel-trace --stats of bench.py --steps 10 --no-extra
#            ab:CMD       an A/B or measurement driver, e.g. "ab:tools/rpc_shapes.py --reps 5"
#            probe:ARGS   tools/_build/mix_probe ARGS
#            latency      tests/cpp/_build/latency_bench at 4 KiB .. 8 MiB -> latency.jsonl
#            crcab        tools/crc_pmc.sh: CRC load-path A/B with FETCH_SIZE (variants from crc_variants.sh)
# e.g. gpurun -- 'bash tools/gpu_round.sh r4val tests,smoke,bench,rocprof'
set -o pipefail
OUT=gpurun_out/${1:?out}
STEPS=${2:?steps}
TAG=${3:-r04}
COMMIT=${4:-unknown}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
IFS=',' read -ra LIST <<< "$STEPS"
n=0
for step in "${LIST[@]}"; do
  n=$((n + 1))
  echo "== $step"
  case "$step" in
    tests)
      AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest_gpu.log" ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest ${step#tests:} -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu_$n.log" 2>&1
      rc=$?; tail -3 "$OUT/pytest_gpu_$n.log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; cat "$OUT/smoke.log" ;;
    pmc)
      bash tools/pmc_prod.sh "$OUT/pmc" "$TAG" "$COMMIT" > "$OUT/pmc.log" 2>&1
      rc=$?; tail -2 "$OUT/pmc.log" | cut -c1-800 ;;
    bench)
      timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; cut -c1-1500 "$OUT/bench.json" ;;
    rocprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o bench -- \
        python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-extra > "$OUT/prof.log" 2>&1
      rc=$?; tail -2 "$OUT/prof.log" ;;
    ab:*)
      timeout -k 10 900 python -u ${step#ab:} > "$OUT/ab_$n.jsonl" 2> "$OUT/ab_$n.err"
      rc=$?; cut -c1-3000 "$OUT/ab_$n.jsonl"; tail -3 "$OUT/ab_$n.err" ;;
    latency)
      for L in 4096 65536 262144 1048576 2097152 4194304 8388608; do
        timeout -k 10 300 tests/cpp/_build/latency_bench $L >> "$OUT/latency.jsonl" 2>> "$OUT/latency.err" || { rc=$?; break; }
        rc=0
      done
      cat "$OUT/latency.jsonl" | cut -c1-400 ;;
    crcab)
      bash tools/crc_pmc.sh "$OUT/crc" crc_coal1 crc_coal0 > "$OUT/crc.log" 2>&1
      rc=$?; tail -2 "$OUT/crc.log" | cut -c1-1500 ;;
    probe:*)
      timeout -k 10 300 tools/_build/mix_probe ${step#probe:} > "$OUT/probe_$n.txt" 2>&1
      rc=$?; cat "$OUT/probe_$n.txt" ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $step failed: exit $rc"
    exit $rc
  fi
done
echo "all steps ok"
