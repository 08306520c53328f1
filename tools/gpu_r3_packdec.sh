#!/bin/bash
# PackTracts kernel variants (tests + A/B), the decode mix ceiling and the single-erasure
# ReconstructData U A/B.
set -o pipefail
OUT=gpurun_out/${1:-r3packdec}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pack.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/pack_ab.py --reps 3 > "$OUT/pack_ab.json" 2> "$OUT/pack_ab.err" || exit $?
cut -c1-1500 "$OUT/pack_ab.json"
timeout -k 10 120 tools/_build/mix_probe dec > "$OUT/mix_dec.txt" 2>&1 || exit $?
cat "$OUT/mix_dec.txt"
timeout -k 10 300 python -u tools/dec_ab.py --variants "base:;u2:BLBRS_DEC_U=2;u4c:BLBRS_DEC_U=12;u2c:BLBRS_DEC_U=22" > "$OUT/dec_ab.json" 2> "$OUT/dec_ab.err" || exit $?
cat "$OUT/dec_ab.json"
