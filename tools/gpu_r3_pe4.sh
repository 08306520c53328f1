#!/bin/bash
# The network PackTracts + Encode on 16 KiB tiles (BLBRS_PE_CM_U=4) vs 8 KiB: parity tests
# under the knob, then interleaved A/B at RS(6,3) B=1024, RS(8,3) and RS(12,5) B=512.
set -o pipefail
OUT=gpurun_out/${1:-r3pe4}
mkdir -p "$OUT"
export TMPDIR=/tmp
BLBRS_PE_CM_U=4 timeout -k 10 300 python -u -m pytest tests/test_pack.py tests/test_bitslice.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_u4.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_u4.log"; [ $rc -eq 0 ] || exit $rc
for shape in "6 3 1024" "8 3 512" "12 5 512"; do
  set -- $shape
  timeout -k 10 300 python -u tools/pe_ab.py --k $1 --m $2 --batch $3 --reps 3 --variants "u2:;u4:BLBRS_PE_CM_U=4" > "$OUT/pe_$1_$2.json" 2> "$OUT/pe_$1_$2.err" || exit $?
  cut -c1-700 "$OUT/pe_$1_$2.json"
done
