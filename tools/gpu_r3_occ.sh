#!/bin/bash
# GPU suite, then an occupancy sweep of the compiled-network launches (dynamic-LDS caps)
# against the v_perm path, with PackTracts + Encode (tools/bitslice_ab.py).
set -o pipefail
OUT=gpurun_out/${1:-r3occ}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"; grep -E "FAIL|Error" "$OUT/pytest_gpu.log" | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u tools/bitslice_ab.py --shapes "${SHAPES:-6,3,1024;12,5,512}" --reps 2 --ops encode,verify,encode_crc,pack_encode \
  --variants "perm:BLBRS_BITSLICE=0;net:BLBRS_BITSLICE=2;n2:BLBRS_OCC_LDS=65536+BLBRS_OCC_LDS_ECT=40000;n3:BLBRS_OCC_LDS=54000+BLBRS_OCC_LDS_ECT=37000;n4:BLBRS_OCC_LDS=40000+BLBRS_OCC_LDS_ECT=23000;pe1:BLBRS_PE_CM_WIDE=0" \
  > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?
cut -c1-2500 "$OUT/ab.jsonl"; tail -3 "$OUT/ab.err"
exit $rc
