#!/bin/bash
# Occupancy sweep of the compiled-network launches (dynamic-LDS caps) against the v_perm path.
set -o pipefail
OUT=gpurun_out/${1:-r3occ}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bitslice_ab.py --shapes "${SHAPES:-6,3,1024;8,3,512}" --reps 3 \
  --variants "perm:BLBRS_BITSLICE=0;net:BLBRS_BITSLICE=1;n2:BLBRS_OCC_LDS=65536+BLBRS_OCC_LDS_ECT=40000;n3:BLBRS_OCC_LDS=54000+BLBRS_OCC_LDS_ECT=37000;n4:BLBRS_OCC_LDS=40000+BLBRS_OCC_LDS_ECT=23000" \
  > "$OUT/ab.jsonl" 2> "$OUT/ab.err"
rc=$?
cut -c1-2000 "$OUT/ab.jsonl"; tail -3 "$OUT/ab.err"
exit $rc
