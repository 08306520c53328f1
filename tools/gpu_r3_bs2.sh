#!/bin/bash
# Network tests, then A/B of the network forms: the tree's library (whole-group fold,
# group-major loads) vs the v_perm path, and the variant builds of tools/ect_variants.sh
# (pairs: fold input pairs as loads land; cmorder: input-major loads, stores after the math;
# pairsorder: both).
set -o pipefail
OUT=gpurun_out/${1:-r3bs2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"; grep -E "FAIL|Error" "$OUT/pytest_gpu.log" | head -5
[ $rc -eq 0 ] || exit $rc
SH="6,3,1024;12,5,512;10,4,512;8,3,512"
timeout -k 10 500 python -u tools/bitslice_ab.py --shapes "$SH" --reps 2 --ops encode,verify,encode_crc,pack_encode \
  --variants "perm:BLBRS_BITSLICE=0;net:BLBRS_BITSLICE=2;policy:BLBRS_BITSLICE=1" > "$OUT/ab_main.jsonl" 2> "$OUT/ab_main.err" || exit $?
cut -c1-1500 "$OUT/ab_main.jsonl"
for v in ${VARIANTS:-pairs cmorder pairsorder}; do
  BLBRS_LIB_PATH=tools/_build/variants/$v/libblbrs.so timeout -k 10 400 python -u tools/bitslice_ab.py --shapes "$SH" --reps 2 \
    --ops encode,verify,encode_crc --variants "perm:BLBRS_BITSLICE=0;net:BLBRS_BITSLICE=2" > "$OUT/ab_$v.jsonl" 2> "$OUT/ab_$v.err" || exit $?
  echo "== $v"; cut -c1-1200 "$OUT/ab_$v.jsonl"
done
