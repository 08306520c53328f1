#!/bin/bash
# Round-3 run 4: slicing width of the fused encode+CRC chains (8 / 16 / 32), RS(12,5), (6,3), (10,4).
set -o pipefail
OUT=gpurun_out/${1:-r3ab3}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=tools/_build/variants
for v in s8 s16 s32; do
  echo "== corr $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/corr_$v.log" 2>&1 || exit 1
done
for v in s8 s16 s32; do
  for km in "12 5 512" "6 3 1024" "10 4 512"; do set -- $km
    echo "== ab $v $1,$2" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 200 python -u tools/ect_ab.py --k $1 --m $2 --batch $3 --reps 3 --iters 3 > "$OUT/ab$1$2_$v.json" 2>&1 || exit 1
  done
done
echo "exit 0"; for f in "$OUT"/ab*.json; do echo "$f: $(tail -1 $f)"; done
