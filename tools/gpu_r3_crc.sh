#!/bin/bash
# CRC-32C stream kernel A/B: register ring depth and two chains per wave.
set -o pipefail
OUT=gpurun_out/${1:-r3crc}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=tools/_build/variants
for v in con con4 con2 coni; do
  echo "== corr $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 300 python -u -m pytest tests/test_crc32c.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/corr_$v.log" 2>&1 || exit 1
done
for rep in 1 2; do for v in con con4 con2 coni; do
  echo "== bench $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 120 python -u tools/crc_bench.py > "$OUT/bench_${v}_$rep.txt" 2>&1 || exit 1
done; done
echo "exit 0"; for f in "$OUT"/bench_*.txt; do echo "$f: $(cat $f | tr '\n' ' ')"; done
