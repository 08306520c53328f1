#!/bin/bash
# CRC stream kernel: byte-table matrix applies (tree library) vs column applies (crcold build),
# alternating processes; CRC GPU tests first.
set -o pipefail
OUT=gpurun_out/${1:-r3crc5}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_crc32c.py tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in tab old; do
    if [ $v = old ]; then L=tools/_build/variants/crcold/libblbrs.so; else L=blb_amd/libblbrs.so; fi
    BLBRS_LIB_PATH=$L timeout -k 10 120 python -u tools/crc_bench.py > "$OUT/crc_${v}_$rep.txt" 2>&1 || exit $?
    echo "$v $rep: $(tr '\n' ' ' < $OUT/crc_${v}_$rep.txt)"
  done
done
