#!/bin/bash
# Round-3 run 2: validation suite (rpc pool fix) + fused encode+CRC tile-kernel A/B variants.
set -o pipefail
OUT=gpurun_out/${1:-r3ab1}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=tools/_build/variants
echo "== pytest -m gpu" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
&& for v in base maskacc persist3 persist3m; do
  echo "== correctness $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/corr_$v.log" 2>&1 || exit 1
done \
&& for v in base maskacc persist3 persist3m; do
  echo "== ab125 $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 200 python -u tools/ect_ab.py --k 12 --m 5 --batch 512 --reps 2 --iters 3 > "$OUT/ab125_$v.json" 2>&1 || exit 1
  echo "== ab63 $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 200 python -u tools/ect_ab.py --k 6 --m 3 --batch 1024 --reps 2 --iters 3 > "$OUT/ab63_$v.json" 2>&1 || exit 1
done \
&& echo "== client shape (current)" && timeout -k 10 300 python -u tools/host_paths.py --client-only > "$OUT/client_shape_after.json" 2> "$OUT/client_after.err" \
&& echo "== client shape (r2 lib)" && BLBRS_LIB_PATH=$PWD/tools/_build/libblbrs_r2.so timeout -k 10 300 python -u tools/host_paths.py --client-only > "$OUT/client_shape_before.json" 2> "$OUT/client_before.err"
rc=$?
echo "exit $rc"; tail -3 "$OUT/pytest_gpu.log"; for f in "$OUT"/ab*.json "$OUT"/client_shape_*.json; do echo "$f"; cat "$f"; done
exit $rc
