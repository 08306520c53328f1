#!/bin/bash
# Round-3 run 3: tile-kernel cost split + nibble-address variant (RS(12,5) B=512), and the
# zero-copy vs DMA-staging sweep of host calls (tools/host_paths.py --zc-sweep).
set -o pipefail
OUT=gpurun_out/${1:-r3ab2}
mkdir -p "$OUT"
export TMPDIR=/tmp
V=tools/_build/variants
for v in ship nib2 f1 f2 f4 f7; do
  echo "== ab125 $v" && BLBRS_LIB_PATH=$PWD/$V/$v/libblbrs.so timeout -k 10 200 python -u tools/ect_ab.py --k 12 --m 5 --batch 512 --reps 3 --iters 3 > "$OUT/ab125_$v.json" 2>&1 || exit 1
done
echo "== nib2 correctness" && BLBRS_LIB_PATH=$PWD/$V/nib2/libblbrs.so timeout -k 10 300 python -u -m pytest tests/test_encode_crc.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/corr_nib2.log" 2>&1 \
&& echo "== zc sweep" && timeout -k 10 600 python -u tools/host_paths.py --zc-sweep > "$OUT/zc_sweep.json" 2> "$OUT/zc_sweep.err"
rc=$?
echo "exit $rc"; for f in "$OUT"/ab*.json; do echo "$f: $(tail -1 $f)"; done; tail -2 "$OUT/corr_nib2.log"
exit $rc
