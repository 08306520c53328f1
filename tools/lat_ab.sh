#!/bin/bash
# Same-box A/B of the single-caller latency (tests/cpp/latency_bench) between the in-tree
# library and one variant directory holding another libblbrs.so (loaded via LD_LIBRARY_PATH,
# which overrides the binary's RUNPATH).  Alternates the two, REPS rounds, per piece size.
# usage: tools/lat_ab.sh OUT VARIANT_DIR [REPS]   -> OUT/lat_ab.jsonl (each row tagged)
set -o pipefail
OUT=${1:?out}; VAR=${2:?variant dir}; REPS=${3:-2}
mkdir -p "$OUT"
for r in $(seq 1 "$REPS"); do
  for L in ${LAT_SIZES:-65536 1048576 8388608}; do
    for v in tree variant; do
      if [ $v = variant ]; then lp="$VAR"; else lp=""; fi
      LD_LIBRARY_PATH="$lp" timeout -k 10 120 tests/cpp/_build/latency_bench $L > "$OUT/one.jsonl" 2>> "$OUT/lat_ab.err" || exit $?
      grep steady_state "$OUT/one.jsonl" | grep '"gpu"' | sed "s/^{/{\"lib\": \"$v\", \"rep\": $r, /" >> "$OUT/lat_ab.jsonl"
    done
  done
done
cat "$OUT/lat_ab.jsonl" | cut -c1-160
