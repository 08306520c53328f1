#!/bin/bash
# PackTracts variants on bench.py's overlapping 4 GiB source pool and on distinct sources.
set -o pipefail
OUT=gpurun_out/${1:-r3pack4}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pack_ab.py --reps 3 --variants 0,6,9,10,8 > "$OUT/pool.json" 2> "$OUT/pool.err" || exit $?
cut -c1-1500 "$OUT/pool.json"
timeout -k 10 400 python -u tools/pack_ab.py --reps 3 --variants 0,6,9,10,8 --distinct > "$OUT/distinct.json" 2> "$OUT/distinct.err" || exit $?
cut -c1-1500 "$OUT/distinct.json"
timeout -k 10 400 python -u tools/pe_ab.py --reps 3 --variants "nt:;cached:BLBRS_PE_LDNT=0" > "$OUT/pe63.json" 2> "$OUT/pe63.err" || exit $?
cut -c1-1500 "$OUT/pe63.json"
timeout -k 10 400 python -u tools/pe_ab.py --k 12 --m 5 --batch 512 --reps 3 --variants "nt:;cached:BLBRS_PE_LDNT=0" > "$OUT/pe125.json" 2> "$OUT/pe125.err" || exit $?
cut -c1-1500 "$OUT/pe125.json"
