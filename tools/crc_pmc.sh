#!/bin/bash
# CRC-32C load-path A/B with counters: FETCH_SIZE and a kernel trace of tools/crc_pmc.py
# under the shipped library and the variants named (built by tools/crc_variants.sh).
# usage: tools/crc_pmc.sh OUTDIR [variant ...]
set -o pipefail
out=${1:?out}; shift
mkdir -p $out
export TMPDIR=/tmp
for v in shipped "$@"; do
  if [ $v = shipped ]; then lib=$PWD/blb_amd/libblbrs.so; else lib=$PWD/tools/_build/variants/$v/libblbrs.so; fi
  export BLBRS_LIB_PATH=$lib
  mkdir -p $out/$v
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/$v/fetch -o fetch -- python3 tools/crc_pmc.py > $out/$v/fetch.log 2>&1 \
  && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/$v/trace -o trace -- python3 tools/crc_pmc.py > $out/$v/trace.log 2>&1 \
  || exit 1
done
unset BLBRS_LIB_PATH
python3 tools/crc_pmc_summary.py $out shipped "$@"
