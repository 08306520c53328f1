#!/bin/bash
# SQ counter passes over tools/ect_pmc.py: tools/ect_pmc.sh OUTDIR "ect_pmc args" [LIB]
set -o pipefail
out=$1; args=$2
[ -n "$3" ] && export BLBRS_LIB_PATH=$3
mkdir -p $out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o $name -- python3 tools/ect_pmc.py $args > $out/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
&& run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM \
&& timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 tools/ect_pmc.py $args > $out/trace.log 2>&1 \
&& python3 tools/ect_pmc_summary.py $out
