#!/bin/bash
# PMC passes over tools/pmc_prod.py (one counter group per rocprofv3 run, as gfx950 requires:
# FETCH_SIZE and WRITE_SIZE never share a pass).  Then summarise into profiles/.
# usage: tools/pmc_prod.sh OUTDIR TAG COMMIT
set -o pipefail
out=${1:-gpurun_out/pmc_prod}; tag=${2:-r02}; commit=${3:-unknown}
mkdir -p $out
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $out/$name -o $name -- python3 tools/pmc_prod.py > $out/$name.log 2>&1
}
run fetch FETCH_SIZE \
&& run write WRITE_SIZE \
&& run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
&& run sq2 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 tools/pmc_prod.py > $out/trace.log 2>&1 \
&& python3 tools/pmc_prod_summary.py $out $tag $commit
