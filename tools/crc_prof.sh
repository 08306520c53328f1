#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/crcprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/crcprof/kt -o kt -- python tools/crc_bench.py > gpurun_out/crcprof/kt.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/crcprof/pmc -o pmc -- python tools/crc_bench.py > gpurun_out/crcprof/pmc.log 2>&1
rc=$?
cut -c1-140 gpurun_out/crcprof/kt/kt_kernel_stats.csv | head -5
python3 - <<'PY'
import csv,collections
rows=list(csv.DictReader(open('gpurun_out/crcprof/pmc/pmc_counter_collection.csv')))
agg=collections.defaultdict(float)
for r in rows:
    if 'crc' in r['Kernel_Name']: agg[(r['Kernel_Name'][:40],r['Counter_Name'])]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print(k, v)
PY
exit $rc
