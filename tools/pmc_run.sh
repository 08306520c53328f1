#!/bin/bash
# HBM traffic of the production RS(6,3) encode kernel from PMC counters, calibrated.
# FETCH_SIZE and WRITE_SIZE need separate passes on gfx950 (TCC slots: 3 + 2 > 4).
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o fetch -- tools/_build/tune pmc > gpurun_out/pmc/fetch.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o write -- tools/_build/tune pmc > gpurun_out/pmc/write.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d gpurun_out/pmc/req -o req -- tools/_build/tune pmc > gpurun_out/pmc/req.log 2>&1
rc=$?
find gpurun_out/pmc -name "*.csv" | head -20
exit $rc
