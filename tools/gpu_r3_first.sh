set -o pipefail
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
echo "== cold bench" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/r3/cold -o cold -- python3 tools/cold_bench.py > gpurun_out/r3/cold.json 2> gpurun_out/r3/cold.err \
&& echo "== sq125" && bash tools/ect_pmc.sh gpurun_out/r3/sq125 "--k 12 --m 5 --batch 512" \
&& echo "== sq83" && bash tools/ect_pmc.sh gpurun_out/r3/sq83 "--k 8 --m 3 --batch 512"
rc=$?; echo "exit $rc"; cat gpurun_out/r3/cold.json; exit $rc
