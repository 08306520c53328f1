mkdir -p gpurun_out/r5r
timeout -k 10 240 python3 tools/pack_encode_time.py --reps 4 --bitslice 1,0 > gpurun_out/r5r/shipped.log 2>&1 || exit 1
for v in pe_n4 pe_n1 pe_w2; do
  BLBRS_LIB_PATH=$PWD/tools/_build/variants/$v/libblbrs.so timeout -k 10 240 python3 tools/pack_encode_time.py --reps 4 --bitslice 1,0 > gpurun_out/r5r/$v.log 2>&1 || exit 1
done
grep -h '^{' gpurun_out/r5r/*.log
