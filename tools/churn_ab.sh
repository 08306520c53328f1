# Interleaved A/B of the rpc pool churn extra: shipped library vs tools/_build/variants/$1.
mkdir -p gpurun_out/churn
for rep in 1 2; do
  timeout -k 10 120 python3 tools/churn_ab.py >> gpurun_out/churn/ab.jsonl 2>> gpurun_out/churn/err.txt || exit 1
  BLBRS_LIB_PATH=$PWD/tools/_build/variants/$1/libblbrs.so timeout -k 10 120 python3 tools/churn_ab.py >> gpurun_out/churn/ab.jsonl 2>> gpurun_out/churn/err.txt || exit 1
done
