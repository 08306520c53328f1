set -o pipefail
OUT=gpurun_out/r4h; mkdir -p $OUT; export TMPDIR=/tmp
for v in shipped cfree nochain; do
  if [ $v = shipped ]; then LIB=$PWD/blb_amd/libblbrs.so; else LIB=$PWD/tools/_build/variants/$v/libblbrs.so; fi
  for shape in "--k 6 --m 3 --batch 1024" "--k 12 --m 5 --batch 512"; do
    tag=$v_$(echo $shape | tr -d ' -')
    BLBRS_LIB_PATH=$LIB timeout -k 10 200 python -u tools/ect_ab.py $shape --reps 3 > $OUT/ab_${v}_$(echo $shape | cut -d' ' -f2,4 | tr ' ' _).json 2>>$OUT/err.txt || exit 1
  done
  BLBRS_LIB_PATH=$LIB timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $PWD/$OUT/pmc_$v -o pmc -- python3 tools/ect_ab.py --k 12 --m 5 --batch 512 --reps 1 --iters 1 > $OUT/pmc_$v.log 2>&1 || exit 1
done
for f in $OUT/ab_*.json; do echo "$f $(cat $f)"; done
