#!/bin/bash
# A/B of tuning builds (tools/ect_variants.sh): tools/run_var.sh OUTDIR "ect_ab args" v1 v2 ...
out=$1; args=$2; shift 2
mkdir -p $out
for v in "$@"; do
  BLBRS_LIB_PATH=$PWD/tools/_build/variants/$v/libblbrs.so timeout -k 10 120 python tools/ect_ab.py $args > $out/$v.json || exit 1
  echo "$v $(cat $out/$v.json)"
done
