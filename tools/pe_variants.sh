#!/bin/bash
# A/B of pack+encode builds: tools/pe_variants.sh OUTDIR "pe_ab args" v1 v2 ... (default lib: "cur")
out=$1; args=$2; shift 2
mkdir -p $out
for v in "$@"; do
  if [ "$v" = cur ]; then lib=$PWD/blb_amd/libblbrs.so; else lib=$PWD/tools/_build/variants/$v/libblbrs.so; fi
  BLBRS_LIB_PATH=$lib timeout -k 10 150 python tools/pe_ab.py $args > $out/$v.json 2> $out/$v.err || exit 1
  echo "$v $(cat $out/$v.json)"
done
