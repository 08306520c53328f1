#!/bin/bash
# Builds tuning variants of libblbrs.so for A/B runs (tools/ect_ab.py under BLBRS_LIB_PATH):
#   [SRCS="encode_crc_tile pack_encode"] tools/ect_variants.sh name1:"-DFOO=1" name2:"..."
# -> tools/_build/variants/<name>/libblbrs.so.  Only the files in $SRCS (default
# encode_crc_tile) are rebuilt with the flags; the rest come from blb_amd/_build.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRCS=${SRCS:-encode_crc_tile}
make -s -C $ROOT/blb_amd
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=$ROOT/tools/_build/variants/$name
  mkdir -p $out/obj
  for src in $SRCS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c $ROOT/blb_amd/csrc/$src.hip -o $out/obj/$src.o &
  done
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  out=$ROOT/tools/_build/variants/$name
  objs=""
  for o in $ROOT/blb_amd/_build/*.o; do
    b=$(basename $o .o)
    if [ -f $out/obj/$b.o ]; then objs="$objs $out/obj/$b.o"; else objs="$objs $o"; fi
  done
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libblbrs.so $objs -ldl
  rm -rf $out/obj
done
