#!/bin/bash
# Builds tuning variants of libblbrs.so for A/B runs (tools/ect_ab.py under BLBRS_LIB_PATH):
#   tools/ect_variants.sh name1:"-DFOO=1 -DBAR=2" name2:"..."
# -> tools/_build/variants/<name>/libblbrs.so.  Only the files that read the macros
# (encode_crc_tile.hip) are rebuilt; the rest come from blb_amd/_build.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C $ROOT/blb_amd
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=$ROOT/tools/_build/variants/$name
  mkdir -p $out/obj
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c $ROOT/blb_amd/csrc/encode_crc_tile.hip -o $out/obj/encode_crc_tile.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  out=$ROOT/tools/_build/variants/$name
  objs=$(ls $ROOT/blb_amd/_build/*.o | grep -v encode_crc_tile.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libblbrs.so $objs $out/obj/encode_crc_tile.o
  rm -rf $out/obj
done
