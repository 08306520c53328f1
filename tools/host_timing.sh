#!/bin/bash
# Builds a measurement variant of libblbrs.so whose host path records per-stage times of
# one-stripe host calls (blbrs.hip HT() marks, -DBLBRS_HOST_TIMING) into tools/_build/host_timing/,
# reusing the library build's other objects.  Run a program against it with
#   LD_LIBRARY_PATH=tools/_build/host_timing tests/cpp/_build/latency_bench 4096
# and read the per-stage medians from its stderr at exit.
set -e
cd "$(dirname "$0")/.."
make -s -C blb_amd libblbrs.so
out=tools/_build/host_timing
mkdir -p $out
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -DBLBRS_HOST_TIMING \
  -c blb_amd/csrc/blbrs.hip -o $out/blbrs_timing.o
objs=$(ls blb_amd/_build/*.o | grep -v '/blbrs.o$')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/libblbrs.so $objs $out/blbrs_timing.o -ldl
echo "built $out/libblbrs.so"
