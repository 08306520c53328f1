#!/bin/bash
# AddressSanitizer build of the host runtime and the C++ mirror's tests (host code only: the
# device code is not instrumented).  Run here, on the CPU; the GPU box only runs the result:
#   bash tools/asan_build.sh && gpurun -- 'bash tools/gpu_asan.sh r4asan 3'
# Unlike tests/cpp's rs_test_asan (test code only), the library's host code is instrumented too.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/tools/_build/asan
mkdir -p "$OUT"
pids=()
make -C "$ROOT/blb_amd" _build/rtc_headers.inc >/dev/null   # the device headers rtc.hip embeds
for f in tuning runtime rtc rs_kernels crc32c encode_crc encode_crc_tile pack pack_encode blbrs; do
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer \
    -I"$ROOT/blb_amd/_build" -c "$ROOT/blb_amd/csrc/$f.hip" -o "$OUT/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -fno-gpu-sanitize -fsanitize=address -fno-omit-frame-pointer \
  -o "$OUT/libblbrs.so" "$OUT"/*.o -lhiprtc
rm -f "$OUT"/*.o
/opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -pthread -fsanitize=address -fno-omit-frame-pointer -o "$OUT/rs_test_asan" \
  "$ROOT/tests/cpp/rs_test.cpp" "$ROOT"/blb_amd/host/{reedsolomon,tractserver,client}.cpp \
  -L"$OUT" -lblbrs -Wl,-rpath,'$ORIGIN' -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
ls -la "$OUT"
