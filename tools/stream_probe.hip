// stream_probe.hip -- the access-pattern ceiling of a coding launch, in the bench's own layout.
//
// A trivial-XOR stream that reads R shards and writes W shards of every stripe of a strided
// [B][n][S] batch (shards [0, R) in, [R, R + W) out), with rs_code_kernel's launch shape: 256
// threads, one tile of U 4 KiB chunks per block, every XCD streaming a contiguous eighth of the
// tiles, nontemporal loads and stores.  Same bytes and same order as the coding kernel with no
// GF arithmetic: what the kernel would take if its math were free.  bench.py prints it next to
// each recovery row (measurement only; the library never loads this).
//
// Build: make -C tools _build/libstream_probe.so
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));
constexpr uint32_t kStep = 256 * 16;

template <int R, int W, int U>
__global__ __launch_bounds__(256) void stream_kernel(uint8_t* base, uint64_t shard_stride, uint64_t stripe_stride,
                                                     uint32_t B, uint32_t tps) {
    const uint32_t total = B * tps;
    // as rs_code_kernel: one tile per block, the tiles past grid (< 8) by the first blocks again
    for (uint32_t t = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u; t < total; t += gridDim.x) {
    const uint32_t b = t / tps;
    uint8_t* stripe = base + static_cast<uint64_t>(b) * stripe_stride +
                      static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
    u32x4 x[R][U];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[r][u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(stripe + r * shard_stride + u * kStep));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 acc = x[0][u];
#pragma unroll
        for (int r = 1; r < R; ++r) acc ^= x[r][u];
#pragma unroll
        for (int w = 0; w < W; ++w)
            __builtin_nontemporal_store(acc + u32x4{static_cast<uint32_t>(w), 0u, 0u, 0u},
                                        reinterpret_cast<u32x4*>(stripe + (R + w) * shard_stride + u * kStep));
    }
    }
}

using Fn = void (*)(uint8_t*, uint64_t, uint64_t, uint32_t, uint32_t);

template <int R, int W>
Fn pick_u(int u) {
    switch (u) {
        case 1: return stream_kernel<R, W, 1>;
        case 2: return stream_kernel<R, W, 2>;
        case 4: return stream_kernel<R, W, 4>;
        default: return nullptr;
    }
}
template <int R>
Fn pick_w(int w, int u) {
    switch (w) {
        case 1: return pick_u<R, 1>(u);
        case 2: return pick_u<R, 2>(u);
        case 3: return pick_u<R, 3>(u);
        case 4: return pick_u<R, 4>(u);
        case 5: return pick_u<R, 5>(u);
        default: return nullptr;
    }
}
Fn pick(int r, int w, int u) {
    switch (r) {
        case 6: return pick_w<6>(w, u);
        case 8: return pick_w<8>(w, u);
        case 10: return pick_w<10>(w, u);
        case 12: return pick_w<12>(w, u);
        default: return nullptr;
    }
}

}  // namespace

// Launches one pass on `stream`.  0 = launched, -1 = unsupported shape (R in {6,8,10,12},
// W 1..5, U in {1,2,4}, S a multiple of the tile, 16-byte aligned strides), else the HIP error.
extern "C" int stream_probe(int R, int W, int U, void* base, size_t shard_stride, size_t stripe_stride, size_t B,
                            size_t S, void* stream) {
    const Fn fn = pick(R, W, U);
    const uint64_t tile = static_cast<uint64_t>(kStep) * U;
    if (!fn || !base || B == 0 || S % tile || shard_stride % 16 || stripe_stride % 16) return -1;
    const uint64_t tps = S / tile, total = B * tps;
    if (total > 0x7FFFFFFFull || total < 8) return -1;
    hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(total & ~uint64_t{7})), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<uint8_t*>(base), shard_stride, stripe_stride,
                       static_cast<uint32_t>(B), static_cast<uint32_t>(tps));
    return static_cast<int>(hipGetLastError());
}
