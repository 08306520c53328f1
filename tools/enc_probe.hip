// enc_probe.hip -- launch-shape probe for the RS(6,3) encode's access pattern (bench layout:
// B = 1024 stripes of 9 x 8 MiB shards, data 0..5 read, parity 6..8 written), a trivial XOR
// in place of the GF multiply.  Varies chunks per lane (U), nontemporal loads / stores,
// workgroup size and the block -> tile map, to look for a streaming shape that beats the one
// rs_code_kernel uses (U = 4, nt loads + stores, 256 threads, XCD-contiguous tiles).
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/enc_probe.hip -o tools/_build/enc_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint64_t S = 8ull << 20;
constexpr int K = 6, M = 3;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    else return *reinterpret_cast<const u32x4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = v;
}

// MAP 0: XCD-contiguous (each XCD a contiguous eighth of the (stripe, tile) space, as the
// kernel); 1: dispatch order; 2: XCD-contiguous, tile-major inside the eighth (consecutive
// workgroups take the same column tile of consecutive stripes).
template <int U, bool NTL, bool NTS, int TPB, int MAP>
__global__ __launch_bounds__(TPB) void enc_kernel(uint8_t* base, uint32_t B) {
    constexpr uint32_t kStep = TPB * 16u;
    constexpr uint32_t tps = S / (kStep * U);
    const uint32_t total = B * tps;
    uint32_t t = blockIdx.x;
    if constexpr (MAP != 1) t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
    if (t >= total) return;
    uint32_t b, tile;
    if constexpr (MAP == 2) {
        const uint32_t per = total / 8u, x = t / per, r = t % per, sb = per / tps;  // stripes per XCD
        b = x * sb + r % sb;
        tile = r / sb;
    } else {
        b = t / tps;
        tile = t % tps;
    }
    const uint64_t off = static_cast<uint64_t>(tile) * kStep * U + threadIdx.x * 16u;
    uint8_t* sp = base + static_cast<uint64_t>(b) * (K + M) * S;
    u32x4 x[K][U];
#pragma unroll
    for (int c = 0; c < K; ++c)
#pragma unroll
        for (int u = 0; u < U; ++u) x[c][u] = ld<NTL>(sp + c * S + off + u * kStep);
#pragma unroll
    for (int r = 0; r < M; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            u32x4 a = x[0][u];
#pragma unroll
            for (int c = 1; c < K; ++c) a ^= (c + r) & 1 ? x[c][u] : (x[c][u] << 1);
            st<NTS>(sp + (K + r) * S + off + u * kStep, a);
        }
}

static uint8_t* g_base;
constexpr uint32_t kB = 1024;

template <int U, bool NTL, bool NTS, int TPB, int MAP>
void run(const char* name) {
    constexpr uint32_t tps = S / (TPB * 16u * U);
    const uint32_t grid = (kB * tps + 7) & ~7u;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&] { hipLaunchKernelGGL((enc_kernel<U, NTL, NTS, TPB, MAP>), dim3(grid), dim3(TPB), 0, 0, g_base, kB); };
    launch();
    CK(hipDeviceSynchronize());
    constexpr int reps = 6;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-28s U=%d ntl=%d nts=%d tpb=%4d map=%d : %8.3f ms %8.1f GB/s\n", name, U, int(NTL), int(NTS), TPB, MAP, ms,
           double(kB) * (K + M) * S / ms / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    CK(hipMalloc(&g_base, size_t(kB) * (K + M) * S));
    CK(hipMemset(g_base, 0x3C, size_t(kB) * (K + M) * S));
    for (int rep = 0; rep < 2; ++rep) {
        printf("# rep %d\n", rep);
        run<4, true, true, 256, 0>("kernel shape");
        run<4, false, true, 256, 0>("cached loads");
        run<4, true, false, 256, 0>("cached stores");
        run<4, false, false, 256, 0>("cached both");
        run<2, true, true, 256, 0>("U2");
        run<8, true, true, 256, 0>("U8");
        run<2, true, true, 512, 0>("512 thr U2");
        run<4, true, true, 512, 0>("512 thr U4");
        run<8, true, true, 128, 0>("128 thr U8");
        run<4, true, true, 256, 1>("dispatch order");
        run<4, true, true, 256, 2>("tile-major per XCD");
        run<4, false, true, 256, 2>("tile-major, cached loads");
    }
    return 0;
}
