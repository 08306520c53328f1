// mix_probe.hip -- access-pattern ceilings of the PackTracts and PackTracts+Encode mixes.
//
// The fused pack+encode (pack_encode.hip) reads the tract bytes of k pieces and writes k
// pieces plus m parity; in the bench's layout that is 4.27 shard-equivalents read and 9
// written per RS(6,3) stripe, the pack alone 4.27 read / 6 written.  This probe times a
// trivial-XOR stream with R reads and W writes per stripe (8 MiB shards, one tile of U 4 KiB
// chunks per block, XCD-contiguous, nontemporal), with aligned or misaligned (+5 bytes,
// two loads + v_alignbyte per 16 B, as the pack does) sources, to give each mix its ceiling.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/mix_probe.hip -o tools/_build/mix_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

constexpr uint64_t S = 8ull << 20;
constexpr uint32_t kStep = 256 * 16;

// Stripe b: R source shards at src + (b*R + r)*S (+mis bytes), W destination shards at
// dst + (b*W + w)*S.  Sources and destinations live in separate regions, as tracts and
// pieces do.
template <int R, int W, int U, bool MIS>
__global__ __launch_bounds__(256) void mix_kernel(const uint8_t* src, uint8_t* dst, uint32_t B) {
    const uint32_t tps = S / (kStep * U);
    const uint32_t total = B * tps;
    const uint32_t t = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
    if (t >= total) return;
    const uint32_t b = t / tps;
    const uint64_t off = static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
    u32x4 x[R > 0 ? R : 1][U], y[R > 0 ? R : 1][U];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint8_t* s = src + (static_cast<uint64_t>(b) * R + r) * S + off;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[r][u] = ld(s + u * kStep);
            if (MIS) y[r][u] = ld(s + u * kStep + 16);
        }
    }
    u32x4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        acc[u] = u32x4{b, t, 0u, 0u};
#pragma unroll
        for (int r = 0; r < R; ++r) {
            u32x4 v = x[r][u];
            if (MIS) {
                v.x = __builtin_amdgcn_alignbyte(x[r][u].y, x[r][u].x, 1);
                v.y = __builtin_amdgcn_alignbyte(x[r][u].z, x[r][u].y, 1);
                v.z = __builtin_amdgcn_alignbyte(x[r][u].w, x[r][u].z, 1);
                v.w = __builtin_amdgcn_alignbyte(y[r][u].x, x[r][u].w, 1);
            }
            acc[u] ^= v;
        }
    }
    if constexpr (W == 0) {  // pure read: a store no lane takes keeps the loads alive
        u32x4 f = acc[0];
#pragma unroll
        for (int u = 1; u < U; ++u) f ^= acc[u];
        if (f.x == 0x9E3779B9u && f.y == 0x7F4A7C15u) st(dst + off, f);
    }
#pragma unroll
    for (int w = 0; w < W; ++w) {
        uint8_t* d = dst + (static_cast<uint64_t>(b) * W + w) * S + off;
#pragma unroll
        for (int u = 0; u < U; ++u) st(d + u * kStep, acc[u] + u32x4{static_cast<uint32_t>(w), 0u, 0u, 0u});
    }
}

template <typename F>
double time_ms(F launch, int reps = 6) {
    static hipEvent_t e0 = nullptr, e1 = nullptr;
    if (!e0) { CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); }
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

static uint8_t *g_src, *g_dst;

template <int R, int W, int U, bool MIS>
void run(uint32_t B) {
    const uint32_t grid = (B * (S / (kStep * U)) + 7) & ~7u;
    const double ms = time_ms([&] { hipLaunchKernelGGL((mix_kernel<R, W, U, MIS>), dim3(grid), dim3(256), 0, 0, g_src + (MIS ? 5 : 0), g_dst, B); });
    const double bytes = double(B) * (R + W) * S;
    printf("R=%d W=%d U=%d mis=%d B=%4u : %8.3f ms %8.1f GB/s (read %.1f GB, write %.1f GB)\n", R, W, U, int(MIS), B, ms, bytes / ms / 1e6,
           double(B) * R * S / 1e9, double(B) * W * S / 1e9);
    fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "dec") {
        // RS(6,3) ReconstructData with one data erasure (BASELINE config 3): read 6, write 1.
        const uint32_t B = 1024;
        CK(hipMalloc(&g_src, size_t(B) * 9 * S + 64));
        CK(hipMalloc(&g_dst, size_t(B) * 3 * S));
        CK(hipMemset(g_src, 0x3C, size_t(B) * 9 * S + 64));
        for (int rep = 0; rep < 2; ++rep) {
            printf("# rep %d\n", rep);
            run<6, 1, 4, false>(B);
            run<6, 1, 2, false>(B);
            run<6, 1, 1, false>(B);
            run<6, 0, 4, false>(B);    // the inputs alone (pure read)
            run<9, 0, 2, false>(B);    // Verify's read
            run<6, 3, 4, false>(B);    // encode
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "rpc") {
        // blb's recovery shapes (tools/rpc_shapes.py): the RPC reads k and writes m (every
        // absent slot rebuilt), the client reads k and writes 1..m.  B as in rpc_shapes.py.
        CK(hipMalloc(&g_src, size_t(6400) * S + 64));  // max B*R: 640*10
        CK(hipMalloc(&g_dst, size_t(3072) * S));       // max B*W: 1024*3
        CK(hipMemset(g_src, 0x3C, size_t(6400) * S + 64));
        for (int rep = 0; rep < 2; ++rep) {
            printf("# rep %d\n", rep);
            run<6, 3, 4, false>(1024);  // RS(6,3)
            run<6, 1, 4, false>(1024);
            run<8, 3, 2, false>(768);   // RS(8,3)
            run<8, 3, 4, false>(768);
            run<8, 1, 4, false>(768);
            run<10, 3, 2, false>(640);  // RS(10,3)
            run<10, 1, 2, false>(640);
            run<10, 1, 4, false>(640);
            run<12, 5, 2, false>(480);  // RS(12,5)
            run<12, 5, 1, false>(480);
            run<12, 1, 2, false>(480);
            run<12, 1, 4, false>(480);
        }
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "rs83") {
        // RS(8,3) pack + encode, bench.py's cold_class_extras: 512 stripes, the tracts fill
        // 5.7 of the 8 data pieces (24.5 GB read), 11 shards written (pieces + parity).
        const uint32_t B = 512;
        CK(hipMalloc(&g_src, size_t(B) * 8 * S + 64));  // R <= 8 source shards per stripe
        CK(hipMalloc(&g_dst, size_t(B) * 11 * S));
        CK(hipMemset(g_src, 0x3C, size_t(B) * 8 * S + 64));
        for (int rep = 0; rep < 2; ++rep) {
            printf("# rep %d\n", rep);
            run<8, 3, 2, false>(B);    // the RS(8,3) encode's mix
            run<6, 11, 1, false>(B);   // pack + encode, aligned sources
            run<6, 11, 1, true>(B);    // misaligned sources (two loads + v_alignbyte)
            run<6, 11, 2, false>(B);
            run<0, 11, 1, false>(B);   // pure write
            run<0, 11, 4, false>(B);
        }
        return 0;
    }
    // 1024 stripes' worth of the pack+encode mix: 4 reads x 8 MiB + 9 writes x 8 MiB per stripe.
    const uint32_t B = 1024;
    CK(hipMalloc(&g_src, size_t(B) * 6 * S + 64));
    CK(hipMalloc(&g_dst, size_t(B) * 9 * S));
    CK(hipMemset(g_src, 0x3C, size_t(B) * 6 * S + 64));
    for (int rep = 0; rep < 2; ++rep) {
        printf("# rep %d\n", rep);
        run<6, 3, 4, false>(B);   // the encode's mix (separate regions)
        run<4, 6, 1, false>(B);   // pack
        run<4, 6, 1, true>(B);
        run<4, 6, 2, true>(B);
        run<4, 9, 1, false>(B);   // pack + encode
        run<4, 9, 1, true>(B);
        run<4, 9, 2, false>(B);
        run<4, 9, 2, true>(B);
        run<4, 9, 4, false>(B);
        run<0, 9, 1, false>(B);   // pure write
        run<0, 9, 4, false>(B);
    }
    return 0;
}
