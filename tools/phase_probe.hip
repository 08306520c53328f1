// phase_probe.hip -- does a chip-wide read/write phase split beat the mixed 2:1 stream?
//
// The RS(6,3) encode reads 6 shards and writes 3.  Measured ceilings on one MI355X
// (profiles/r02/hbm): pure read 6.8 TB/s, pure write 6.95 TB/s, but the 2:1 mix only
// 6.2 TB/s -- about 10 % lost to read/write turnaround in the memory controllers.  This probe
// gates every wave on the chip-wide constant clock (s_memrealtime, 100 MHz): loads are issued
// only inside the read window of each period, stores only inside the write window, so all
// channels see one direction at a time.  Trivial XOR compute (the access pattern only).
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/phase_probe.hip -o tools/_build/phase_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

constexpr uint64_t S = 8ull << 20;
constexpr uint32_t kStep = 256 * 16;

// Baseline: one tile (U chunks of 4 KiB per shard) per block, XCD-contiguous, as shipped.
template <int U>
__global__ __launch_bounds__(256) void mixed_kernel(uint8_t* base, uint32_t B) {
    const uint32_t tps = S / (kStep * U);
    const uint32_t total = B * tps;
    const uint32_t t = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
    if (t >= total) return;
    const uint32_t b = t / tps;
    uint8_t* s = base + b * 9 * S + static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
    u32x4 x[6][U];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) x[r][u] = ld(s + r * S + u * kStep);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32x4 a = x[0][u] ^ x[1][u] ^ x[2][u];
        const u32x4 c = x[3][u] ^ x[4][u] ^ x[5][u];
        st(s + 6 * S + u * kStep, a ^ c);
        st(s + 7 * S + u * kStep, a);
        st(s + 8 * S + u * kStep, c);
    }
}

// Store with explicit gfx950 cache-policy bits (vector stores only).
template <int SP>
__device__ __forceinline__ void st_pol(uint8_t* p, u32x4 v) {
    if constexpr (SP == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (SP == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
constexpr const char* kPolName[6] = {"plain", "nt", "sc1", "sc1 nt", "sc0 sc1", "sc0 sc1 nt"};

// The shipped grid's access pattern with store policy SP and nontemporal (LNT) or plain loads.
template <int SP, bool LNT>
__global__ __launch_bounds__(256) void policy_kernel(uint8_t* base, uint32_t B) {
    constexpr int U = 4;
    const uint32_t tps = S / (kStep * U);
    const uint32_t total = B * tps;
    const uint32_t t = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
    if (t >= total) return;
    const uint32_t b = t / tps;
    uint8_t* s = base + b * 9 * S + static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
    u32x4 x[6][U];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) x[r][u] = LNT ? ld(s + r * S + u * kStep) : *reinterpret_cast<const u32x4*>(s + r * S + u * kStep);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32x4 a = x[0][u] ^ x[1][u] ^ x[2][u];
        const u32x4 c = x[3][u] ^ x[4][u] ^ x[5][u];
        st_pol<SP>(s + 6 * S + u * kStep, a ^ c);
        st_pol<SP>(s + 7 * S + u * kStep, a);
        st_pol<SP>(s + 8 * S + u * kStep, c);
    }
}

// One tile per block of NTH threads (U 16-byte chunks per lane per shard): tile = NTH*16*U
// bytes per shard, XCD-contiguous.  Does a larger contiguous tile per block (fewer,
// longer concurrent streams) raise the read-6/write-3 ceiling?
template <int NTH, int U>
__global__ __launch_bounds__(NTH) void wide_kernel(uint8_t* base, uint32_t B) {
    constexpr uint32_t step = NTH * 16;
    const uint32_t tps = S / (step * U);
    const uint32_t total = B * tps;
    const uint32_t t = (blockIdx.x % 8u) * (gridDim.x / 8u) + blockIdx.x / 8u;
    if (t >= total) return;
    const uint32_t b = t / tps;
    uint8_t* s = base + b * 9 * S + static_cast<uint64_t>(t - b * tps) * step * U + threadIdx.x * 16;
    u32x4 x[6][U];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) x[r][u] = ld(s + r * S + u * step);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32x4 a = x[0][u] ^ x[1][u] ^ x[2][u];
        const u32x4 c = x[3][u] ^ x[4][u] ^ x[5][u];
        st(s + 6 * S + u * step, a ^ c);
        st(s + 7 * S + u * step, a);
        st(s + 8 * S + u * step, c);
    }
}

__device__ __forceinline__ void wait_window(uint64_t period, uint64_t lo, uint64_t hi) {
    // Spin (sleeping) until clock mod period is in [lo, hi).  Terminates: the clock runs.
    for (;;) {
        const uint64_t ph = wall_clock64() % period;
        if (ph >= lo && ph < hi) return;
        __builtin_amdgcn_s_sleep(2);
    }
}

// Persistent: each block walks groups of U tiles (grid-stride over the XCD's contiguous
// range); with period > 0 loads wait for [0, rd) and stores for [rd, period).
template <int U>
__global__ __launch_bounds__(256) void phased_kernel(uint8_t* base, uint32_t B, uint64_t period, uint64_t rd) {
    const uint32_t tps = S / (kStep * U);
    const uint32_t total = B * tps;
    const uint32_t per_xcd = (total + 7) / 8;
    const uint32_t xcd = blockIdx.x % 8u;
    const uint32_t blocks_per_xcd = gridDim.x / 8u;
    const uint32_t lo = xcd * per_xcd;
    const uint32_t hi = min(total, lo + per_xcd);
    for (uint32_t t = lo + blockIdx.x / 8u; t < hi; t += blocks_per_xcd) {
        const uint32_t b = t / tps;
        uint8_t* s = base + b * 9 * S + static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
        if (period) wait_window(period, 0, rd);
        u32x4 x[6][U];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) x[r][u] = ld(s + r * S + u * kStep);
        u32x4 a[U], c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = x[0][u] ^ x[1][u] ^ x[2][u]; c[u] = x[3][u] ^ x[4][u] ^ x[5][u]; }
        if (period) wait_window(period, rd, period);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            st(s + 6 * S + u * kStep, a[u] ^ c[u]);
            st(s + 7 * S + u * kStep, a[u]);
            st(s + 8 * S + u * kStep, c[u]);
        }
    }
}

template <typename F>
double time_ms(F launch, int reps = 8) {
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

int main(int argc, char** argv) {
    const uint32_t B = argc > 1 ? static_cast<uint32_t>(atoi(argv[1])) : 1024;
    const size_t bytes = size_t(B) * 9 * S;
    const double alg = double(B) * 9 * S;
    uint8_t* base = nullptr;
    CK(hipMalloc(&base, bytes));
    CK(hipMemset(base, 0x5B, bytes));
    int rate_khz = 0, cus = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const double tick_us = 1e3 / rate_khz;
    printf("# B=%u  %.1f GB  wall clock %d kHz (%.3f us/tick)  CUs %d\n", B, alg / 1e9, rate_khz, tick_us, cus);

    auto report = [&](const char* tag, double ms) { printf("%-48s %8.3f ms %8.1f GB/s\n", tag, ms, alg / ms / 1e6); fflush(stdout); };
    char tag[128];
    if (argc > 2 && std::string(argv[2]) == "wide") {  // phase_probe B wide: tile-size sweep
        for (int rep = 0; rep < 3; ++rep) {
            printf("# wide rep %d\n", rep);
#define WIDE(NTH, U, LDS) { const uint32_t g = (B * (S / (NTH * 16u * U)) + 7) & ~7u; \
            snprintf(tag, sizeof tag, "wide threads=%4d U=%d tile=%3u KiB lds=%3u KiB", NTH, U, NTH * 16 * U / 1024, LDS); \
            report(tag, time_ms([&] { hipLaunchKernelGGL((wide_kernel<NTH, U>), dim3(g), dim3(NTH), LDS * 1024, 0, base, B); })); }
            WIDE(256, 4, 0) WIDE(256, 4, 96) WIDE(512, 4, 0) WIDE(512, 2, 0) WIDE(1024, 2, 0) WIDE(1024, 1, 0) WIDE(256, 8, 0) WIDE(512, 4, 96)
#undef WIDE
        }
        CK(hipFree(base));
        return 0;
    }
    if (argc > 2) {  // phase_probe B policy: store cache-policy A/B on the encode's pattern
        const uint32_t g4 = (B * (S / (kStep * 4)) + 7) & ~7u;
        for (int rep = 0; rep < 3; ++rep) {
            printf("# policy rep %d\n", rep);
            report("mixed U=4 builtin nt loads + nt stores", time_ms([&] { hipLaunchKernelGGL(mixed_kernel<4>, dim3(g4), dim3(256), 0, 0, base, B); }));
#define POL(SP, L) snprintf(tag, sizeof tag, "policy stores=%s loads=%s", kPolName[SP], L ? "nt" : "plain"); \
            report(tag, time_ms([&] { hipLaunchKernelGGL((policy_kernel<SP, L>), dim3(g4), dim3(256), 0, 0, base, B); }));
            POL(0, true) POL(1, true) POL(2, true) POL(3, true) POL(4, true) POL(5, true) POL(1, false) POL(0, false)
#undef POL
        }
        CK(hipFree(base));
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        printf("# rep %d\n", rep);
        const uint32_t g4 = (B * (S / (kStep * 4)) + 7) & ~7u;
        report("mixed U=4 one tile per block", time_ms([&] { hipLaunchKernelGGL(mixed_kernel<4>, dim3(g4), dim3(256), 0, 0, base, B); }));
        int bpc4 = 0, bpc2 = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc4, reinterpret_cast<const void*>(phased_kernel<4>), 256, 0));
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc2, reinterpret_cast<const void*>(phased_kernel<2>), 256, 0));
        for (int U : {2, 4}) {
            const int bpc = U == 4 ? bpc4 : bpc2;
            const int grid = cus * bpc;
            auto run = [&](uint64_t period, uint64_t rd) {
                return time_ms([&] {
                    if (U == 4) hipLaunchKernelGGL(phased_kernel<4>, dim3(grid), dim3(256), 0, 0, base, B, period, rd);
                    else hipLaunchKernelGGL(phased_kernel<2>, dim3(grid), dim3(256), 0, 0, base, B, period, rd);
                });
            };
            snprintf(tag, sizeof tag, "persistent U=%d bpc=%d ungated", U, bpc);
            report(tag, run(0, 0));
            for (double period_us : {6.0, 8.0, 10.0, 12.0, 14.0, 16.0, 20.0, 24.0}) {
                for (double frac : {0.60, 0.70}) {
                    const uint64_t p = static_cast<uint64_t>(period_us / tick_us + 0.5);
                    const uint64_t r = static_cast<uint64_t>(p * frac + 0.5);
                    snprintf(tag, sizeof tag, "persistent U=%d gated period=%4.0fus rd=%.2f", U, period_us, frac);
                    report(tag, run(p, r));
                }
            }
        }
    }
    CK(hipFree(base));
    return 0;
}
