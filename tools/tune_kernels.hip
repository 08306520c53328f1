// tune_kernels.hip -- standalone MI355X tuning harness for the RS coding kernel.
// Measures, on the BASELINE workload (RS(6,3), B stripes of 8 MiB shards, strided):
//   * the access-pattern ceiling: read R shards / write W shards with trivial XOR compute;
//   * rs_code_kernel variants: chunks per lane U, nontemporal policy NT, grid size.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tune_kernels.hip -o tools/_build/tune
#include "../blb_amd/csrc/rs_kernels.hip"
#include "../blb_amd/csrc/gf256.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace blbrs;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

// Pattern kernel: each lane reads U 16B chunks from each of R shards, XORs them and writes
// the XOR to W shards.
template <int R, int W, int U, int NT, int XCD = 0>
__global__ __launch_bounds__(256) void pattern_kernel(uint8_t* base, uint64_t shard_stride, uint64_t stripe_stride,
                                                      uint32_t B, uint32_t tps, uint32_t* sink) {
    constexpr uint32_t kStep = 256 * 16;
    const uint32_t total = B * tps;
    uint32_t keep = 0;
    uint32_t bid = blockIdx.x;
    if (XCD) bid = (bid % 8) * (gridDim.x / 8) + bid / 8;  // XCD x owns a contiguous block range
    for (uint32_t t = bid; t < total; t += gridDim.x) {
        const uint32_t b = t / tps;
        const uint64_t off = static_cast<uint64_t>(t - b * tps) * kStep * U + threadIdx.x * 16;
        uint8_t* s = base + b * stripe_stride + off;
        V4 x[R][U];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int u = 0; u < U; ++u) x[r][u] = ld16<NT>(s + r * shard_stride + u * kStep);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            V4 a{0, 0, 0, 0};
#pragma unroll
            for (int r = 0; r < R; ++r) { a.x ^= x[r][u].x; a.y ^= x[r][u].y; a.z ^= x[r][u].z; a.w ^= x[r][u].w; }
            if constexpr (W == 0) keep ^= a.x ^ a.y ^ a.z ^ a.w;
#pragma unroll
            for (int w = 0; w < W; ++w) st16<NT>(s + (R + w) * shard_stride + u * kStep, a);
        }
    }
    if (W == 0 && keep == 0x9E3779B9u) sink[0] = keep;
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

template <typename F>
double time_ms(F launch, int reps = 10) {
    static Timer t;
    launch(); launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t.a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(t.b));
    CK(hipEventSynchronize(t.b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t.a, t.b));
    return ms / reps;
}

static uint8_t* g_base;
static uint32_t* g_sink;
static const uint64_t S = 8ull << 20;
static uint32_t B = 1024;

template <int R, int W, int U, int NT, int XCD = 0>
void run_pattern(int grid) {
    const uint64_t ss = S, bs = 9 * S;
    const uint32_t tps = static_cast<uint32_t>(S / (4096 * U));
    double ms = time_ms([&] { hipLaunchKernelGGL((pattern_kernel<R, W, U, NT, XCD>), dim3(grid), dim3(256), 0, 0,
                                                 g_base, ss, bs, B, tps, g_sink); });
    const double bytes = double(B) * (R + W) * S;
    printf("pattern XCD=%d R=%d W=%d U=%d NT=%d grid=%6d : %8.3f ms  %7.1f GB/s\n", XCD, R, W, U, NT, grid, ms, bytes / ms / 1e6);
}

// Pattern ceiling at a wider shape: stripes of R+W shards packed back to back in the same
// buffer (as shape() views it for rs_code_kernel), so the two are directly comparable.
template <int R, int W, int U>
void run_pattern_shape() {
    const uint64_t ss = S, bs = uint64_t(R + W) * S;
    const uint32_t nb = static_cast<uint32_t>(uint64_t(B) * 9 * S / bs);
    const uint32_t tps = static_cast<uint32_t>(S / (4096 * U));
    const int grid = static_cast<int>(nb * tps) & ~7;
    double ms = time_ms([&] { hipLaunchKernelGGL((pattern_kernel<R, W, U, 3, 1>), dim3(grid), dim3(256), 0, 0,
                                                 g_base, ss, bs, nb, tps, g_sink); });
    const double bytes = double(nb) * (R + W) * S;
    printf("pattern R=%2d W=%d U=%d B=%4u : %8.3f ms  %7.1f GB/s  %7.1f GiB/s data\n", R, W, U, nb, ms, bytes / ms / 1e6,
           double(nb) * R * S / (ms * 1e-3) / double(1u << 30));
}

template <int U, int NT, int K = 6, int MR = 3, int MODE = 0>
void run_rs(CodeArgs a, int grid, const char* tag, int remap = 0) {
    a.xcd_remap = remap;
    a.tiles_per_stripe = static_cast<uint32_t>(S / (kTileBytes * U));
    auto fn = rs_code_kernel<K, MR, MODE, 0, U, NT>;
    int bpc = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, reinterpret_cast<const void*>(fn), 256, 0));
    if (grid <= 0) grid = 256 * bpc * (-grid == 0 ? 1 : -grid);
    if (grid == 1) grid = static_cast<int>(a.B * a.tiles_per_stripe);
    if (MODE == 1) {  // make the parity consistent first (same tables), else every wave flags
        hipLaunchKernelGGL((rs_code_kernel<K, MR, 0, 0, U, 3>), dim3(grid), dim3(256), 0, 0, a);
        CK(hipMemset(a.mismatch, 0, 4 * a.B));
        CK(hipDeviceSynchronize());
    }
    double ms = time_ms([&] { hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, a); });
    const int kk = K ? K : a.k;
    const double bytes = double(a.B) * (kk + MR) * S;
    int32_t bad = 0;
    if (MODE == 1) {
        std::vector<int32_t> f(a.B);
        CK(hipMemcpy(f.data(), a.mismatch, 4 * a.B, hipMemcpyDeviceToHost));
        for (int32_t v : f) bad += v;
    }
    printf("%s", bad ? "[MISMATCH] " : "");
    printf("K=%2d MR=%d MODE=%d %-6s remap=%d U=%d NT=%d bpc=%d grid=%7d : %8.3f ms  %7.1f GB/s  %7.1f GiB/s data\n",
           kk, MR, MODE, tag, remap, U, NT, bpc, grid, ms, bytes / ms / 1e6,
           double(a.B) * kk * S / (ms * 1e-3) / double(1u << 30));
}

// Zero-copy: the coding kernel reads/writes pinned host stripes directly over PCIe.
static void zero_copy_probe() {
    const uint32_t nb = 24;
    const size_t bytes = size_t(nb) * 9 * S;
    for (unsigned flags : {0u /*default*/, 0x40000000u /*hipHostMallocNonCoherent*/}) {
        uint8_t* h = nullptr;
        if (hipHostMalloc(&h, bytes, flags) != hipSuccess) { printf("hostmalloc %x failed\n", flags); continue; }
        memset(h, 0x37, bytes);
        std::vector<uint32_t> tab(6 * 3 * 5, 0x03020100u);
        int32_t idx[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
        uint32_t* d_tab; int32_t* d_idx;
        CK(hipMalloc(&d_tab, tab.size() * 4));
        CK(hipMalloc(&d_idx, sizeof(idx)));
        CK(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d_idx, idx, sizeof(idx), hipMemcpyHostToDevice));
        CodeArgs c{};
        c.tables = d_tab; c.in_idx = d_idx; c.out_idx = d_idx + 6; c.base = h;
        c.shard_stride = S; c.stripe_stride = 9 * S; c.B = nb; c.S = S; c.k = 6; c.rows = 3; c.aligned = 1;
        for (int u : {2, 4}) {
            c.tiles_per_stripe = static_cast<uint32_t>(S / (4096 * u));
            const uint32_t total = nb * c.tiles_per_stripe;
            for (int grid : {1024, 4096, static_cast<int>(total & ~7u)}) {
                c.xcd_remap = 1;
                double ms = time_ms([&] {
                    if (u == 4) hipLaunchKernelGGL((rs_code_kernel<6, 3, 0, 0, 4, 3>), dim3(grid), dim3(256), 0, 0, c);
                    else hipLaunchKernelGGL((rs_code_kernel<6, 3, 0, 0, 2, 3>), dim3(grid), dim3(256), 0, 0, c);
                }, 3);
                printf("zero-copy flags=%x U=%d grid=%7d : %8.3f ms  %6.2f GiB/s data  (%5.1f GB/s rd, %5.1f GB/s wr)\n",
                       flags, u, grid, ms, double(nb) * 6 * S / (ms * 1e-3) / double(1u << 30),
                       double(nb) * 6 * S / ms / 1e6, double(nb) * 3 * S / ms / 1e6);
            }
        }
        CK(hipHostFree(h));
        CK(hipFree(d_tab)); CK(hipFree(d_idx));
    }
}

// Shard / stripe stride padding: do 9 streams exactly 8 MiB apart alias in the HBM
// channel/bank hash?  Same kernel, same bytes, different layouts.
static void stride_probe(CodeArgs a) {
    const size_t cap = size_t(B) * 9 * S;
    for (int rep = 0; rep < 2; ++rep)
        for (uint64_t pad : {0ull, 256ull, 4096ull, 65536ull, 1ull << 20, 3ull << 12}) {
            for (int mode = 0; mode < 2; ++mode) {  // 0: pad shards, 1: pad stripes only
                CodeArgs c = a;
                c.shard_stride = mode == 0 ? S + pad : S;
                c.stripe_stride = mode == 0 ? 9 * (S + pad) : 9 * S + pad;
                c.B = static_cast<uint32_t>((cap - 9 * (S + pad)) / c.stripe_stride);
                if (c.B > 1000) c.B = 1000;
                c.tiles_per_stripe = static_cast<uint32_t>(S / 16384);
                c.xcd_remap = 1;
                const int grid = static_cast<int>(c.B * c.tiles_per_stripe) & ~7;
                double ms = time_ms([&] { hipLaunchKernelGGL((rs_code_kernel<6, 3, 0, 0, 4, 3>), dim3(grid), dim3(256), 0, 0, c); });
                printf("stride pad=%8llu %s B=%u : %8.3f ms  %7.1f GB/s\n", (unsigned long long)pad,
                       mode == 0 ? "shard " : "stripe", c.B, ms, double(c.B) * 9 * S / ms / 1e6);
            }
        }
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "zc") { zero_copy_probe(); return 0; }
    const bool ntab = argc > 1 && std::string(argv[1]) == "nt";
    const bool occ = argc > 1 && std::string(argv[1]) == "occ";
    const bool stride = argc > 1 && std::string(argv[1]) == "stride";
    const bool pmc = argc > 1 && std::string(argv[1]) == "pmc";
    const bool ceil = argc > 1 && std::string(argv[1]) == "ceil";
    if (argc > 1 && !pmc && !stride && !ceil && !ntab && !occ) B = static_cast<uint32_t>(atoi(argv[1]));
    const size_t total = size_t(B) * 9 * S;
    CK(hipMalloc(&g_base, total));
    CK(hipMalloc(&g_sink, 64));
    CK(hipMemset(g_base, 0x5B, total));
    // tables for RS(6,3)
    Mat mat;
    build_matrix(6, 3, mat);
    std::vector<uint32_t> tab(17 * 8 * 5, 0x03020100u);
    int32_t idx[32];
    for (int i = 0; i < 32; ++i) idx[i] = i;
    uint32_t* d_tab; int32_t* d_idx;
    CK(hipMalloc(&d_tab, tab.size() * 4));
    CK(hipMalloc(&d_idx, sizeof(idx)));
    CK(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_idx, idx, sizeof(idx), hipMemcpyHostToDevice));
    int32_t* d_flags;
    CK(hipMalloc(&d_flags, 1 << 20));
    CK(hipMemset(d_flags, 0, 1 << 20));
    CodeArgs a{};
    a.tables = d_tab; a.in_idx = d_idx; a.out_idx = d_idx + 6; a.base = g_base;
    a.shard_stride = S; a.stripe_stride = 9 * S; a.B = B; a.S = S; a.k = 6; a.rows = 3; a.aligned = 1;
    a.mismatch = d_flags;
    // same 72 GiB buffer re-viewed for the other shapes
    auto shape = [&](int k, int rows) {
        CodeArgs c = a;
        c.k = k; c.rows = rows; c.out_idx = d_idx + k;
        c.stripe_stride = uint64_t(k + rows) * S;
        c.B = static_cast<uint32_t>(total / c.stripe_stride);
        return c;
    };

    printf("# B=%u stripes x 9 shards x 8 MiB = %.1f GiB\n", B, total / double(1ull << 30));
    if (stride) { stride_probe(a); return 0; }
    if (pmc) {
        // Counter calibration (one launch each, run under rocprofv3 --pmc):
        //   pattern R=9 W=0: reads exactly B*9*S bytes, writes nothing;
        //   pattern R=1 W=1: reads B*S, writes B*S (same nt 16-B/lane access as the kernel);
        //   rs_code_kernel<6,3,0,0,4,3>: the production RS(6,3) encode.
        const uint32_t all4 = static_cast<uint32_t>(B * (S / 16384));
        hipLaunchKernelGGL((pattern_kernel<9, 0, 4, 3, 1>), dim3(all4 & ~7u), dim3(256), 0, 0, g_base, S, 9 * S, B,
                           static_cast<uint32_t>(S / 16384), g_sink);
        hipLaunchKernelGGL((pattern_kernel<1, 1, 4, 3, 1>), dim3(all4 & ~7u), dim3(256), 0, 0, g_base, S, 9 * S, B,
                           static_cast<uint32_t>(S / 16384), g_sink);
        CodeArgs c = a;
        c.tiles_per_stripe = static_cast<uint32_t>(S / 16384);
        c.xcd_remap = 1;
        hipLaunchKernelGGL((rs_code_kernel<6, 3, 0, 0, 4, 3>), dim3(all4 & ~7u), dim3(256), 0, 0, c);
        CK(hipDeviceSynchronize());
        printf("pmc launches done: read_bytes=%.0f copy_bytes=%.0f+%.0f rs63_bytes=%.0f+%.0f\n", double(B) * 9 * S,
               double(B) * S, double(B) * S, double(B) * 6 * S, double(B) * 3 * S);
        return 0;
    }
    if (occ) {
        // Occupancy of the shipped encode grid, capped by an unused dynamic LDS allocation:
        // 0 = natural (VGPR-limited), 56 KiB = at most 2 blocks per CU, 96 KiB = 1 block per CU.
        CodeArgs c = a;
        c.tiles_per_stripe = static_cast<uint32_t>(S / 16384);
        c.xcd_remap = 1;
        const int grid = static_cast<int>(c.B * c.tiles_per_stripe) & ~7;
        const double bytes = double(c.B) * 9 * S;
        for (int rep = 0; rep < 3; ++rep)
            for (unsigned lds : {0u, 56u << 10, 96u << 10}) {
                double ms = time_ms([&] { hipLaunchKernelGGL((rs_code_kernel<6, 3, 0, 0, 4, 3>), dim3(grid), dim3(256), lds, 0, c); });
                printf("occ rep %d rs63 U=4 dyn_lds=%6u : %8.3f ms  %7.1f GB/s\n", rep, lds, ms, bytes / ms / 1e6);
                const uint32_t tps4 = static_cast<uint32_t>(S / 16384);
                ms = time_ms([&] { hipLaunchKernelGGL((pattern_kernel<6, 3, 4, 3, 1>), dim3(grid), dim3(256), lds, 0, g_base, S, 9 * S, B, tps4, g_sink); });
                printf("occ rep %d pattern R6W3 U=4 dyn_lds=%6u : %8.3f ms  %7.1f GB/s\n", rep, lds, ms, bytes / ms / 1e6);
                fflush(stdout);
            }
        return 0;
    }
    if (ntab) {
        // Cache policy of the shipped grid (one tile per block, XCD remap, U = 4): NT bit 0 =
        // nontemporal loads, bit 1 = nontemporal stores.  Plain stores land in L2 / MALL.
        for (int rep = 0; rep < 3; ++rep) {
            printf("# nt rep %d\n", rep);
            run_rs<4, 3>(a, 1, "nt3", 1);
            run_rs<4, 1>(a, 1, "nt1", 1);
            run_rs<4, 2>(a, 1, "nt2", 1);
            run_rs<4, 0>(a, 1, "nt0", 1);
        }
        return 0;
    }
    if (ceil) {
        // Wide-shape question: is RS(10,4)/RS(12,5) below its own
        // access-pattern ceiling, or is the ceiling itself lower than RS(6,3)'s?
        for (int rep = 0; rep < 2; ++rep) {
            printf("# ceil rep %d\n", rep);
            run_pattern_shape<6, 3, 4>();
            run_rs<4, 3>(a, 1, "all", 1);
            run_pattern_shape<10, 4, 2>();
            run_pattern_shape<10, 4, 4>();
            run_rs<2, 3, 10, 4>(shape(10, 4), 1, "rs104", 1);
            run_pattern_shape<12, 5, 2>();
            run_pattern_shape<12, 5, 4>();
            run_rs<2, 3, 12, 5>(shape(12, 5), 1, "rs125", 1);
            run_pattern_shape<10, 2, 2>();
            run_rs<2, 3, 10, 2>(shape(10, 2), 1, "dec2", 1);
            run_pattern_shape<6, 1, 4>();
            run_rs<4, 3, 6, 1>(shape(6, 1), 1, "dec1", 1);
        }
        return 0;
    }
    for (int rep = 0; rep < 1; ++rep) {
        printf("# rep %d\n", rep);
        run_rs<4, 3>(a, 1, "all", 1);
        run_rs<2, 3>(a, 1, "all", 1);
        run_rs<4, 3, 6, 1>(shape(6, 1), 1, "dec1", 1);
        run_rs<2, 3, 6, 1>(shape(6, 1), 1, "dec1", 1);
        run_rs<4, 1, 6, 3, 1>(a, 1, "verify", 1);
        run_rs<2, 1, 6, 3, 1>(a, 1, "verify", 1);
        run_pattern<9, 0, 4, 3, 1>(static_cast<int>(B * (S / 16384)) & ~7);
        run_rs<4, 3, 10, 4>(shape(10, 4), 1, "rs104", 1);
        run_rs<2, 3, 10, 4>(shape(10, 4), 1, "rs104", 1);
        run_rs<4, 3, 10, 2>(shape(10, 2), 1, "dec2", 1);
        run_rs<2, 3, 10, 2>(shape(10, 2), 1, "dec2", 1);
        run_rs<4, 3, 12, 5>(shape(12, 5), 1, "rs125", 1);
        run_rs<2, 3, 12, 5>(shape(12, 5), 1, "rs125", 1);
        run_rs<4, 3, 8, 3>(shape(8, 3), 1, "rs83", 1);
        run_rs<2, 3, 8, 3>(shape(8, 3), 1, "rs83", 1);
        run_rs<4, 3, 0, 3>(shape(17, 3), 1, "gen17", 1);
        run_rs<2, 3, 0, 3>(shape(17, 3), 1, "gen17", 1);
        run_rs<1, 3, 0, 3>(shape(17, 3), 1, "gen17", 1);
        run_rs<4, 1, 10, 4, 1>(shape(10, 4), 1, "ver104", 1);
        run_rs<2, 1, 10, 4, 1>(shape(10, 4), 1, "ver104", 1);
        run_rs<4, 3, 4, 2>(shape(4, 2), 1, "rs42", 1);
        run_rs<2, 3, 4, 2>(shape(4, 2), 1, "rs42", 1);
        run_rs<4, 3, 10, 1>(shape(10, 1), 1, "dec1w", 1);
        run_rs<2, 3, 10, 1>(shape(10, 1), 1, "dec1w", 1);
    }
    return 0;
}
