// rbs_ab.hip -- A/B of the run-time-coefficient bit-plane kernel (rs_rbs.hpp) against the
// v_perm table kernel (rs_code.hpp) on one device-resident batch, interleaved in one process.
//
// Shape: B stripes of (k + rows) shards of S bytes, strided, inputs = shards 0..k-1, outputs =
// shards k..k+rows-1, random non-zero coefficients (a decode pass's shape).  Both kernels run
// on the same buffer; the bit-plane kernel's output is compared byte for byte with the table
// kernel's before timing.  Prints one JSON line.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I blb_amd/csrc -I tools tools/rbs_ab.hip -o tools/_build/rbs_ab
// usage: rbs_ab [k rows B S reps]   (k = 12 or 10 compiled; rows 1..5)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "gf256.hpp"
#include "rs_rbs.hpp"

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

using namespace blbrs;

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        x ^= x >> 15;
        x *= 2246822519u;
        x ^= x >> 13;
        p[i] = x;
    }
}

__global__ void diff_kernel(const uint4* a, const uint4* b, size_t n, unsigned long long* bad) {
    unsigned long long local = 0;
    for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x) {
        const uint4 x = a[i], y = b[i];
        local += (x.x != y.x) + (x.y != y.y) + (x.z != y.z) + (x.w != y.w);
    }
    if (local) atomicAdd(bad, local);
}

template <int K, int MR>
void launch_tab(const CodeArgs& a, unsigned grid) {
    hipLaunchKernelGGL((code::rs_code_kernel<K, MR, 0, 0, 2, 3>), dim3(grid), dim3(kThreads), 0, 0, a);
}
template <int MR>
void launch_rbs(const CodeArgs& a, const uint32_t* coef8, unsigned grid) {
    hipLaunchKernelGGL((code::rs_rbs_kernel<MR, 0>), dim3(grid), dim3(kThreads), 0, 0, a, coef8);
}

int main(int argc, char** argv) {
    const int k = argc > 1 ? std::atoi(argv[1]) : 12;
    const int rows = argc > 2 ? std::atoi(argv[2]) : 5;
    const uint32_t B = argc > 3 ? std::atoi(argv[3]) : 480;
    const size_t S = argc > 4 ? std::strtoull(argv[4], nullptr, 0) : (size_t{8} << 20);
    const int reps = argc > 5 ? std::atoi(argv[5]) : 7;
    if ((k != 12 && k != 10) || rows < 1 || rows > 5) {
        std::printf("{\"error\": \"k must be 10 or 12, rows 1..5\"}\n");
        return 2;
    }
    const int n = k + rows;
    const size_t total = static_cast<size_t>(B) * n * S;
    uint8_t* base = nullptr;
    CK(hipMalloc(&base, total));
    CK(hipMemset(base, 0, total));
    for (uint32_t b = 0; b < B; ++b)
        hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(base + static_cast<size_t>(b) * n * S),
                           static_cast<size_t>(k) * S / 4, 97531u + b);
    CK(hipDeviceSynchronize());

    std::mt19937 rng(4242);
    Mat coef(static_cast<size_t>(rows) * k);
    for (auto& c : coef) c = static_cast<uint8_t>(1 + rng() % 255);
    const std::vector<uint32_t> tab = perm_tables(coef, rows, k);
    std::vector<uint32_t> c8(static_cast<size_t>(k) * 2, 0);
    for (int c = 0; c < k; ++c)
        for (int r = 0; r < rows; ++r) c8[2 * c + r / 4] |= static_cast<uint32_t>(coef[r * k + c]) << (8 * (r % 4));
    std::vector<int32_t> in_idx(k), out_idx(rows);
    for (int c = 0; c < k; ++c) in_idx[c] = c;
    for (int r = 0; r < rows; ++r) out_idx[r] = k + r;
    uint32_t *d_tab = nullptr, *d_c8 = nullptr;
    int32_t *d_in = nullptr, *d_out = nullptr;
    CK(hipMalloc(&d_tab, tab.size() * 4));
    CK(hipMalloc(&d_c8, c8.size() * 4));
    CK(hipMalloc(&d_in, k * 4));
    CK(hipMalloc(&d_out, rows * 4));
    CK(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_c8, c8.data(), c8.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_in, in_idx.data(), k * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_out, out_idx.data(), rows * 4, hipMemcpyHostToDevice));

    CodeArgs a{};
    a.tables = d_tab;
    a.in_idx = d_in;
    a.out_idx = d_out;
    a.base = base;
    a.shard_stride = S;
    a.stripe_stride = static_cast<uint64_t>(n) * S;
    a.nshards = n;
    a.B = B;
    a.S = S;
    a.k = k;
    a.rows = rows;
    a.aligned = 1;
    const uint64_t tile = static_cast<uint64_t>(kTileBytes) * 2;
    const uint64_t tps = (S + tile - 1) / tile;
    a.tiles_per_stripe = static_cast<uint32_t>(tps);
    const uint64_t tiles = static_cast<uint64_t>(B) * tps;
    unsigned grid = static_cast<unsigned>(tiles);
    a.xcd_remap = 0;
    if (tiles >= 64) {
        grid = static_cast<unsigned>(tiles & ~uint64_t{7});
        a.xcd_remap = 1;
    }

    auto tab_run = [&] {
        if (k == 12) {
            switch (rows) {
                case 1: launch_tab<12, 1>(a, grid); break;
                case 2: launch_tab<12, 2>(a, grid); break;
                case 3: launch_tab<12, 3>(a, grid); break;
                case 4: launch_tab<12, 4>(a, grid); break;
                default: launch_tab<12, 5>(a, grid); break;
            }
        } else {
            switch (rows) {
                case 1: launch_tab<10, 1>(a, grid); break;
                case 2: launch_tab<10, 2>(a, grid); break;
                case 3: launch_tab<10, 3>(a, grid); break;
                case 4: launch_tab<10, 4>(a, grid); break;
                default: launch_tab<10, 5>(a, grid); break;
            }
        }
    };
    auto rbs_run = [&] {
        switch (rows) {
            case 1: launch_rbs<1>(a, d_c8, grid); break;
            case 2: launch_rbs<2>(a, d_c8, grid); break;
            case 3: launch_rbs<3>(a, d_c8, grid); break;
            case 4: launch_rbs<4>(a, d_c8, grid); break;
            default: launch_rbs<5>(a, d_c8, grid); break;
        }
    };

    // Bit-exactness: the table kernel's outputs, then the bit-plane kernel's over the same slots.
    const size_t out_bytes_per_stripe = static_cast<size_t>(rows) * S;
    uint8_t* ref = nullptr;
    CK(hipMalloc(&ref, out_bytes_per_stripe * std::min<uint32_t>(B, 8)));
    tab_run();
    CK(hipDeviceSynchronize());
    const uint32_t nchk = std::min<uint32_t>(B, 8);
    for (uint32_t i = 0; i < nchk; ++i) {
        const uint32_t sb = i * (B / nchk);
        CK(hipMemcpy(ref + i * out_bytes_per_stripe, base + static_cast<size_t>(sb) * n * S + static_cast<size_t>(k) * S,
                     out_bytes_per_stripe, hipMemcpyDeviceToDevice));
    }
    CK(hipMemset(base, 0xA5, 0));
    for (uint32_t b = 0; b < B; ++b) CK(hipMemsetAsync(base + static_cast<size_t>(b) * n * S + static_cast<size_t>(k) * S, 0x5A, out_bytes_per_stripe));
    rbs_run();
    CK(hipDeviceSynchronize());
    unsigned long long* d_bad = nullptr;
    CK(hipMalloc(&d_bad, 8));
    CK(hipMemset(d_bad, 0, 8));
    for (uint32_t i = 0; i < nchk; ++i) {
        const uint32_t sb = i * (B / nchk);
        hipLaunchKernelGGL(diff_kernel, dim3(1024), dim3(256), 0, 0,
                           reinterpret_cast<const uint4*>(ref + i * out_bytes_per_stripe),
                           reinterpret_cast<const uint4*>(base + static_cast<size_t>(sb) * n * S + static_cast<size_t>(k) * S),
                           out_bytes_per_stripe / 16, d_bad);
    }
    unsigned long long bad = 0;
    CK(hipMemcpy(&bad, d_bad, 8, hipMemcpyDeviceToHost));

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ta, tb;
    for (int r = 0; r < reps; ++r) {
        for (int v = 0; v < 2; ++v) {
            CK(hipEventRecord(e0, 0));
            if (v == 0) tab_run();
            else rbs_run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            (v == 0 ? ta : tb).push_back(ms);
        }
    }
    std::sort(ta.begin(), ta.end());
    std::sort(tb.begin(), tb.end());
    const double bytes = static_cast<double>(B) * (k + rows) * S;
    const double ma = ta[ta.size() / 2], mb = tb[tb.size() / 2];
    std::printf("{\"k\": %d, \"rows\": %d, \"B\": %u, \"S\": %zu, \"reps\": %d, \"tables_ms\": %.3f, \"rbs_ms\": %.3f, "
                "\"tables_GBps\": %.1f, \"rbs_GBps\": %.1f, \"rbs_over_tables\": %.4f, \"mismatched_words\": %llu}\n",
                k, rows, B, S, reps, ma, mb, bytes / ma / 1e6, bytes / mb / 1e6, mb / ma, bad);
    return bad ? 3 : 0;
}
