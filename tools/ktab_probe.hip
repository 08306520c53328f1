// ktab_probe.hip -- can a kernel read a stale pointer table through the scalar cache?
//
// The library's pointer-table path (rs_code_kernel<.., ADDR = 1, ..>) reads each stripe's shard
// pointers with scalar loads (as_const, constant address space) from a device table that the
// host rewrites before every call: hipMemcpyAsync(tab_dev, tab_host, H2D, s) then the launch on
// the same stream (runtime.hip Worker::upload_table, PtrLease::upload, the batcher's lanes).
// If the scalar cache of a CU kept the table's lines from an earlier launch, the kernel would
// dereference an earlier call's pointers -- memory that may be freed or unregistered since.
//
// This probe reproduces exactly that sequence without dereferencing anything: each launch
// compares every table entry it reads (scalar loads, every workgroup) with the value the host
// wrote for this launch and counts mismatches.  Patterns:
//   sync   : one stream; per iteration write host table, H2D copy, launch, stream sync
//   nosync : one stream, two host tables alternated, no sync between iterations
//   threads: T threads, each its own stream and table (the worker pool / batcher lanes)
// Output: one JSON line per pattern.  Any mismatch means the cache served stale table lines.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

using cu64 = const uint64_t __attribute__((address_space(4)))*;

// Every workgroup reads the whole table with scalar loads (uniform addresses) and compares.
__global__ __launch_bounds__(64) void probe(const uint64_t* tab, uint32_t n, uint64_t expect, uint32_t* bad,
                                            uint64_t* seen) {
    const cu64 t = (cu64)(uintptr_t)tab;
    uint32_t nb = 0;
    uint64_t first = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t v = t[i];
        if (v != expect + i) {
            if (!nb) first = v;
            ++nb;
        }
    }
    if (nb && threadIdx.x == 0) {
        atomicAdd(bad, nb);
        seen[0] = first;  // vector store: the last stale value any workgroup saw
    }
}

struct Lane {
    hipStream_t s;
    uint64_t* host[2];
    uint64_t* dev;
    uint32_t* bad;
    uint64_t* seen;
    hipEvent_t copied[2];
};

static void make_lane(Lane& l, uint32_t n) {
    CK(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking));
    for (auto& h : l.host) CK(hipHostMalloc(reinterpret_cast<void**>(&h), n * 8, hipHostMallocDefault));
    CK(hipMalloc(reinterpret_cast<void**>(&l.dev), n * 8));
    CK(hipMalloc(reinterpret_cast<void**>(&l.bad), 4));
    CK(hipMalloc(reinterpret_cast<void**>(&l.seen), 8));
    CK(hipMemset(l.bad, 0, 4));
    for (auto& e : l.copied) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
}

// One lane's iterations; returns mismatching entries observed.
static uint32_t run_lane(Lane& l, uint32_t n, int iters, int grid, bool sync, uint64_t tag0) {
    for (int it = 0; it < iters; ++it) {
        uint64_t* h = l.host[sync ? 0 : (it & 1)];
        if (!sync && it >= 2) CK(hipEventSynchronize(l.copied[it & 1]));  // its copy of iteration it-2 is done
        const uint64_t tag = tag0 + (static_cast<uint64_t>(it) << 20);
        for (uint32_t i = 0; i < n; ++i) h[i] = tag + i;
        CK(hipMemcpyAsync(l.dev, h, n * 8, hipMemcpyHostToDevice, l.s));
        if (!sync) CK(hipEventRecord(l.copied[it & 1], l.s));
        hipLaunchKernelGGL(probe, dim3(grid), dim3(64), 0, l.s, l.dev, n, tag, l.bad, l.seen);
        CK(hipGetLastError());
        if (sync) CK(hipStreamSynchronize(l.s));
    }
    CK(hipStreamSynchronize(l.s));
    uint32_t bad = 0;
    CK(hipMemcpy(&bad, l.bad, 4, hipMemcpyDeviceToHost));
    return bad;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const int grid = argc > 2 ? std::atoi(argv[2]) : 2048;
    const int nthreads = argc > 3 ? std::atoi(argv[3]) : 8;
    const uint32_t n = argc > 4 ? static_cast<uint32_t>(std::atoi(argv[4])) : 72;  // 8 stripes x 9 shards
    for (int pattern = 0; pattern < 3; ++pattern) {
        const char* name = pattern == 0 ? "sync" : pattern == 1 ? "nosync" : "threads";
        const int T = pattern == 2 ? nthreads : 1;
        std::vector<Lane> lanes(T);
        for (auto& l : lanes) make_lane(l, n);
        std::vector<uint32_t> bad(T, 0);
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] { bad[t] = run_lane(lanes[t], n, iters, grid, pattern != 1, uint64_t(t + 1) << 50); });
        for (auto& x : th) x.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t total = 0;
        for (uint32_t b : bad) total += b;
        std::printf("{\"pattern\": \"%s\", \"threads\": %d, \"iters\": %d, \"grid\": %d, \"entries\": %u, "
                    "\"launches\": %d, \"stale_entries_seen\": %llu, \"seconds\": %.2f}\n",
                    name, T, iters, grid, n, T * iters, static_cast<unsigned long long>(total), s);
        std::fflush(stdout);
        for (auto& l : lanes) {
            CK(hipStreamDestroy(l.s));
            for (auto& h : l.host) CK(hipHostFree(h));
            CK(hipFree(l.dev));
            CK(hipFree(l.bad));
            CK(hipFree(l.seen));
            for (auto& e : l.copied) CK(hipEventDestroy(e));
        }
    }
    return 0;
}
