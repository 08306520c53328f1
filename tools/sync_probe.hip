// sync_probe.hip -- where a small host call's ~20 us goes: launch, kernel, and the wait for it.
//
// Models the library's small staged call (blbrs.hip host_run, one unit): the CPU copies k = 6
// pageable inputs of S bytes into pinned, device-mapped staging, one kernel reads them in place
// over PCIe and writes one S-byte output into the staging, the CPU waits, then copies the output
// to a pageable buffer.  Only the wait differs between modes:
//   stream_sync   hipStreamSynchronize (the library's choice)
//   event_sync    hipEventRecord + hipEventSynchronize
//   stream_query  spin on hipStreamQuery
//   flag_spin     the kernel's last workgroup stores a sequence number to a coherent pinned word
//                 (release, system scope) after a device-scope completion count; the CPU spins on
//                 it (bounded: 1 s, then the run fails)
// Each mode runs `iters` calls per round, rounds interleave the modes; one JSON line per
// (S, mode) with p50/p99 of the whole call and of the launch API alone.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/sync_probe.hip -o tools/_build/sync_probe
// usage: sync_probe [iters rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::printf("{\"error\": \"%s at line %d\"}\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

constexpr int kK = 6;

struct Args {
    const uint4* in[kK];
    uint4* out;
    uint32_t* count;      // device memory, reset by the last workgroup
    uint32_t* host_flag;  // coherent pinned word (flag_spin), or null
    uint32_t seq;
    uint32_t n16;
};

__global__ __launch_bounds__(256) void xor_kernel(Args a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < a.n16) {
        uint4 v = a.in[0][i];
#pragma unroll
        for (int j = 1; j < kK; ++j) {
            const uint4 w = a.in[j][i];
            v.x ^= w.x;
            v.y ^= w.y;
            v.z ^= w.z;
            v.w ^= w.w;
        }
        a.out[i] = v;
    }
    if (!a.host_flag) return;
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t done = __hip_atomic_fetch_add(a.count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == gridDim.x - 1) {
            __hip_atomic_store(a.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.host_flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

using Clock = std::chrono::steady_clock;
static double us(Clock::time_point a, Clock::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const char* names[] = {"stream_sync", "event_sync", "stream_query", "flag_spin"};
    const size_t sizes[] = {4096, 65536, 262144};
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t* count = nullptr;
    CK(hipMalloc(&count, 4));
    CK(hipMemset(count, 0, 4));
    uint32_t* flag = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent | hipHostMallocMapped));
    *flag = 0;
    uint32_t* flag_dev = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&flag_dev), flag, 0));
    uint32_t seq = 0;
    {
        // hipPointerGetAttributes, which the library calls per touched shard (rt::device_view):
        // a pageable heap pointer (fails), a pinned one, a device one.
        std::vector<uint8_t> heap(1 << 16);
        void* dptr = nullptr;
        CK(hipMalloc(&dptr, 4096));
        const void* ptrs[3] = {heap.data() + 64, flag, dptr};
        const char* kinds[3] = {"pageable", "pinned", "device"};
        for (int kind = 0; kind < 3; ++kind) {
            std::vector<double> t;
            for (int it = 0; it < 20000; ++it) {
                hipPointerAttribute_t attr;
                const auto a0 = Clock::now();
                if (hipPointerGetAttributes(&attr, ptrs[kind]) != hipSuccess) (void)hipGetLastError();
                t.push_back(us(a0, Clock::now()));
            }
            std::sort(t.begin(), t.end());
            std::printf("{\"op\": \"hipPointerGetAttributes\", \"kind\": \"%s\", \"p50_us\": %.3f, \"p99_us\": %.3f}\n",
                        kinds[kind], t[t.size() / 2], t[t.size() * 99 / 100]);
        }
        CK(hipFree(dptr));
    }
    for (size_t S : sizes) {
        uint8_t* stage = nullptr;
        CK(hipHostMalloc(reinterpret_cast<void**>(&stage), (kK + 1) * S, hipHostMallocPortable | hipHostMallocMapped));
        uint8_t* stage_dev = nullptr;
        CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&stage_dev), stage, 0));
        std::vector<std::vector<uint8_t>> src(kK, std::vector<uint8_t>(S));
        for (int j = 0; j < kK; ++j)
            for (size_t b = 0; b < S; ++b) src[j][b] = static_cast<uint8_t>(b * 31 + j * 7 + 1);
        std::vector<uint8_t> want(S), got(S);
        for (size_t b = 0; b < S; ++b) {
            uint8_t x = 0;
            for (int j = 0; j < kK; ++j) x ^= src[j][b];
            want[b] = x;
        }
        Args a{};
        for (int j = 0; j < kK; ++j) a.in[j] = reinterpret_cast<const uint4*>(stage_dev + j * S);
        a.out = reinterpret_cast<uint4*>(stage_dev + kK * S);
        a.count = count;
        a.n16 = static_cast<uint32_t>(S / 16);
        const unsigned grid = static_cast<unsigned>((S / 16 + 255) / 256);
        std::vector<std::vector<double>> call(4), launch(4);
        long bad = 0;
        for (int r = 0; r < rounds + 1; ++r)  // round 0 warms up
            for (int m = 0; m < 4; ++m)
                for (int it = 0; it < iters; ++it) {
                    const auto t0 = Clock::now();
                    for (int j = 0; j < kK; ++j) std::memcpy(stage + j * S, src[j].data(), S);
                    a.host_flag = m == 3 ? flag_dev : nullptr;
                    a.seq = ++seq;
                    const auto t1 = Clock::now();
                    hipLaunchKernelGGL(xor_kernel, dim3(grid), dim3(256), 0, s, a);
                    const auto t2 = Clock::now();
                    if (m == 0) {
                        CK(hipStreamSynchronize(s));
                    } else if (m == 1) {
                        CK(hipEventRecord(ev, s));
                        CK(hipEventSynchronize(ev));
                    } else if (m == 2) {
                        hipError_t q;
                        while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
                        }
                        CK(q);
                    } else {
                        const auto lim = t2 + std::chrono::seconds(1);
                        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != a.seq)
                            if (Clock::now() > lim) {
                                std::printf("{\"error\": \"flag_spin timed out\", \"S\": %zu}\n", S);
                                CK(hipStreamSynchronize(s));
                                return 1;
                            }
                    }
                    std::memcpy(got.data(), stage + kK * S, S);
                    const auto t3 = Clock::now();
                    if (r > 0) {
                        call[m].push_back(us(t0, t3));
                        launch[m].push_back(us(t1, t2));
                    }
                    if (it == 0 && std::memcmp(got.data(), want.data(), S) != 0) ++bad;
                    std::memset(stage + kK * S, 0, 16);
                }
        CK(hipStreamSynchronize(s));
        for (int m = 0; m < 4; ++m) {
            auto& c = call[m];
            auto& l = launch[m];
            std::sort(c.begin(), c.end());
            std::sort(l.begin(), l.end());
            std::printf("{\"S\": %zu, \"mode\": \"%s\", \"calls\": %zu, \"call_p50_us\": %.2f, \"call_p99_us\": %.2f, "
                        "\"launch_p50_us\": %.2f, \"mismatched_rounds\": %ld}\n",
                        S, names[m], c.size(), c[c.size() / 2], c[c.size() * 99 / 100], l[l.size() / 2], bad);
        }
        std::fflush(stdout);
        CK(hipHostFree(stage));
    }
    CK(hipHostFree(flag));
    CK(hipFree(count));
    CK(hipEventDestroy(ev));
    CK(hipStreamDestroy(s));
    return 0;
}
