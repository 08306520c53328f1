// Host-call throughput through the C ABI, with and without the batcher.
//   reconstruct (default): client degraded reads -- T threads x R calls
//     of ReconstructData on RS(6,3) stripes of L-byte pinned pieces, one missing data shard, a
//     fresh encoder per call (client/blb/reconstruct.go:172);
//   rverify: the recovery RPCs' reconstructAndVerify (store.go:1132-1142), one data shard
//     missing, as reconstruct (the random bytes never verify; the work is the same);
//   encode: concurrent RSEncode RPCs (§8f row 1) -- T threads x R calls of Encode on RS(6,3)
//     stripes of L-byte pinned increments (store.go:1099; EncodeIncrementSize 4 MiB, 1 MiB in
//     tests), one encoder per RPC.
// No Python in the loop.
//   build: see tools/Makefile (target batch_bench); run: tools/_build/batch_bench [T] [R] [encode|rverify]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/blb_rs.h"

static void check(int rc, const char* what) {
    if (rc) {
        std::fprintf(stderr, "%s failed: %d %s\n", what, rc, blbrs_last_error());
        std::exit(1);
    }
}

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 64;
    const int R = argc > 2 ? std::atoi(argv[2]) : 50;
    const bool encode = argc > 3 && std::strcmp(argv[3], "encode") == 0;
    const bool rverify = argc > 3 && std::strcmp(argv[3], "rverify") == 0;  // reconstructAndVerify
    const int k = 6, m = 3, n = k + m;
    {  // cost of the per-shard pointer classification under T-way contention
        uint8_t* p = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), 1 << 20, hipHostMallocDefault) != hipSuccess) return 1;
        const int N = 20000;
        std::vector<std::thread> th;
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                hipPointerAttribute_t a;
                for (int i = 0; i < N; ++i) (void)hipPointerGetAttributes(&a, p + (t * 64 + i) % (1 << 20));
            });
        for (auto& x : th) x.join();
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("{\"probe\": \"hipPointerGetAttributes\", \"threads\": %d, \"calls_per_s\": %.0f}\n", T,
                    T * static_cast<double>(N) / el);
        (void)hipHostFree(p);
    }
    std::vector<size_t> lengths =
        encode ? std::vector<size_t>{size_t{64} << 10, size_t{256} << 10, size_t{1} << 20, size_t{4} << 20}
               : std::vector<size_t>{size_t{4} << 10, size_t{16} << 10, size_t{64} << 10, size_t{256} << 10, size_t{1} << 20};
    if (const char* e = std::getenv("BB_LENGTHS")) {  // e.g. "131072,262144"
        lengths.clear();
        for (const char* p = e; *p;) {
            char* end = nullptr;
            lengths.push_back(std::strtoull(p, &end, 0));
            p = *end == ',' ? end + 1 : end;
            if (end == p && *p) break;
        }
    }
    for (size_t L : lengths) {
        // Per-thread pinned stripe + output.
        std::vector<uint8_t*> bufs(static_cast<size_t>(T) * (n + 1));
        for (auto& p : bufs) {
            if (hipHostMalloc(reinterpret_cast<void**>(&p), L, hipHostMallocDefault) != hipSuccess) return 1;
            for (size_t i = 0; i < L; ++i) p[i] = static_cast<uint8_t>(std::rand());
        }
        for (int batched = 0; batched < 2; ++batched) {
            for (int window_us : batched ? std::vector<int>{0, 50, 200} : std::vector<int>{0}) {
                blbrs_batcher* b = nullptr;
                if (batched) check(blbrs_batcher_new(T, window_us, &b), "batcher_new");
                auto client = [&](int t, int reps) {
                    for (int r = 0; r < reps; ++r) {
                        blbrs_encoder* enc = nullptr;
                        check(blbrs_new(k, m, &enc), "new");
                        if (b) check(blbrs_encoder_set_batcher(enc, b), "set_batcher");
                        std::vector<uint8_t*> sh(n);
                        std::vector<size_t> lens(n, L);
                        for (int i = 0; i < n; ++i) sh[i] = bufs[static_cast<size_t>(t) * (n + 1) + i];
                        if (encode) {
                            check(blbrs_encode(enc, sh.data(), lens.data()), "encode");
                        } else if (rverify) {  // store.go:1132-1142; the bytes are random, so ok = 0
                            sh[1] = bufs[static_cast<size_t>(t) * (n + 1) + n];
                            lens[1] = 0;
                            int ok = 0;
                            check(blbrs_reconstruct_verify(enc, sh.data(), lens.data(), &ok), "reconstruct_verify");
                        } else {
                            sh[1] = bufs[static_cast<size_t>(t) * (n + 1) + n];  // output
                            lens[1] = 0;
                            check(blbrs_reconstruct_data(enc, sh.data(), lens.data()), "reconstruct_data");
                        }
                        blbrs_free(enc);
                    }
                };
                {  // warm plans and every thread's worker / staging before timing
                    std::vector<std::thread> w;
                    for (int t = 0; t < T; ++t) w.emplace_back(client, t, 2);
                    for (auto& x : w) x.join();
                }
                uint64_t r0 = 0, l0 = 0;
                if (b) check(blbrs_batcher_stats(b, &r0, &l0), "stats");
                std::vector<std::thread> th;
                const auto t0 = std::chrono::steady_clock::now();
                for (int t = 0; t < T; ++t) th.emplace_back(client, t, R);
                for (auto& x : th) x.join();
                const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                uint64_t r1 = 0, l1 = 0;
                if (b) check(blbrs_batcher_stats(b, &r1, &l1), "stats");
                const double calls = static_cast<double>(T) * R;
                std::printf("{\"op\": \"%s\", \"piece_bytes\": %zu, \"mode\": \"%s\", \"window_us\": %d, \"threads\": %d, "
                            "\"calls\": %.0f, \"calls_per_s\": %.0f, \"GiBps_data_read\": %.3f, \"us_per_call_latency\": %.1f, "
                            "\"calls_per_launch\": %.2f}\n",
                            encode ? "encode" : rverify ? "reconstruct_verify" : "reconstruct_data", L, batched ? "batched" : "per_call", window_us, T, calls,
                            calls / el,
                            calls * k * L / el / (1u << 30), el * 1e6 / R,
                            b ? static_cast<double>(r1 - r0) / static_cast<double>(l1 - l0 ? l1 - l0 : 1) : 1.0);
                std::fflush(stdout);
                if (b) blbrs_batcher_free(b);
            }
        }
        for (auto p : bufs) (void)hipHostFree(p);
    }
    return 0;
}
