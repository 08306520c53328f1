// Single-caller latency of blb's client degraded read (client/blb/reconstruct.go:65-195) through
// the C ABI, next to the CPU restatement (oracle/rs_oracle.c) -- no Python in the loop.
//
// blb serialises client reconstructs: defaultMaxReconstructInFlight = 1 (reconstruct.go:18-20,
// 35-45, 73-74), so what a reader sees is ONE call's latency.  Per read, the client does
//   enc, e := reedsolomon.New(n, m)          (reconstruct.go:166)
//   data[targetIdx] = thisB[0:0:length]      (the caller's pageable buffer, blob.go ReadAt)
//   enc.ReconstructData(data)                (k good replies in, 1.. missing data rows out)
// and the replies are RPC buffers: rpc.GetBuffer keeps pieces up to 128 KiB + ExtraRoom in plain
// (pageable) memory and pools larger ones (pkg/rpc/pool.go:28-43) -- pinned by the drop-in's pool
// (blbrs_buffer_get), so those are read in place.
//
// Timed per call, GPU: blbrs_new + blbrs_reconstruct_data + blbrs_free.  CPU (the restatement,
// klauspost@925cb01's algorithm): New's matrix (rso_build_matrix) + the sub-matrix inversion +
// the rows' multiply (rso_code, AVX2 as klauspost's galMulAVX2), on 1 thread and on T threads.
//
//   first call of an erasure pattern: 1 missing data piece, the k - 1 other data pieces + one
//     parity piece present, over every (target, parity) of blb's classes RS(6,3), RS(8,3),
//     RS(10,3), RS(12,5) (internal/core/StorageClass.go) = 132 patterns, each timed once on its
//     first call (host plan: inversion; device plan: table upload).  A 2-row call per class runs
//     first, so the process's one-time costs (stream worker, staging) are not in these numbers.
//   steady state: RS(6,3), target 1, parity 6 present, R calls.
// Every GPU result is compared with the CPU's bytes (outside the timed region).
//
// LAT_POOL_ALL=1: every reply is a pool buffer, whatever its size -- blb's rpc pool patched to
// pool requests of <= 128 KiB + ExtraRoom too (blbrs_buffer_get serves them from its small
// class), so small replies are read in place instead of staged.
//
//   usage: latency_bench SIZE [R] [T]     (one size per process: plans are per process)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include <sched.h>

#include "../../include/blb_rs.h"

extern "C" {
int rso_build_matrix(int k, int m, uint8_t* out);
int rso_invert(int n, const uint8_t* in, uint8_t* out);
void rso_code(const uint8_t* rows, int in_count, int out_count, const uint8_t* const* inputs, uint8_t* const* outputs,
              size_t n, int use_avx2, int threads);
int rso_encode(int k, int m, uint8_t* const* shards, const size_t* lens, int use_avx2, int threads);
}

namespace {

using Clock = std::chrono::steady_clock;

double us_since(Clock::time_point t0) { return std::chrono::duration<double, std::micro>(Clock::now() - t0).count(); }

void check(int rc, const char* what) {
    if (rc) {
        std::fprintf(stderr, "%s failed: %d %s\n", what, rc, blbrs_last_error());
        std::exit(1);
    }
}

constexpr size_t kSmallMax = (size_t{128} << 10) + (size_t{64} << 10);  // pool.go:31
const bool kPoolAll = [] {
    const char* e = std::getenv("LAT_POOL_ALL");
    return e && *e && *e != '0';
}();

// One stripe of class (k, m) at piece length L: pieces as blb's RPC layer hands them over.
struct Stripe {
    int k, m;
    size_t L;
    std::vector<uint8_t*> piece;  // k + m
    bool pooled;
    size_t cap = 0;               // bytes each piece holds (a pool class can exceed L)
    Stripe(int k_, int m_, size_t L_, std::mt19937_64& rng)
        : k(k_), m(m_), L(L_), piece(k_ + m_), pooled(kPoolAll || L_ > kSmallMax) {
        cap = (L + 63) / 64 * 64;
        for (auto& p : piece) {
            if (pooled) {
                check(blbrs_buffer_get(L, &p, &cap), "buffer_get");
            } else {
                p = static_cast<uint8_t*>(std::aligned_alloc(64, (L + 63) / 64 * 64));
            }
        }
        for (int i = 0; i < k; ++i)
            for (size_t b = 0; b < L; b += 8) {
                const uint64_t v = rng();
                std::memcpy(piece[i] + b, &v, std::min<size_t>(8, L - b));
            }
        std::vector<size_t> lens(k + m, L);
        if (rso_encode(k, m, piece.data(), lens.data(), 1, 1) != 0) std::exit(1);
    }
    ~Stripe() {
        for (auto p : piece) {
            if (pooled) (void)blbrs_buffer_put(p);
            else std::free(p);
        }
    }
};

// klauspost New + ReconstructData(shards) on the CPU for present = `present`, output = out.
void cpu_call(const Stripe& s, const std::vector<int>& present, int target, uint8_t* out, int threads) {
    const int k = s.k, m = s.m;
    std::vector<uint8_t> mat(static_cast<size_t>(k + m) * k);
    (void)rso_build_matrix(k, m, mat.data());  // New
    std::vector<int> valid;
    for (int i = 0; i < k + m && static_cast<int>(valid.size()) < k; ++i)
        if (std::find(present.begin(), present.end(), i) != present.end()) valid.push_back(i);
    std::vector<uint8_t> sub(static_cast<size_t>(k) * k), dec(static_cast<size_t>(k) * k);
    for (int r = 0; r < k; ++r) std::memcpy(&sub[static_cast<size_t>(r) * k], &mat[static_cast<size_t>(valid[r]) * k], k);
    (void)rso_invert(k, sub.data(), dec.data());
    std::vector<const uint8_t*> in(k);
    for (int r = 0; r < k; ++r) in[r] = s.piece[valid[r]];
    uint8_t* outs[1] = {out};
    rso_code(&dec[static_cast<size_t>(target) * k], k, 1, in.data(), outs, s.L, 1, threads);
}

// The drop-in's call: New + ReconstructData + (Go's GC of the encoder).
// Every other missing data slot gets `spare` (klauspost allocates one; the Go shim does the same).
double gpu_call(const Stripe& s, const std::vector<int>& present, int target, uint8_t* out, uint8_t* spare = nullptr) {
    const int n = s.k + s.m;
    std::vector<uint8_t*> sh(n, nullptr);
    std::vector<size_t> lens(n, 0);
    for (int i = 0; i < s.k; ++i) sh[i] = spare;
    for (int i : present) {
        sh[i] = s.piece[i];
        lens[i] = s.L;
    }
    sh[target] = out;  // thisB[0:0:length]: capacity, no length
    const auto t0 = Clock::now();
    blbrs_encoder* enc = nullptr;
    check(blbrs_new(s.k, s.m, &enc), "new");
    check(blbrs_reconstruct_data(enc, sh.data(), lens.data()), "reconstruct_data");
    blbrs_free(enc);
    return us_since(t0);
}

struct Dist {
    double p50, p99, mean, max;
    size_t n;
};
Dist dist(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    double sum = 0;
    for (double x : v) sum += x;
    auto at = [&](double q) { return v[std::min(v.size() - 1, static_cast<size_t>(q * (v.size() - 1) + 0.5))]; };
    return {at(0.5), at(0.99), sum / v.size(), v.back(), v.size()};
}

void print(const char* what, const char* side, int threads, size_t L, const Dist& d) {
    std::printf("{\"row\": \"%s\", \"side\": \"%s\", \"threads\": %d, \"piece_bytes\": %zu, \"calls\": %zu, "
                "\"p50_us\": %.1f, \"p99_us\": %.1f, \"mean_us\": %.1f, \"max_us\": %.1f}\n",
                what, side, threads, L, d.n, d.p50, d.p99, d.mean, d.max);
    std::fflush(stdout);
}

int job_threads() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) != 0) return 1;
    return std::min(CPU_COUNT(&set), 16);  // the GPU box gives a job 16 CPUs (its cgroup share)
}

}  // namespace

int main(int argc, char** argv) {
    const size_t L = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 4096;
    const int R = argc > 2 ? std::atoi(argv[2]) : 0;  // 0: as many as ~1.5 s allows (<= 5000)
    const int T = argc > 3 ? std::atoi(argv[3]) : job_threads();
    std::mt19937_64 rng(L * 7919 + 3);
    const int classes[][2] = {{6, 3}, {8, 3}, {10, 3}, {12, 5}};
    std::vector<uint8_t> out_gpu(L), out_cpu(L), spare(L);
    int bad = 0;

    // The process's first call (worker streams, pinned staging, tables of its pattern).
    {
        Stripe s(6, 3, L, rng);
        std::vector<int> present = {2, 3, 4, 5, 6, 7};
        std::vector<double> t = {gpu_call(s, present, 0, out_gpu.data(), spare.data())};
        print("process_first_call", "gpu", 0, L, dist(t));
    }

    // First call of each 1-row erasure pattern.
    std::vector<double> first_gpu, first_cpu1;
    for (const auto& c : classes) {
        const int k = c[0], m = c[1];
        Stripe s(k, m, L, rng);
        {  // class warm-up with a 2-row pattern outside the sample
            std::vector<int> present;
            for (int i = 2; i < k + 2; ++i) present.push_back(i);
            (void)gpu_call(s, present, 0, out_gpu.data(), spare.data());
        }
        for (int target = 0; target < k; ++target)
            for (int p = k; p < k + m; ++p) {
                std::vector<int> present;
                for (int i = 0; i < k; ++i)
                    if (i != target) present.push_back(i);
                present.push_back(p);
                std::memset(out_gpu.data(), 0xA5, L);
                first_gpu.push_back(gpu_call(s, present, target, out_gpu.data()));
                const auto t0 = Clock::now();
                cpu_call(s, present, target, out_cpu.data(), 1);
                first_cpu1.push_back(us_since(t0));
                if (std::memcmp(out_gpu.data(), s.piece[target], L) || std::memcmp(out_cpu.data(), s.piece[target], L))
                    ++bad;
            }
    }
    print("first_call_of_pattern", "gpu", 0, L, dist(first_gpu));
    print("first_call_of_pattern", "cpu", 1, L, dist(first_cpu1));

    // Steady state: one pattern, repeated.
    Stripe s(6, 3, L, rng);
    const std::vector<int> present = {0, 2, 3, 4, 5, 6};
    const int target = 1;
    int reps = R;
    if (reps <= 0) {
        const auto t0 = Clock::now();
        (void)gpu_call(s, present, target, out_gpu.data());
        const double one = std::max(1.0, us_since(t0));
        reps = static_cast<int>(std::clamp(1.5e6 / one, 50.0, 5000.0));
    }
    for (int threads : {0, 1, T}) {
        if (threads == T && T == 1) continue;
        std::vector<double> t;
        t.reserve(reps);
        for (int r = 0; r < std::min(reps, 10); ++r) {  // warm (page faults, OpenMP team)
            if (threads == 0) (void)gpu_call(s, present, target, out_gpu.data());
            else cpu_call(s, present, target, out_cpu.data(), threads);
        }
        for (int r = 0; r < reps; ++r) {
            if (threads == 0) {
                t.push_back(gpu_call(s, present, target, out_gpu.data()));
            } else {
                const auto t0 = Clock::now();
                cpu_call(s, present, target, out_cpu.data(), threads);
                t.push_back(us_since(t0));
            }
        }
        uint8_t* got = threads == 0 ? out_gpu.data() : out_cpu.data();
        if (std::memcmp(got, s.piece[target], L)) ++bad;
        print("steady_state", threads == 0 ? "gpu" : "cpu", threads, L, dist(t));
    }
    // Cold inputs: every call reads a stripe (and writes an output) last touched long before --
    // a ring of distinct stripes larger than the host's last-level cache, visited in order --
    // as replies fresh off the network are for the CPU's caches (round 6).
    // The steady-state rows above reuse one stripe, so the CPU side runs cache-hot there.
    {
        constexpr size_t kColdBytes = size_t{768} << 20;  // > the 256 MB L3 of the box's EPYC 9575F
        const size_t per = static_cast<size_t>(6 + 3) * s.cap + L;  // pieces as allocated + the output
        const int nring = static_cast<int>(std::clamp<size_t>(kColdBytes / per + 1, 8, 20000));
        std::vector<Stripe*> ring;
        std::vector<uint8_t*> outs;
        for (int i = 0; i < nring; ++i) {
            ring.push_back(new Stripe(6, 3, L, rng));
            outs.push_back(static_cast<uint8_t*>(std::aligned_alloc(64, (L + 63) / 64 * 64)));
            std::memset(outs.back(), 0, L);
        }
        const int creps = std::min(reps, 4 * nring);
        for (int side = 0; side < 2; ++side) {
            std::vector<double> t;
            t.reserve(creps);
            for (int r = 0; r < creps; ++r) {
                const Stripe& cs = *ring[r % nring];
                uint8_t* o = outs[r % nring];
                if (side == 0) {
                    t.push_back(gpu_call(cs, present, target, o));
                } else {
                    const auto t0 = Clock::now();
                    cpu_call(cs, present, target, o, 1);
                    t.push_back(us_since(t0));
                }
                if (r < nring && std::memcmp(o, cs.piece[target], L)) ++bad;
            }
            print("steady_state_cold_inputs", side == 0 ? "gpu" : "cpu", side == 0 ? 0 : 1, L, dist(t));
        }
        std::printf("{\"row\": \"cold_ring\", \"piece_bytes\": %zu, \"stripes\": %d, \"ring_bytes\": %zu}\n", L, nring,
                    static_cast<size_t>(nring) * per);
        for (auto* x : ring) delete x;
        for (auto* o : outs) std::free(o);
    }
    std::printf("{\"row\": \"check\", \"piece_bytes\": %zu, \"mismatches\": %d, \"inputs\": \"%s\"}\n", L, bad,
                s.pooled ? "pool (pinned)" : "pageable");
    return bad ? 2 : 0;
}
