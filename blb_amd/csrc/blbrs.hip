// blbrs.hip -- the C ABI (include/blb_rs.h) of the MI355X RS engine.
//
// What lives here (the kernels are in rs_kernels.hip, the per-device runtime in runtime.hip):
//   * reedsolomon.New equivalent: (k+m) x k matrix build (gf256.hpp), argument checks with
//     klauspost's error values, a device list per encoder.
//   * Coding plans: for each (operation, erasure pattern) the coefficient rows, their
//     v_perm lookup tables and shard index lists, uploaded once per device and cached on
//     the encoder -- the counterpart of klauspost's inversion tree (decode matrices
//     cached by invalid-index set) but holding device-ready tables.
//   * Host-memory Encoder methods (Encode / Verify / Reconstruct / ReconstructData) with
//     klauspost's shard conventions; each call runs on the least-loaded device of its
//     encoder on a leased stream worker, so concurrent callers (goroutines through cgo)
//     never share a stream and never depend on the calling thread's HIP device.
//   * Device-resident batched entry points (on the device owning the stripes, on caller
//     streams), multi-device parts, and the host-batch encoder split over the device list.
//   * The reconstruct batcher (client degraded reads).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/blb_rs.h"
#include "crc32c.hpp"
#include "encode_crc.hpp"
#include "gf256.hpp"
#include "gf_bitslice.hpp"
#include "pack.hpp"
#include "rs_kernels.hpp"
#include "rtc.hpp"
#include "runtime.hpp"
#include "tuning.hpp"

using namespace blbrs;
using rt::aligned16;
using rt::fail;
using rt::hip_fail;
using rt::round_up;

#define HIP_TRY(expr) BLBRS_HIP_TRY(expr)

// Host-side stage timing of one-stripe host calls, for measurement builds only
// (tools/host_timing.sh: -DBLBRS_HOST_TIMING; the library build compiles HT() to nothing).
// Marks: 0 blbrs_new entry, 1 its return, 2 the call's checks and plan lookup done, 3 the device
// and lane picked, 4 worker, device plans and shard classification done, 5 inputs staged and
// the table tagged, 6 launched, 7 the kernels' completion seen, 8 outputs copied out,
// 9 blbrs_free returned.  Per-stage medians go to stderr at exit.
#ifdef BLBRS_HOST_TIMING
namespace ht {
constexpr int kMarks = 10;
thread_local std::chrono::steady_clock::time_point g_t[kMarks];
thread_local int g_next = 0;
std::mutex g_mu;
std::vector<std::vector<double>> g_us(kMarks);
inline void mark(int i) {
    if (i == 0) g_next = 0;
    if (i != g_next) {  // out of order (another path): drop this call
        g_next = -1;
        return;
    }
    g_t[i] = std::chrono::steady_clock::now();
    g_next = i + 1;
    if (i == kMarks - 1) {
        std::lock_guard<std::mutex> g(g_mu);
        for (int j = 1; j < kMarks; ++j)
            g_us[j].push_back(std::chrono::duration<double, std::micro>(g_t[j] - g_t[j - 1]).count());
    }
}
struct Dump {
    ~Dump() {
        std::lock_guard<std::mutex> g(g_mu);
        std::fprintf(stderr, "{\"host_timing_us_p50\": [");
        for (int j = 1; j < kMarks; ++j) {
            auto v = g_us[j];
            std::sort(v.begin(), v.end());
            std::fprintf(stderr, "%s%.3f", j > 1 ? ", " : "", v.empty() ? -1.0 : v[v.size() / 2]);
        }
        std::fprintf(stderr, "], \"calls\": %zu}\n", g_us[1].size());
    }
} g_dump;
}  // namespace ht
#define HT(i) ht::mark(i)
#else
#define HT(i) ((void)0)
#endif

namespace {

// ---------------------------------------------------------------------------------------
// Coding plans
// ---------------------------------------------------------------------------------------

// One kernel pass: <= kMaxRows output rows over k_in inputs.
struct Pass {
    int k_in = 0, rows = 0;
    int nstore = -1;  // store+verify plans: rows [0, nstore) of this pass are stored
    bool parity = false;  // rows = encode parity rows 0..rows-1 of k_in (compiled network)
    std::vector<int32_t> in_idx, out_idx;
    std::vector<uint32_t> tables;
    Mat coef;  // rows x k_in coefficients (a run-time network is generated from them, rtc.hpp)
};

// Host description of an operation: rows x k_in coefficients, split into passes.
struct HostPlan {
    int k_in = 0;
    std::vector<int32_t> in_idx;   // inputs (shard indices)
    std::vector<int32_t> out_idx;  // outputs (shard indices), one per row
    Mat rows;                      // out_idx.size() x k_in
    int nstore = -1;               // store+verify plan: the first nstore rows are written, the
                                   // rest compared (-1: a plain store / verify plan)
    std::vector<Pass> passes;
};

void split_passes(HostPlan& p) {
    const int nrows = static_cast<int>(p.out_idx.size());
    for (int r0 = 0; r0 < nrows; r0 += kMaxRows) {
        Pass ps;
        ps.k_in = p.k_in;
        ps.rows = std::min(kMaxRows, nrows - r0);
        if (p.nstore >= 0) ps.nstore = std::max(0, std::min(ps.rows, p.nstore - r0));
        ps.in_idx = p.in_idx;
        ps.out_idx.assign(p.out_idx.begin() + r0, p.out_idx.begin() + r0 + ps.rows);
        Mat sub(p.rows.begin() + static_cast<size_t>(r0) * p.k_in,
                p.rows.begin() + static_cast<size_t>(r0 + ps.rows) * p.k_in);
        ps.tables = perm_tables(sub, ps.rows, p.k_in);
        ps.parity = bs::is_parity_rows(sub.data(), ps.rows, p.k_in);
        ps.coef = std::move(sub);
        p.passes.push_back(std::move(ps));
    }
}

// Device copy of a HostPlan on one device.
struct DevPass {
    void* mem = nullptr;
    const int32_t* in_idx = nullptr;
    const int32_t* out_idx = nullptr;
    const uint32_t* tables = nullptr;
    std::vector<int32_t> in_idx_h, out_idx_h;  // host copies (one-stripe small calls resolve entries)
    int k_in = 0, rows = 0;
    int nstore = -1;
    bool parity = false;
    Mat coef;
    std::shared_ptr<rtc::NetSlot> net;  // run-time network lookups of this pass (rtc.hpp)
};
struct DevPlan {
    std::vector<DevPass> passes;
    int device = -1;
    ~DevPlan() {
        rt::DeviceGuard g;
        if (g.enter(device) != BLBRS_OK) return;
        for (auto& p : passes)
            if (p.mem) (void)hipFree(p.mem);
    }
};

// Uploads on the current device (== device).
std::atomic<uint64_t> g_host_plans{0}, g_device_plans{0};  // blbrs_plan_stats

int upload(const HostPlan& hp, int device, std::unique_ptr<DevPlan>& out) {
    g_device_plans.fetch_add(1, std::memory_order_relaxed);
    auto dp = std::make_unique<DevPlan>();
    dp->device = device;
    for (const Pass& ps : hp.passes) {
        DevPass d;
        d.k_in = ps.k_in;
        d.rows = ps.rows;
        d.nstore = ps.nstore;
        d.parity = ps.parity;
        d.coef = ps.coef;
        d.in_idx_h = ps.in_idx;
        d.out_idx_h = ps.out_idx;
        d.net = std::make_shared<rtc::NetSlot>();
        const size_t n_in = ps.in_idx.size() * 4, n_out = round_up(ps.out_idx.size() * 4, 16);
        const size_t off_out = round_up(n_in, 16), off_tab = off_out + n_out;
        const size_t bytes = off_tab + ps.tables.size() * 4;
        std::vector<uint8_t> host(bytes, 0);
        std::memcpy(host.data(), ps.in_idx.data(), n_in);
        std::memcpy(host.data() + off_out, ps.out_idx.data(), ps.out_idx.size() * 4);
        std::memcpy(host.data() + off_tab, ps.tables.data(), ps.tables.size() * 4);
        HIP_TRY(hipMalloc(&d.mem, bytes));
        dp->passes.push_back(d);  // owned from here on (freed by ~DevPlan)
        HIP_TRY(rt::upload_pinned(d.mem, host.data(), bytes));
        auto* base = static_cast<uint8_t*>(d.mem);
        dp->passes.back().in_idx = reinterpret_cast<const int32_t*>(base);
        dp->passes.back().out_idx = reinterpret_cast<const int32_t*>(base + off_out);
        dp->passes.back().tables = reinterpret_cast<const uint32_t*>(base + off_tab);
    }
    out = std::move(dp);
    return BLBRS_OK;
}

// "E" = encode; "R" + ('d' data only | 'a' all | 'v' all + verify) + present bits.
std::string plan_key(bool encode, const std::vector<uint8_t>& present, bool data_only, bool verify = false) {
    if (encode) return "E";
    std::string key(present.size() + 2, '0');
    key[0] = 'R';
    key[1] = verify ? 'v' : data_only ? 'd' : 'a';
    for (size_t i = 0; i < present.size(); ++i) key[i + 2] = present[i] ? '1' : '0';
    return key;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Encoder
// ---------------------------------------------------------------------------------------

// Matrix and plan caches of one (k, m).  Shared by every blbrs_encoder handle with that
// shape: blb makes a fresh reedsolomon.New(n, m) per client reconstruct
// (client/blb/reconstruct.go:166), and a shared core keeps those calls from rebuilding
// and re-uploading plans -- and lets a batcher merge them.
struct EncoderCore {
    int k = 0, m = 0;
    Mat matrix;  // (k+m) x k systematic encoding matrix
    std::mutex mu;
    std::map<std::string, std::shared_ptr<HostPlan>> host_plans;
    std::map<std::pair<int, std::string>, std::unique_ptr<DevPlan>> dev_plans;

    // Encode / Verify: parity rows of M over the k data shards.
    std::shared_ptr<HostPlan> encode_plan() {
        std::lock_guard<std::mutex> g(mu);
        auto& slot = host_plans["E"];
        if (!slot) {
            auto p = std::make_shared<HostPlan>();
            p->k_in = k;
            for (int i = 0; i < k; ++i) p->in_idx.push_back(i);
            for (int i = 0; i < m; ++i) p->out_idx.push_back(k + i);
            p->rows.assign(matrix.begin() + static_cast<size_t>(k) * k, matrix.end());
            split_passes(*p);
            slot = p;
            g_host_plans.fetch_add(1, std::memory_order_relaxed);
        }
        return slot;
    }

    // Reconstruct(dataOnly): inputs = first k present shards ascending (klauspost
    // reedsolomon.go reconstruct), rows = inv(M[valid]) rows of missing data shards, then
    // (unless data_only) P[j] * inv(M[valid]) for missing parity j -- one pass produces
    // every missing shard straight from the k survivors.  Returns nullptr + rc on error.
    std::shared_ptr<HostPlan> decode_plan(const std::vector<uint8_t>& present, bool data_only, int* rc) {
        const std::string key = plan_key(false, present, data_only);
        std::lock_guard<std::mutex> g(mu);
        auto& slot = host_plans[key];
        if (slot) return slot;
        auto p = std::make_shared<HostPlan>();
        const int n = k + m;
        for (int i = 0; i < n && static_cast<int>(p->in_idx.size()) < k; ++i)
            if (present[i]) p->in_idx.push_back(i);
        Mat sub(static_cast<size_t>(k) * k), dec;
        for (int r = 0; r < k; ++r)
            std::memcpy(&sub[static_cast<size_t>(r) * k], &matrix[static_cast<size_t>(p->in_idx[r]) * k], k);
        if (!invert(sub, k, dec)) {
            host_plans.erase(key);
            *rc = fail(BLBRS_ERR_SINGULAR, "matrix is singular");
            return nullptr;
        }
        p->k_in = k;
        for (int i = 0; i < k; ++i)
            if (!present[i]) {
                p->out_idx.push_back(i);
                p->rows.insert(p->rows.end(), dec.begin() + static_cast<size_t>(i) * k,
                               dec.begin() + static_cast<size_t>(i + 1) * k);
            }
        if (!data_only)
            for (int i = k; i < n; ++i)
                if (!present[i]) {
                    Mat prow(matrix.begin() + static_cast<size_t>(i) * k,
                             matrix.begin() + static_cast<size_t>(i + 1) * k);
                    Mat r = matmul(prow, 1, k, dec, k);
                    p->out_idx.push_back(i);
                    p->rows.insert(p->rows.end(), r.begin(), r.end());
                }
        split_passes(*p);
        slot = p;
        g_host_plans.fetch_add(1, std::memory_order_relaxed);
        return slot;
    }

    // reconstructAndVerify in one pass (store.go:1132-1142): inputs = the first k present
    // shards, as for Reconstruct; rows = every missing shard (stored), then every present
    // shard the decode does not read (compared).  Verify after Reconstruct recomputes the
    // parity from the rebuilt data: the inputs and the rebuilt shards agree with it by
    // construction (M[valid] * inv(M[valid]) = I), so what it checks is exactly the present
    // shards outside the inputs -- all parity, since data shards come first.  k + m - k = m
    // rows: every shard is read or written once (k + m shard passes instead of 2k + m + e).
    std::shared_ptr<HostPlan> decode_verify_plan(const std::vector<uint8_t>& present, int* rc) {
        const std::string key = plan_key(false, present, false, true);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = host_plans.find(key);
            if (it != host_plans.end() && it->second) return it->second;
        }
        auto dp = decode_plan(present, false, rc);  // inputs, inverse, missing rows
        if (!dp) return nullptr;
        auto p = std::make_shared<HostPlan>();
        p->k_in = dp->k_in;
        p->in_idx = dp->in_idx;
        p->out_idx = dp->out_idx;
        p->rows = dp->rows;
        p->nstore = static_cast<int>(dp->out_idx.size());
        std::vector<uint8_t> is_in(k + m, 0);
        for (int32_t i : p->in_idx) is_in[i] = 1;
        // P[e] * inv(M[valid]) for the extra present shards: reuse the decode's inverse.
        Mat sub(static_cast<size_t>(k) * k), dec;
        for (int r = 0; r < k; ++r)
            std::memcpy(&sub[static_cast<size_t>(r) * k], &matrix[static_cast<size_t>(p->in_idx[r]) * k], k);
        if (!invert(sub, k, dec)) {
            *rc = fail(BLBRS_ERR_SINGULAR, "matrix is singular");
            return nullptr;
        }
        for (int i = 0; i < k + m; ++i)
            if (present[i] && !is_in[i]) {
                Mat row(matrix.begin() + static_cast<size_t>(i) * k, matrix.begin() + static_cast<size_t>(i + 1) * k);
                Mat r = matmul(row, 1, k, dec, k);
                p->out_idx.push_back(i);
                p->rows.insert(p->rows.end(), r.begin(), r.end());
            }
        split_passes(*p);
        std::lock_guard<std::mutex> g(mu);
        auto& slot = host_plans[key];
        if (!slot) {
            slot = p;
            g_host_plans.fetch_add(1, std::memory_order_relaxed);
        }
        return slot;
    }

    // Device tables for `hp` on `device` (uploaded on first use; the caller has made
    // `device` current).
    int dev_plan(const std::string& key, const HostPlan& hp, int device, const DevPlan** out) {
        std::lock_guard<std::mutex> g(mu);
        auto& slot = dev_plans[{device, key}];
        if (!slot) {
            int rc = upload(hp, device, slot);
            if (rc != BLBRS_OK) {
                dev_plans.erase({device, key});
                return rc;
            }
        }
        *out = slot.get();
        return BLBRS_OK;
    }
};

struct blbrs_encoder {
    std::shared_ptr<EncoderCore> core;
    int k = 0, m = 0;
    std::atomic<blbrs_batcher*> batcher{nullptr};  // routes host Encode / Reconstruct[Data] (blbrs_encoder_set_batcher)
    std::mutex dev_mu;
    std::vector<int> devices;   // explicit list, or empty until the default list is resolved
    bool resolved = false;
    std::atomic<unsigned> rr{0};

    std::shared_ptr<HostPlan> encode_plan() { return core->encode_plan(); }
    std::shared_ptr<HostPlan> decode_plan(const std::vector<uint8_t>& present, bool data_only, int* rc) {
        return core->decode_plan(present, data_only, rc);
    }
    std::shared_ptr<HostPlan> decode_verify_plan(const std::vector<uint8_t>& present, int* rc) {
        return core->decode_verify_plan(present, rc);
    }
    int dev_plan(const std::string& key, const HostPlan& hp, int device, const DevPlan** out) {
        return core->dev_plan(key, hp, device, out);
    }
    // The device list: explicit (checked once) or the process default (resolved once).
    int lanes(std::vector<int>* out) {
        std::lock_guard<std::mutex> g(dev_mu);
        if (!resolved) {
            int rc = devices.empty() ? rt::default_devices(&devices) : rt::check_devices(devices);
            if (rc) return rc;
            resolved = true;
        }
        *out = devices;
        return BLBRS_OK;
    }
};

namespace {

// Cores live for the process.  blb's client makes a reedsolomon.New per degraded read and drops
// it (client/blb/reconstruct.go:166); with cores owned by their handles, every such read freed
// the core, its device plans with it, and the next read inverted and uploaded its plan again
// (hipMalloc + hipMemcpy + hipFree per call, ~45 us of a 4 KiB read: profiles/r05/latency).
// Freeing device plans could also race a kernel still queued on a caller's stream by an
// asynchronous *_dev call whose encoder had just been dropped.  A process uses a handful of
// (k, m) classes, and a plan's device memory is a few KB.
std::mutex g_cores_mu;
std::map<std::pair<int, int>, std::shared_ptr<EncoderCore>>& cores() {
    static auto* m = new std::map<std::pair<int, int>, std::shared_ptr<EncoderCore>>();  // never destroyed
    return *m;
}

// The shared core for (k, m); nullptr when the matrix cannot be built.
std::shared_ptr<EncoderCore> core_for(int k, int m) {
    std::lock_guard<std::mutex> g(g_cores_mu);
    auto& c = cores()[{k, m}];
    if (c) return c;
    auto fresh = std::make_shared<EncoderCore>();
    fresh->k = k;
    fresh->m = m;
    if (!build_matrix(k, m, fresh->matrix)) {
        cores().erase({k, m});
        return nullptr;
    }
    c = fresh;
    return c;
}

// Addressing of one batch of stripes on the device.
struct Stripes {
    uint8_t* base = nullptr;  // strided form
    uint64_t shard_stride = 0, stripe_stride = 0;
    const uint64_t* ptrs = nullptr;  // device pointer table form
    const uint64_t* inl = nullptr;   //   or an inline table (host memory, copied into the launch)
    uint32_t ninline = 0;            //   of this many entries (<= kInlinePtrs)
    uint32_t nshards = 0;
    bool aligned = false;
    uint32_t tag = 0;                // the table's tag (rt::tag_entries)
    uint32_t* fault = nullptr;       //   and the record its launches report a wrong entry to
    // A small host call (store passes only): every pass on rs_small_kernel, the last one
    // publishing done_seq to done_word when that is set (rs_small.hpp).
    bool small = false;
    uint32_t* done_word = nullptr;
    uint32_t* done_count = nullptr;
    uint32_t done_seq = 0;
};

// Launch every pass of `plan` over `batch` stripes.
int run_plan(const DevPlan& plan, const Stripes& st, size_t batch, size_t S, Mode mode,
             int32_t* mismatch, hipStream_t stream) {
    if (batch == 0 || S == 0) return BLBRS_OK;
    if (batch > 0x7FFFFFFFull) return fail(BLBRS_ERR_INVALID_ARG, "batch too large");
    for (const DevPass& ps : plan.passes) {
        CodeArgs a{};
        a.tables = ps.tables;
        a.in_idx = ps.in_idx;
        a.out_idx = ps.out_idx;
        a.base = st.base;
        a.ptrs = st.ptrs;
        a.shard_stride = st.shard_stride;
        a.stripe_stride = st.stripe_stride;
        a.nshards = st.nshards;
        a.B = static_cast<uint32_t>(batch);
        a.S = S;
        a.k = ps.k_in;
        a.rows = ps.rows;
        a.aligned = st.aligned ? 1 : 0;
        a.mismatch = mismatch;
        a.parity = ps.parity ? 1 : 0;
        a.ptr_tag = st.tag;
        a.fault = st.fault;
        if (st.ninline) {
            if (st.ninline > static_cast<uint32_t>(kInlinePtrs)) return fail(BLBRS_ERR_INVALID_ARG, "inline table too long");
            std::memcpy(a.inl, st.inl, st.ninline * sizeof(uint64_t));
        }
        if (st.small && mode == Mode::kStore) {
            const bool last = &ps == &plan.passes.back();
            uint32_t* word = last ? st.done_word : nullptr;
            // One stripe with an inline table: the kernel gets the pass's entries resolved.
            hipError_t e = batch == 1 && st.ninline
                               ? launch_small1(a, ps.in_idx_h.data(), ps.out_idx_h.data(), word, st.done_count,
                                               st.done_seq, stream)
                               : hipErrorNotSupported;
            if (e == hipErrorNotSupported) e = launch_small(a, word, st.done_count, st.done_seq, stream);
            if (e != hipSuccess) return hip_fail(e, "launch rs_small_kernel");
            continue;
        }
        Mode m = mode;
        if (mode == Mode::kStoreVerify) {  // per pass: all stored, all compared, or mixed
            a.nstore = ps.nstore;
            m = ps.nstore == ps.rows ? Mode::kStore : ps.nstore == 0 ? Mode::kVerify : Mode::kStoreVerify;
        }
        // Wide passes the library has no compiled network for (decode rows; encode rows of k
        // outside the compiled list) take a network generated for their coefficients once it is
        // loaded; until then, and on failure, the table kernel.
        rtc::NetKernel* net = nullptr;
        const bool aot = bs::use(ps.parity, ps.k_in, ps.rows, bs::kWideCode);  // compiled encode network
        if (!aot && bs::mode() != 0 && rtc::eligible(ps.k_in, ps.rows)) {
            auto& slot = ps.net->k[static_cast<int>(m)][st.base ? 0 : 1];
            rtc::NetKernel* nk = slot.load(std::memory_order_acquire);
            if (!nk) {
                nk = rtc::request(plan.device, ps.k_in, ps.rows, m, st.base != nullptr, ps.coef.data());
                slot.store(nk, std::memory_order_release);
            }
            net = nk;
        }
        hipError_t e = launch_code(a, m, stream, net);
        if (e != hipSuccess) return hip_fail(e, "launch rs_code_kernel");
    }
    return BLBRS_OK;
}

// klauspost checkShards / shardSize.
int check_shards(int n, const size_t* lens, bool nilok, size_t* size) {
    size_t s = 0;
    for (int i = 0; i < n; ++i)
        if (lens[i]) { s = lens[i]; break; }
    if (s == 0) return fail(BLBRS_ERR_SHARD_NO_DATA, "no shard data");
    for (int i = 0; i < n; ++i)
        if (lens[i] != s && (lens[i] != 0 || !nilok)) return fail(BLBRS_ERR_SHARD_SIZE, "shard sizes do not match");
    *size = s;
    return BLBRS_OK;
}

// The device a device-resident call runs on: the owner of `p` when it is device memory,
// else the calling thread's current device (pinned host memory is mapped on every device).
int device_of(const void* p, int* dev) {
    int n = 0;
    int rc = rt::device_count(&n);
    if (rc) return rc;
    uint64_t view = 0;
    int owner = -1;
    if (p && rt::device_view(p, &view, &owner) && owner >= 0) {
        *dev = owner;
        return BLBRS_OK;
    }
    HIP_TRY(hipGetDevice(dev));
    return BLBRS_OK;
}

// One step of a host-memory call: a plan run in store or verify mode.
struct Step {
    std::string key;
    const HostPlan* hp;
    Mode mode;
};

// Host-memory coding of `batch` stripes (shards = batch x n pointers, stripe-major) on
// device `dev` (already current).  Steps run in order over each stripe, so a later step
// sees what an earlier one wrote (Reconstruct then Verify = reconstructAndVerify,
// store.go:1132-1142, in one device round trip).  Shards read by a step and not produced by
// an earlier step are copied in once; shards written by store steps are copied out.
// `known` (one stripe, optional): the caller's device views of the n shards (0 = pageable), so
// each shard's pointer attributes are looked up once per call.
int host_run(blbrs_encoder* enc, const std::vector<Step>& steps, uint8_t* const* shards, size_t batch, size_t S,
             int* ok, int dev, const uint64_t* known = nullptr) {
    rt::WorkerLease w;
    int rc = w.acquire(dev);
    if (rc) return rc;
    rt::note_call(dev);
    const int n = enc->k + enc->m;
    std::vector<const DevPlan*> plans(steps.size(), nullptr);
    std::vector<char> produced(n, 0), need_in(n, 0), is_out(n, 0), touched(n, 0);
    bool verify = false;
    for (size_t t = 0; t < steps.size(); ++t) {
        if ((rc = enc->dev_plan(steps[t].key, *steps[t].hp, dev, &plans[t]))) return rc;
        const HostPlan& hp = *steps[t].hp;
        for (int32_t i : hp.in_idx) {
            touched[i] = 1;
            if (!produced[i]) need_in[i] = 1;
        }
        for (size_t r = 0; r < hp.out_idx.size(); ++r) {
            const int32_t i = hp.out_idx[r];
            touched[i] = 1;
            const bool store = steps[t].mode == Mode::kStore ||
                               (steps[t].mode == Mode::kStoreVerify && static_cast<int>(r) < hp.nstore);
            if (store) {
                produced[i] = 1;
                is_out[i] = 1;
            } else {
                verify = true;
                if (!produced[i]) need_in[i] = 1;
            }
        }
    }
    auto drain = [&](int rc_) {
        (void)hipStreamSynchronize(w->s[0]);
        (void)hipStreamSynchronize(w->s[1]);
        return rc_;
    };
    // A single-launch call (the two forms below, or one unit of the slot pipeline) runs on the
    // small-call kernel and ends on its completion word when it is small and has no verify flag
    // to copy back; otherwise on a stream wait.
    size_t call_bytes = 0;
    for (int i = 0; i < n; ++i) call_bytes += touched[i] ? batch * S : 0;
    bool use_done =
        !verify && S <= rt::kDoneMaxPiece && call_bytes <= rt::kDoneMaxBytes && tune::get(tune::kDoneWord) != 0;
    if (use_done && w->ensure_done() != BLBRS_OK) use_done = false;  // no word to spin on: the stream wait
    auto launch_steps = [&](const Stripes& st, size_t nb, size_t len, int* rc_out) {
        *rc_out = BLBRS_OK;
        const uint32_t seq = use_done ? w->next_done_seq() : 0;
        for (size_t t = 0; t < steps.size(); ++t) {
            Stripes x = st;
            x.small = use_done;
            if (use_done && t + 1 == steps.size()) {
                x.done_word = w->done_dev;
                x.done_count = w->done_count;
                x.done_seq = seq;
            }
            if ((*rc_out = run_plan(*plans[t], x, nb, len, steps[t].mode, w->flag, w->s[0]))) return seq;
        }
        return seq;
    };
    // Per-slot addressing: device shards and pinned host shards are used in place (pinned ones
    // read and written by the kernels over PCIe, both link directions busy at once); only
    // pageable shards are staged.  blb's degraded read has k pool buffers in and the user's
    // pageable Blob.ReadAt buffer out (client/blb/reconstruct.go:172-173, blob.go:59): one staged
    // slot, not k + 1.  (Rounds 2-4 also staged pinned inputs of read-dominated calls by DMA when
    // more than 3 calls were in flight; that path went with the device staging)
    std::vector<uint64_t> view(batch * n, 0);
    std::vector<char> pageable(batch * n, 0);
    int max_staged = 0;  // staged touched slots of the worst stripe
    for (size_t b = 0; b < batch; ++b) {
        int ns = 0;
        for (int i = 0; i < n; ++i) {
            if (!touched[i]) continue;
            int owner = -1;
            const bool visible = known && batch == 1 ? (view[i] = known[i]) != 0
                                                     : rt::device_view(shards[b * n + i], &view[b * n + i], &owner);
            if (!visible) {
                pageable[b * n + i] = 1;
                ++ns;
            }
        }
        max_staged = std::max(max_staged, ns);
    }
    if (max_staged == 0) {
        // Everything in place: one launch per step over the whole batch.
        HT(4);
        Stripes st;
        st.nshards = n;
        st.fault = w->fault;
        uint64_t inl[kInlinePtrs];
        if (view.size() <= static_cast<size_t>(kInlinePtrs)) {  // one stripe: the table rides in the launch
            st.tag = rt::next_table_tag();
            if ((rc = rt::tag_entries(view.data(), view.size(), st.tag, inl, &st.aligned))) return rc;
            st.inl = inl;
            st.ninline = static_cast<uint32_t>(view.size());
        } else if ((rc = w->upload_table(view.data(), view.size(), &st.ptrs, &st.aligned, &st.tag))) {
            return drain(rc);
        }
        hipError_t e = hipSuccess;
        if (verify) e = hipMemsetAsync(w->flag, 0, sizeof(int32_t), w->s[0]);
        if (e != hipSuccess) return drain(hip_fail(e, "hipMemsetAsync"));
        HT(5);
        const uint32_t seq = launch_steps(st, batch, S, &rc);
        HT(6);
        if (rc) return drain(rc);
        if (use_done) {
            if ((rc = w->wait_done(seq))) return drain(rc);
        } else {
            if (verify && (rc = w->ensure_bounce(0))) return drain(rc);  // the pinned flag word
            if (verify) e = hipMemcpyAsync(w->flag_host, w->flag, sizeof(int32_t), hipMemcpyDeviceToHost, w->s[0]);
            const hipError_t f = hipStreamSynchronize(w->s[0]);
            if (e == hipSuccess) e = f;
            if (e != hipSuccess) return drain(hip_fail(e, "zero-copy call"));
        }
        HT(7);
        if ((rc = rt::check_fault(w->fault, "host call"))) return rc;
        if (ok) *ok = verify && *w->flag_host ? 0 : 1;
        HT(8);
        return BLBRS_OK;
    }
    // Pageable shards are never handed to HIP's copy engines: HIP pins pageable memory on the
    // fly for such copies, and the GPU suite's intermittent illegal-address fault appeared in
    // exactly that kind of copy after the tests that register, unregister and stage thousands
    // of heap buffers.  They go through the worker's pinned, device-mapped staging
    // instead: the CPU copies inputs in, the kernels read and write the staging in place, the
    // CPU copies outputs out.
    //
    // Small calls (one unit): blb's degraded read of a piece up to 128 KiB + ExtraRoom has its k
    // replies in plain memory (rpc.GetBuffer does not pool them, pkg/rpc/pool.go:31) and writes
    // the user's pageable buffer (client/blb/reconstruct.go:172-173): one launch per step, one
    // sync, and the tagged pointer table rides in the launch arguments (one stripe) or in the
    // staging (more).  DMA staging cost ~100 us per 4 KiB read.
    const bool inline_tab = batch * n <= static_cast<size_t>(kInlinePtrs);
    const size_t tab_bytes = inline_tab ? 0 : round_up(batch * n * sizeof(uint64_t), 256);
    size_t bounce_bytes = tab_bytes;
    const size_t Sb = round_up(S, 256);
    for (size_t x = 0; x < batch * n; ++x) bounce_bytes += pageable[x] ? Sb : 0;
    if (bounce_bytes <= rt::kBounceMaxBytes) {
        HT(4);
        if ((rc = w->ensure_bounce(bounce_bytes))) return rc;
        uint8_t* const hb = w->bounce;
        std::vector<size_t> at(batch * n, 0);
        size_t pos = tab_bytes;
        for (size_t b = 0; b < batch; ++b)
            for (int i = 0; i < n; ++i) {
                const size_t x = b * n + i;
                if (!touched[i] || !pageable[x]) continue;
                at[x] = pos;
                view[x] = w->bounce_dev + pos;
                if (need_in[i]) std::memcpy(hb + pos, shards[x], S);
                pos += Sb;
            }
        Stripes st;
        st.nshards = n;
        st.fault = w->fault;
        st.tag = rt::next_table_tag();
        uint64_t inl[kInlinePtrs];
        if ((rc = rt::tag_entries(view.data(), view.size(), st.tag, inline_tab ? inl : reinterpret_cast<uint64_t*>(hb),
                                  &st.aligned)))
            return rc;
        if (inline_tab) {
            st.inl = inl;
            st.ninline = static_cast<uint32_t>(view.size());
        } else {
            st.ptrs = reinterpret_cast<const uint64_t*>(w->bounce_dev);  // read over PCIe (rare: many stripes)
        }
        hipError_t e = hipSuccess;
        if (verify) e = hipMemsetAsync(w->flag, 0, sizeof(int32_t), w->s[0]);
        if (e != hipSuccess) return drain(hip_fail(e, "hipMemsetAsync"));
        HT(5);
        const uint32_t seq = launch_steps(st, batch, S, &rc);
        HT(6);
        if (rc) return drain(rc);
        if (use_done) {
            if ((rc = w->wait_done(seq))) return drain(rc);
        } else {
            if (verify) e = hipMemcpyAsync(w->flag_host, w->flag, sizeof(int32_t), hipMemcpyDeviceToHost, w->s[0]);
            const hipError_t f = hipStreamSynchronize(w->s[0]);
            if (e == hipSuccess) e = f;
            if (e != hipSuccess) return drain(hip_fail(e, "staged call"));
        }
        HT(7);
        if ((rc = rt::check_fault(w->fault, "host call"))) return rc;
        for (size_t b = 0; b < batch; ++b)
            for (int i = 0; i < n; ++i) {
                const size_t x = b * n + i;
                if (touched[i] && pageable[x] && is_out[i]) std::memcpy(shards[x], hb + at[x], S);
            }
        if (ok) *ok = verify && *w->flag_host ? 0 : 1;
        HT(8);
        return BLBRS_OK;
    }
    // Larger calls: units of (stripe, column chunk) alternate over two slots of the staging, in
    // order on s[0].  Before unit u fills its slot, the CPU waits for unit u - 2 (the slot's
    // previous user, event ev[slot]) and copies that unit's outputs out; so the CPU fills one slot
    // while the kernels work in the other.  A slot holds the unit's pageable shards (and, past
    // kInlinePtrs entries, its tagged table); the rest are addressed in place at the chunk's
    // column.  Staging per worker: 2 x kPinnedSlotBytes.
    //
    // A stripe is split into about kPipelineUnits column chunks of at least kMinUnitBytes (both
    // measured: 1 MiB as 4 x 256 KiB, 8 MiB as 8 x 1 MiB), so the
    // CPU's copies of one chunk overlap the kernels of the next even for a single stripe (blb's
    // degraded read: one 8 MiB piece copied out while the rest is still decoding).
    size_t chunk = S;
    const size_t slot_tab = n <= kInlinePtrs ? 0 : round_up(static_cast<size_t>(n) * sizeof(uint64_t), 256);
    if (slot_tab + static_cast<size_t>(max_staged) * Sb > rt::kPinnedSlotBytes)
        chunk = std::max<size_t>(4096, (rt::kPinnedSlotBytes - slot_tab) / max_staged / 4096 * 4096);
    constexpr size_t kPipelineUnits = 8, kMinUnitBytes = size_t{256} << 10;
    if (batch < kPipelineUnits && chunk > kMinUnitBytes) {
        const size_t want = batch * ((S + chunk - 1) / chunk) >= kPipelineUnits
                                ? chunk
                                : std::max(kMinUnitBytes, round_up((S + kPipelineUnits / batch - 1) / (kPipelineUnits / batch),
                                                                   size_t{64} << 10));
        chunk = std::min(chunk, want);
    }
    const size_t cp = round_up(chunk, 256);
    const size_t slot_bytes = slot_tab + static_cast<size_t>(max_staged) * cp;
    if ((rc = w->ensure_bounce(2 * slot_bytes))) return rc;
    if ((rc = w->ensure_events())) return rc;
    const size_t per_stripe = (S + chunk - 1) / chunk, units = batch * per_stripe;
    const bool one_done = use_done && units == 1;
    uint32_t done_seq = 0;
    hipError_t e = hipSuccess;
    if (verify) e = hipMemsetAsync(w->flag, 0, sizeof(int32_t), w->s[0]);
    if (e != hipSuccess) return drain(hip_fail(e, "hipMemsetAsync"));
    // Copies the outputs of unit u (finished) from its slot to the caller's pageable shards.
    auto copy_out = [&](size_t u) {
        const size_t b = u / per_stripe, off = (u % per_stripe) * chunk, len = std::min(chunk, S - off);
        const uint8_t* slot = w->bounce + (u & 1) * slot_bytes + slot_tab;
        for (int i = 0, r = 0; i < n; ++i) {
            if (!touched[i] || !pageable[b * n + i]) continue;
            if (is_out[i]) std::memcpy(shards[b * n + i] + off, slot + static_cast<size_t>(r) * cp, len);
            ++r;
        }
    };
    for (size_t u = 0; u < units; ++u) {
        const size_t b = u / per_stripe, off = (u % per_stripe) * chunk, len = std::min(chunk, S - off);
        const size_t sl = u & 1;
        if (u >= 2) {
            if ((e = hipEventSynchronize(w->ev[sl])) != hipSuccess) return drain(hip_fail(e, "staged call"));
            if ((rc = rt::check_fault(w->fault, "host call"))) return drain(rc);
            copy_out(u - 2);
        }
        uint8_t* const slot = w->bounce + sl * slot_bytes;
        const uint64_t slot_dev = w->bounce_dev + sl * slot_bytes;
        uint64_t entries[256];  // n <= 256 (blbrs_new)
        for (int i = 0, r = 0; i < n; ++i) {
            entries[i] = 0;
            if (!touched[i]) continue;
            if (pageable[b * n + i]) {
                const size_t at = slot_tab + static_cast<size_t>(r++) * cp;
                if (need_in[i]) std::memcpy(slot + at, shards[b * n + i] + off, len);
                entries[i] = slot_dev + at;
            } else {
                entries[i] = view[b * n + i] + off;
            }
        }
        Stripes st;
        st.nshards = n;
        st.fault = w->fault;
        st.tag = rt::next_table_tag();
        uint64_t inl[kInlinePtrs];
        if ((rc = rt::tag_entries(entries, n, st.tag, slot_tab ? reinterpret_cast<uint64_t*>(slot) : inl, &st.aligned)))
            return drain(rc);
        if (slot_tab) {
            st.ptrs = reinterpret_cast<const uint64_t*>(slot_dev);
        } else {
            st.inl = inl;
            st.ninline = static_cast<uint32_t>(n);
        }
        if (one_done) {  // a single unit: the small call's kernel and its completion word
            done_seq = launch_steps(st, 1, len, &rc);
            if (rc) return drain(rc);
            continue;
        }
        for (size_t t = 0; t < steps.size(); ++t)
            if ((rc = run_plan(*plans[t], st, 1, len, steps[t].mode, w->flag, w->s[0]))) return drain(rc);
        if ((e = hipEventRecord(w->ev[sl], w->s[0])) != hipSuccess) return drain(hip_fail(e, "staged call"));
    }
    if (verify) e = hipMemcpyAsync(w->flag_host, w->flag, sizeof(int32_t), hipMemcpyDeviceToHost, w->s[0]);
    if (e != hipSuccess) return drain(hip_fail(e, "staged call"));
    if (units >= 2) {  // the next-to-last unit's copy overlaps the last unit's kernels
        if ((e = hipEventSynchronize(w->ev[(units - 2) & 1])) != hipSuccess) return drain(hip_fail(e, "staged call"));
        if ((rc = rt::check_fault(w->fault, "host call"))) return drain(rc);
        copy_out(units - 2);
    }
    if (one_done) {
        if ((rc = w->wait_done(done_seq))) return drain(rc);
    } else if ((e = hipStreamSynchronize(w->s[0])) != hipSuccess) {
        return drain(hip_fail(e, "staged call"));
    }
    if ((rc = rt::check_fault(w->fault, "host call"))) return rc;
    copy_out(units - 1);
    if (ok) *ok = verify && *w->flag_host ? 0 : 1;
    return BLBRS_OK;
}

// A host-memory call: pick the device (the owner of any device-memory shard, else the
// least-loaded entry of the encoder's list), make it current for the call and run.
int host_call(blbrs_encoder* enc, const std::vector<Step>& steps, uint8_t* const* shards, size_t S, int* ok) {
    std::vector<int> lanes;
    int rc = enc->lanes(&lanes);
    if (rc) return rc;
    const int n = enc->k + enc->m;
    // Device-memory shards pin the call to their device; they must all be on one device
    // (a kernel dereferencing another GPU's HBM would need peer access).
    int dev = -1;
    uint64_t known[256] = {};  // n <= 256 (blbrs_new); 0 = pageable (or NULL)
    for (int i = 0; i < n; ++i) {
        int owner = -1;
        if (shards[i] && rt::device_view(shards[i], &known[i], &owner) && owner >= 0) {
            if (dev >= 0 && owner != dev) return fail(BLBRS_ERR_INVALID_ARG, "shards on different devices");
            dev = owner;
        }
    }
    int occ = 0;
    if (dev < 0) {
        // Host shards: prefer a GPU on the NUMA node holding them (pool and registered buffers
        // know their node; pageable memory gives no preference).
        int node = -1;
        for (int i = 0; i < n && node < 0; ++i)
            if (shards[i]) node = rt::host_numa_node(shards[i]);
        const size_t li = rt::pick_lane(lanes, enc->rr, node);
        dev = lanes[li];
        occ = rt::lane_keys(lanes)[li].second;
    }
    rt::LoadTicket ticket;
    ticket.take(dev, occ, static_cast<uint64_t>(n) * S);
    rt::DeviceGuard guard;
    if ((rc = guard.enter(dev))) return rc;
    HT(3);
    return host_run(enc, steps, shards, 1, S, ok, dev, known);
}

std::vector<uint8_t> present_vec(const blbrs_encoder* enc, const uint8_t* present) {
    std::vector<uint8_t> p(enc->k + enc->m);
    for (int i = 0; i < enc->k + enc->m; ++i) p[i] = present[i] ? 1 : 0;
    return p;
}

// ---- batched host calls ----
//
// client/blb/reconstruct.go:65-195 calls ReconstructData once per degraded read, on one
// stripe of `length`-byte pieces; MaxInFlight (:19,35-45) lets many run at once.  The
// tractserver runs one RSEncode per control RPC (up to RejectCtlReqThreshold = 1000 at once,
// internal/tractserver/config.go:91), each an Encode per 4 MiB increment (store.go:1099).
// Alone, each call is a launch plus a stream round trip for a few KiB..MiB of work.  A batcher
// collects the calls that arrive within `window_us` (or until `max_batch` are waiting) and
// runs them as ONE launch per (shape, erasure pattern, length) group over a device pointer
// table, with one stream sync for the whole batch.  Each device has a queue drained by two
// lanes (own stream and table each): while one lane's batch runs and syncs, the other
// collects the next -- the batches pipeline.  Shards in pinned or device memory are used in
// place; pageable shards are staged by the CALLING thread through a pooled pinned buffer.
struct BatchReq {
    EncoderCore* core = nullptr;
    std::shared_ptr<HostPlan> hp;   // store step (encode / decode plan); null = verify only
    std::shared_ptr<HostPlan> vp;   // verify step after it (the encode plan); null = none
    bool mixed = false;             // hp is a store+verify plan (reconstructAndVerify, one pass)
    std::string key;                // group key: plan key, "+V" when verifying
    int ok = 0;                     // verify result (vp set or mixed)
    std::vector<uint64_t> views;  // device-visible address per shard slot (0 = unused)
    size_t S = 0;
    int dev = -1;                 // device that must run it (device-memory shards), -1 = any
    std::chrono::steady_clock::time_point arrival;
    int rc = BLBRS_OK;
    std::string msg;              // error text, re-raised on the caller's thread
    // Completion: per request, so a finished batch wakes only its own callers (a shared
    // condition variable woke every waiting caller on every batch and serialised them on the
    // queue mutex: 64 callers of 64 KiB pieces ran at 77k calls/s against 96k per call).
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
};

}  // namespace

struct blbrs_batcher {
    struct Queue {
        std::deque<BatchReq*> q;
        std::condition_variable cv;
    };
    struct Lane {
        int device = 0;
        hipStream_t stream = nullptr;
        uint64_t* tab_host = nullptr;
        uint64_t* tab_dev = nullptr;
        size_t tab_cap = 0;
        int32_t* flags_host = nullptr;  // per-stripe Verify mismatch flags
        int32_t* flags_dev = nullptr;
        size_t flags_cap = 0;
        uint32_t* fault = nullptr;      // pinned record of the lane's table checks
        std::thread th;
    };
    size_t max_batch = 64;
    std::chrono::microseconds window{200};
    std::vector<int> devices;  // distinct devices
    std::mutex mu;
    std::map<int, Queue> queues;
    std::vector<std::unique_ptr<Lane>> lanes;
    std::atomic<unsigned> rr{0};
    bool stop = false;
    std::atomic<uint64_t> launches{0}, requests{0};

    void run(Lane* lane) {
        rt::DeviceGuard guard;
        if (guard.enter(lane->device) != BLBRS_OK) return;
        Queue& qu = queues[lane->device];
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            qu.cv.wait(lk, [&] { return stop || !qu.q.empty(); });
            if (qu.q.empty()) return;  // stop requested and nothing left
            const auto deadline = qu.q.front()->arrival + window;
            qu.cv.wait_until(lk, deadline, [&] { return stop || qu.q.size() >= max_batch; });
            if (qu.q.empty()) continue;  // the other lane took them
            std::vector<BatchReq*> batch;
            while (!qu.q.empty() && batch.size() < max_batch) {
                batch.push_back(qu.q.front());
                qu.q.pop_front();
            }
            if (!qu.q.empty()) qu.cv.notify_one();
            lk.unlock();
            process(lane, batch);
            for (BatchReq* r : batch) {
                // Notify under the request's lock: once it is released the caller may return
                // and destroy the request.
                std::lock_guard<std::mutex> g(r->m);
                r->done = true;
                r->cv.notify_one();
            }
            lk.lock();
        }
    }

    int upload(Lane* lane, const std::vector<uint64_t>& table, const uint64_t** dev_out, bool* aligned, uint32_t* tag) {
        if (table.size() > lane->tab_cap) {
            if (lane->tab_host) (void)hipHostFree(lane->tab_host);
            if (lane->tab_dev) (void)hipFree(lane->tab_dev);
            lane->tab_host = nullptr;
            lane->tab_dev = nullptr;
            lane->tab_cap = 0;
            const size_t cap = std::max<size_t>(table.size(), 1024);
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&lane->tab_host), cap * 8, hipHostMallocDefault));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&lane->tab_dev), cap * 8));
            lane->tab_cap = cap;
        }
        *tag = rt::next_table_tag();
        if (int rc = rt::tag_entries(table.data(), table.size(), *tag, lane->tab_host, aligned)) return rc;
        HIP_TRY(hipMemcpyAsync(lane->tab_dev, lane->tab_host, table.size() * 8, hipMemcpyHostToDevice, lane->stream));
        *dev_out = lane->tab_dev;
        return BLBRS_OK;
    }

    int flags(Lane* lane, size_t count) {
        if (count > lane->flags_cap) {
            if (lane->flags_host) (void)hipHostFree(lane->flags_host);
            if (lane->flags_dev) (void)hipFree(lane->flags_dev);
            lane->flags_host = nullptr;
            lane->flags_dev = nullptr;
            lane->flags_cap = 0;
            const size_t cap = std::max<size_t>(count, 256);
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&lane->flags_host), cap * 4, hipHostMallocDefault));
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&lane->flags_dev), cap * 4));
            lane->flags_cap = cap;
        }
        HIP_TRY(hipMemsetAsync(lane->flags_dev, 0, count * 4, lane->stream));
        return BLBRS_OK;
    }

    void process(Lane* lane, std::vector<BatchReq*>& batch) {
        // Handles of one (k, m) share a core, so calls from different encoders merge.  The
        // groups share the lane's table, so they run one after the other.  A group runs its
        // store step (encode / decode) and then, for Verify / ReconstructAndVerify, the encode
        // plan in verify mode over the same table: per-stripe mismatch flags come back with
        // the one sync (store.go:1132-1142 in one round trip for the whole group).
        std::map<std::tuple<EncoderCore*, std::string, size_t>, std::vector<BatchReq*>> groups;
        for (BatchReq* r : batch) groups[{r->core, r->key, r->S}].push_back(r);
        rt::LoadTicket ticket;
        ticket.take(lane->device);
        for (auto& [gk, reqs] : groups) {
            EncoderCore* core = std::get<0>(gk);
            const size_t S = std::get<2>(gk), n = static_cast<size_t>(core->k + core->m);
            const BatchReq& r0 = *reqs[0];
            const std::string plan_key_ = std::get<1>(gk).substr(0, std::get<1>(gk).size() - (r0.vp ? 2 : 0));
            const DevPlan* plan = nullptr;
            const DevPlan* vplan = nullptr;
            int rc = BLBRS_OK;
            if (r0.hp) rc = core->dev_plan(plan_key_, *r0.hp, lane->device, &plan);
            if (rc == BLBRS_OK && r0.vp) rc = core->dev_plan("E", *r0.vp, lane->device, &vplan);
            if (rc == BLBRS_OK) {
                std::vector<uint64_t> table(reqs.size() * n);
                for (size_t j = 0; j < reqs.size(); ++j)
                    std::copy(reqs[j]->views.begin(), reqs[j]->views.end(), table.begin() + j * n);
                Stripes st;
                st.nshards = static_cast<uint32_t>(n);
                st.fault = lane->fault;
                rc = upload(lane, table, &st.ptrs, &st.aligned, &st.tag);
                if (rc == BLBRS_OK && plan && r0.mixed) {
                    rc = flags(lane, reqs.size());
                    if (rc == BLBRS_OK)
                        rc = run_plan(*plan, st, reqs.size(), S, Mode::kStoreVerify, lane->flags_dev, lane->stream);
                    if (rc == BLBRS_OK) {
                        const hipError_t e = hipMemcpyAsync(lane->flags_host, lane->flags_dev, reqs.size() * 4,
                                                            hipMemcpyDeviceToHost, lane->stream);
                        if (e != hipSuccess) rc = hip_fail(e, "batched verify flags");
                    }
                } else if (rc == BLBRS_OK && plan) {
                    rc = run_plan(*plan, st, reqs.size(), S, Mode::kStore, nullptr, lane->stream);
                }
                if (rc == BLBRS_OK && vplan) {
                    rc = flags(lane, reqs.size());
                    if (rc == BLBRS_OK)
                        rc = run_plan(*vplan, st, reqs.size(), S, Mode::kVerify, lane->flags_dev, lane->stream);
                    if (rc == BLBRS_OK) {
                        const hipError_t e = hipMemcpyAsync(lane->flags_host, lane->flags_dev, reqs.size() * 4,
                                                            hipMemcpyDeviceToHost, lane->stream);
                        if (e != hipSuccess) rc = hip_fail(e, "batched verify flags");
                    }
                }
                if (rc == BLBRS_OK) launches.fetch_add(1);
                // The table is rewritten by the next group: wait for this one's launches.
                const hipError_t e = hipStreamSynchronize(lane->stream);
                if (rc == BLBRS_OK && e != hipSuccess) rc = hip_fail(e, "batched call");
                if (rc == BLBRS_OK) rc = rt::check_fault(lane->fault, "batched call");
            }
            for (size_t j = 0; j < reqs.size(); ++j) {
                BatchReq* r = reqs[j];
                r->rc = rc;
                if (rc != BLBRS_OK) r->msg = rt::last_error();
                else if (r->vp || r->mixed) r->ok = lane->flags_host[j] == 0;
            }
        }
        requests.fetch_add(batch.size());
    }

    // Queue `r` (mu held): on its required device, else the device with the shortest queue.
    void enqueue(BatchReq* r) {
        int dev = r->dev;  // batched_call has checked that a required device has a queue
        if (dev < 0) {
            const size_t start = rr.fetch_add(1) % devices.size();
            dev = devices[start];
            size_t best = queues[dev].q.size();
            for (size_t j = 1; j < devices.size(); ++j) {
                const int d = devices[(start + j) % devices.size()];
                if (queues[d].q.size() < best) {
                    best = queues[d].q.size();
                    dev = d;
                }
            }
        }
        Queue& qu = queues[dev];
        qu.q.push_back(r);
        if (qu.q.size() == 1 || qu.q.size() >= max_batch) qu.cv.notify_one();
    }

    void shutdown() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            for (auto& [d, qu] : queues) qu.cv.notify_all();
        }
        for (auto& l : lanes)
            if (l->th.joinable()) l->th.join();  // drains the queues first
        for (auto& l : lanes) {
            rt::DeviceGuard guard;
            if (guard.enter(l->device) != BLBRS_OK) continue;
            if (l->stream) (void)hipStreamDestroy(l->stream);
            if (l->tab_host) (void)hipHostFree(l->tab_host);
            if (l->tab_dev) (void)hipFree(l->tab_dev);
            if (l->flags_host) (void)hipHostFree(l->flags_host);
            if (l->flags_dev) (void)hipFree(l->flags_dev);
            if (l->fault) (void)hipHostFree(l->fault);
        }
    }
};

namespace {

// The host Encode / Reconstruct / ReconstructData of one stripe through `b` (blocking).  `hp`
// is the encode or decode plan (at least one output), `key` its cache key; argument checks
// have been done.
int batched_call(blbrs_batcher* b, blbrs_encoder* enc, const std::string& key, std::shared_ptr<HostPlan> hp,
                 std::shared_ptr<HostPlan> vp, uint8_t* const* shards, size_t S, int* ok, bool mixed = false) {
    const int n = enc->k + enc->m;
    BatchReq req;
    req.core = enc->core.get();
    req.hp = hp;
    req.vp = vp;
    req.mixed = mixed;
    req.key = vp ? key + "+V" : key;
    req.S = S;
    req.views.assign(n, 0);
    // Slots the steps touch; the store step's outputs are written, every other slot is read.
    // Pageable slots get a staging slot: read ones are copied in, written ones copied out.
    std::vector<char> touched(n, 0), written(n, 0);
    if (hp) {
        for (int32_t i : hp->in_idx) touched[i] = 1;
        for (size_t r = 0; r < hp->out_idx.size(); ++r) {
            touched[hp->out_idx[r]] = 1;
            if (!mixed || static_cast<int>(r) < hp->nstore) written[hp->out_idx[r]] = 1;
        }
    }
    if (vp) {
        for (int32_t i : vp->in_idx) touched[i] = 1;
        for (int32_t i : vp->out_idx) touched[i] = 1;
    }
    const size_t Sp = round_up(S, 256);
    size_t nstaged = 0;
    std::vector<int> slot(n, -1);
    for (int i = 0; i < n; ++i) {
        if (!touched[i]) continue;
        int owner = -1;
        if (!rt::device_view(shards[i], &req.views[i], &owner)) {
            slot[i] = static_cast<int>(nstaged++);
        } else if (owner >= 0) {
            if (req.dev >= 0 && req.dev != owner)
                return fail(BLBRS_ERR_INVALID_ARG, "shards on different devices");
            req.dev = owner;
        }
    }
    struct Staging {
        uint8_t* p = nullptr;
        ~Staging() {
            if (p) (void)rt::pool_put(p);
        }
    } stage;
    if (nstaged) {
        size_t cap = 0;
        int rc = rt::pool_get(nstaged * Sp, &stage.p, &cap, /*internal=*/true);
        if (rc) return rc;
        for (int i = 0; i < n; ++i) {
            if (slot[i] < 0) continue;
            uint8_t* p = stage.p + static_cast<size_t>(slot[i]) * Sp;
            if (!written[i]) std::memcpy(p, shards[i], S);
            if (!rt::device_view(p, &req.views[i])) return fail(BLBRS_ERR_HIP, "pinned staging has no device mapping");
        }
    }
    if (req.dev >= 0 && !b->queues.count(req.dev))  // queues is fixed after make_batcher
        return fail(BLBRS_ERR_INVALID_ARG, "shards live on device " + std::to_string(req.dev) +
                                               ", which is not in the batcher's device list");
    req.arrival = std::chrono::steady_clock::now();
    {
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->stop) return fail(BLBRS_ERR_INVALID_ARG, "batcher is shutting down");
        b->enqueue(&req);
    }
    {
        std::unique_lock<std::mutex> lk(req.m);
        req.cv.wait(lk, [&] { return req.done; });
    }
    if (req.rc != BLBRS_OK) return fail(req.rc, req.msg);
    for (int i = 0; i < n; ++i)
        if (written[i] && slot[i] >= 0) std::memcpy(shards[i], stage.p + static_cast<size_t>(slot[i]) * Sp, S);
    if (ok) *ok = req.ok;
    return BLBRS_OK;
}

int make_batcher(int max_batch, int window_us, std::vector<int> devs, blbrs_batcher** out) {
    std::sort(devs.begin(), devs.end());
    devs.erase(std::unique(devs.begin(), devs.end()), devs.end());
    auto* b = new blbrs_batcher();
    b->max_batch = static_cast<size_t>(max_batch);
    b->window = std::chrono::microseconds(window_us);
    b->devices = devs;
    // Launch lanes per device queue (default 2: one batch collects while the previous runs);
    // $BLBRS_BATCH_LANES = 1..8 overrides it (tuning).
    int nlanes = 2;
    if (const char* env = std::getenv("BLBRS_BATCH_LANES"); env && *env) nlanes = std::min(8, std::max(1, std::atoi(env)));
    for (int d : devs) {
        b->queues[d];
        for (int j = 0; j < nlanes; ++j) {
            auto lane = std::make_unique<blbrs_batcher::Lane>();
            lane->device = d;
            rt::DeviceGuard guard;
            int rc = guard.enter(d);
            hipError_t e = hipSuccess;
            if (rc == BLBRS_OK) e = hipStreamCreateWithFlags(&lane->stream, hipStreamNonBlocking);
            if (rc == BLBRS_OK && e == hipSuccess) rc = rt::alloc_fault_record(&lane->fault);
            if (rc != BLBRS_OK || e != hipSuccess) {
                b->shutdown();
                delete b;
                return rc ? rc : hip_fail(e, "hipStreamCreate");
            }
            b->lanes.push_back(std::move(lane));
        }
    }
    for (auto& l : b->lanes) {
        blbrs_batcher::Lane* lp = l.get();
        l->th = std::thread([b, lp] { b->run(lp); });
    }
    *out = b;
    return BLBRS_OK;
}

// Device-resident calls: the stripes' owner device, current for the call.
struct DevCall {
    rt::DeviceGuard guard;
    int dev = 0;
    int enter(const void* p) {
        int rc = device_of(p, &dev);
        if (rc) return rc;
        return guard.enter(dev);
    }
};

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

static int new_encoder(int data_shards, int parity_shards, std::vector<int> devices, blbrs_encoder** out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (data_shards <= 0 || parity_shards <= 0)
        return fail(BLBRS_ERR_INV_SHARD_NUM, "cannot create Encoder with zero or less data/parity shards");
    if (data_shards + parity_shards > 256)
        return fail(BLBRS_ERR_MAX_SHARD_NUM, "cannot create Encoder with more than 256 data+parity shards");
    auto core = core_for(data_shards, parity_shards);
    if (!core) return fail(BLBRS_ERR_SINGULAR, "matrix is singular");
    auto* e = new blbrs_encoder();
    e->core = std::move(core);
    e->k = data_shards;
    e->m = parity_shards;
    e->devices = std::move(devices);
    *out = e;
    return BLBRS_OK;
}

int blbrs_new(int data_shards, int parity_shards, blbrs_encoder** out) {
    HT(0);
    const int rc = new_encoder(data_shards, parity_shards, {}, out);
    HT(1);
    return rc;
}

int blbrs_new_on(int data_shards, int parity_shards, const int* devices, int ndevices, blbrs_encoder** out) {
    if (out) *out = nullptr;
    if (!devices || ndevices <= 0) return fail(BLBRS_ERR_INVALID_ARG, "empty device list");
    std::vector<int> devs(devices, devices + ndevices);
    for (int d : devs)
        if (d < 0) return fail(BLBRS_ERR_INVALID_ARG, "negative device id");
    return new_encoder(data_shards, parity_shards, std::move(devs), out);
}

int blbrs_encoder_devices(blbrs_encoder* enc, int* out, int cap, int* n) {
    if (!enc || !n || (cap > 0 && !out)) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    std::vector<int> lanes;
    int rc = enc->lanes(&lanes);
    if (rc) return rc;
    *n = static_cast<int>(lanes.size());
    for (int i = 0; i < cap && i < *n; ++i) out[i] = lanes[i];
    return BLBRS_OK;
}

int blbrs_encoder_lane_stats(blbrs_encoder* enc, int lane, blbrs_lane_stats* out) {
    if (!enc || !out || lane < 0) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    std::vector<int> lanes;
    int rc = enc->lanes(&lanes);
    if (rc) return rc;
    if (static_cast<size_t>(lane) >= lanes.size()) return fail(BLBRS_ERR_INVALID_ARG, "lane out of range");
    const auto key = rt::lane_keys(lanes)[lane];
    return rt::lane_stats(key.first, key.second, out);
}

int blbrs_set_default_devices(const int* devices, int ndevices) {
    if (ndevices < 0 || (ndevices > 0 && !devices)) return fail(BLBRS_ERR_INVALID_ARG, "bad device list");
    return rt::set_default_devices(std::vector<int>(devices, devices + ndevices));
}

void blbrs_free(blbrs_encoder* enc) {
    delete enc;
    HT(9);
}
int blbrs_data_shards(const blbrs_encoder* enc) { return enc ? enc->k : 0; }
int blbrs_parity_shards(const blbrs_encoder* enc) { return enc ? enc->m : 0; }

int blbrs_encoder_compiled_network(const blbrs_encoder* enc) {
    if (!enc) return 0;
    const auto hp = enc->core->encode_plan();
    int code = 1, tile = 1, pack = 1, rtc_net = 1;
    for (const Pass& ps : hp->passes) {
        code &= bs::use(ps.parity, ps.k_in, ps.rows, bs::kWideCode) ? 1 : 0;
        tile &= bs::use(ps.parity, ps.k_in, ps.rows, bs::kWideTile) ? 1 : 0;
        pack &= bs::use(ps.parity, ps.k_in, ps.rows, bs::kWidePack) ? 1 : 0;
        rtc_net &= !bs::use(ps.parity, ps.k_in, ps.rows, bs::kWideCode) && bs::mode() != 0 &&
                   rtc::eligible(ps.k_in, ps.rows) ? 1 : 0;
    }
    return (code ? BLBRS_NET_CODE : 0) | (tile ? BLBRS_NET_TILE : 0) | (pack ? BLBRS_NET_PACK : 0) |
           (rtc_net ? BLBRS_NET_RTC : 0);
}

int blbrs_device_numa_node(int device, int* node) {
    if (!node || device < 0) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    *node = rt::device_numa_node(device);
    return BLBRS_OK;
}

int blbrs_set_device_numa_node(int device, int node) { return rt::set_device_numa_node(device, node); }

int blbrs_host_numa_node(const void* p, int* node) {
    if (!node) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    *node = rt::host_numa_node(p);
    return BLBRS_OK;
}

int blbrs_lane_policy(const int* nodes, const int64_t* loads, size_t n, size_t start, int node, size_t* lane) {
    if (!nodes || !loads || !lane || n == 0 || start >= n) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    *lane = rt::pick_lane_policy(nodes, loads, n, start, node);
    return BLBRS_OK;
}

int blbrs_rtc_get_stats(blbrs_rtc_stats* out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    const rtc::Stats s = rtc::stats();
    out->requested = s.requested;
    out->compiled = s.compiled;
    out->loaded = s.loaded;
    out->failed = s.failed;
    out->pending = s.pending;
    out->compile_ms = s.compile_ms;
    return BLBRS_OK;
}

int blbrs_rtc_compile(int k, int rows, const uint8_t* coef, int mode, int strided, void* code, size_t cap,
                      size_t* len) {
    if (k < 1 || k > 16 || rows < 1 || rows > kMaxRows || !coef || mode < 0 || mode > 2)
        return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    std::string log;
    std::vector<char> obj;
    if (!rtc::compile_only(k, rows, static_cast<Mode>(mode), strided != 0, coef, &log, &obj))
        return fail(BLBRS_ERR_HIP, "hipRTC: " + log.substr(0, 2000));
    if (len) *len = obj.size();
    if (code) {
        if (cap < obj.size()) return fail(BLBRS_ERR_INVALID_ARG, "code buffer too small");
        std::memcpy(code, obj.data(), obj.size());
    }
    return BLBRS_OK;
}

int blbrs_rtc_wait(long timeout_ms) {
    return rtc::wait_idle(timeout_ms) ? BLBRS_OK : fail(BLBRS_ERR_LIMIT, "run-time networks still compiling");
}

int blbrs_rtc_network_source(int k, int rows, const uint8_t* coef, char* out, size_t cap, int* ops) {
    if (k < 1 || rows < 1 || k > 256 || rows > 256 || !coef || !out) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    int n = 0;
    const std::string src = rtc::network_source(k, rows, coef, &n);
    if (src.size() + 1 > cap) return fail(BLBRS_ERR_INVALID_ARG, "buffer too small");
    std::memcpy(out, src.c_str(), src.size() + 1);
    if (ops) *ops = n;
    return BLBRS_OK;
}

int blbrs_matrix(const blbrs_encoder* enc, uint8_t* out, size_t cap) {
    if (!enc || !out) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    const Mat& mat = enc->core->matrix;
    if (cap < mat.size()) return fail(BLBRS_ERR_INVALID_ARG, "buffer too small");
    std::memcpy(out, mat.data(), mat.size());
    return BLBRS_OK;
}

int blbrs_encode(blbrs_encoder* enc, uint8_t* const* shards, const size_t* lens) {
    if (!enc || !shards || !lens) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    const int n = enc->k + enc->m;
    size_t S = 0;
    int rc = check_shards(n, lens, false, &S);
    if (rc) return rc;
    for (int i = 0; i < n; ++i)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    auto hp = enc->encode_plan();
    if (blbrs_batcher* b = enc->batcher.load()) return batched_call(b, enc, "E", hp, nullptr, shards, S, nullptr);
    return host_call(enc, {Step{"E", hp.get(), Mode::kStore}}, shards, S, nullptr);
}

int blbrs_verify(blbrs_encoder* enc, const uint8_t* const* shards, const size_t* lens, int* ok) {
    if (!enc || !shards || !lens || !ok) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    const int n = enc->k + enc->m;
    size_t S = 0;
    int rc = check_shards(n, lens, false, &S);
    if (rc) return rc;
    for (int i = 0; i < n; ++i)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    auto hp = enc->encode_plan();
    if (blbrs_batcher* b = enc->batcher.load())
        return batched_call(b, enc, "V", nullptr, hp, const_cast<uint8_t* const*>(shards), S, ok);
    return host_call(enc, {Step{"E", hp.get(), Mode::kVerify}}, const_cast<uint8_t* const*>(shards), S, ok);
}

static int reconstruct_host(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens, bool data_only,
                            int* verify_ok) {
    if (!enc || !shards || !lens) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    const int n = enc->k + enc->m;
    size_t S = 0;
    int rc = check_shards(n, lens, true, &S);
    if (rc) return rc;
    std::vector<uint8_t> present(n);
    int npresent = 0;
    for (int i = 0; i < n; ++i) {
        present[i] = lens[i] != 0;
        npresent += present[i];
    }
    auto ep = enc->encode_plan();
    blbrs_batcher* b = enc->batcher.load();
    if (npresent == n) {  // nothing to rebuild; reconstructAndVerify still verifies
        if (!verify_ok) return BLBRS_OK;
        for (int i = 0; i < n; ++i)
            if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
        if (b) return batched_call(b, enc, "V", nullptr, ep, shards, S, verify_ok);
        return host_call(enc, {Step{"E", ep.get(), Mode::kVerify}}, shards, S, verify_ok);
    }
    if (npresent < enc->k) return fail(BLBRS_ERR_TOO_FEW_SHARDS, "too few shards given");
    auto hp = enc->decode_plan(present, data_only, &rc);
    if (!hp) return rc;
    for (int32_t i : hp->in_idx)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    for (int32_t i : hp->out_idx)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "missing shard has no output buffer");
    // reconstructAndVerify: one pass that writes the missing shards and compares the present
    // shards the decode does not read (EncoderCore::decode_verify_plan).
    std::shared_ptr<HostPlan> vp;
    if (verify_ok && !hp->out_idx.empty()) {
        vp = enc->decode_verify_plan(present, &rc);
        if (!vp) return rc;
        for (int32_t i : vp->out_idx)
            if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    }
    if (b && !hp->out_idx.empty()) {
        rc = vp ? batched_call(b, enc, plan_key(false, present, false, true), vp, nullptr, shards, S, verify_ok, true)
                : batched_call(b, enc, plan_key(false, present, data_only), hp, nullptr, shards, S, nullptr);
        if (rc) return rc;
        for (int32_t i : hp->out_idx) lens[i] = S;
        return BLBRS_OK;
    }
    std::vector<Step> steps;
    if (vp) steps.push_back(Step{plan_key(false, present, false, true), vp.get(), Mode::kStoreVerify});
    else if (!hp->out_idx.empty()) steps.push_back(Step{plan_key(false, present, data_only), hp.get(), Mode::kStore});
    else if (verify_ok) steps.push_back(Step{"E", ep.get(), Mode::kVerify});
    if (steps.empty()) return BLBRS_OK;  // data_only with only parity missing
    HT(2);
    rc = host_call(enc, steps, shards, S, verify_ok);
    if (rc) return rc;
    for (int32_t i : hp->out_idx) lens[i] = S;
    return BLBRS_OK;
}

int blbrs_reconstruct(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens) {
    return reconstruct_host(enc, shards, lens, false, nullptr);
}

int blbrs_reconstruct_data(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens) {
    return reconstruct_host(enc, shards, lens, true, nullptr);
}

int blbrs_reconstruct_verify(blbrs_encoder* enc, uint8_t* const* shards, size_t* lens, int* ok) {
    if (!ok) return fail(BLBRS_ERR_INVALID_ARG, "ok is NULL");
    *ok = 0;
    return reconstruct_host(enc, shards, lens, false, ok);
}

// ---- device-resident batched path ----

static int dev_stripes_strided(uint8_t* stripes, size_t shard_stride, size_t stripe_stride, size_t batch,
                               size_t shard_len, Stripes* st) {
    if (!stripes) return fail(BLBRS_ERR_INVALID_ARG, "stripes is NULL");
    if (shard_stride < shard_len || (batch > 1 && stripe_stride < shard_len))
        return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than shard length");
    st->base = stripes;
    st->shard_stride = shard_stride;
    st->stripe_stride = stripe_stride;
    st->aligned = aligned16(reinterpret_cast<uintptr_t>(stripes)) && aligned16(shard_stride) &&
                  aligned16(stripe_stride);
    return BLBRS_OK;
}

// Runs `hp` on the current device `dev`.
static int dev_run(blbrs_encoder* enc, int dev, const std::string& key, const HostPlan& hp, const Stripes& st,
                   size_t batch, size_t S, Mode mode, int32_t* mismatch, void* stream) {
    const DevPlan* plan = nullptr;
    int rc = enc->dev_plan(key, hp, dev, &plan);
    if (rc) return rc;
    return run_plan(*plan, st, batch, S, mode, mismatch, static_cast<hipStream_t>(stream));
}

int blbrs_encode_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                     size_t batch, size_t shard_len, void* stream) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    Stripes st;
    int rc = dev_stripes_strided(stripes, shard_stride, stripe_stride, batch, shard_len, &st);
    if (rc) return rc;
    DevCall dc;
    if ((rc = dc.enter(stripes))) return rc;
    auto hp = enc->encode_plan();
    return dev_run(enc, dc.dev, "E", *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

// A caller's device pointer table, tagged; its launches report to the device's record (the call
// is asynchronous: blbrs_table_fault_take reads it once the caller's stream has run).
static int upload_ptrs(uint8_t* const* ptrs, size_t count, hipStream_t stream, rt::PtrLease& lease, int dev,
                       Stripes* st) {
    std::vector<uint64_t> v(count);
    for (size_t i = 0; i < count; ++i) {
        if (!ptrs[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
        v[i] = reinterpret_cast<uint64_t>(ptrs[i]);
    }
    st->fault = rt::device_fault_record(dev);
    if (!st->fault) return fail(BLBRS_ERR_HIP, "no fault record for device " + std::to_string(dev));
    return lease.upload(v.data(), count, stream, &st->ptrs, &st->aligned, &st->tag);
}

int blbrs_encode_dev_ptrs(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                          void* stream) {
    if (!enc || !shard_ptrs) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    const int n = enc->k + enc->m;
    DevCall dc;
    int rc = dc.enter(shard_ptrs[0]);
    if (rc) return rc;
    rt::PtrLease lease;
    Stripes st;
    if ((rc = upload_ptrs(shard_ptrs, batch * n, static_cast<hipStream_t>(stream), lease, dc.dev, &st)))
        return rc;
    st.nshards = n;
    auto hp = enc->encode_plan();
    return dev_run(enc, dc.dev, "E", *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

static int dev_decode_plan(blbrs_encoder* enc, const uint8_t* present, int data_only,
                           std::shared_ptr<HostPlan>* hp, std::string* key, bool* nothing) {
    if (!present) return fail(BLBRS_ERR_INVALID_ARG, "present is NULL");
    auto pv = present_vec(enc, present);
    int np = 0;
    for (uint8_t p : pv) np += p;
    *nothing = false;
    if (np == enc->k + enc->m) { *nothing = true; return BLBRS_OK; }
    if (np < enc->k) return fail(BLBRS_ERR_TOO_FEW_SHARDS, "too few shards given");
    int rc = BLBRS_OK;
    *hp = enc->decode_plan(pv, data_only != 0, &rc);
    if (!*hp) return rc;
    if ((*hp)->out_idx.empty()) *nothing = true;
    *key = plan_key(false, pv, data_only != 0);
    return BLBRS_OK;
}

int blbrs_reconstruct_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                          size_t batch, size_t shard_len, const uint8_t* present, int data_only, void* stream) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    std::shared_ptr<HostPlan> hp;
    std::string key;
    bool nothing = false;
    int rc = dev_decode_plan(enc, present, data_only, &hp, &key, &nothing);
    if (rc || nothing || batch == 0 || shard_len == 0) return rc;
    Stripes st;
    if ((rc = dev_stripes_strided(stripes, shard_stride, stripe_stride, batch, shard_len, &st))) return rc;
    DevCall dc;
    if ((rc = dc.enter(stripes))) return rc;
    return dev_run(enc, dc.dev, key, *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

int blbrs_reconstruct_dev_ptrs(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                               const uint8_t* present, int data_only, void* stream) {
    if (!enc || !shard_ptrs) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    std::shared_ptr<HostPlan> hp;
    std::string key;
    bool nothing = false;
    int rc = dev_decode_plan(enc, present, data_only, &hp, &key, &nothing);
    if (rc || nothing || batch == 0 || shard_len == 0) return rc;
    const int n = enc->k + enc->m;
    DevCall dc;
    if ((rc = dc.enter(shard_ptrs[hp->in_idx[0]]))) return rc;
    rt::PtrLease lease;
    Stripes st;
    if ((rc = upload_ptrs(shard_ptrs, batch * n, static_cast<hipStream_t>(stream), lease, dc.dev, &st)))
        return rc;
    st.nshards = n;
    return dev_run(enc, dc.dev, key, *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

int blbrs_verify_dev(blbrs_encoder* enc, const uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                     size_t batch, size_t shard_len, int32_t* mismatch_dev, void* stream) {
    if (!enc || !mismatch_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0) return BLBRS_OK;
    DevCall dc;
    int rc = dc.enter(mismatch_dev);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(mismatch_dev, 0, batch * sizeof(int32_t), static_cast<hipStream_t>(stream)));
    if (shard_len == 0) return BLBRS_OK;
    Stripes st;
    if ((rc = dev_stripes_strided(const_cast<uint8_t*>(stripes), shard_stride, stripe_stride, batch, shard_len,
                                  &st)))
        return rc;
    auto hp = enc->encode_plan();
    return dev_run(enc, dc.dev, "E", *hp, st, batch, shard_len, Mode::kVerify, mismatch_dev, stream);
}

int blbrs_reconstruct_verify_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                                 size_t batch, size_t shard_len, const uint8_t* present, int32_t* mismatch_dev,
                                 void* stream) {
    if (!enc || !mismatch_dev || !present) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    auto pv = present_vec(enc, present);
    int np = 0;
    for (uint8_t x : pv) np += x;
    if (np == enc->k + enc->m)  // nothing to rebuild: reconstructAndVerify is a Verify
        return blbrs_verify_dev(enc, stripes, shard_stride, stripe_stride, batch, shard_len, mismatch_dev, stream);
    if (np < enc->k) return fail(BLBRS_ERR_TOO_FEW_SHARDS, "too few shards given");
    if (batch == 0) return BLBRS_OK;
    DevCall dc;
    int rc = dc.enter(mismatch_dev);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(mismatch_dev, 0, batch * sizeof(int32_t), static_cast<hipStream_t>(stream)));
    if (shard_len == 0) return BLBRS_OK;
    auto vp = enc->decode_verify_plan(pv, &rc);
    if (!vp) return rc;
    Stripes st;
    if ((rc = dev_stripes_strided(stripes, shard_stride, stripe_stride, batch, shard_len, &st))) return rc;
    return dev_run(enc, dc.dev, plan_key(false, pv, false, true), *vp, st, batch, shard_len, Mode::kStoreVerify,
                   mismatch_dev, stream);
}

int blbrs_verify_dev_ptrs(blbrs_encoder* enc, const uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                          int32_t* mismatch_dev, void* stream) {
    if (!enc || !shard_ptrs || !mismatch_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0) return BLBRS_OK;
    DevCall dc;
    int rc = dc.enter(mismatch_dev);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(mismatch_dev, 0, batch * sizeof(int32_t), static_cast<hipStream_t>(stream)));
    if (shard_len == 0) return BLBRS_OK;
    const int n = enc->k + enc->m;
    rt::PtrLease lease;
    Stripes st;
    if ((rc = upload_ptrs(const_cast<uint8_t* const*>(shard_ptrs), batch * n, static_cast<hipStream_t>(stream),
                          lease, dc.dev, &st)))
        return rc;
    st.nshards = n;
    auto hp = enc->encode_plan();
    return dev_run(enc, dc.dev, "E", *hp, st, batch, shard_len, Mode::kVerify, mismatch_dev, stream);
}

// ---- multi-device parts ----

static int check_parts(const blbrs_dev_part* parts, size_t nparts, size_t shard_len) {
    if (nparts && !parts) return fail(BLBRS_ERR_INVALID_ARG, "parts is NULL");
    for (size_t p = 0; p < nparts; ++p) {
        if (parts[p].batch == 0) continue;
        Stripes st;
        int rc = dev_stripes_strided(parts[p].stripes, parts[p].shard_stride, parts[p].stripe_stride, parts[p].batch,
                                     shard_len, &st);
        if (rc) return fail(rc, "part " + std::to_string(p) + ": " + rt::last_error());
    }
    return BLBRS_OK;
}

int blbrs_encode_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    int rc = check_parts(parts, nparts, shard_len);
    if (rc || shard_len == 0) return rc;
    for (size_t p = 0; p < nparts; ++p) {
        const blbrs_dev_part& x = parts[p];
        if (!x.batch) continue;
        if ((rc = blbrs_encode_dev(enc, x.stripes, x.shard_stride, x.stripe_stride, x.batch, shard_len, x.stream)))
            return fail(rc, "part " + std::to_string(p) + ": " + rt::last_error());
    }
    return BLBRS_OK;
}

int blbrs_reconstruct_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len,
                            const uint8_t* present, int data_only) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    int rc = check_parts(parts, nparts, shard_len);
    if (rc) return rc;
    std::shared_ptr<HostPlan> hp;
    std::string key;
    bool nothing = false;
    if ((rc = dev_decode_plan(enc, present, data_only, &hp, &key, &nothing)) || nothing || shard_len == 0) return rc;
    for (size_t p = 0; p < nparts; ++p) {
        const blbrs_dev_part& x = parts[p];
        if (!x.batch) continue;
        if ((rc = blbrs_reconstruct_dev(enc, x.stripes, x.shard_stride, x.stripe_stride, x.batch, shard_len, present,
                                        data_only, x.stream)))
            return fail(rc, "part " + std::to_string(p) + ": " + rt::last_error());
    }
    return BLBRS_OK;
}

int blbrs_verify_parts(blbrs_encoder* enc, const blbrs_dev_part* parts, size_t nparts, size_t shard_len,
                       int32_t* const* mismatch_dev) {
    if (!enc || (nparts && !mismatch_dev)) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    int rc = check_parts(parts, nparts, shard_len);
    if (rc) return rc;
    for (size_t p = 0; p < nparts; ++p) {
        const blbrs_dev_part& x = parts[p];
        if (!x.batch) continue;
        if ((rc = blbrs_verify_dev(enc, x.stripes, x.shard_stride, x.stripe_stride, x.batch, shard_len,
                                   mismatch_dev[p], x.stream)))
            return fail(rc, "part " + std::to_string(p) + ": " + rt::last_error());
    }
    return BLBRS_OK;
}

// ---- streaming host path ----

// The copy-engine form of BASELINE config 5 (nstreams >= 1): pinned host stripes -> a device ring
// -> host parity.  Stripe b goes to slot b % R on stream b % R: hipMemcpyAsync of its k data
// shards into the slot, rs_code_kernel over the slot (strided, device-resident), hipMemcpyAsync
// of its m parity shards back.  One stream per slot keeps a slot's reuse in order, and R streams
// overlap the H2D, kernel and D2H of consecutive stripes (PCIe is full duplex).  Every shard is
// pinned, device-visible host memory: the library never hands HIP a pageable range to copy
// (DESIGN §4h); the caller checked.
static int dma_run(blbrs_encoder* enc, const HostPlan& hp, uint8_t* const* shards, size_t batch, size_t S, int dev,
                   int nstreams) {
    const int k = enc->k, n = enc->k + enc->m;
    const DevPlan* plan = nullptr;
    int rc = enc->dev_plan("E", hp, dev, &plan);
    if (rc) return rc;
    const int R = std::max(1, std::min(nstreams, 8));
    const size_t pitch = round_up(S, 256), slot = pitch * n;
    std::vector<hipStream_t> s(R, nullptr);
    uint8_t* ring = nullptr;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&ring), slot * static_cast<size_t>(std::min<size_t>(R, batch)));
    for (int i = 0; i < R && e == hipSuccess; ++i) e = hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    for (size_t b = 0; b < batch && e == hipSuccess; ++b) {
        const int r = static_cast<int>(b % R);
        uint8_t* base = ring + static_cast<size_t>(r) * slot;
        for (int i = 0; i < k && e == hipSuccess; ++i)
            e = hipMemcpyAsync(base + static_cast<size_t>(i) * pitch, shards[b * n + i], S, hipMemcpyHostToDevice, s[r]);
        if (e != hipSuccess) break;
        Stripes st;
        st.base = base;
        st.shard_stride = pitch;
        st.stripe_stride = slot;
        st.nshards = static_cast<uint32_t>(n);
        st.aligned = true;
        if ((rc = run_plan(*plan, st, 1, S, Mode::kStore, nullptr, s[r]))) break;
        for (int i = k; i < n && e == hipSuccess; ++i)
            e = hipMemcpyAsync(shards[b * n + i], base + static_cast<size_t>(i) * pitch, S, hipMemcpyDeviceToHost, s[r]);
    }
    for (auto& x : s)
        if (x) {
            const hipError_t f = hipStreamSynchronize(x);
            if (e == hipSuccess) e = f;
            (void)hipStreamDestroy(x);
        }
    if (ring) (void)hipFree(ring);
    if (rc) return rc;
    return e == hipSuccess ? BLBRS_OK : hip_fail(e, "host batch (copy engines)");
}

int blbrs_encode_host_batch(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                            int nstreams) {
    if (nstreams < 0) return fail(BLBRS_ERR_INVALID_ARG, "nstreams must be >= 0");
    if (!enc || !shard_ptrs) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    const size_t n = static_cast<size_t>(enc->k + enc->m);
    for (size_t i = 0; i < batch * n; ++i)
        if (!shard_ptrs[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    std::vector<int> lanes;
    int rc = enc->lanes(&lanes);
    if (rc) return rc;
    auto hp = enc->encode_plan();
    const std::vector<Step> steps{Step{"E", hp.get(), Mode::kStore}};
    // Contiguous split of the stripes over the device list (multigpu.stripe_range's rule).
    const size_t parts = std::min(lanes.size(), batch);
    struct Part {
        int dev, occ;
        size_t start, count;
        int rc = BLBRS_OK;
        std::string msg;
    };
    std::vector<Part> ps;
    const auto keys = rt::lane_keys(lanes);
    const size_t base = batch / parts, extra = batch % parts;
    for (size_t p = 0, start = 0; p < parts; ++p) {
        const size_t count = base + (p < extra ? 1 : 0);
        ps.push_back(Part{lanes[p], keys[p].second, start, count});
        start += count;
    }
    auto run_part = [&](Part& p) {
        rt::LoadTicket ticket;
        ticket.take(p.dev, p.occ, static_cast<uint64_t>(p.count) * n * shard_len);
        rt::DeviceGuard guard;
        p.rc = guard.enter(p.dev);
        // nstreams >= 1 and every shard of the part pinned: the copy-engine pipeline; otherwise
        // the kernels code pinned shards in place and pageable ones are staged by CPU copies.
        bool dma = nstreams >= 1;
        for (size_t i = 0; dma && i < p.count * n; ++i) {
            uint64_t view = 0;
            int owner = -1;
            dma = rt::device_view(shard_ptrs[p.start * n + i], &view, &owner) && owner < 0;
        }
        if (p.rc == BLBRS_OK && dma) p.rc = dma_run(enc, *hp, shard_ptrs + p.start * n, p.count, shard_len, p.dev, nstreams);
        else if (p.rc == BLBRS_OK) p.rc = host_run(enc, steps, shard_ptrs + p.start * n, p.count, shard_len, nullptr, p.dev);
        if (p.rc != BLBRS_OK) p.msg = rt::last_error();
    };
    std::vector<std::thread> th;
    for (size_t p = 1; p < parts; ++p) th.emplace_back(run_part, std::ref(ps[p]));
    run_part(ps[0]);
    for (auto& t : th) t.join();
    for (size_t p = 0; p < parts; ++p)
        if (ps[p].rc != BLBRS_OK)
            return fail(ps[p].rc, "device " + std::to_string(ps[p].dev) + " (stripes " + std::to_string(ps[p].start) +
                                      ".." + std::to_string(ps[p].start + ps[p].count) + "): " + ps[p].msg);
    return BLBRS_OK;
}

// ---- CRC-32C ----

int blbrs_crc32c_dev_at(const uint8_t* data, size_t stride, size_t batch, size_t len, size_t block, size_t phase,
                        const uint32_t* seeds_dev, uint32_t* out_dev, void* stream) {
    if (batch == 0 || len == 0) return BLBRS_OK;
    if (!data || !out_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch > 1 && stride < len) return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than length");
    if (block == 0) {
        block = len;
        phase = 0;
    }
    if (phase >= block) return fail(BLBRS_ERR_INVALID_ARG, "phase must be smaller than the block");
    DevCall dc;
    int rc = dc.enter(data);
    if (rc) return rc;
    hipError_t e = crc32c_blocks(data, stride, batch, len, block, phase, seeds_dev, out_dev,
                                 static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "crc32c_blocks");
    return BLBRS_OK;
}

int blbrs_crc32c_dev(const uint8_t* data, size_t stride, size_t batch, size_t len, size_t block,
                     uint32_t* out_dev, void* stream) {
    return blbrs_crc32c_dev_at(data, stride, batch, len, block, 0, nullptr, out_dev, stream);
}

int blbrs_encode_crc_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                         size_t batch, size_t shard_len, size_t block, uint32_t* crc_out_dev, void* stream) {
    return blbrs_encode_crc_dev_at(enc, stripes, shard_stride, stripe_stride, batch, shard_len, block, 0, nullptr,
                                   crc_out_dev, stream);
}

// Coding pass of plan `hp` (encode or decode) fused with the CRC-32C of its output rows:
// crc[(j * batch + b) * nblocks + i] for output row j (hp->out_idx order).
static int code_crc_dev(blbrs_encoder* enc, const std::string& key, const HostPlan& hp, uint8_t* stripes,
                        size_t shard_stride, size_t stripe_stride, size_t batch, size_t shard_len, size_t block,
                        size_t phase, const uint32_t* seeds_dev, uint32_t* crc_out_dev, void* stream) {
    if (block == 0) {
        block = shard_len;
        phase = 0;
    }
    if (phase >= block) return fail(BLBRS_ERR_INVALID_ARG, "phase must be smaller than the block");
    Stripes st;
    int rc = dev_stripes_strided(stripes, shard_stride, stripe_stride, batch, shard_len, &st);
    if (rc) return rc;
    DevCall dc;
    if ((rc = dc.enter(stripes))) return rc;
    const DevPlan* plan = nullptr;
    if ((rc = enc->dev_plan(key, hp, dc.dev, &plan))) return rc;
    if (block > shard_len + phase) block = shard_len + phase;  // one block
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (plan->passes.size() == 1) {
        const DevPass& ps = plan->passes[0];
        EncodeCrcArgs a{};
        a.tables = ps.tables;
        a.in_idx = ps.in_idx;
        a.out_idx = ps.out_idx;
        a.base = stripes;
        a.shard_stride = shard_stride;
        a.stripe_stride = stripe_stride;
        a.B = static_cast<uint32_t>(batch);
        a.S = shard_len;
        a.block = block;
        a.k = ps.k_in;
        a.rows = ps.rows;
        a.crc = crc_out_dev;
        a.phase = phase;
        a.seeds = seeds_dev;
        a.parity = ps.parity;
        if (encode_crc_supported(a)) {
            const hipError_t e = launch_encode_crc(a, s);
            if (e != hipSuccess) return hip_fail(e, "launch encode_crc_kernel");
            return BLBRS_OK;
        }
    }
    // Shapes without a fused instantiation (or unaligned): the coding pass, then the CRC of
    // each output row -- same results, one more read of the outputs.
    if ((rc = run_plan(*plan, st, batch, shard_len, Mode::kStore, nullptr, s))) return rc;
    const size_t nblocks = (shard_len + phase + block - 1) / block;
    for (size_t j = 0; j < hp.out_idx.size(); ++j) {
        const hipError_t e = crc32c_blocks(stripes + static_cast<size_t>(hp.out_idx[j]) * shard_stride, stripe_stride,
                                           batch, shard_len, block, phase, seeds_dev ? seeds_dev + j * batch : nullptr,
                                           crc_out_dev + j * batch * nblocks, s);
        if (e != hipSuccess) return hip_fail(e, "crc32c_blocks");
    }
    return BLBRS_OK;
}

int blbrs_encode_crc_dev_at(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                            size_t batch, size_t shard_len, size_t block, size_t phase, const uint32_t* seeds_dev,
                            uint32_t* crc_out_dev, void* stream) {
    if (!enc || !crc_out_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    if (batch > 0x7FFFFFFFull) return fail(BLBRS_ERR_INVALID_ARG, "batch too large");
    auto hp = enc->encode_plan();
    return code_crc_dev(enc, "E", *hp, stripes, shard_stride, stripe_stride, batch, shard_len, block, phase, seeds_dev,
                        crc_out_dev, stream);
}

int blbrs_reconstruct_crc_dev_at(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                                 size_t batch, size_t shard_len, const uint8_t* present, int data_only, size_t block,
                                 size_t phase, const uint32_t* seeds_dev, uint32_t* crc_out_dev, void* stream) {
    if (!enc || !crc_out_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    std::shared_ptr<HostPlan> hp;
    std::string key;
    bool nothing = false;
    int rc = dev_decode_plan(enc, present, data_only, &hp, &key, &nothing);
    if (rc || nothing || batch == 0 || shard_len == 0) return rc;
    if (batch > 0x7FFFFFFFull) return fail(BLBRS_ERR_INVALID_ARG, "batch too large");
    return code_crc_dev(enc, key, *hp, stripes, shard_stride, stripe_stride, batch, shard_len, block, phase, seeds_dev,
                        crc_out_dev, stream);
}

int blbrs_crc32c(const uint8_t* data, size_t len, size_t block, uint32_t* out) {
    if (!data || !out) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (len == 0) return BLBRS_OK;
    if (block == 0) block = len;
    std::vector<int> lanes;
    int rc = rt::default_devices(&lanes);
    if (rc) return rc;
    static std::atomic<unsigned> rr{0};
    uint64_t view = 0;
    int owner = -1;
    const bool visible = rt::device_view(data, &view, &owner);
    const int dev = owner >= 0 ? owner : lanes[rt::pick_lane(lanes, rr, rt::host_numa_node(data))];
    rt::LoadTicket ticket;
    ticket.take(dev, 0, len);
    rt::DeviceGuard guard;
    if ((rc = guard.enter(dev))) return rc;
    rt::WorkerLease w;
    if ((rc = w.acquire(dev))) return rc;
    rt::note_call(dev);
    const size_t nblocks = (len + block - 1) / block;
    const hipStream_t s = w->s[0];
    uint32_t* dout = nullptr;  // nblocks entries + one seed word
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&dout), (nblocks + 1) * 4, s));
    // The CRCs come back through pinned memory: `out` may be pageable, and pageable memory is
    // never handed to HIP's copy engines.
    uint8_t* pout = nullptr;
    size_t pcap = 0;
    if ((rc = rt::pool_get(nblocks * 4, &pout, &pcap, /*internal=*/true))) {
        (void)hipFreeAsync(dout, s);
        (void)hipStreamSynchronize(s);
        return rc;
    }
    struct PoolBack {
        uint8_t* p;
        ~PoolBack() { (void)rt::pool_put(p); }
    } pout_back{pout};
    hipError_t e = hipSuccess;
    if (visible) {
        // Pinned / device memory: in place.
        e = crc32c_blocks(reinterpret_cast<const uint8_t*>(view), len, 1, len, block, 0, nullptr, dout, s);
    } else {
        // Pageable: chunks of at most one slot through the worker's pinned staging, two slots
        // alternating: the CPU copies chunk c in while the kernel reads chunk c - 1 in place
        // (device-mapped pinned memory).  With block <= the slot a chunk is whole blocks; a
        // longer block (a whole bulk frame) is continued across chunks: the chunk at offset
        // `off` starts (off mod block) bytes into block off / block, whose CRC so far is the
        // seed (crc32.Update) and which the chunk's first entry overwrites.
        const size_t slot = rt::kPinnedSlotBytes;
        const size_t C = block <= slot ? slot / block * block : slot;
        const size_t cs = round_up(std::min(C, len), 256);
        if ((rc = w->ensure_bounce(2 * cs)) || (rc = w->ensure_events())) {
            (void)hipFreeAsync(dout, s);
            (void)hipStreamSynchronize(s);
            return rc;
        }
        uint32_t* seed = dout + nblocks;
        size_t c = 0;
        for (size_t off = 0; off < len && e == hipSuccess; off += C, ++c) {
            const size_t clen = std::min(C, len - off), phase = off % block, first = off / block;
            const size_t sl = c & 1;
            if (c >= 2 && (e = hipEventSynchronize(w->ev[sl])) != hipSuccess) break;
            std::memcpy(w->bounce + sl * cs, data + off, clen);
            const uint8_t* src = reinterpret_cast<const uint8_t*>(w->bounce_dev + sl * cs);
            if (phase) e = hipMemcpyAsync(seed, dout + first, 4, hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess) e = crc32c_blocks(src, clen, 1, clen, block, phase, phase ? seed : nullptr, dout + first, s);
            if (e == hipSuccess) e = hipEventRecord(w->ev[sl], s);
        }
    }
    if (e == hipSuccess) e = hipMemcpyAsync(pout, dout, nblocks * 4, hipMemcpyDeviceToHost, s);
    (void)hipFreeAsync(dout, s);
    const hipError_t f = hipStreamSynchronize(s);
    if (e == hipSuccess) e = f;
    if (e != hipSuccess) return hip_fail(e, "crc32c");
    std::memcpy(out, pout, nblocks * 4);
    return BLBRS_OK;
}

// ---- batched client reconstructs ----

int blbrs_batcher_new(int max_batch, int window_us, blbrs_batcher** out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (max_batch <= 0 || window_us < 0) return fail(BLBRS_ERR_INVALID_ARG, "max_batch must be > 0, window_us >= 0");
    std::vector<int> devs;
    int rc = rt::default_devices(&devs);
    if (rc) return rc;
    return make_batcher(max_batch, window_us, devs, out);
}

int blbrs_batcher_new_on(int max_batch, int window_us, const int* devices, int ndevices, blbrs_batcher** out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (max_batch <= 0 || window_us < 0) return fail(BLBRS_ERR_INVALID_ARG, "max_batch must be > 0, window_us >= 0");
    if (!devices || ndevices <= 0) return fail(BLBRS_ERR_INVALID_ARG, "empty device list");
    std::vector<int> devs(devices, devices + ndevices);
    int rc = rt::check_devices(devs);
    if (rc) return rc;
    return make_batcher(max_batch, window_us, devs, out);
}

void blbrs_batcher_free(blbrs_batcher* b) {
    if (!b) return;
    b->shutdown();
    delete b;
}

int blbrs_batcher_stats(const blbrs_batcher* b, uint64_t* requests, uint64_t* launches) {
    if (!b || !requests || !launches) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    *requests = b->requests.load();
    *launches = b->launches.load();
    return BLBRS_OK;
}

int blbrs_encoder_set_batcher(blbrs_encoder* enc, blbrs_batcher* b) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    enc->batcher.store(b);
    return BLBRS_OK;
}

// ---- PackTracts ----

// checkTractSpec (store.go:996-1009) per piece, plus the device table: piece starts, then
// {src (device view), offset, length, piece} per extent.
static int build_pack_table(size_t npieces, size_t piece_len, const blbrs_pack_extent* extents, size_t nextents,
                            std::vector<uint64_t>* out) {
    std::vector<uint64_t>& table = *out;
    table.assign(npieces + 1 + 4 * nextents, 0);
    uint64_t* ex = table.data() + npieces + 1;
    size_t next_piece = 0;
    uint64_t end = 0;
    const uint8_t* last_src = nullptr;
    uint64_t last_view = 0;
    for (size_t i = 0; i < nextents; ++i) {
        const blbrs_pack_extent& x = extents[i];
        if (x.piece >= npieces || x.piece + 1 < next_piece)
            return fail(BLBRS_ERR_INVALID_ARG, "extent " + std::to_string(i) + ": piece out of range or out of order");
        while (next_piece <= x.piece) {
            table[next_piece++] = i;
            end = 0;
        }
        if (x.offset < end || x.length > piece_len || x.offset > piece_len - x.length)
            return fail(BLBRS_ERR_INVALID_ARG, "extent " + std::to_string(i) + " overlaps, is out of order or exceeds the piece");
        end = x.offset + x.length;
        uint64_t sview = 0;
        if (x.length) {
            if (!x.src) return fail(BLBRS_ERR_INVALID_ARG, "extent " + std::to_string(i) + ": NULL source");
            if (x.src == last_src) {
                sview = last_view;
            } else if (!rt::device_view(x.src, &sview)) {
                return fail(BLBRS_ERR_INVALID_ARG, "extent " + std::to_string(i) + ": source is not device-accessible");
            }
            last_src = x.src;
            last_view = sview;
        }
        ex[4 * i] = sview;
        ex[4 * i + 1] = x.offset;
        ex[4 * i + 2] = x.length;
        ex[4 * i + 3] = x.piece;
    }
    while (next_piece <= npieces) table[next_piece++] = nextents;
    return BLBRS_OK;
}

int blbrs_pack_dev(uint8_t* dst, size_t dst_stride, size_t npieces, size_t piece_len,
                   const blbrs_pack_extent* extents, size_t nextents, void* stream) {
    if (npieces == 0 || piece_len == 0) {
        if (nextents) return fail(BLBRS_ERR_INVALID_ARG, "extents given for empty pieces");
        return BLBRS_OK;
    }
    if (!dst || (nextents && !extents)) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (npieces > 1 && dst_stride < piece_len) return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than piece length");
    DevCall dc;
    int rc = dc.enter(dst);
    if (rc) return rc;
    uint64_t dview = 0;
    if (!rt::device_view(dst, &dview)) return fail(BLBRS_ERR_INVALID_ARG, "pack destination is not device-accessible");
    std::vector<uint64_t> table;
    if ((rc = build_pack_table(npieces, piece_len, extents, nextents, &table))) return rc;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    rt::PtrLease lease;
    const uint64_t* tdev = nullptr;
    bool unused = false;
    if ((rc = lease.upload(table.data(), table.size(), s, &tdev, &unused))) return rc;
    hipError_t e = pack_pieces(reinterpret_cast<uint8_t*>(dview), dst_stride, npieces, piece_len, tdev, s);
    if (e != hipSuccess) return hip_fail(e, "pack_pieces");
    return BLBRS_OK;
}

int blbrs_pack_encode_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                          size_t batch, size_t shard_len, const blbrs_pack_extent* extents, size_t nextents,
                          void* stream) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    if (batch == 0 || shard_len == 0) {
        if (nextents) return fail(BLBRS_ERR_INVALID_ARG, "extents given for empty pieces");
        return BLBRS_OK;
    }
    if (nextents && !extents) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch > 0x7FFFFFFFull) return fail(BLBRS_ERR_INVALID_ARG, "batch too large");
    Stripes st;
    int rc = dev_stripes_strided(stripes, shard_stride, stripe_stride, batch, shard_len, &st);
    if (rc) return rc;
    DevCall dc;
    if ((rc = dc.enter(stripes))) return rc;
    const size_t npieces = batch * static_cast<size_t>(enc->k);
    std::vector<uint64_t> table;
    if ((rc = build_pack_table(npieces, shard_len, extents, nextents, &table))) return rc;
    auto hp = enc->encode_plan();
    const DevPlan* plan = nullptr;
    if ((rc = enc->dev_plan("E", *hp, dc.dev, &plan))) return rc;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    PackEncodeArgs a{};
    const bool one_pass = plan->passes.size() == 1;
    if (one_pass) {
        a.tables = plan->passes[0].tables;
        a.out_idx = plan->passes[0].out_idx;
        a.base = stripes;
        a.shard_stride = shard_stride;
        a.stripe_stride = stripe_stride;
        a.S = shard_len;
        a.B = static_cast<uint32_t>(batch);
        a.k = static_cast<uint32_t>(enc->k);
        a.rows = static_cast<uint32_t>(plan->passes[0].rows);
        a.nextents = nextents;
        a.parity = plan->passes[0].parity;
    }
    const bool fused = one_pass && pack_encode_supported(a);
    // The extent table and (fused) the pre-pass's layout descriptors share one slot of the
    // caller-stream ring: reused only after the stream has run this call's launches.
    rt::PtrLease lease;
    const uint64_t* tdev = nullptr;
    bool unused = false;
    void* scratch = nullptr;
    if ((rc = lease.upload(table.data(), table.size(), s, &tdev, &unused, nullptr,
                           fused ? pack_encode_scratch_bytes(a) : 0, &scratch)))
        return rc;
    if (fused) {
        a.table = tdev;
        a.scratch = scratch;
        const hipError_t e = launch_pack_encode(a, s);
        if (e != hipSuccess) return hip_fail(e, "launch pack_encode_kernel");
        return BLBRS_OK;
    }
    // No fused instantiation: PackTracts into the data shards, then Encode (same bytes).
    hipError_t e = pack_pieces(stripes, shard_stride, npieces, shard_len, tdev, s, static_cast<uint32_t>(enc->k),
                               stripe_stride);
    if (e != hipSuccess) return hip_fail(e, "pack_pieces");
    return run_plan(*plan, st, batch, shard_len, Mode::kStore, nullptr, s);
}

// ---- pinned host memory ----

int blbrs_buffer_get(size_t n, uint8_t** out, size_t* cap) {
    if (!out || !cap) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    return rt::pool_get(n, out, cap);
}

int blbrs_buffer_put(uint8_t* p) { return rt::pool_put(p); }

int blbrs_buffer_register(void* p, size_t n) { return rt::pool_register(p, n); }

int blbrs_buffer_unregister(void* p) { return rt::pool_unregister(p); }

int blbrs_pool_set_live_limit(size_t bytes) { return rt::pool_set_live_limit(bytes); }

int blbrs_pool_set_idle_limit(size_t bytes) { return rt::pool_set_idle_limit(bytes); }

int blbrs_get_pool_stats(blbrs_pool_stats* out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    return rt::pool_stats(out);
}

int blbrs_host_alloc(size_t n, void** out) {
    if (!out || n == 0) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument or zero length");
    *out = nullptr;
    int nd = 0;
    int rc = rt::device_count(&nd);
    if (rc) return rc;
    HIP_TRY(hipHostMalloc(out, n, hipHostMallocDefault));
    return BLBRS_OK;
}

int blbrs_host_free(void* p) {
    if (!p) return BLBRS_OK;
    rt::note_released(p, 0, "blbrs_host_free");
    HIP_TRY(hipHostFree(p));
    return BLBRS_OK;
}

int blbrs_host_register(void* p, size_t n) {
    if (!p || n == 0) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument or zero length");
    int nd = 0;
    int rc = rt::device_count(&nd);
    if (rc) return rc;
    HIP_TRY(hipHostRegister(p, n, hipHostRegisterPortable | hipHostRegisterMapped));
    return BLBRS_OK;
}

int blbrs_host_unregister(void* p) {
    if (!p) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    rt::note_released(p, 0, "blbrs_host_unregister");
    HIP_TRY(hipHostUnregister(p));
    return BLBRS_OK;
}

// ---- runtime limits ----

int blbrs_set_worker_limit(int per_device) { return rt::set_worker_limit(per_device); }

int blbrs_get_device_stats(int device, blbrs_device_stats* out) {
    if (!out || device < 0) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    return rt::device_stats(device, out);
}

int blbrs_debug_watch_faults(void) { return rt::watch_faults(); }

int blbrs_plan_stats(uint64_t* host_plans, uint64_t* device_plans) {
    if (!host_plans || !device_plans) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    *host_plans = g_host_plans.load();
    *device_plans = g_device_plans.load();
    return BLBRS_OK;
}

int blbrs_trim(void) {
    rt::trim_workers();
    rt::pool_trim();
    return BLBRS_OK;
}

int blbrs_table_fault_take(int device, blbrs_table_fault* out, int* found) {
    if (!out || !found || device < 0) return fail(BLBRS_ERR_INVALID_ARG, "bad argument");
    *found = 0;
    *out = blbrs_table_fault{};
    uint32_t* rec = rt::device_fault_record(device);
    if (!rec) return fail(BLBRS_ERR_HIP, "no fault record for device " + std::to_string(device));
    volatile uint32_t* v = rec;
    if (!v[0]) return BLBRS_OK;
    const uint64_t e = (static_cast<uint64_t>(v[5]) << 32) | v[4];
    out->stripe = v[1];
    out->slot = v[2];
    out->launch_tag = v[3];
    out->entry_tag = static_cast<uint32_t>(e >> kPtrTagShift);
    out->address = e & kPtrMask;
    *found = 1;
    for (int i = 0; i < rt::kFaultWords; ++i) v[i] = 0;
    return BLBRS_OK;
}

int blbrs_debug_corrupt_next_table(int slot) {
    if (slot < 0) return fail(BLBRS_ERR_INVALID_ARG, "negative slot");
    rt::corrupt_next_table(slot);
    return BLBRS_OK;
}

// ---- misc ----

int blbrs_set_device(int device) {
    HIP_TRY(hipSetDevice(device));
    return BLBRS_OK;
}

int blbrs_device_count(int* count) {
    if (!count) return fail(BLBRS_ERR_INVALID_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return BLBRS_OK;
}

const char* blbrs_last_error(void) { return rt::last_error().c_str(); }

const char* blbrs_version(void) { return "blbrs 0.2.0 (gfx950; klauspost/reedsolomon@925cb01d6510 semantics)"; }

const char* blbrs_strerror(int code) {
    switch (code) {
        case BLBRS_OK: return "ok";
        case BLBRS_ERR_INV_SHARD_NUM: return "cannot create Encoder with zero or less data/parity shards";
        case BLBRS_ERR_MAX_SHARD_NUM: return "cannot create Encoder with more than 256 data+parity shards";
        case BLBRS_ERR_TOO_FEW_SHARDS: return "too few shards given";
        case BLBRS_ERR_SHARD_NO_DATA: return "no shard data";
        case BLBRS_ERR_SHARD_SIZE: return "shard sizes do not match";
        case BLBRS_ERR_SINGULAR: return "matrix is singular";
        case BLBRS_ERR_INVALID_ARG: return "invalid argument";
        case BLBRS_ERR_HIP: return "HIP runtime error";
        case BLBRS_ERR_NO_DEVICE: return "no HIP device";
        case BLBRS_ERR_LIMIT: return "pinned-memory live limit reached";
        default: return "unknown error";
    }
}

}  // extern "C"
