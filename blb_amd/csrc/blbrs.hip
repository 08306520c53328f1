// blbrs.hip -- host runtime + C ABI (include/blb_rs.h) of the MI355X RS engine.
//
// What lives here (the kernels are in rs_kernels.hip):
//   * reedsolomon.New equivalent: (k+m) x k matrix build (gf256.hpp), argument checks with
//     klauspost's error values.
//   * Coding plans: for each (operation, erasure pattern) the coefficient rows, their
//     v_perm lookup tables and shard index lists, uploaded once per device and cached on
//     the encoder -- the counterpart of klauspost's inversion tree (decode matrices
//     cached by invalid-index set) but holding device-ready tables.
//   * Host-memory Encoder methods (Encode / Verify / Reconstruct / ReconstructData) with
//     klauspost's shard conventions, each call borrowing a per-device stream worker so
//     concurrent callers (goroutines through cgo) never share a stream.
//   * Device-resident batched entry points on caller streams, and the pinned-host
//     streaming encoder (H2D / kernel / D2H overlapped over several streams).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
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
#include "pack.hpp"
#include "gf256.hpp"
#include "rs_kernels.hpp"

using namespace blbrs;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    g_last_error = m;
    return BLBRS_ERR_HIP;
}

#define HIP_TRY(expr)                                         \
    do {                                                      \
        hipError_t e_ = (expr);                               \
        if (e_ != hipSuccess) return hip_fail(e_, #expr);     \
    } while (0)

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------------------
// Coding plans
// ---------------------------------------------------------------------------------------

// One kernel pass: <= kMaxRows output rows over k_in inputs.
struct Pass {
    int k_in = 0, rows = 0;
    std::vector<int32_t> in_idx, out_idx;
    std::vector<uint32_t> tables;
};

// Host description of an operation: rows x k_in coefficients, split into passes.
struct HostPlan {
    int k_in = 0;
    std::vector<int32_t> in_idx;   // inputs (shard indices)
    std::vector<int32_t> out_idx;  // outputs (shard indices), one per row
    Mat rows;                      // out_idx.size() x k_in
    std::vector<Pass> passes;
};

void split_passes(HostPlan& p) {
    const int nrows = static_cast<int>(p.out_idx.size());
    for (int r0 = 0; r0 < nrows; r0 += kMaxRows) {
        Pass ps;
        ps.k_in = p.k_in;
        ps.rows = std::min(kMaxRows, nrows - r0);
        ps.in_idx = p.in_idx;
        ps.out_idx.assign(p.out_idx.begin() + r0, p.out_idx.begin() + r0 + ps.rows);
        Mat sub(p.rows.begin() + static_cast<size_t>(r0) * p.k_in,
                p.rows.begin() + static_cast<size_t>(r0 + ps.rows) * p.k_in);
        ps.tables = perm_tables(sub, ps.rows, p.k_in);
        p.passes.push_back(std::move(ps));
    }
}

// Device copy of a HostPlan on one device.
struct DevPass {
    void* mem = nullptr;
    const int32_t* in_idx = nullptr;
    const int32_t* out_idx = nullptr;
    const uint32_t* tables = nullptr;
    int k_in = 0, rows = 0;
};
struct DevPlan {
    std::vector<DevPass> passes;
    int device = -1;
    ~DevPlan() {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return;
        if (hipSetDevice(device) != hipSuccess) return;
        for (auto& p : passes)
            if (p.mem) (void)hipFree(p.mem);
        (void)hipSetDevice(cur);
    }
};

int upload(const HostPlan& hp, int device, std::unique_ptr<DevPlan>& out) {
    auto dp = std::make_unique<DevPlan>();
    dp->device = device;
    for (const Pass& ps : hp.passes) {
        DevPass d;
        d.k_in = ps.k_in;
        d.rows = ps.rows;
        const size_t n_in = ps.in_idx.size() * 4, n_out = round_up(ps.out_idx.size() * 4, 16);
        const size_t off_out = round_up(n_in, 16), off_tab = off_out + n_out;
        const size_t bytes = off_tab + ps.tables.size() * 4;
        std::vector<uint8_t> host(bytes, 0);
        std::memcpy(host.data(), ps.in_idx.data(), n_in);
        std::memcpy(host.data() + off_out, ps.out_idx.data(), ps.out_idx.size() * 4);
        std::memcpy(host.data() + off_tab, ps.tables.data(), ps.tables.size() * 4);
        HIP_TRY(hipMalloc(&d.mem, bytes));
        dp->passes.push_back(d);  // owned from here on (freed by ~DevPlan)
        HIP_TRY(hipMemcpy(d.mem, host.data(), bytes, hipMemcpyHostToDevice));
        auto* base = static_cast<uint8_t*>(d.mem);
        dp->passes.back().in_idx = reinterpret_cast<const int32_t*>(base);
        dp->passes.back().out_idx = reinterpret_cast<const int32_t*>(base + off_out);
        dp->passes.back().tables = reinterpret_cast<const uint32_t*>(base + off_tab);
    }
    out = std::move(dp);
    return BLBRS_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Encoder
// ---------------------------------------------------------------------------------------

// Matrix and plan caches of one (k, m).  Shared by every blbrs_encoder handle with that
// shape: blb makes a fresh reedsolomon.New(n, m) per client reconstruct
// (client/blb/reconstruct.go:172), and a shared core keeps those calls from rebuilding
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
        }
        return slot;
    }

    // Reconstruct(dataOnly): inputs = first k present shards ascending (klauspost
    // reedsolomon.go reconstruct), rows = inv(M[valid]) rows of missing data shards, then
    // (unless data_only) P[j] * inv(M[valid]) for missing parity j -- one pass produces
    // every missing shard straight from the k survivors.  Returns nullptr + rc on error.
    std::shared_ptr<HostPlan> decode_plan(const std::vector<uint8_t>& present, bool data_only, int* rc) {
        std::string key(present.size() + 2, '0');
        key[0] = 'R';
        key[1] = data_only ? 'd' : 'a';
        for (size_t i = 0; i < present.size(); ++i) key[i + 2] = present[i] ? '1' : '0';
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
        return slot;
    }

    // Device tables for `hp` on `device` (uploaded on first use).
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
    std::atomic<blbrs_batcher*> batcher{nullptr};  // routes host Reconstruct[Data] (blbrs_encoder_set_batcher)
    std::shared_ptr<HostPlan> encode_plan() { return core->encode_plan(); }
    std::shared_ptr<HostPlan> decode_plan(const std::vector<uint8_t>& present, bool data_only, int* rc) {
        return core->decode_plan(present, data_only, rc);
    }
    int dev_plan(const std::string& key, const HostPlan& hp, int device, const DevPlan** out) {
        return core->dev_plan(key, hp, device, out);
    }
};

namespace {

std::mutex g_cores_mu;
std::map<std::pair<int, int>, std::weak_ptr<EncoderCore>> g_cores;

// The shared core for (k, m); nullptr when the matrix cannot be built.
std::shared_ptr<EncoderCore> core_for(int k, int m) {
    std::lock_guard<std::mutex> g(g_cores_mu);
    auto& w = g_cores[{k, m}];
    if (auto c = w.lock()) return c;
    auto c = std::make_shared<EncoderCore>();
    c->k = k;
    c->m = m;
    if (!build_matrix(k, m, c->matrix)) return nullptr;
    w = c;
    return c;
}

std::string plan_key(bool encode, const std::vector<uint8_t>& present, bool data_only) {
    if (encode) return "E";
    std::string key(present.size() + 2, '0');
    key[0] = 'R';
    key[1] = data_only ? 'd' : 'a';
    for (size_t i = 0; i < present.size(); ++i) key[i + 2] = present[i] ? '1' : '0';
    return key;
}

// Addressing of one batch of stripes on the device.
struct Stripes {
    uint8_t* base = nullptr;  // strided form
    uint64_t shard_stride = 0, stripe_stride = 0;
    const uint64_t* ptrs = nullptr;  // device pointer table form
    uint32_t nshards = 0;
    bool aligned = false;
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
        hipError_t e = launch_code(a, mode, stream);
        if (e != hipSuccess) return hip_fail(e, "launch rs_code_kernel");
    }
    return BLBRS_OK;
}

// ---- per-device resources ----

// Stream worker for host-memory calls: its own streams and device staging buffer.
struct Worker {
    hipStream_t s[2] = {nullptr, nullptr};
    uint8_t* dbuf = nullptr;
    size_t cap = 0;
    int32_t* dflag = nullptr;
    int device = -1;
    int ensure(size_t bytes) {
        if (bytes <= cap) return BLBRS_OK;
        if (dbuf) (void)hipFree(dbuf);
        dbuf = nullptr;
        cap = 0;
        HIP_TRY(hipMalloc(&dbuf, bytes));
        cap = bytes;
        return BLBRS_OK;
    }
};

// Pinned + device slot for uploading pointer tables of the *_ptrs entry points.
struct PtrSlot {
    std::mutex mu;
    uint64_t* host = nullptr;
    uint64_t* dev = nullptr;
    size_t cap = 0;  // entries
    hipEvent_t done = nullptr;
};

struct Device {
    std::mutex mu;
    std::vector<Worker*> idle;
    static constexpr int kSlots = 8;
    PtrSlot slots[kSlots];
    std::atomic<unsigned> next_slot{0};
};

std::mutex g_dev_mu;
std::map<int, Device*> g_devices;  // never freed (process lifetime)

Device& device_ctx(int dev) {
    std::lock_guard<std::mutex> g(g_dev_mu);
    auto& d = g_devices[dev];
    if (!d) d = new Device();
    return *d;
}

int current_device(int* dev) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return fail(BLBRS_ERR_NO_DEVICE, "no HIP device visible");
    HIP_TRY(hipGetDevice(dev));
    return BLBRS_OK;
}

struct WorkerLease {
    Device* d = nullptr;
    Worker* w = nullptr;
    ~WorkerLease() {
        if (w) {
            std::lock_guard<std::mutex> g(d->mu);
            d->idle.push_back(w);
        }
    }
};

int lease_worker(WorkerLease& lease) {
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    Device& d = device_ctx(dev);
    lease.d = &d;
    {
        std::lock_guard<std::mutex> g(d.mu);
        if (!d.idle.empty()) {
            lease.w = d.idle.back();
            d.idle.pop_back();
            return BLBRS_OK;
        }
    }
    auto* w = new Worker();
    w->device = dev;
    for (auto& s : w->s) HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&w->dflag, sizeof(int32_t)));
    lease.w = w;
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

bool aligned16(uintptr_t x) { return (x & 15u) == 0; }

// Upload a host array of device pointers to a device pointer table on `stream`.  The
// slot's event keeps it busy until the kernels that read it have run.
struct PtrLease {
    PtrSlot* slot = nullptr;
    hipStream_t stream = nullptr;
    ~PtrLease() {
        if (slot) {
            (void)hipEventRecord(slot->done, stream);
            slot->mu.unlock();
        }
    }
};

int upload_table(const uint64_t* ptrs, size_t count, hipStream_t stream, PtrLease& lease,
                 const uint64_t** dev_out, bool* aligned) {
    int dev = 0;
    int rc = current_device(&dev);
    if (rc) return rc;
    Device& d = device_ctx(dev);
    PtrSlot& s = d.slots[d.next_slot.fetch_add(1) % Device::kSlots];
    s.mu.lock();
    if (!s.done) {
        hipError_t e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e != hipSuccess) { s.mu.unlock(); return hip_fail(e, "hipEventCreate"); }
    } else {
        hipError_t e = hipEventSynchronize(s.done);
        if (e != hipSuccess) { s.mu.unlock(); return hip_fail(e, "hipEventSynchronize"); }
    }
    if (s.cap < count) {
        if (s.host) (void)hipHostFree(s.host);
        if (s.dev) (void)hipFree(s.dev);
        s.host = nullptr;
        s.dev = nullptr;
        s.cap = 0;
        const size_t cap = std::max<size_t>(count, 1024);
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&s.host), cap * 8, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.dev), cap * 8);
        if (e != hipSuccess) { s.mu.unlock(); return hip_fail(e, "ptr table alloc"); }
        s.cap = cap;
    }
    bool al = true;
    for (size_t i = 0; i < count; ++i) {
        s.host[i] = ptrs[i];
        al = al && aligned16(s.host[i]);
    }
    lease.slot = &s;
    lease.stream = stream;
    HIP_TRY(hipMemcpyAsync(s.dev, s.host, count * 8, hipMemcpyHostToDevice, stream));
    *dev_out = s.dev;
    *aligned = al;
    return BLBRS_OK;
}

int upload_ptrs(uint8_t* const* ptrs, size_t count, hipStream_t stream, PtrLease& lease,
                const uint64_t** dev_out, bool* aligned) {
    std::vector<uint64_t> v(count);
    for (size_t i = 0; i < count; ++i) {
        if (!ptrs[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
        v[i] = reinterpret_cast<uint64_t>(ptrs[i]);
    }
    return upload_table(v.data(), count, stream, lease, dev_out, aligned);
}

// Address under which the GPU can access `p`: device memory as is, pinned host memory
// (hipHostMalloc / hipHostRegister) through its device mapping.  False for pageable memory.
bool device_view(const void* p, uint64_t* out) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the sticky error
        return false;
    }
    if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
        *out = reinterpret_cast<uint64_t>(p);
        return true;
    }
    if (attr.type == hipMemoryTypeHost && attr.devicePointer && attr.hostPointer) {
        *out = reinterpret_cast<uint64_t>(attr.devicePointer) +
               (reinterpret_cast<uintptr_t>(p) - reinterpret_cast<uintptr_t>(attr.hostPointer));
        return true;
    }
    return false;
}

// One step of a host-memory call: a plan run in store or verify mode.
struct Step {
    std::string key;
    const HostPlan* hp;
    Mode mode;
};

// Host-memory coding.  Steps run in order over the same stripe, so a later step sees what
// an earlier one wrote (Reconstruct then Verify = reconstructAndVerify, store.go:1132-1142,
// in one device round trip).  Shards read by a step and not produced by an earlier step
// are copied in once; shards written by store steps are copied out.
int host_run(blbrs_encoder* enc, const std::vector<Step>& steps, uint8_t* const* shards, size_t S, int* ok) {
    WorkerLease lease;
    int rc = lease_worker(lease);
    if (rc) return rc;
    Worker& w = *lease.w;
    const int n = enc->k + enc->m;
    std::vector<const DevPlan*> plans(steps.size(), nullptr);
    std::vector<char> produced(n, 0), need_in(n, 0), is_out(n, 0), touched(n, 0);
    bool verify = false;
    for (size_t t = 0; t < steps.size(); ++t) {
        if ((rc = enc->dev_plan(steps[t].key, *steps[t].hp, w.device, &plans[t]))) return rc;
        const HostPlan& hp = *steps[t].hp;
        for (int32_t i : hp.in_idx) {
            touched[i] = 1;
            if (!produced[i]) need_in[i] = 1;
        }
        for (int32_t i : hp.out_idx) {
            touched[i] = 1;
            if (steps[t].mode == Mode::kStore) {
                produced[i] = 1;
                is_out[i] = 1;
            } else {
                verify = true;
                if (!produced[i]) need_in[i] = 1;
            }
        }
    }
    // Zero-copy: when every shard the steps touch is pinned (or device) memory, the kernels
    // read and write it in place over PCIe -- no staging, and both link directions busy at
    // once (RS(6,3): 50.8 GiB/s of data vs 37.3 through copy engines; profiles/r01/zc.txt).
    {
        std::vector<uint64_t> view(n, 0);
        bool all = true;
        for (int i = 0; i < n && all; ++i)
            if (touched[i]) all = device_view(shards[i], &view[i]);
        if (all) {
            PtrLease pl;
            Stripes st;
            st.nshards = n;
            if ((rc = upload_table(view.data(), n, w.s[0], pl, &st.ptrs, &st.aligned))) return rc;
            if (verify) HIP_TRY(hipMemsetAsync(w.dflag, 0, sizeof(int32_t), w.s[0]));
            for (size_t t = 0; t < steps.size(); ++t)
                if ((rc = run_plan(*plans[t], st, 1, S, steps[t].mode, w.dflag, w.s[0]))) return rc;
            int32_t flag = 0;
            if (verify) HIP_TRY(hipMemcpyAsync(&flag, w.dflag, sizeof(int32_t), hipMemcpyDeviceToHost, w.s[0]));
            HIP_TRY(hipStreamSynchronize(w.s[0]));
            if (ok) *ok = flag ? 0 : 1;
            return BLBRS_OK;
        }
    }
    // Staged: 1 MiB column chunks alternate over the worker's two streams, so the H2D of
    // chunk j+1 overlaps the kernels and D2H of chunk j.
    const size_t Sp = round_up(S, 256);  // padded shard stride keeps every shard 16B-aligned
    if ((rc = w.ensure(static_cast<size_t>(n) * Sp))) return rc;
    const size_t chunk = S <= (size_t{2} << 20) ? S : (size_t{1} << 20);
    hipEvent_t ev = nullptr;
    if (verify) {
        HIP_TRY(hipMemsetAsync(w.dflag, 0, sizeof(int32_t), w.s[0]));
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev, w.s[0]));
        HIP_TRY(hipStreamWaitEvent(w.s[1], ev, 0));
    }
    int j = 0;
    for (size_t off = 0; off < S; off += chunk, ++j) {
        const size_t len = std::min(chunk, S - off);
        hipStream_t s = w.s[j & 1];
        for (int i = 0; i < n; ++i)
            if (need_in[i])
                HIP_TRY(hipMemcpyAsync(w.dbuf + static_cast<size_t>(i) * Sp + off, shards[i] + off, len,
                                       hipMemcpyHostToDevice, s));
        Stripes st;
        st.base = w.dbuf + off;
        st.shard_stride = Sp;
        st.stripe_stride = static_cast<uint64_t>(n) * Sp;
        st.aligned = aligned16(off);
        for (size_t t = 0; t < steps.size(); ++t)
            if ((rc = run_plan(*plans[t], st, 1, len, steps[t].mode, w.dflag, s))) return rc;
        for (int i = 0; i < n; ++i)
            if (is_out[i])
                HIP_TRY(hipMemcpyAsync(shards[i] + off, w.dbuf + static_cast<size_t>(i) * Sp + off, len,
                                       hipMemcpyDeviceToHost, s));
    }
    int32_t flag = 0;
    if (verify) {
        HIP_TRY(hipEventRecord(ev, w.s[1]));
        HIP_TRY(hipStreamWaitEvent(w.s[0], ev, 0));
        HIP_TRY(hipMemcpyAsync(&flag, w.dflag, sizeof(int32_t), hipMemcpyDeviceToHost, w.s[0]));
    }
    HIP_TRY(hipStreamSynchronize(w.s[0]));
    HIP_TRY(hipStreamSynchronize(w.s[1]));
    if (ev) (void)hipEventDestroy(ev);
    if (ok) *ok = flag ? 0 : 1;
    return BLBRS_OK;
}

int host_code(blbrs_encoder* enc, const std::string& key, const HostPlan& hp, uint8_t* const* shards,
              size_t S, Mode mode, int* ok) {
    return host_run(enc, {Step{key, &hp, mode}}, shards, S, ok);
}

int current_dev_or_fail(int* dev) { return current_device(dev); }

std::vector<uint8_t> present_vec(const blbrs_encoder* enc, const uint8_t* present) {
    std::vector<uint8_t> p(enc->k + enc->m);
    for (int i = 0; i < enc->k + enc->m; ++i) p[i] = present[i] ? 1 : 0;
    return p;
}

// ---- batched host reconstructs ----
//
// client/blb/reconstruct.go:65-195 calls ReconstructData once per degraded read, on one
// stripe of `length`-byte pieces; MaxInFlight (:19,35-45) lets many run at once.  Alone,
// each call is a launch plus a stream round trip for a few KiB..MiB of work.  A batcher
// collects the calls that arrive within `window_us` (or until `max_batch` are waiting) and
// runs them as ONE launch per (encoder, erasure pattern, length) group over a device
// pointer table, with one stream sync for the whole batch.  Shards in pinned or device
// memory are used in place; pageable shards are staged by the CALLING thread through its
// own pinned buffer, so the memcpys of concurrent callers run in parallel.
struct BatchReq {
    blbrs_encoder* enc = nullptr;
    std::shared_ptr<HostPlan> hp;
    std::string key;
    std::vector<uint64_t> views;  // device-visible address per shard slot (0 = unused)
    size_t S = 0;
    std::chrono::steady_clock::time_point arrival;
    int rc = BLBRS_OK;
    bool done = false;
};

// Per-thread pinned staging for pageable shards.
struct PinnedStage {
    uint8_t* p = nullptr;
    size_t cap = 0;
    ~PinnedStage() {
        if (p) (void)hipHostFree(p);
    }
    int ensure(size_t bytes) {
        if (bytes <= cap) return BLBRS_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&p), bytes, hipHostMallocDefault));
        cap = bytes;
        return BLBRS_OK;
    }
};

}  // namespace

struct blbrs_batcher {
    int device = 0;
    size_t max_batch = 64;
    std::chrono::microseconds window{200};
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::condition_variable cv_in, cv_done;
    std::deque<BatchReq*> q;
    bool stop = false;
    std::thread th;
    std::atomic<uint64_t> launches{0}, requests{0};

    void run() {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_in.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop requested and nothing left
            const auto deadline = q.front()->arrival + window;
            cv_in.wait_until(lk, deadline, [&] { return stop || q.size() >= max_batch; });
            std::vector<BatchReq*> batch;
            while (!q.empty() && batch.size() < max_batch) {
                batch.push_back(q.front());
                q.pop_front();
            }
            lk.unlock();
            process(batch);
            lk.lock();
            for (BatchReq* r : batch) r->done = true;
            cv_done.notify_all();
        }
    }

    void process(std::vector<BatchReq*>& batch) {
        // Handles of one (k, m) share a core, so calls from different encoders merge.
        std::map<std::tuple<EncoderCore*, std::string, size_t>, std::vector<BatchReq*>> groups;
        for (BatchReq* r : batch) groups[{r->enc->core.get(), r->key, r->S}].push_back(r);
        for (auto& [gk, reqs] : groups) {
            EncoderCore* enc = std::get<0>(gk);
            const size_t S = std::get<2>(gk), n = static_cast<size_t>(enc->k + enc->m);
            const DevPlan* plan = nullptr;
            int rc = enc->dev_plan(std::get<1>(gk), *reqs[0]->hp, device, &plan);
            if (rc == BLBRS_OK) {
                std::vector<uint64_t> table(reqs.size() * n);
                for (size_t j = 0; j < reqs.size(); ++j)
                    std::copy(reqs[j]->views.begin(), reqs[j]->views.end(), table.begin() + j * n);
                PtrLease pl;
                Stripes st;
                st.nshards = static_cast<uint32_t>(n);
                rc = upload_table(table.data(), table.size(), stream, pl, &st.ptrs, &st.aligned);
                if (rc == BLBRS_OK) rc = run_plan(*plan, st, reqs.size(), S, Mode::kStore, nullptr, stream);
                if (rc == BLBRS_OK) launches.fetch_add(1);
            }
            for (BatchReq* r : reqs) r->rc = rc;
        }
        const hipError_t e = hipStreamSynchronize(stream);
        if (e != hipSuccess) {
            const int rc = hip_fail(e, "batched reconstruct");
            for (BatchReq* r : batch) r->rc = rc;
        }
        requests.fetch_add(batch.size());
    }
};

namespace {

// The host Reconstruct / ReconstructData of one stripe through `b` (blocking).  `hp` is
// the decode plan with at least one output; argument checks have been done.
int batched_reconstruct(blbrs_batcher* b, blbrs_encoder* enc, const std::string& key,
                        std::shared_ptr<HostPlan> hp, uint8_t* const* shards, size_t S) {
    static thread_local PinnedStage stage;
    const int n = enc->k + enc->m;
    BatchReq req;
    req.enc = enc;
    req.hp = hp;
    req.key = key;
    req.S = S;
    req.views.assign(n, 0);
    // Slots touched by the plan: inputs then outputs; pageable ones get a staging slot.
    std::vector<std::pair<int, bool>> touched;
    for (int32_t i : hp->in_idx) touched.push_back({i, true});
    for (int32_t i : hp->out_idx) touched.push_back({i, false});
    const size_t Sp = round_up(S, 256);
    size_t nstaged = 0;
    std::vector<int> slot(n, -1);
    for (auto [i, in] : touched) {
        (void)in;
        if (!device_view(shards[i], &req.views[i])) slot[i] = static_cast<int>(nstaged++);
    }
    if (nstaged) {
        int rc = stage.ensure(nstaged * Sp);
        if (rc) return rc;
        for (auto [i, in] : touched) {
            if (slot[i] < 0) continue;
            uint8_t* p = stage.p + static_cast<size_t>(slot[i]) * Sp;
            if (in) std::memcpy(p, shards[i], S);
            if (!device_view(p, &req.views[i])) return fail(BLBRS_ERR_HIP, "pinned staging has no device mapping");
        }
    }
    req.arrival = std::chrono::steady_clock::now();
    {
        std::unique_lock<std::mutex> lk(b->mu);
        if (b->stop) return fail(BLBRS_ERR_INVALID_ARG, "batcher is shutting down");
        b->q.push_back(&req);
        if (b->q.size() >= b->max_batch) b->cv_in.notify_one();
        else if (b->q.size() == 1) b->cv_in.notify_one();
        b->cv_done.wait(lk, [&] { return req.done; });
    }
    if (req.rc != BLBRS_OK) return req.rc;
    for (int32_t i : hp->out_idx)
        if (slot[i] >= 0) std::memcpy(shards[i], stage.p + static_cast<size_t>(slot[i]) * Sp, S);
    return BLBRS_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int blbrs_new(int data_shards, int parity_shards, blbrs_encoder** out) {
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
    *out = e;
    return BLBRS_OK;
}

void blbrs_free(blbrs_encoder* enc) { delete enc; }
int blbrs_data_shards(const blbrs_encoder* enc) { return enc ? enc->k : 0; }
int blbrs_parity_shards(const blbrs_encoder* enc) { return enc ? enc->m : 0; }

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
    return host_code(enc, "E", *hp, shards, S, Mode::kStore, nullptr);
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
    return host_code(enc, "E", *hp, const_cast<uint8_t* const*>(shards), S, Mode::kVerify, ok);
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
    if (npresent == n) {  // nothing to rebuild; reconstructAndVerify still verifies
        if (!verify_ok) return BLBRS_OK;
        for (int i = 0; i < n; ++i)
            if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
        return host_code(enc, "E", *ep, shards, S, Mode::kVerify, verify_ok);
    }
    if (npresent < enc->k) return fail(BLBRS_ERR_TOO_FEW_SHARDS, "too few shards given");
    auto hp = enc->decode_plan(present, data_only, &rc);
    if (!hp) return rc;
    for (int32_t i : hp->in_idx)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    for (int32_t i : hp->out_idx)
        if (!shards[i]) return fail(BLBRS_ERR_INVALID_ARG, "missing shard has no output buffer");
    blbrs_batcher* b = verify_ok ? nullptr : enc->batcher.load();
    if (b && !hp->out_idx.empty()) {
        if ((rc = batched_reconstruct(b, enc, plan_key(false, present, data_only), hp, shards, S))) return rc;
        for (int32_t i : hp->out_idx) lens[i] = S;
        return BLBRS_OK;
    }
    std::vector<Step> steps;
    if (!hp->out_idx.empty()) steps.push_back(Step{plan_key(false, present, data_only), hp.get(), Mode::kStore});
    if (verify_ok) steps.push_back(Step{"E", ep.get(), Mode::kVerify});
    if (steps.empty()) return BLBRS_OK;  // data_only with only parity missing
    rc = host_run(enc, steps, shards, S, verify_ok);
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

static int dev_stripes_strided(const blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride,
                               size_t stripe_stride, size_t batch, size_t shard_len, Stripes* st) {
    if (!stripes) return fail(BLBRS_ERR_INVALID_ARG, "stripes is NULL");
    const int n = enc->k + enc->m;
    if (shard_stride < shard_len || (batch > 1 && stripe_stride < shard_len))
        return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than shard length");
    (void)n;
    st->base = stripes;
    st->shard_stride = shard_stride;
    st->stripe_stride = stripe_stride;
    st->aligned = aligned16(reinterpret_cast<uintptr_t>(stripes)) && aligned16(shard_stride) &&
                  aligned16(stripe_stride);
    return BLBRS_OK;
}

static int dev_run(blbrs_encoder* enc, const std::string& key, const HostPlan& hp, const Stripes& st,
                   size_t batch, size_t S, Mode mode, int32_t* mismatch, void* stream) {
    int dev = 0;
    int rc = current_dev_or_fail(&dev);
    if (rc) return rc;
    const DevPlan* plan = nullptr;
    if ((rc = enc->dev_plan(key, hp, dev, &plan))) return rc;
    return run_plan(*plan, st, batch, S, mode, mismatch, static_cast<hipStream_t>(stream));
}

int blbrs_encode_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                     size_t batch, size_t shard_len, void* stream) {
    if (!enc) return fail(BLBRS_ERR_INVALID_ARG, "enc is NULL");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    Stripes st;
    int rc = dev_stripes_strided(enc, stripes, shard_stride, stripe_stride, batch, shard_len, &st);
    if (rc) return rc;
    auto hp = enc->encode_plan();
    return dev_run(enc, "E", *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

int blbrs_encode_dev_ptrs(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                          void* stream) {
    if (!enc || !shard_ptrs) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    const int n = enc->k + enc->m;
    PtrLease lease;
    Stripes st;
    int rc = upload_ptrs(shard_ptrs, batch * n, static_cast<hipStream_t>(stream), lease, &st.ptrs, &st.aligned);
    if (rc) return rc;
    st.nshards = n;
    auto hp = enc->encode_plan();
    return dev_run(enc, "E", *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
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
    if ((rc = dev_stripes_strided(enc, stripes, shard_stride, stripe_stride, batch, shard_len, &st))) return rc;
    return dev_run(enc, key, *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
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
    PtrLease lease;
    Stripes st;
    if ((rc = upload_ptrs(shard_ptrs, batch * n, static_cast<hipStream_t>(stream), lease, &st.ptrs, &st.aligned)))
        return rc;
    st.nshards = n;
    return dev_run(enc, key, *hp, st, batch, shard_len, Mode::kStore, nullptr, stream);
}

int blbrs_verify_dev(blbrs_encoder* enc, const uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                     size_t batch, size_t shard_len, int32_t* mismatch_dev, void* stream) {
    if (!enc || !mismatch_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0) return BLBRS_OK;
    HIP_TRY(hipMemsetAsync(mismatch_dev, 0, batch * sizeof(int32_t), static_cast<hipStream_t>(stream)));
    if (shard_len == 0) return BLBRS_OK;
    Stripes st;
    int rc = dev_stripes_strided(enc, const_cast<uint8_t*>(stripes), shard_stride, stripe_stride, batch,
                                 shard_len, &st);
    if (rc) return rc;
    auto hp = enc->encode_plan();
    return dev_run(enc, "E", *hp, st, batch, shard_len, Mode::kVerify, mismatch_dev, stream);
}

int blbrs_verify_dev_ptrs(blbrs_encoder* enc, const uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                          int32_t* mismatch_dev, void* stream) {
    if (!enc || !shard_ptrs || !mismatch_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0) return BLBRS_OK;
    HIP_TRY(hipMemsetAsync(mismatch_dev, 0, batch * sizeof(int32_t), static_cast<hipStream_t>(stream)));
    if (shard_len == 0) return BLBRS_OK;
    const int n = enc->k + enc->m;
    PtrLease lease;
    Stripes st;
    int rc = upload_ptrs(const_cast<uint8_t* const*>(shard_ptrs), batch * n, static_cast<hipStream_t>(stream),
                         lease, &st.ptrs, &st.aligned);
    if (rc) return rc;
    st.nshards = n;
    auto hp = enc->encode_plan();
    return dev_run(enc, "E", *hp, st, batch, shard_len, Mode::kVerify, mismatch_dev, stream);
}

// ---- streaming host path ----

int blbrs_encode_host_batch(blbrs_encoder* enc, uint8_t* const* shard_ptrs, size_t batch, size_t shard_len,
                            int nstreams) {
    if (!enc || !shard_ptrs) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    const int n = enc->k + enc->m, k = enc->k;
    for (size_t i = 0; i < batch * n; ++i)
        if (!shard_ptrs[i]) return fail(BLBRS_ERR_INVALID_ARG, "NULL shard pointer");
    if (nstreams < 1) nstreams = 3;
    if (nstreams > 8) nstreams = 8;
    int dev = 0;
    int rc = current_dev_or_fail(&dev);
    if (rc) return rc;
    auto hp = enc->encode_plan();
    const DevPlan* plan = nullptr;
    if ((rc = enc->dev_plan("E", *hp, dev, &plan))) return rc;

    // Pinned stripes: one zero-copy launch over the whole batch (see host_code).
    {
        std::vector<uint64_t> view(batch * n, 0);
        bool all = true;
        for (size_t i = 0; i < batch * n && all; ++i) all = device_view(shard_ptrs[i], &view[i]);
        if (all) {
            hipStream_t s = nullptr;
            HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            {
                PtrLease pl;
                Stripes st;
                st.nshards = n;
                rc = upload_table(view.data(), view.size(), s, pl, &st.ptrs, &st.aligned);
                if (rc == BLBRS_OK) rc = run_plan(*plan, st, batch, shard_len, Mode::kStore, nullptr, s);
            }
            hipError_t e = hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
            if (rc) return rc;
            if (e != hipSuccess) return hip_fail(e, "zero-copy encode");
            return BLBRS_OK;
        }
    }

    const size_t Sp = round_up(shard_len, 256);
    const size_t slot_bytes = static_cast<size_t>(n) * Sp;
    std::vector<hipStream_t> streams(nstreams, nullptr);
    uint8_t* dbuf = nullptr;
    auto cleanup = [&]() {
        for (auto s : streams)
            if (s) { (void)hipStreamSynchronize(s); (void)hipStreamDestroy(s); }
        if (dbuf) (void)hipFree(dbuf);
    };
    for (auto& s : streams) {
        hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        if (e != hipSuccess) { cleanup(); return hip_fail(e, "hipStreamCreate"); }
    }
    hipError_t e = hipMalloc(&dbuf, slot_bytes * nstreams);
    if (e != hipSuccess) { dbuf = nullptr; cleanup(); return hip_fail(e, "hipMalloc staging"); }
    for (size_t b = 0; b < batch && rc == BLBRS_OK; ++b) {
        const int si = static_cast<int>(b % nstreams);
        hipStream_t s = streams[si];
        uint8_t* slot = dbuf + slot_bytes * si;
        for (int i = 0; i < k && e == hipSuccess; ++i)
            e = hipMemcpyAsync(slot + i * Sp, shard_ptrs[b * n + i], shard_len, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { rc = hip_fail(e, "H2D"); break; }
        Stripes st;
        st.base = slot;
        st.shard_stride = Sp;
        st.stripe_stride = slot_bytes;
        st.aligned = true;
        rc = run_plan(*plan, st, 1, shard_len, Mode::kStore, nullptr, s);
        for (int i = k; i < n && rc == BLBRS_OK && e == hipSuccess; ++i)
            e = hipMemcpyAsync(shard_ptrs[b * n + i], slot + i * Sp, shard_len, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess) rc = hip_fail(e, "D2H");
    }
    cleanup();
    return rc;
}

// ---- CRC-32C ----

int blbrs_crc32c_dev(const uint8_t* data, size_t stride, size_t batch, size_t len, size_t block,
                     uint32_t* out_dev, void* stream) {
    if (batch == 0 || len == 0) return BLBRS_OK;
    if (!data || !out_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch > 1 && stride < len) return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than length");
    int dev = 0;
    int rc = current_dev_or_fail(&dev);
    if (rc) return rc;
    if (block == 0) block = len;
    hipError_t e = crc32c_blocks(data, stride, batch, len, block, out_dev, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) return hip_fail(e, "crc32c_blocks");
    return BLBRS_OK;
}

int blbrs_encode_crc_dev(blbrs_encoder* enc, uint8_t* stripes, size_t shard_stride, size_t stripe_stride,
                         size_t batch, size_t shard_len, size_t block, uint32_t* crc_out_dev, void* stream) {
    if (!enc || !crc_out_dev) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (batch == 0 || shard_len == 0) return BLBRS_OK;
    if (batch > 0x7FFFFFFFull) return fail(BLBRS_ERR_INVALID_ARG, "batch too large");
    Stripes st;
    int rc = dev_stripes_strided(enc, stripes, shard_stride, stripe_stride, batch, shard_len, &st);
    if (rc) return rc;
    int dev = 0;
    if ((rc = current_dev_or_fail(&dev))) return rc;
    auto hp = enc->encode_plan();
    const DevPlan* plan = nullptr;
    if ((rc = enc->dev_plan("E", *hp, dev, &plan))) return rc;
    if (block == 0 || block > shard_len) block = shard_len;
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
        if (encode_crc_supported(a)) {
            const hipError_t e = launch_encode_crc(a, s);
            if (e != hipSuccess) return hip_fail(e, "launch encode_crc_kernel");
            return BLBRS_OK;
        }
    }
    // Shapes without a fused instantiation (or unaligned): the coding pass, then the CRC of
    // each parity row -- same results, one more read of the parity.
    if ((rc = run_plan(*plan, st, batch, shard_len, Mode::kStore, nullptr, s))) return rc;
    const size_t nblocks = (shard_len + block - 1) / block;
    for (int j = 0; j < enc->m; ++j) {
        const hipError_t e = crc32c_blocks(stripes + static_cast<size_t>(enc->k + j) * shard_stride, stripe_stride,
                                           batch, shard_len, block, crc_out_dev + j * batch * nblocks, s);
        if (e != hipSuccess) return hip_fail(e, "crc32c_blocks");
    }
    return BLBRS_OK;
}

int blbrs_crc32c(const uint8_t* data, size_t len, size_t block, uint32_t* out) {
    if (!data || !out) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (len == 0) return BLBRS_OK;
    if (block == 0) block = len;
    WorkerLease lease;
    int rc = lease_worker(lease);
    if (rc) return rc;
    Worker& w = *lease.w;
    const size_t nblocks = (len + block - 1) / block;
    uint64_t view = 0;
    const uint8_t* src = nullptr;
    if (device_view(data, &view)) {
        src = reinterpret_cast<const uint8_t*>(view);  // pinned / device memory: in place
    } else {
        if ((rc = w.ensure(round_up(len, 256)))) return rc;
        HIP_TRY(hipMemcpyAsync(w.dbuf, data, len, hipMemcpyHostToDevice, w.s[0]));
        src = w.dbuf;
    }
    uint32_t* dout = nullptr;
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&dout), nblocks * 4, w.s[0]));
    hipError_t e = crc32c_blocks(src, len, 1, len, block, dout, w.s[0]);
    if (e == hipSuccess) e = hipMemcpyAsync(out, dout, nblocks * 4, hipMemcpyDeviceToHost, w.s[0]);
    (void)hipFreeAsync(dout, w.s[0]);
    if (e == hipSuccess) e = hipStreamSynchronize(w.s[0]);
    if (e != hipSuccess) return hip_fail(e, "crc32c");
    return BLBRS_OK;
}

// ---- batched client reconstructs ----

int blbrs_batcher_new(int max_batch, int window_us, blbrs_batcher** out) {
    if (!out) return fail(BLBRS_ERR_INVALID_ARG, "out is NULL");
    *out = nullptr;
    if (max_batch <= 0 || window_us < 0) return fail(BLBRS_ERR_INVALID_ARG, "max_batch must be > 0, window_us >= 0");
    int dev = 0;
    int rc = current_dev_or_fail(&dev);
    if (rc) return rc;
    auto* b = new blbrs_batcher();
    b->device = dev;
    b->max_batch = static_cast<size_t>(max_batch);
    b->window = std::chrono::microseconds(window_us);
    hipError_t e = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete b;
        return hip_fail(e, "hipStreamCreate");
    }
    b->th = std::thread([b] { b->run(); });
    *out = b;
    return BLBRS_OK;
}

void blbrs_batcher_free(blbrs_batcher* b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->mu);
        b->stop = true;
    }
    b->cv_in.notify_all();
    b->th.join();  // drains the queue first
    (void)hipStreamDestroy(b->stream);
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

int blbrs_pack_dev(uint8_t* dst, size_t dst_stride, size_t npieces, size_t piece_len,
                   const blbrs_pack_extent* extents, size_t nextents, void* stream) {
    if (npieces == 0 || piece_len == 0) {
        if (nextents) return fail(BLBRS_ERR_INVALID_ARG, "extents given for empty pieces");
        return BLBRS_OK;
    }
    if (!dst || (nextents && !extents)) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    if (npieces > 1 && dst_stride < piece_len) return fail(BLBRS_ERR_INVALID_ARG, "stride smaller than piece length");
    int dev = 0;
    int rc = current_dev_or_fail(&dev);
    if (rc) return rc;
    uint64_t dview = 0;
    if (!device_view(dst, &dview)) return fail(BLBRS_ERR_INVALID_ARG, "pack destination is not device-accessible");
    // checkTractSpec (store.go:996-1009) per piece, plus the table: piece starts, then
    // {src, offset, length, piece} per extent.
    std::vector<uint64_t> table(npieces + 1 + 4 * nextents);
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
            } else if (!device_view(x.src, &sview)) {
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
    const hipStream_t s = static_cast<hipStream_t>(stream);
    PtrLease lease;
    const uint64_t* tdev = nullptr;
    bool unused = false;
    if ((rc = upload_table(table.data(), table.size(), s, lease, &tdev, &unused))) return rc;
    hipError_t e = pack_pieces(reinterpret_cast<uint8_t*>(dview), dst_stride, npieces, piece_len, tdev, s);
    if (e != hipSuccess) return hip_fail(e, "pack_pieces");
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

const char* blbrs_last_error(void) { return g_last_error.c_str(); }

const char* blbrs_version(void) { return "blbrs 0.1.0 (gfx950; klauspost/reedsolomon@925cb01d6510 semantics)"; }

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
        default: return "unknown error";
    }
}

}  // extern "C"
