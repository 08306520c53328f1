// runtime.hip -- host runtime of libblbrs (see runtime.hpp).
#include "runtime.hpp"

#include "tuning.hpp"

#include <dlfcn.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <shared_mutex>
#include <cstring>
#include <map>
#include <memory>
#include <unordered_map>

namespace blbrs {
namespace rt {

// ---------------------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------------------

namespace {
thread_local std::string g_last_error;
}

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return BLBRS_ERR_HIP;
}

void set_last_error(const std::string& msg) { g_last_error = msg; }
const std::string& last_error() { return g_last_error; }

// ---------------------------------------------------------------------------------------
// devices
// ---------------------------------------------------------------------------------------

namespace {

std::mutex g_defaults_mu;
std::vector<int> g_defaults;   // empty = not chosen yet

constexpr int kMaxDevices = 64;
std::atomic<int64_t> g_load[kMaxDevices];
std::atomic<uint64_t> g_stage_bytes[kMaxDevices];
std::atomic<uint64_t> g_done_waits[kMaxDevices], g_done_fallbacks[kMaxDevices];

void stage_add(int dev, int64_t delta) {
    if (dev >= 0 && dev < kMaxDevices) g_stage_bytes[dev].fetch_add(static_cast<uint64_t>(delta));
}

}  // namespace

int device_count(int* n) {
    int c = 0;
    const hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c <= 0) {
        (void)hipGetLastError();
        return fail(BLBRS_ERR_NO_DEVICE, "no HIP device visible");
    }
    *n = std::min(c, kMaxDevices);
    return BLBRS_OK;
}

int check_devices(const std::vector<int>& devs) {
    if (devs.empty()) return fail(BLBRS_ERR_INVALID_ARG, "empty device list");
    int n = 0;
    int rc = device_count(&n);
    if (rc) return rc;
    for (int d : devs)
        if (d < 0 || d >= n)
            return fail(BLBRS_ERR_INVALID_ARG, "device " + std::to_string(d) + " is not visible (" +
                                                   std::to_string(n) + " devices)");
    return BLBRS_OK;
}

int default_devices(std::vector<int>* out) {
    std::lock_guard<std::mutex> g(g_defaults_mu);
    if (g_defaults.empty()) {
        int n = 0;
        int rc = device_count(&n);
        if (rc) return rc;
        std::vector<int> devs;
        if (const char* env = std::getenv("BLBRS_DEVICES"); env && *env) {
            const char* p = env;
            while (*p) {
                char* end = nullptr;
                const long d = std::strtol(p, &end, 10);
                if (end == p) break;
                devs.push_back(static_cast<int>(d));
                p = *end == ',' ? end + 1 : end;
            }
            if ((rc = check_devices(devs))) return fail(rc, "BLBRS_DEVICES: " + last_error());
        } else {
            for (int d = 0; d < n; ++d) devs.push_back(d);
        }
        g_defaults = devs;
    }
    *out = g_defaults;
    return BLBRS_OK;
}

int set_default_devices(const std::vector<int>& devs) {
    if (!devs.empty()) {
        int rc = check_devices(devs);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> g(g_defaults_mu);
    g_defaults = devs;  // empty: resolved again from $BLBRS_DEVICES / all visible
    return BLBRS_OK;
}

DeviceGuard::~DeviceGuard() {
    if (prev_ >= 0) (void)hipSetDevice(prev_);
}

int DeviceGuard::enter(int dev) {
    int cur = 0;
    BLBRS_HIP_TRY(hipGetDevice(&cur));
    if (prev_ < 0) prev_ = cur;
    if (cur != dev) BLBRS_HIP_TRY(hipSetDevice(dev));
    return BLBRS_OK;
}

void load_add(int dev, int delta) {
    if (dev >= 0 && dev < kMaxDevices) g_load[dev].fetch_add(delta, std::memory_order_relaxed);
}

int64_t load_of(int dev) {
    return dev >= 0 && dev < kMaxDevices ? g_load[dev].load(std::memory_order_relaxed) : 0;
}

namespace {

struct LaneLoad {
    std::atomic<uint64_t> calls{0}, bytes{0};
    std::atomic<int64_t> in_calls{0}, in_bytes{0};
};
LaneLoad g_lanes[kMaxDevices][kMaxLaneOcc];

LaneLoad* lane_of(int dev, int occ) {
    if (dev < 0 || dev >= kMaxDevices || occ < 0) return nullptr;
    return &g_lanes[dev][std::min(occ, kMaxLaneOcc - 1)];
}

}  // namespace

std::vector<std::pair<int, int>> lane_keys(const std::vector<int>& devs) {
    std::vector<std::pair<int, int>> keys(devs.size());
    for (size_t i = 0; i < devs.size(); ++i) {
        int occ = 0;
        for (size_t j = 0; j < i; ++j) occ += devs[j] == devs[i];
        keys[i] = {devs[i], std::min(occ, kMaxLaneOcc - 1)};
    }
    return keys;
}

size_t pick_lane_policy(const int* nodes, const int64_t* loads, size_t n, size_t start, int node) {
    size_t best = start, best_local = n;
    for (size_t j = 0; j < n; ++j) {
        const size_t i = (start + j) % n;
        if (loads[i] < loads[best]) best = i;
        if (node >= 0 && nodes[i] == node && (best_local == n || loads[i] < loads[best_local])) best_local = i;
    }
    if (best_local < n && loads[best_local] <= loads[best] + kNumaSlackBytes) return best_local;
    return best;
}

size_t pick_lane(const std::vector<int>& lanes, std::atomic<unsigned>& rr, int node) {
    const size_t n = lanes.size();
    const auto keys = lane_keys(lanes);
    std::vector<int64_t> loads(n);
    std::vector<int> nodes(n, -1);
    for (size_t i = 0; i < n; ++i) {
        const LaneLoad* l = lane_of(keys[i].first, keys[i].second);
        loads[i] = l ? l->in_bytes.load(std::memory_order_relaxed) : 0;
        if (node >= 0) nodes[i] = device_numa_node(keys[i].first);
    }
    return pick_lane_policy(nodes.data(), loads.data(), n, rr.fetch_add(1, std::memory_order_relaxed) % n, node);
}

namespace {

// Device -> NUMA node, -2 = not looked up yet.
std::atomic<int> g_dev_node[kMaxDevices];
std::once_flag g_dev_node_once;

int read_device_node(int dev) {
    char bdf[64] = {};
    if (hipDeviceGetPCIBusId(bdf, sizeof bdf, dev) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    std::string path = "/sys/bus/pci/devices/";
    for (const char* c = bdf; *c; ++c) path += static_cast<char>(std::tolower(static_cast<unsigned char>(*c)));
    path += "/numa_node";
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node;
}

// The node of the page at p (get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)), -1 if unknown.
int page_node(const void* p) {
    int node = -1;
    constexpr unsigned long kMpolFNode = 1, kMpolFAddr = 2;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0ul, p, kMpolFNode | kMpolFAddr) != 0) return -1;
    return node;
}

// Pool-handed and registered host buffers -> their node (recorded once per buffer).
struct NodeMap {
    std::shared_mutex mu;
    std::map<uintptr_t, std::pair<size_t, int>> ranges;  // base -> (length, node)
};
NodeMap& node_map() {
    static NodeMap* m = new NodeMap();
    return *m;
}
void note_range(const void* p, size_t n) {
    const int node = page_node(p);
    NodeMap& m = node_map();
    std::unique_lock<std::shared_mutex> g(m.mu);
    m.ranges[reinterpret_cast<uintptr_t>(p)] = {n, node};
}
void drop_range(const void* p) {
    NodeMap& m = node_map();
    std::unique_lock<std::shared_mutex> g(m.mu);
    m.ranges.erase(reinterpret_cast<uintptr_t>(p));
}

}  // namespace

int device_numa_node(int dev) {
    if (dev < 0 || dev >= kMaxDevices) return -1;
    std::call_once(g_dev_node_once, [] {
        for (auto& v : g_dev_node) v.store(-2);
    });
    int v = g_dev_node[dev].load(std::memory_order_acquire);
    if (v == -2) {
        v = read_device_node(dev);
        int expect = -2;
        if (!g_dev_node[dev].compare_exchange_strong(expect, v)) v = expect;
    }
    return v;
}

int set_device_numa_node(int dev, int node) {
    if (dev < 0 || dev >= kMaxDevices || node < -1) return fail(BLBRS_ERR_INVALID_ARG, "bad device or node");
    (void)device_numa_node(dev);  // initialise the table
    g_dev_node[dev].store(node, std::memory_order_release);
    return BLBRS_OK;
}

int host_numa_node(const void* p) {
    if (!p) return -1;
    NodeMap& m = node_map();
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::shared_lock<std::shared_mutex> g(m.mu);
    auto it = m.ranges.upper_bound(a);
    if (it == m.ranges.begin()) return -1;
    --it;
    return a < it->first + it->second.first ? it->second.second : -1;
}

void LoadTicket::take(int d, int o, uint64_t b) {
    dev = d;
    occ = o;
    bytes = b;
    load_add(d, 1);
    if (LaneLoad* l = lane_of(d, o)) {
        l->calls.fetch_add(1, std::memory_order_relaxed);
        l->bytes.fetch_add(b, std::memory_order_relaxed);
        l->in_calls.fetch_add(1, std::memory_order_relaxed);
        l->in_bytes.fetch_add(static_cast<int64_t>(b), std::memory_order_relaxed);
    }
}

LoadTicket::~LoadTicket() {
    if (dev < 0) return;
    load_add(dev, -1);
    if (LaneLoad* l = lane_of(dev, occ)) {
        l->in_calls.fetch_sub(1, std::memory_order_relaxed);
        l->in_bytes.fetch_sub(static_cast<int64_t>(bytes), std::memory_order_relaxed);
    }
}

int lane_stats(int dev, int occ, blbrs_lane_stats* out) {
    const LaneLoad* l = lane_of(dev, occ);
    if (!l) return fail(BLBRS_ERR_INVALID_ARG, "no such lane");
    out->calls = l->calls.load();
    out->bytes = l->bytes.load();
    out->inflight_calls = l->in_calls.load();
    out->inflight_bytes = l->in_bytes.load();
    return BLBRS_OK;
}

bool device_view(const void* p, uint64_t* view, int* owner) {
    if (owner) *owner = -1;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the sticky error
        return false;
    }
    if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) {
        *view = reinterpret_cast<uint64_t>(p);
        if (owner) *owner = attr.device;
        return true;
    }
    if (attr.type == hipMemoryTypeHost && attr.devicePointer && attr.hostPointer) {
        *view = reinterpret_cast<uint64_t>(attr.devicePointer) +
                (reinterpret_cast<uintptr_t>(p) - reinterpret_cast<uintptr_t>(attr.hostPointer));
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------------------
// pointer-table check
// ---------------------------------------------------------------------------------------

namespace {
std::atomic<uint32_t> g_tag{0};
std::atomic<int> g_corrupt_slot{-1};
std::mutex g_fault_mu;
std::map<int, uint32_t*> g_dev_fault;  // process lifetime
}  // namespace

uint32_t next_table_tag() {
    for (;;) {
        const uint32_t t = g_tag.fetch_add(1, std::memory_order_relaxed) & 0xFFFFu;
        if (t) return t;
    }
}

int tag_entries(const uint64_t* ptrs, size_t count, uint32_t tag, uint64_t* out, bool* aligned) {
    bool al = true;
    for (size_t i = 0; i < count; ++i) {
        if (ptrs[i] > kPtrMask)
            return fail(BLBRS_ERR_INVALID_ARG, "shard address above the 48-bit address space (entry " + std::to_string(i) + ")");
        out[i] = ptrs[i] | static_cast<uint64_t>(tag) << kPtrTagShift;
        al = al && aligned16(ptrs[i]);
    }
    if (const int c = g_corrupt_slot.exchange(-1); c >= 0 && static_cast<size_t>(c) < count)
        out[c] = ptrs[c] | static_cast<uint64_t>(tag ^ 0x5A5Au) << kPtrTagShift;
    *aligned = al;
    return BLBRS_OK;
}

void corrupt_next_table(int slot) { g_corrupt_slot.store(slot); }

int alloc_fault_record(uint32_t** out) {
    *out = nullptr;
    void* p = nullptr;
    BLBRS_HIP_TRY(hipHostMalloc(&p, kFaultWords * 4, hipHostMallocDefault));
    std::memset(p, 0, kFaultWords * 4);
    *out = static_cast<uint32_t*>(p);
    return BLBRS_OK;
}

uint32_t* device_fault_record(int dev) {
    std::lock_guard<std::mutex> g(g_fault_mu);
    uint32_t*& r = g_dev_fault[dev];
    if (!r && alloc_fault_record(&r) != BLBRS_OK) r = nullptr;
    return r;
}

int check_fault(uint32_t* rec, const char* what) {
    if (!rec) return BLBRS_OK;
    volatile uint32_t* v = rec;
    if (!v[0]) return BLBRS_OK;
    const uint64_t e = (static_cast<uint64_t>(v[5]) << 32) | v[4];
    const std::string msg = std::string(what) + ": pointer table entry of stripe " + std::to_string(v[1]) + " slot " +
                            std::to_string(v[2]) + " holds 0x" + [&] {
                                char b[32];
                                std::snprintf(b, sizeof b, "%016llx", static_cast<unsigned long long>(e));
                                return std::string(b);
                            }() + " (tag " + std::to_string(e >> kPtrTagShift) + ", launch tag " + std::to_string(v[3]) +
                            "); the stripe was not coded";
    for (int i = 0; i < kFaultWords; ++i) v[i] = 0;
    return fail(BLBRS_ERR_HIP, msg);
}

// ---------------------------------------------------------------------------------------
// stream workers
// ---------------------------------------------------------------------------------------

int Worker::ensure_events() {
    for (auto& e : ev)
        if (!e) BLBRS_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return BLBRS_OK;
}

int Worker::ensure_bounce(size_t bytes) {
    if (!flag_host) BLBRS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&flag_host), 64, hipHostMallocDefault));
    if (bytes <= bounce_cap) return BLBRS_OK;
    note_released(bounce, bounce_cap, "worker staging (grown)");
    if (bounce) {
        // Calls that ended on a completion word leave their launch's tail on the streams.
        for (auto& x : s) (void)hipStreamSynchronize(x);
        (void)hipHostFree(bounce);
    }
    stage_add(device, -static_cast<int64_t>(bounce_cap));
    bounce = nullptr;
    bounce_dev = 0;
    bounce_cap = 0;
    const size_t cap = round_up(std::max<size_t>(bytes, size_t{64} << 10), size_t{64} << 10);
    BLBRS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&bounce), cap, hipHostMallocDefault));
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, bounce, 0);
    if (e != hipSuccess || !d) {
        (void)hipHostFree(bounce);
        bounce = nullptr;
        return hip_fail(e != hipSuccess ? e : hipErrorInvalidValue, "bounce buffer device mapping");
    }
    bounce_dev = reinterpret_cast<uint64_t>(d);
    bounce_cap = cap;
    stage_add(device, static_cast<int64_t>(cap));  // reported as the device's staging bytes
    return BLBRS_OK;
}

int Worker::upload_table(const uint64_t* ptrs, size_t count, const uint64_t** dev_out, bool* aligned,
                         uint32_t* tag) {
    if (count > tab_cap) {
        // The previous copy out of tab_host completes before the tables are released.
        for (auto& x : s) (void)hipStreamSynchronize(x);
        note_released(tab_host, tab_cap * 8, "worker table host (grown)");
        note_released(tab_dev, tab_cap * 8, "worker table device (grown)");
        if (tab_host) (void)hipHostFree(tab_host);
        if (tab_dev) (void)hipFree(tab_dev);
        tab_host = nullptr;
        tab_dev = nullptr;
        tab_cap = 0;
        const size_t cap = std::max<size_t>(round_up(count, 64), 256);
        BLBRS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&tab_host), cap * 8, hipHostMallocDefault));
        BLBRS_HIP_TRY(hipMalloc(reinterpret_cast<void**>(&tab_dev), cap * 8));
        tab_cap = cap;
    }
    *tag = next_table_tag();
    if (int rc = tag_entries(ptrs, count, *tag, tab_host, aligned)) return rc;
    BLBRS_HIP_TRY(hipMemcpyAsync(tab_dev, tab_host, count * 8, hipMemcpyHostToDevice, s[0]));
    *dev_out = tab_dev;
    return BLBRS_OK;
}

int Worker::ensure_done() {
    if (done_host) return BLBRS_OK;
    uint32_t* h = nullptr;
    BLBRS_HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h), 64, hipHostMallocCoherent | hipHostMallocMapped));
    *h = 0;
    void* d = nullptr;
    uint32_t* cnt = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e == hipSuccess && !d) e = hipErrorInvalidValue;
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&cnt), sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), s[0]);
    if (e == hipSuccess) e = hipStreamSynchronize(s[0]);
    if (e != hipSuccess) {
        if (cnt) (void)hipFree(cnt);
        (void)hipHostFree(h);
        return hip_fail(e, "completion word");
    }
    done_host = h;
    done_dev = static_cast<uint32_t*>(d);
    done_count = cnt;
    return BLBRS_OK;
}

uint32_t Worker::next_done_seq() {
    const uint32_t cur = __atomic_load_n(done_host, __ATOMIC_ACQUIRE);
    do ++done_seq;
    while (done_seq == 0 || done_seq == cur);
    return done_seq;
}

int Worker::wait_done(uint32_t seq) {
    using Clock = std::chrono::steady_clock;
    const auto limit = Clock::now() + std::chrono::microseconds(kDoneSpinUs);
    for (uint32_t spins = 1;; ++spins) {
        if (__atomic_load_n(done_host, __ATOMIC_ACQUIRE) == seq) {
            if (device >= 0 && device < kMaxDevices) g_done_waits[device].fetch_add(1, std::memory_order_relaxed);
            return BLBRS_OK;
        }
        if (spins % 64 == 0 && Clock::now() > limit) break;
        __builtin_ia32_pause();
    }
    if (device >= 0 && device < kMaxDevices) g_done_fallbacks[device].fetch_add(1, std::memory_order_relaxed);
    hipError_t e = hipStreamSynchronize(s[0]);
    if (e != hipSuccess) return hip_fail(e, "small call");
    if (__atomic_load_n(done_host, __ATOMIC_ACQUIRE) != seq) {
        // The launches finished without publishing (none carried the word): restart the count.
        e = hipMemsetAsync(done_count, 0, sizeof(uint32_t), s[0]);
        if (e == hipSuccess) e = hipStreamSynchronize(s[0]);
        if (e != hipSuccess) return hip_fail(e, "completion word reset");
    }
    return BLBRS_OK;
}

void Worker::destroy() {
    for (auto& x : s)
        if (x) {
            (void)hipStreamSynchronize(x);
            (void)hipStreamDestroy(x);
            x = nullptr;
        }
    note_released(flag, 4, "worker flag (destroy)");
    note_released(tab_host, tab_cap * 8, "worker table host (destroy)");
    note_released(tab_dev, tab_cap * 8, "worker table device (destroy)");
    note_released(bounce, bounce_cap, "worker staging (destroy)");
    if (flag) (void)hipFree(flag);
    if (tab_host) (void)hipHostFree(tab_host);
    if (tab_dev) (void)hipFree(tab_dev);
    if (fault) (void)hipHostFree(fault);
    if (bounce) (void)hipHostFree(bounce);
    if (flag_host) (void)hipHostFree(flag_host);
    if (done_host) (void)hipHostFree(done_host);
    if (done_count) (void)hipFree(done_count);
    done_host = done_dev = done_count = nullptr;
    for (auto& e : ev)
        if (e) (void)hipEventDestroy(e);
    stage_add(device, -static_cast<int64_t>(bounce_cap));
    fault = nullptr;
    bounce = nullptr;
    flag_host = nullptr;
    ev[0] = ev[1] = nullptr;
    bounce_dev = 0;
    bounce_cap = 0;
    flag = nullptr;
    tab_host = nullptr;
    tab_dev = nullptr;
    tab_cap = 0;
}

namespace {

std::atomic<int> g_worker_limit{8};

struct DevicePool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Worker*> idle;
    int live = 0;  // created and not destroyed
    uint64_t waits = 0;
    std::atomic<uint64_t> calls{0};
};

std::mutex g_pools_mu;
std::map<int, DevicePool*> g_pools;  // process lifetime

DevicePool& pool_of(int dev) {
    std::lock_guard<std::mutex> g(g_pools_mu);
    auto& p = g_pools[dev];
    if (!p) p = new DevicePool();
    return *p;
}

// Creates a worker on the current device (== dev); on failure everything made is released.
int make_worker(int dev, Worker** out) {
    auto* w = new Worker();
    w->device = dev;
    hipError_t e = hipSuccess;
    for (auto& x : w->s)
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&w->flag, sizeof(int32_t));
    if (e == hipSuccess && alloc_fault_record(&w->fault) != BLBRS_OK) e = hipErrorOutOfMemory;
    if (e != hipSuccess) {
        w->destroy();
        delete w;
        return hip_fail(e, "stream worker setup");
    }
    *out = w;
    return BLBRS_OK;
}

}  // namespace

WorkerLease::~WorkerLease() {
    if (!w_) return;
    DevicePool& p = pool_of(w_->device);
    {
        std::lock_guard<std::mutex> g(p.mu);
        p.idle.push_back(w_);
    }
    p.cv.notify_one();
}

int WorkerLease::acquire(int dev) {
    DevicePool& p = pool_of(dev);
    {
        std::unique_lock<std::mutex> lk(p.mu);
        bool waited = false;
        for (;;) {
            if (!p.idle.empty()) {
                w_ = p.idle.back();
                p.idle.pop_back();
                return BLBRS_OK;
            }
            if (p.live < g_worker_limit.load()) {
                ++p.live;  // reserve the slot, build outside the lock
                break;
            }
            if (!waited) {
                ++p.waits;
                waited = true;
            }
            p.cv.wait(lk);
        }
    }
    Worker* w = nullptr;
    const int rc = make_worker(dev, &w);
    if (rc) {
        {
            std::lock_guard<std::mutex> g(p.mu);
            --p.live;
        }
        p.cv.notify_one();
        return rc;
    }
    w_ = w;
    return BLBRS_OK;
}

int set_worker_limit(int per_device) {
    if (per_device < 1) return fail(BLBRS_ERR_INVALID_ARG, "worker limit must be >= 1");
    g_worker_limit.store(per_device);
    std::lock_guard<std::mutex> g(g_pools_mu);
    for (auto& [d, p] : g_pools) p->cv.notify_all();
    return BLBRS_OK;
}

int worker_limit() { return g_worker_limit.load(); }

void note_call(int dev) { pool_of(dev).calls.fetch_add(1, std::memory_order_relaxed); }

int device_stats(int dev, blbrs_device_stats* out) {
    DevicePool& p = pool_of(dev);
    std::lock_guard<std::mutex> g(p.mu);
    out->workers = static_cast<uint64_t>(p.live);
    out->idle = p.idle.size();
    out->waits = p.waits;
    out->staging_bytes = dev >= 0 && dev < kMaxDevices ? g_stage_bytes[dev].load() : 0;
    out->calls = p.calls.load();
    out->inflight = load_of(dev);
    const bool in = dev >= 0 && dev < kMaxDevices;
    out->done_waits = in ? g_done_waits[dev].load(std::memory_order_relaxed) : 0;
    out->done_fallbacks = in ? g_done_fallbacks[dev].load(std::memory_order_relaxed) : 0;
    return BLBRS_OK;
}

void trim_workers() {
    std::vector<std::pair<int, DevicePool*>> pools;
    {
        std::lock_guard<std::mutex> g(g_pools_mu);
        for (auto& [d, p] : g_pools) pools.emplace_back(d, p);
    }
    for (auto& [d, p] : pools) {
        std::vector<Worker*> idle;
        {
            std::lock_guard<std::mutex> g(p->mu);
            idle.swap(p->idle);
            p->live -= static_cast<int>(idle.size());
        }
        if (idle.empty()) continue;
        DeviceGuard guard;
        if (guard.enter(d) != BLBRS_OK) continue;
        for (Worker* w : idle) {
            w->destroy();
            delete w;
        }
        p->cv.notify_all();
    }
}

// ---------------------------------------------------------------------------------------
// pointer tables on caller streams
// ---------------------------------------------------------------------------------------

struct PtrSlot {
    std::mutex mu;
    uint64_t* host = nullptr;
    uint64_t* dev = nullptr;
    size_t cap = 0;        // entries of `host`
    size_t dev_bytes = 0;  // bytes of `dev`: the table, then scratch (PtrLease::upload `extra`)
    hipEvent_t done = nullptr;
};

namespace {

struct SlotRing {
    static constexpr int kSlots = 16;
    PtrSlot slots[kSlots];
    std::atomic<unsigned> next{0};
};

std::mutex g_rings_mu;
std::map<int, SlotRing*> g_rings;  // process lifetime

SlotRing& ring_of(int dev) {
    std::lock_guard<std::mutex> g(g_rings_mu);
    auto& r = g_rings[dev];
    if (!r) r = new SlotRing();
    return *r;
}

}  // namespace

PtrLease::~PtrLease() {
    if (slot_) {
        (void)hipEventRecord(slot_->done, stream_);
        slot_->mu.unlock();
    }
}

int PtrLease::upload(const uint64_t* ptrs, size_t count, hipStream_t stream, const uint64_t** dev_out,
                     bool* aligned, uint32_t* tag, size_t extra, void** extra_out) {
    int dev = 0;
    BLBRS_HIP_TRY(hipGetDevice(&dev));
    SlotRing& r = ring_of(dev);
    const size_t need = round_up(std::max<size_t>(count, 1) * 8, 256) + extra;
    PtrSlot* pick = nullptr;
    if (extra) {
        // Scratch-carrying uploads (pack_encode's descriptors, ~100 MB at blb's shapes) prefer an
        // idle slot that is already big enough, so a stream of calls does not reallocate scratch
        // in every slot of the ring.
        const unsigned start = r.next.load(std::memory_order_relaxed);
        for (int j = 0; j < SlotRing::kSlots && !pick; ++j) {
            PtrSlot& c = r.slots[(start + j) % SlotRing::kSlots];
            if (c.dev_bytes < need || !c.mu.try_lock()) continue;
            if (!c.done || hipEventQuery(c.done) == hipSuccess) pick = &c;
            else c.mu.unlock();
        }
        (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    }
    if (!pick) {
        pick = &r.slots[r.next.fetch_add(1) % SlotRing::kSlots];
        pick->mu.lock();
    }
    PtrSlot& s = *pick;
    if (!s.done) {
        const hipError_t e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e != hipSuccess) {
            s.mu.unlock();
            return hip_fail(e, "hipEventCreate");
        }
    } else {
        const hipError_t e = hipEventSynchronize(s.done);
        if (e != hipSuccess) {
            s.mu.unlock();
            return hip_fail(e, "hipEventSynchronize");
        }
    }
    const size_t tab_bytes = round_up(std::max<size_t>(count, 1) * 8, 256);
    if (s.cap < count || s.dev_bytes < tab_bytes + extra) {
        // The slot's previous launches are done (the event wait above).
        if (s.host) (void)hipHostFree(s.host);
        if (s.dev) (void)hipFree(s.dev);
        s.host = nullptr;
        s.dev = nullptr;
        s.cap = 0;
        s.dev_bytes = 0;
        const size_t cap = std::max<size_t>(count, 1024);
        const size_t dev_bytes = std::max(round_up(cap * 8, 256), tab_bytes + extra);
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&s.host), cap * 8, hipHostMallocDefault);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&s.dev), dev_bytes);
        if (e != hipSuccess) {
            s.mu.unlock();
            return hip_fail(e, "ptr table alloc");
        }
        s.cap = cap;
        s.dev_bytes = dev_bytes;
    }
    if (extra_out) *extra_out = extra ? reinterpret_cast<uint8_t*>(s.dev) + tab_bytes : nullptr;
    if (tag) {
        *tag = next_table_tag();
        if (int rc = tag_entries(ptrs, count, *tag, s.host, aligned)) {
            s.mu.unlock();
            return rc;
        }
    } else {
        bool al = true;
        for (size_t i = 0; i < count; ++i) {
            s.host[i] = ptrs[i];
            al = al && aligned16(ptrs[i]);
        }
        *aligned = al;
    }
    slot_ = &s;
    stream_ = stream;
    BLBRS_HIP_TRY(hipMemcpyAsync(s.dev, s.host, count * 8, hipMemcpyHostToDevice, stream));
    *dev_out = s.dev;
    return BLBRS_OK;
}

namespace {
struct Released {
    uint64_t lo = 0, hi = 0;
    const char* what = nullptr;
    uint64_t seq = 0;
};
constexpr size_t kReleasedRing = 4096;
std::mutex g_rel_mu;
Released g_rel[kReleasedRing];
uint64_t g_rel_seq = 0;

hsa_status_t on_system_event(const hsa_amd_event_t* e, void*) {
    if (!e || e->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
    const uint64_t a = e->memory_fault.virtual_address;
    std::fprintf(stderr, "blbrs: GPU memory fault at 0x%llx (reason mask 0x%x)\n", static_cast<unsigned long long>(a),
                 e->memory_fault.fault_reason_mask);
    std::unique_lock<std::mutex> g(g_rel_mu, std::try_to_lock);
    if (g.owns_lock()) {
        // The fault address is a page (or coarser) address: report ranges within 2 MiB of it.
        constexpr uint64_t kNear = 2ull << 20;
        int shown = 0;
        for (size_t i = 0; i < kReleasedRing && shown < 32; ++i) {
            const Released& r = g_rel[i];
            if (!r.what || a + kNear < r.lo || a >= r.hi + kNear) continue;
            std::fprintf(stderr, "blbrs:   released #%llu (%llu ago) %s [0x%llx, 0x%llx)%s\n",
                         static_cast<unsigned long long>(r.seq), static_cast<unsigned long long>(g_rel_seq - r.seq),
                         r.what, static_cast<unsigned long long>(r.lo), static_cast<unsigned long long>(r.hi),
                         a >= r.lo && a < r.hi ? "  <-- contains the address" : "");
            ++shown;
        }
        std::fprintf(stderr, "blbrs:   %d released range(s) near it of %llu released; live pool/registered node: %d\n", shown,
                     static_cast<unsigned long long>(g_rel_seq), host_numa_node(reinterpret_cast<const void*>(a)));
    }
    return HSA_STATUS_SUCCESS;
}
}  // namespace

void note_released(const void* p, size_t n, const char* what) {
    if (!p) return;
    std::lock_guard<std::mutex> g(g_rel_mu);
    Released& r = g_rel[g_rel_seq % kReleasedRing];
    r.lo = reinterpret_cast<uint64_t>(p);
    r.hi = r.lo + n;
    r.what = what;
    r.seq = ++g_rel_seq;
}

int watch_faults() {
    static std::once_flag once;
    static hsa_status_t st = HSA_STATUS_SUCCESS;
    static std::string why;
    std::call_once(once, [] {
        // HIP's initialisation initialises the HSA runtime it loaded (never a second copy, DESIGN
        // §4h); the handler is looked up in that runtime, not linked.
        (void)hipFree(nullptr);
        using Reg = hsa_status_t (*)(hsa_amd_system_event_callback_t, void*);
        void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
        Reg reg = h ? reinterpret_cast<Reg>(dlsym(h, "hsa_amd_register_system_event_handler")) : nullptr;
        st = reg ? reg(on_system_event, nullptr) : HSA_STATUS_ERROR;
        if (!h) why = "libhsa-runtime64.so.1 is not loaded";
        else if (!reg) why = "hsa_amd_register_system_event_handler not found";
        else if (st != HSA_STATUS_SUCCESS) why = "hsa_amd_register_system_event_handler: status " + std::to_string(st);
    });
    return st == HSA_STATUS_SUCCESS ? BLBRS_OK : fail(BLBRS_ERR_HIP, why);
}

hipError_t upload_pinned(void* dev, const void* src, size_t n) {
    if (n == 0) return hipSuccess;
    static std::mutex mu;
    static uint8_t* buf = nullptr;  // process lifetime
    static size_t cap = 0;
    std::lock_guard<std::mutex> g(mu);
    if (n > cap) {
        if (buf) (void)hipHostFree(buf);  // the previous upload was synchronous
        buf = nullptr;
        cap = 0;
        const size_t want = round_up(std::max<size_t>(n, 64 << 10), 64 << 10);
        const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&buf), want, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        cap = want;
    }
    std::memcpy(buf, src, n);
    return hipMemcpy(dev, buf, n, hipMemcpyHostToDevice);
}

// ---------------------------------------------------------------------------------------
// pinned buffer pool -- rpc.GetBuffer / PutBuffer (pkg/rpc/pool.go:16-62)
// ---------------------------------------------------------------------------------------
//
// Same capacity classes as blb's pool: 1 MiB, 4 MiB and 8 MiB (+ disk.ExtraRoom = one 64 KiB
// ChecksumFile block, pkg/disk/checksum_file.go:27), plus a 128 KiB + ExtraRoom class for the
// library's own staging of small pageable shards (blb does not pool that size).  Larger
// requests get an exact allocation, freed on Put.  Buffers are pinned and mapped for every
// device (hipHostMallocDefault = portable | mapped), so the coding kernels read and write them
// in place over PCIe.  Like sync.Pool, Get never blocks; idle buffers above the idle limit are
// freed on Put.
//
// Lifetime.  blb's pool is a sync.Pool (pkg/rpc/pool.go:22-26): a buffer that is never
// PutBuffer'd is simply garbage-collected, and blb relies on that (reconstruct.go:126-152
// drops errored and straggling replies; bulk_codec.go:212-221 returns on a read error with
// the buffer it took).  Library-owned buffers cannot follow the GC, so callers with that
// pattern register memory they own instead (pool_register: the Go shim registers Go-heap
// buffers and unregisters them from a finalizer), and every pinned byte -- handed out or
// registered -- counts against a live limit: past it the pool refuses (BLBRS_ERR_LIMIT) and
// the caller uses pageable memory, which the engine stages.

namespace {

constexpr size_t kExtraRoom = 64 << 10;
constexpr size_t kClasses[] = {(size_t{128} << 10) + kExtraRoom, (size_t{1} << 20) + kExtraRoom,
                               (size_t{4} << 20) + kExtraRoom, (size_t{8} << 20) + kExtraRoom};
constexpr int kNumClasses = 4;

struct HostPool {
    std::mutex mu;
    std::vector<uint8_t*> free_list[kNumClasses];
    std::unordered_map<uint8_t*, size_t> live;        // every buffer handed out -> capacity
    std::unordered_map<uintptr_t, size_t> registered;  // caller memory pinned -> length
    size_t idle_bytes = 0, live_bytes = 0, registered_bytes = 0;
    size_t idle_limit = size_t{4} << 30;
    size_t live_limit = size_t{16} << 30;  // 0 = none
    uint64_t gets = 0, puts = 0, allocs = 0, frees = 0, registrations = 0, rejects = 0;

    // Room for `bytes` more pinned bytes under the live limit (mu held).
    bool room_for(size_t bytes) const {
        return live_limit == 0 || live_bytes + registered_bytes + bytes <= live_limit;
    }
};

HostPool& host_pool() {
    static HostPool* p = new HostPool();  // process lifetime
    return *p;
}

int class_of(size_t cap) {
    for (int c = 0; c < kNumClasses; ++c)
        if (cap == kClasses[c]) return c;
    return -1;
}

int limit_fail(HostPool& p, size_t want) {
    ++p.rejects;
    return fail(BLBRS_ERR_LIMIT, "pinned live limit reached (" + std::to_string(p.live_bytes + p.registered_bytes) +
                                     " + " + std::to_string(want) + " > " + std::to_string(p.live_limit) + " bytes)");
}

}  // namespace

int pool_get(size_t n, uint8_t** out, size_t* cap, bool internal) {
    *out = nullptr;
    if (n == 0) return fail(BLBRS_ERR_INVALID_ARG, "zero-length buffer");
    HostPool& p = host_pool();
    size_t want = n;
    int c = 0;
    while (c < kNumClasses && n > kClasses[c]) ++c;
    if (c < kNumClasses) want = kClasses[c];
    {
        std::lock_guard<std::mutex> g(p.mu);
        ++p.gets;
        if (!internal && !p.room_for(want)) return limit_fail(p, want);
        if (c < kNumClasses && !p.free_list[c].empty()) {
            uint8_t* b = p.free_list[c].back();
            p.free_list[c].pop_back();
            p.idle_bytes -= want;
            p.live[b] = want;
            p.live_bytes += want;
            *out = b;
            *cap = want;
            return BLBRS_OK;
        }
        // Reserve the bytes before allocating outside the lock, so that concurrent gets
        // cannot overshoot the limit together.
        p.live_bytes += want;
    }
    int nd = 0;
    int rc = device_count(&nd);
    uint8_t* b = nullptr;
    hipError_t e = hipSuccess;
    if (rc == BLBRS_OK) e = hipHostMalloc(reinterpret_cast<void**>(&b), want, hipHostMallocDefault);
    std::lock_guard<std::mutex> g(p.mu);
    if (rc != BLBRS_OK || e != hipSuccess) {
        p.live_bytes -= want;
        return rc != BLBRS_OK ? rc : hip_fail(e, "hipHostMalloc");
    }
    ++p.allocs;
    p.live[b] = want;
    *out = b;
    *cap = want;
    note_range(b, want);  // its NUMA node, for the lane pick (pick_lane)
    return BLBRS_OK;
}

int pool_put(uint8_t* b) {
    if (!b) return BLBRS_OK;
    HostPool& p = host_pool();
    bool free_it = false;
    size_t cap = 0;
    {
        std::lock_guard<std::mutex> g(p.mu);
        auto it = p.live.find(b);
        if (it == p.live.end()) return fail(BLBRS_ERR_INVALID_ARG, "buffer was not allocated by blbrs_buffer_get");
        cap = it->second;
        p.live.erase(it);
        p.live_bytes -= cap;
        ++p.puts;
        const int c = class_of(cap);
        if (c >= 0 && p.idle_bytes + cap <= p.idle_limit) {
            p.free_list[c].push_back(b);
            p.idle_bytes += cap;
        } else {
            free_it = true;
            ++p.frees;
        }
    }
    if (free_it) {
        drop_range(b);
        note_released(b, cap, "pool buffer (hipHostFree on put)");
        BLBRS_HIP_TRY(hipHostFree(b));
    }
    return BLBRS_OK;
}

int pool_register(void* ptr, size_t n) {
    if (!ptr || n == 0) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument or zero length");
    HostPool& p = host_pool();
    const uintptr_t key = reinterpret_cast<uintptr_t>(ptr);
    {
        std::lock_guard<std::mutex> g(p.mu);
        if (p.registered.count(key)) return fail(BLBRS_ERR_INVALID_ARG, "memory is already registered");
        if (!p.room_for(n)) return limit_fail(p, n);
        p.registered[key] = n;  // reserved; undone below if pinning fails
        p.registered_bytes += n;
    }
    int nd = 0;
    int rc = device_count(&nd);
    hipError_t e = hipSuccess;
    if (rc == BLBRS_OK) e = hipHostRegister(ptr, n, hipHostRegisterPortable | hipHostRegisterMapped);
    std::lock_guard<std::mutex> g(p.mu);
    if (rc != BLBRS_OK || e != hipSuccess) {
        p.registered.erase(key);
        p.registered_bytes -= n;
        if (e != hipSuccess) (void)hipGetLastError();
        return rc != BLBRS_OK ? rc : hip_fail(e, "hipHostRegister");
    }
    ++p.registrations;
    note_range(ptr, n);  // its NUMA node, for the lane pick (pick_lane)
    return BLBRS_OK;
}

int pool_unregister(void* ptr) {
    if (!ptr) return fail(BLBRS_ERR_INVALID_ARG, "NULL argument");
    HostPool& p = host_pool();
    const uintptr_t key = reinterpret_cast<uintptr_t>(ptr);
    size_t n = 0;
    {
        std::lock_guard<std::mutex> g(p.mu);
        auto it = p.registered.find(key);
        if (it == p.registered.end()) return fail(BLBRS_ERR_INVALID_ARG, "memory was not registered by blbrs_buffer_register");
        n = it->second;
        p.registered.erase(it);
        p.registered_bytes -= n;
    }
    drop_range(ptr);
    note_released(ptr, n, "registered host buffer (hipHostUnregister)");
    BLBRS_HIP_TRY(hipHostUnregister(ptr));
    return BLBRS_OK;
}

int pool_set_idle_limit(size_t bytes) {
    HostPool& p = host_pool();
    {
        std::lock_guard<std::mutex> g(p.mu);
        p.idle_limit = bytes;
    }
    if (bytes == 0) pool_trim();
    return BLBRS_OK;
}

int pool_set_live_limit(size_t bytes) {
    HostPool& p = host_pool();
    std::lock_guard<std::mutex> g(p.mu);
    p.live_limit = bytes;
    return BLBRS_OK;
}

int pool_stats(blbrs_pool_stats* out) {
    HostPool& p = host_pool();
    std::lock_guard<std::mutex> g(p.mu);
    out->gets = p.gets;
    out->puts = p.puts;
    out->allocs = p.allocs;
    out->frees = p.frees;
    out->live_bytes = p.live_bytes;
    out->idle_bytes = p.idle_bytes;
    out->registered_bytes = p.registered_bytes;
    out->registrations = p.registrations;
    out->live_limit = p.live_limit;
    out->limit_rejects = p.rejects;
    return BLBRS_OK;
}

void pool_trim() {
    HostPool& p = host_pool();
    std::vector<std::pair<uint8_t*, size_t>> drop;
    {
        std::lock_guard<std::mutex> g(p.mu);
        for (int c = 0; c < kNumClasses; ++c) {
            for (uint8_t* b : p.free_list[c]) drop.emplace_back(b, kClasses[c]);
            p.free_list[c].clear();
        }
        p.idle_bytes = 0;
        p.frees += drop.size();
    }
    for (auto [b, cap] : drop) {
        drop_range(b);
        note_released(b, cap, "pool buffer (hipHostFree on trim)");
        (void)hipHostFree(b);
    }
}

}  // namespace rt
}  // namespace blbrs
