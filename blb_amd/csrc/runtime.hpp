// runtime.hpp -- the host runtime under libblbrs's C ABI: errors, device selection, the
// bounded per-device stream-worker pool, pointer-table upload and the pinned buffer pool.
//
// blb calls the RS engine from many goroutines at once: one per RSEncode RPC, bounded only by
// the tractserver's pendingSem / RejectCtlReqThreshold = 1000 (internal/tractserver/
// config.go:91, server.go:553-582), one per curator chunk encode (internal/curator/
// pack_tracts.go:187-196) and one per client degraded read (client/blb/reconstruct.go:65-195).
// cgo runs each on some OS thread whose current HIP device means nothing (goroutines migrate),
// so every call here picks its device itself and leaves the caller's current device as it
// found it:
//   * host-memory calls go to the least-loaded device of the encoder's device list;
//   * device-resident calls run on the device that owns the stripes.
// Workers (two streams, a bounded staging ring, a pointer table and a verify flag) are
// capped per device; a call that finds none idle waits for one instead of growing HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/blb_rs.h"
#include "rs_kernels.hpp"

namespace blbrs {
namespace rt {

// ---- errors (thread-local message, as blbrs_last_error() reports it) ----
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);
void set_last_error(const std::string& msg);
const std::string& last_error();

#define BLBRS_HIP_TRY(expr)                                          \
    do {                                                             \
        hipError_t e_ = (expr);                                      \
        if (e_ != hipSuccess) return ::blbrs::rt::hip_fail(e_, #expr); \
    } while (0)

inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline bool aligned16(uintptr_t x) { return (x & 15u) == 0; }

// ---- devices ----

// Number of visible HIP devices; BLBRS_ERR_NO_DEVICE when there are none.
int device_count(int* n);
// The process default device list: blbrs_set_default_devices(), else $BLBRS_DEVICES
// ("0,1,..."), else every visible device.
int default_devices(std::vector<int>* out);
int set_default_devices(const std::vector<int>& devs);
// Every entry in [0, device_count).
int check_devices(const std::vector<int>& devs);

// Scoped hipSetDevice: restores the calling thread's device on destruction.
class DeviceGuard {
 public:
    DeviceGuard() = default;
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
    ~DeviceGuard();
    int enter(int dev);

 private:
    int prev_ = -1;
};

// Load accounting.  A device list may repeat a device: entry i is lane (dev, occ) where occ
// counts the earlier entries naming the same device, so [0, 0] is two lanes on GPU 0 and an
// encoder on [0, 1] shares lane (0, 0) with every other list that names GPU 0 once.  Each lane
// counts calls and bytes (cumulative and in flight); each device counts calls in flight.
constexpr int kMaxLaneOcc = 16;
void load_add(int dev, int delta);
int64_t load_of(int dev);
// (dev, occ) of every entry of a device list.
std::vector<std::pair<int, int>> lane_keys(const std::vector<int>& devs);
// Index into `lanes` of the entry with the fewest BYTES in flight (a 4 KiB degraded read and
// an 8 MiB increment do not weigh the same); ties rotate through `rr`.  With `node` >= 0 (the
// NUMA node holding the call's host shards) the lanes of GPUs attached to that node are
// preferred: the least-loaded local lane wins unless it carries more than kNumaSlackBytes
// beyond the least-loaded lane overall (then the host link is the smaller cost than the wait).
constexpr int64_t kNumaSlackBytes = int64_t{64} << 20;
size_t pick_lane(const std::vector<int>& lanes, std::atomic<unsigned>& rr, int node = -1);
// The policy itself, over explicit lane nodes and loads, starting the scan at `start` (tests).
size_t pick_lane_policy(const int* nodes, const int64_t* loads, size_t n, size_t start, int node);

// NUMA topology.  device_numa_node: the node the GPU's PCIe root sits on
// (/sys/bus/pci/devices/<bdf>/numa_node), cached; -1 when unknown; set_device_numa_node
// overrides it (containers without sysfs, tests).  host_numa_node: the node of the page at p
// for memory the pool handed out or registered (recorded once per buffer, with
// get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR) on its first page), -1 for anything else.
int device_numa_node(int dev);
int set_device_numa_node(int dev, int node);
int host_numa_node(const void* p);
int lane_stats(int dev, int occ, blbrs_lane_stats* out);

// Holds one call's load on a lane (and its device) for the call's duration.
struct LoadTicket {
    int dev = -1, occ = 0;
    uint64_t bytes = 0;
    void take(int d, int o = 0, uint64_t b = 0);
    ~LoadTicket();
};

// Address under which the GPU reaches `p`: device memory as is, pinned host memory
// (hipHostMalloc / hipHostRegister) through its device mapping.  False for pageable memory.
// *owner = the device holding device memory, -1 for host memory.
bool device_view(const void* p, uint64_t* view, int* owner = nullptr);

// ---- pointer-table check (rs_code.hpp stripe_table_ok) ----
//
// Every shard-pointer table the library uploads is tagged: entry = address | tag << 48, with a
// 16-bit tag drawn per upload.  The coding kernel compares each entry it is about to use with the
// tag of ITS launch; a stripe with a wrong entry -- one left over from another call, or not an
// address the host wrote at all -- is skipped instead of dereferenced, and the first such entry
// is recorded in a pinned, device-mapped record of the table's owner (worker, batcher lane, or
// the device's record for tables on caller streams).  The host reads the record after the call's
// sync: free when clear, a named error when not.  Round 4 saw two illegal-address faults whose
// cause inside the runtime stayed unpinned; a stale or foreign table entry is now
// reported instead of faulting the GPU.
constexpr int kFaultWords = 8;  // valid, stripe, slot, expected tag, entry lo, entry hi, -, -
uint32_t next_table_tag();      // 1 .. 0xFFFF, cycling
// out[i] = ptrs[i] | tag << 48; INVALID_ARG for an address at or above 2^48.  *aligned: every
// address 16-byte aligned.
int tag_entries(const uint64_t* ptrs, size_t count, uint32_t tag, uint64_t* out, bool* aligned);
// A zeroed pinned record mapped for every device.
int alloc_fault_record(uint32_t** out);
// Process-wide record of `dev` (tables on caller streams: the *_ptrs entry points).
uint32_t* device_fault_record(int dev);
// BLBRS_OK when `rec` is clear; else clears it and fails with BLBRS_ERR_HIP naming the entry.
int check_fault(uint32_t* rec, const char* what);
// Test hook (blbrs_debug_corrupt_next_table): the next tagged upload writes entry `slot` with a
// wrong tag (its address intact).
void corrupt_next_table(int slot);

// ---- stream workers ----

// Host calls whose pageable bytes (inputs and outputs, plus the pointer table) fit in this go
// through the worker's pinned bounce buffer: CPU copies in, the kernel reads and writes it in
// place over PCIe, CPU copies out -- one launch and one sync instead of a DMA per shard.
constexpr size_t kBounceMaxBytes = size_t{512} << 10;
// Larger calls with pageable shards are cut into units that alternate over two slots of the same
// pinned staging, each at most this big: the CPU fills one slot while the kernel works in the
// other.  Pageable memory is never handed to HIP's copy engines.
constexpr size_t kPinnedSlotBytes = size_t{8} << 20;
// Single-launch host calls touching at most this many shard bytes, with no verify flag to read
// back, run on rs_small_kernel and end on its completion word (rs_small.hpp; BLBRS_DONE_WORD,
// default on): the word arrives ~3 us before the stream's completion signal would wake the
// caller (tools/sync_probe.hip).  The spin bound covers such a kernel many times
// over; past it the thread waits for the stream.
// Pieces above kDoneMaxPiece keep rs_code_kernel and the stream wait: from 128 KiB a single
// caller gains nothing (128 KiB ties, 256 KiB is 2-5 us slower) and 64 concurrent per-call
// callers lose 20-31 % of their calls/s, while up to 64 KiB the word saves 4.5-7 us a call and
// costs concurrent callers at most 5-10 % at 64 KiB (profiles/r06/concurrency/).
constexpr size_t kDoneMaxBytes = size_t{2} << 20;
constexpr size_t kDoneMaxPiece = size_t{64} << 10;
constexpr int kDoneSpinUs = 2000;

struct Worker {
    int device = -1;
    hipStream_t s[2] = {nullptr, nullptr};
    int32_t* flag = nullptr;        // verify mismatch flag (device)
    uint64_t* tab_host = nullptr;   // pinned pointer table
    uint64_t* tab_dev = nullptr;
    size_t tab_cap = 0;             // entries
    uint32_t* fault = nullptr;      // pinned record of the worker's table checks
    uint8_t* bounce = nullptr;      // pinned, device-mapped staging of pageable shards (CPU copies in
    uint64_t bounce_dev = 0;        //   and out; the kernels read and write it in place)
    size_t bounce_cap = 0;
    int32_t* flag_host = nullptr;   // pinned landing word of the verify flag
    hipEvent_t ev[2] = {nullptr, nullptr};  // staging slot reuse (created on first use)
    // Completion word of small calls (rs_small.hpp SmallArgs, created on first use): a coherent
    // pinned word the call's last launch publishes its sequence number to, its device view, and
    // the device-memory count of finished workgroups behind it.
    uint32_t* done_host = nullptr;
    uint32_t* done_dev = nullptr;
    uint32_t* done_count = nullptr;
    uint32_t done_seq = 0;
    int ensure_bounce(size_t bytes);
    int ensure_events();
    int ensure_done();
    // The next sequence number (never 0, never the word's current value).
    uint32_t next_done_seq();
    // Ends a call whose last launch on s[0] carries word `seq`: spins on the word for up to
    // kDoneSpinUs, then waits for s[0] instead (which reports a fault; a finished launch that
    // never published -- none was made -- restarts the count).  Counted per device.
    int wait_done(uint32_t seq);
    // Copies `count` device addresses, tagged (*tag), to the worker's device table on stream s[0].
    int upload_table(const uint64_t* ptrs, size_t count, const uint64_t** dev_out, bool* aligned, uint32_t* tag);
    void destroy();
};

// Exclusive use of one worker of `dev` for the duration of a call.  acquire() waits while
// the device already has the maximum number of workers and none is idle.
class WorkerLease {
 public:
    WorkerLease() = default;
    WorkerLease(const WorkerLease&) = delete;
    WorkerLease& operator=(const WorkerLease&) = delete;
    ~WorkerLease();
    int acquire(int dev);
    Worker& operator*() const { return *w_; }
    Worker* operator->() const { return w_; }

 private:
    Worker* w_ = nullptr;
};

int set_worker_limit(int per_device);
int worker_limit();
int device_stats(int dev, blbrs_device_stats* out);
void note_call(int dev);
// Frees idle workers of every device (streams, staging, tables).
void trim_workers();

// ---- pointer tables for calls on caller streams (the *_ptrs entry points) ----
struct PtrSlot;
class PtrLease {
 public:
    PtrLease() = default;
    PtrLease(const PtrLease&) = delete;
    PtrLease& operator=(const PtrLease&) = delete;
    ~PtrLease();
    // Uploads on `stream` (current device); the slot stays busy until the stream has run the
    // kernels that read it.  With `tag`, a shard-pointer table: entries tagged (*tag set).
    // `extra` > 0: the slot's device buffer also holds `extra` bytes of scratch after the table
    // (256-byte aligned, *extra_out), free for the launches on `stream` that read the table.
    int upload(const uint64_t* ptrs, size_t count, hipStream_t stream, const uint64_t** dev_out, bool* aligned,
               uint32_t* tag = nullptr, size_t extra = 0, void** extra_out = nullptr);

 private:
    PtrSlot* slot_ = nullptr;
    hipStream_t stream_ = nullptr;
};

// ---- GPU memory-fault watch (diagnostics) ----
// Records a host or device range the library releases (unregistered, freed), kept in a ring of
// the last few thousand; a GPU memory fault reported by the HSA runtime is printed with the ranges
// of that ring and of the live pool / registrations that hold the faulting address.
void note_released(const void* p, size_t n, const char* what);
int watch_faults();  // registers the HSA system event handler once

// Synchronous upload of n bytes of host data through a pinned bounce (pageable memory is never
// handed to HIP's copy engines).  For small, rare uploads: plans, constant tables.
hipError_t upload_pinned(void* dev, const void* src, size_t n);

// ---- pinned buffer pool (rpc.GetBuffer / PutBuffer over pinned, device-mapped memory) ----
// Every pinned byte the pool hands out or registers counts against the live limit; past it
// pool_get / pool_register fail with BLBRS_ERR_LIMIT and callers fall back to pageable
// memory.  `internal` = the library's own transient staging (bounded by the calls in
// flight), which is counted but never refused.
int pool_get(size_t n, uint8_t** out, size_t* cap, bool internal = false);
int pool_put(uint8_t* p);
int pool_register(void* p, size_t n);
int pool_unregister(void* p);
int pool_set_idle_limit(size_t bytes);
int pool_set_live_limit(size_t bytes);
int pool_stats(blbrs_pool_stats* out);
void pool_trim();

}  // namespace rt
}  // namespace blbrs
