// rtc.hpp -- decode networks compiled at run time (hipRTC), one per erasure pattern.
//
// Encode's coefficients are fixed, so its bit-plane XOR networks are compiled into the library
// (gf_bitslice.hpp).  A decode pass's rows -- inv(M[valid]) for missing data,
// P * inv(M[valid]) for missing parity -- depend on which shards are present, i.e. on the
// erasure pattern of the call (klauspost reedsolomon.go reconstruct; blb's recovery RPC
// rebuilds every absent slot, internal/tractserver/store.go:1062-1102).  On wide shapes the
// v_perm table multiply is VALU-bound there too, so for such a pass this module can generate the
// pass's network as straight-line code, compile rs_code_kernel<K, MR, MODE, ADDR, U, NT, Net> (rs_code.hpp) with hipRTC
// against the library's own device headers, and loads it on the device.  The device plan caches
// the kernel next to the pass's tables -- the counterpart of klauspost's inversion tree, one
// level further: a compiled kernel per cached inverse.
//
// On by default again since round 6 (knob BLBRS_RTC = 1; off in round 5).  Only RS(12,5)-wide
// multi-row passes take a network (k + rows > BLBRS_RTC_WIDE = 13, rows >= 2): blb's recovery
// RPC and the client's multi-row ReconstructData at its widest class.  There the v_perm table
// kernel keeps the SIMD's VALU ~97 % busy, and under sustained load it fell to 1.05-1.07x of the
// trivial-XOR stream, while the network stayed within 0.99-1.01x in every process measured
// (DESIGN §4h, round 6).  The device fault once suspected of module loads was raised by HIP's
// in-place lock of pageable test arrays, in every round-5 run whose log survives.
// hipRTC is opened with dlopen on the first request, never linked, so a process that never runs
// such a pass (or sets BLBRS_RTC = 0) never maps it or comgr.
// BLBRS_RTC = 1 compiles on a background thread: the pass keeps the table kernel until its
// network is compiled, so no call waits on the compiler.  That thread makes no HIP call (hipRTC
// is host-only); the code object is loaded (hipModuleLoadData) by the next launch that wants it,
// in the launching thread (ready()).  Compiles and loads share one lock, a launch never waits for
// it, and the compiler thread lives for the whole process and is joined at exit, before comgr's
// static destructors run.  BLBRS_RTC = 2 compiles and loads in the calling thread on first use.
// A compile or load failure (or hipRTC missing) leaves the pass on tables (blbrs_rtc_get_stats).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "rs_kernels.hpp"

namespace blbrs {
namespace rtc {

struct NetKernel {
    std::atomic<hipFunction_t> fn{nullptr};  // set once loaded
    std::atomic<int> state{0};               // 0 compiling, 2 compiled (not loaded), 1 ready, -1 failed
    std::atomic<const void*> code{nullptr};  // the compiled code object (the compile cache's; set with state 2)
    int device = 0;                          // the device it is loaded on
    int u = 0;                               // 16-byte chunks per lane per tile
    int ops = 0;                             // VALU ops of the generated network per 8-dword group
};

// Per-pass lookup cache (mode x addressing), kept in the device plan.  The generated source
// depends on nothing but the pass (no knob shapes it), so an entry never goes stale.
struct NetSlot {
    std::atomic<NetKernel*> k[3][2] = {};
};

// Whether a pass of `rows` rows over `k` inputs may take a run-time network (the knob
// BLBRS_RTC is on, rows >= 2 and k + rows > BLBRS_RTC_WIDE); cheap, called per launch.
bool eligible(int k, int rows);

// The network kernel for (device, rows x k coefficients, mode, addressing), requesting its
// compilation on first use.  Returns nullptr when not eligible; otherwise an entry that stays
// valid for the life of the process (fn == nullptr until it is ready; a shared entry that never
// becomes ready once the process holds kMaxEntries kernels).
NetKernel* request(int device, int k, int rows, Mode mode, bool strided, const uint8_t* coef);

// The loaded kernel of `nk`, loading its compiled code object on nk->device in the calling thread
// when that has not happened yet; nullptr while it compiles or after a failure.  Called per launch.
// wait = false (launches): nullptr instead of waiting while another compile or load holds comgr.
hipFunction_t ready(NetKernel* nk, bool wait = false);

// The generated network's source for rows x k coefficients (tests, tools).
std::string network_source(int k, int rows, const uint8_t* coef, int* ops);

// Compiles the kernel request() would build, without loading it (no device needed); true on
// success, else false with the compiler log.  Adds to the compile cache.
bool compile_only(int k, int rows, Mode mode, bool strided, const uint8_t* coef, std::string* log,
                  std::vector<char>* code = nullptr);

struct Stats {
    uint64_t requested = 0, compiled = 0, loaded = 0, failed = 0, pending = 0;
    double compile_ms = 0;  // total compile time
};
Stats stats();
// Blocks until no compile is queued or running, or timeout_ms passes (< 0: forever); true when
// idle.  A compiled network is loaded by the next launch that wants it.
bool wait_idle(long timeout_ms);
// The compiler log of the first failure ("" if none).
std::string first_failure();

}  // namespace rtc
}  // namespace blbrs
