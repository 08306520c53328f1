// rs_kernels.hpp -- launch interface of the GF(2^8) coding kernels (rs_kernels.hip).
// The struct and constants are also compiled by hipRTC (rtc.hip); the host launch interface
// is not.
#pragma once
#include "dev_common.hpp"

namespace blbrs {

// One coding pass: out[r] = XOR_c coef[r][c] * in[c] over every byte column of every
// stripe in the batch.  The same kernel serves Encode (rows = parity rows of M),
// Reconstruct[Data] (rows = inv(M[valid]) and P*inv(M[valid])) and Verify (rows = parity
// rows, outputs compared instead of stored).
// Pointer tables of at most this many entries travel in the kernel arguments (CodeArgs::inl).
constexpr int kInlinePtrs = 32;

struct CodeArgs {
    const uint32_t* tables;   // device: [rows][k][5] v_perm lookup words (gf256.hpp)
    const int32_t* in_idx;    // device: [k] shard index (within a stripe) of input c
    const int32_t* out_idx;   // device: [rows] shard index of output r
    uint8_t* base;            // strided addressing when non-null
    uint64_t shard_stride;    //   shard i of stripe b at base + b*stripe_stride + i*shard_stride
    uint64_t stripe_stride;
    const uint64_t* ptrs;     // pointer-table addressing when base == null: [B][nshards]
    uint32_t nshards;         //   k+m entries per stripe
    uint32_t B;               // stripes in the batch
    uint64_t S;               // shard length in bytes
    uint32_t tiles_per_stripe;  // set by launch_code()
    int32_t k;                // inputs per stripe
    int32_t rows;             // outputs per stripe (<= kMaxRows)
    int32_t aligned;          // every shard address 16-byte aligned (vector path allowed)
    int32_t* mismatch;        // verify: [B] flags (device)
    int32_t xcd_remap;        // set by launch_code(): block b starts at tile (b%8)*(grid/8) + b/8
    int32_t nstore;           // kStoreVerify: rows [0, nstore) are stored, the rest compared
    int32_t parity;           // rows = encode parity rows 0..rows-1 of k: the compiled network
                              //   (gf_bitslice.hpp) where the shape has one
    // Pointer-table check (ADDR = 1): every entry carries its table's 16-bit tag in bits 48-63
    // (TableFault in runtime.hpp).  A stripe whose entries do not all carry ptr_tag is not
    // touched; the kernel records the first entry it finds wrong in *fault (host-mapped).
    uint32_t* fault;          // [8]: valid, stripe, slot, expected tag, entry lo, entry hi
    uint32_t ptr_tag;
    // Inline table (base == ptrs == null): a host call of one stripe passes its k + m tagged
    // entries here, so the kernel reads no table from memory.  A table in pinned host memory
    // cost a dependent PCIe round trip per entry checked (~10 us of a 4 KiB RS(6,3) read), one in
    // device memory an upload per call.
    uint64_t inl[kInlinePtrs];
};

// Table entries: the device address in bits 0-47 (every GPU and host address the runtime hands
// out is below 2^48), the table's tag above.
constexpr int kPtrTagShift = 48;
constexpr uint64_t kPtrMask = (uint64_t{1} << kPtrTagShift) - 1;

constexpr int kThreads = 256;
constexpr int kBytesPerThread = 16;                       // one dwordx4 per shard per lane
constexpr int kTileBytes = kThreads * kBytesPerThread;    // byte columns per block-iteration
constexpr int kMaxRows = 8;                               // outputs per pass

// kStoreVerify: one pass of reconstructAndVerify (store.go:1132-1142) -- the first nstore
// rows (the missing shards) are written, the others (present shards the decode did not read)
// are compared, so every shard is read or written once.
enum class Mode : int { kStore = 0, kVerify = 1, kStoreVerify = 2 };

// 16-byte chunks per lane per tile of the network kernels (compiled encode networks and run-time
// decode networks alike): 4 in store mode when k + rows <= 9, else 2.  The network holds fewer
// registers than the table multiply (no bit groups, no table operands), so verify keeps U = 2 on
// every shape (RS(12,5): 154 VGPRs).
constexpr int network_u(int k, int rows, int mode) { return mode == 0 ? (k + rows <= 9 ? 4 : 2) : 2; }

#ifndef __HIPCC_RTC__
namespace rtc {
struct NetKernel;
}
// Launches one pass over args.B stripes on `stream` (grid, tiles and XCD mapping chosen
// here); returns hipSuccess or the launch error.  `net`: the pass's run-time network
// (rtc.hpp), used when loaded, else the ahead-of-time kernel.
hipError_t launch_code(const CodeArgs& args, Mode mode, hipStream_t stream, rtc::NetKernel* net = nullptr);

// Name of the kernel instantiation launch_code() would pick (for profiling/tests).
const char* kernel_name(int k, int rows, Mode mode, bool parity = false);
// A store pass of a small host call on rs_small_kernel (rs_small.hpp): one workgroup per 4 KiB
// column chunk of each stripe, pointer-table addressing.  With done_word set, the launch's last
// workgroup publishes `seq` there (done_count: the device word counting workgroups, at 0).
hipError_t launch_small(const CodeArgs& args, uint32_t* done_word, uint32_t* done_count, uint32_t seq,
                        hipStream_t stream);
// The same for ONE stripe with an inline table (args.inl): the kernel (rs_small1_kernel) gets
// the pass's tagged entries in plan order (in_idx / out_idx: the pass's host index lists), so
// it loads no index or table entry itself.  hipErrorNotSupported for shapes it has no kernel for
// (k outside the compiled list, more than 5 rows): the caller uses launch_small.
hipError_t launch_small1(const CodeArgs& args, const int32_t* in_idx, const int32_t* out_idx, uint32_t* done_word,
                         uint32_t* done_count, uint32_t seq, hipStream_t stream);
#endif


}  // namespace blbrs
