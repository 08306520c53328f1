// rs_small.hpp -- the latency kernel of small host calls (device code; rs_kernels.hip only).
//
// blb's degraded read is one ReconstructData of a few KiB to a few hundred KiB per piece
// (client/blb/reconstruct.go:166-173), with MaxInFlight = 1: what matters is the call's
// latency, ~20 us at 4 KiB against the HBM kernels' milliseconds.  Its shards are read and
// written over PCIe in place (pinned pool buffers or the worker's pinned staging), so a launch
// costs one PCIe round trip per dependent group of loads plus the wait for the stream.
// rs_small_kernel takes two pieces of that off (profiles/r06/latency_floor/):
//  * one workgroup per (stripe, 4 KiB column chunk), every input's 16-byte piece of a lane
//    loaded before any is waited for -- compiled K of 9..16 (RS(10,x), RS(12,x)) as one group of
//    16, where rs_code_kernel's partial-tile path issues two groups of 8, two round trips
//    (its 4 KiB RS(12,x) decode took 10.8 us of kernel against 6.0 at RS(6,3));
//  * a completion word: the last workgroup to finish publishes the call's sequence number to a
//    coherent pinned word once every workgroup's stores are visible to the host, and the calling
//    thread spins on that word instead of waiting for the stream's completion signal
//    (tools/sync_probe.hip: 14.1 -> 10.9 us per 4 KiB call).
// Store mode only (the calls that use it copy no verify flag back), pointer-table addressing
// (host calls), the v_perm table multiply of rs_code.hpp.  The HBM kernels are not touched:
// rs_code_kernel's code is unchanged by this header.
#pragma once
#include "rs_code.hpp"

namespace blbrs {
namespace code {

struct SmallArgs {
    CodeArgs c;               // tiles_per_stripe = 4 KiB chunks per stripe (launch_code)
    uint32_t* done_word;      // coherent pinned word (device view); null: a pass before the last
    uint32_t* done_count;     // device memory: finished workgroups, left at 0
    uint32_t done_seq;        // the call's sequence number (never 0)
};

// One group of 16 inputs: every load issued before any math (sched_barrier; left alone the
// scheduler sinks the second half's loads into the first half's math), the math in two halves
// of 8 so that each unrolled body stays under the unroller's limit (one loop of 16 was left
// rolled, its registers indexed through scratch).
template <int MR>
__device__ __forceinline__ void madd8(const CodeArgs& a, const V4 (&xin)[kSlowBatch], int c0, int cn,
                                      uint32_t (&acc)[MR][4]) {
#pragma unroll
    for (int j = 0; j < kSlowBatch; ++j) {
        if (j >= cn) break;
        const int c = c0 + j;
        uint32_t x[4];
        unpack(xin[j], x);
        madd<MR, 4>(Groups<4>(x), [&](int r) { return as_const(a.tables) + (static_cast<uint32_t>(r) * a.k + c) * 5; },
                    acc, a.rows);
    }
}

template <int MR>
__device__ __forceinline__ void code_chunk_vec16(const CodeArgs& a, uint32_t b, uint64_t off) {
    const ci32 in_idx = as_const(a.in_idx);
    uint32_t acc[MR][4] = {};
    for (int c0 = 0; c0 < a.k; c0 += 2 * kSlowBatch) {
        const int cn = a.k - c0 < 2 * kSlowBatch ? a.k - c0 : 2 * kSlowBatch;
        V4 lo[kSlowBatch], hi[kSlowBatch];
#pragma unroll
        for (int j = 0; j < kSlowBatch; ++j) lo[j] = ld16<0>(shard_ptr<1>(a, b, in_idx[c0 + (j < cn ? j : 0)]) + off);
#pragma unroll
        for (int j = 0; j < kSlowBatch; ++j) {
            const int jj = kSlowBatch + j;
            hi[j] = ld16<0>(shard_ptr<1>(a, b, in_idx[c0 + (jj < cn ? jj : 0)]) + off);
        }
        __builtin_amdgcn_sched_barrier(0);
        madd8<MR>(a, lo, c0, cn < kSlowBatch ? cn : kSlowBatch, acc);
        if (cn > kSlowBatch) madd8<MR>(a, hi, c0 + kSlowBatch, cn - kSlowBatch, acc);
    }
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r >= a.rows) break;
        st16<0>(shard_ptr<1>(a, b, as_const(a.out_idx)[r]) + off, pack(acc[r]));
    }
}

// Each workgroup makes its stores (outputs and the table-check record) visible to the host, then
// counts itself finished; the last one resets the count and publishes the sequence number with a
// system-scope release.  A workgroup that faults never counts, so the host's bounded spin ends
// in the stream wait that reports the fault.
__device__ __forceinline__ void signal_done(const SmallArgs& s) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t before = __hip_atomic_fetch_add(s.done_count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (before == gridDim.x - 1) {
            __hip_atomic_store(s.done_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(s.done_word, s.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// K: compiled input count (0 = runtime k); MR: bound on the rows.
template <int K, int MR>
__global__ __launch_bounds__(kThreads) void rs_small_kernel(SmallArgs s) {
    const CodeArgs& a = s.c;
    const uint32_t chunks = a.tiles_per_stripe;
    const uint32_t total = a.B * chunks;
    for (uint32_t t = blockIdx.x; t < total; t += gridDim.x) {
        const uint32_t b = t / chunks;
        if (!stripe_table_ok<1>(a, b)) continue;
        const uint64_t chunk0 = static_cast<uint64_t>(t - b * chunks) * kTileBytes;
        if (a.aligned && chunk0 + kTileBytes <= a.S) {  // uniform over the block
            const uint64_t off = chunk0 + static_cast<uint64_t>(threadIdx.x) * kBytesPerThread;
            if constexpr (K > kSlowBatch) {
                code_chunk_vec16<MR>(a, b, off);
            } else if constexpr (K == 0) {
                if (a.k > kSlowBatch) code_chunk_vec16<MR>(a, b, off);
                else code_chunk_vec<MR, 0, 1>(a, b, off);
            } else {
                code_chunk_vec<MR, 0, 1>(a, b, off);
            }
        } else {
            code_tile_slow<MR, 0, 1, 1>(a, b, chunk0);  // ragged end or unaligned shards: bytes
        }
    }
    if (s.done_word) signal_done(s);
}

}  // namespace code
}  // namespace blbrs
