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
// (host calls), the v_perm table multiply of rs_code.hpp.  A call of one stripe with an inline
// table -- blb's degraded read -- takes rs_small1_kernel (below), which also drops the chain of
// dependent index and table-entry loads.  The HBM kernels are not touched: rs_code_kernel's code
// is unchanged by this header.
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
// system-scope release (a grid of one publishes without counting).  A workgroup that faults never counts, so the host's bounded spin ends
// in the stream wait that reports the fault.
__device__ __forceinline__ void signal_done(uint32_t* word, uint32_t* count, uint32_t seq) {
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0 && gridDim.x == 1) {  // one workgroup (a 4 KiB piece): nothing to count
        __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (threadIdx.x == 0) {
        const uint32_t before = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (before == gridDim.x - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
    if (s.done_word) signal_done(s.done_word, s.done_count, s.done_seq);
}

// ---- one stripe, entries resolved by the host ----
//
// rs_small_kernel (and rs_code_kernel's partial tiles) find a shard's address through two
// dependent scalar loads -- the plan's index, then the table entry at that index -- and the
// table check walks every entry the same way before the first data load: ~30 serialized scalar
// round trips for an RS(6,3) decode (the 4 KiB kernel took 8.7 us against 3.8 for the same PCIe
// reads in tools/sync_probe.hip).  A one-stripe call with an inline table (blb's degraded read,
// a single increment) needs none of that: the host hands the kernel the pass's tagged entries
// in plan order, so the tag check and every address come from constant-offset loads of the
// kernel arguments, the coefficient tables from constant offsets of one pointer, and every input
// load issues before the first wait.
constexpr int kSmall1MaxIn = 16;

struct Small1Args {
    const uint32_t* tables;         // device: [rows][k][5] v_perm words (the pass's plan)
    uint64_t S;                     // shard bytes
    uint32_t* fault;                // host-mapped table-check record (rs_code.hpp stripe_table_ok's format)
    uint32_t* done_word;            // completion word, or null (a pass before the last)
    uint32_t* done_count;
    uint32_t done_seq;
    uint32_t ptr_tag;
    uint32_t chunks;                // 4 KiB column chunks
    int32_t rows;                   // <= MR
    int32_t aligned;                // every entry 16-byte aligned
    uint64_t in_e[kSmall1MaxIn];    // tagged entries of the inputs, in plan order
    uint64_t out_e[kMaxRows];       // and of the outputs
    uint8_t in_slot[kSmall1MaxIn];  // their slots in the stripe (fault reports)
    uint8_t out_slot[kMaxRows];
};

__device__ __forceinline__ uint8_t* entry_ptr(uint64_t e) { return reinterpret_cast<uint8_t*>(e & kPtrMask); }

// Inputs [J0, J1) of a K-input pass into acc: unrolled over a range of at most 8 inputs so that
// the body stays under the unroller's limit.
template <int K, int MR, int J0, int J1, int NV>
__device__ __forceinline__ void madd_range(const Small1Args& s, const V4 (&x)[K], uint32_t (&acc)[MR][NV]) {
#pragma unroll
    for (int j = J0; j < J1; ++j) {
        uint32_t w[4];
        unpack(x[j], w);
        madd<MR, 4>(Groups<4>(w), [&](int r) { return as_const(s.tables) + (r * K + j) * 5; }, acc, s.rows);
    }
}

template <int K, int MR>
__global__ __launch_bounds__(kThreads) void rs_small1_kernel(Small1Args s) {
    static_assert(K > 0 && K <= kSmall1MaxIn && MR <= kMaxRows, "shape");
    int bad = -1;  // the first entry with a wrong tag: input j, or K + output r
#pragma unroll
    for (int j = K - 1; j >= 0; --j)
        if (static_cast<uint32_t>(s.in_e[j] >> kPtrTagShift) != s.ptr_tag) bad = j;
    if (bad < 0) {
#pragma unroll
        for (int r = MR - 1; r >= 0; --r)
            if (r < s.rows && static_cast<uint32_t>(s.out_e[r] >> kPtrTagShift) != s.ptr_tag) bad = K + r;
    }
    if (bad >= 0) {  // nothing is dereferenced; the host fails the call naming the slot
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const uint64_t e = bad < K ? s.in_e[bad] : s.out_e[bad - K];
            s.fault[1] = 0u;
            s.fault[2] = bad < K ? s.in_slot[bad] : s.out_slot[bad - K];
            s.fault[3] = s.ptr_tag;
            s.fault[4] = static_cast<uint32_t>(e);
            s.fault[5] = static_cast<uint32_t>(e >> 32);
            __threadfence_system();
            s.fault[0] = 1u;
        }
    } else {
        for (uint32_t t = blockIdx.x; t < s.chunks; t += gridDim.x) {
            const uint64_t chunk0 = static_cast<uint64_t>(t) * kTileBytes;
            const uint64_t off = chunk0 + static_cast<uint64_t>(threadIdx.x) * kBytesPerThread;
            V4 x[K];
            uint32_t acc[MR][4] = {};
            if (s.aligned && chunk0 + kTileBytes <= s.S) {  // uniform: every lane holds a whole 16 B
#pragma unroll
                for (int j = 0; j < K; ++j) x[j] = ld16<0>(entry_ptr(s.in_e[j]) + off);
                __builtin_amdgcn_sched_barrier(0);
                madd_range<K, MR, 0, (K < 8 ? K : 8), 4>(s, x, acc);
                if constexpr (K > 8) madd_range<K, MR, 8, K, 4>(s, x, acc);
#pragma unroll
                for (int r = 0; r < MR; ++r)
                    if (r < s.rows) st16<0>(entry_ptr(s.out_e[r]) + off, pack(acc[r]));
            } else if (off < s.S) {  // the ragged end, or unaligned shards: per lane
                const uint32_t nb = static_cast<uint32_t>(s.S - off < 16 ? s.S - off : 16);
                const bool vec = s.aligned && nb == 16;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    const uint8_t* p = entry_ptr(s.in_e[j]) + off;
                    x[j] = vec ? ld16<0>(p) : load_bytes(p, nb);
                }
                madd_range<K, MR, 0, (K < 8 ? K : 8), 4>(s, x, acc);
                if constexpr (K > 8) madd_range<K, MR, 8, K, 4>(s, x, acc);
#pragma unroll
                for (int r = 0; r < MR; ++r) {
                    if (r >= s.rows) break;
                    uint8_t* q = entry_ptr(s.out_e[r]) + off;
                    if (vec) st16<0>(q, pack(acc[r]));
                    else store_bytes(q, pack(acc[r]), nb);
                }
            }
        }
    }
    if (s.done_word) signal_done(s.done_word, s.done_count, s.done_seq);
}

}  // namespace code
}  // namespace blbrs
