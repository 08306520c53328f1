// rs_code.hpp -- the GF(2^8) coding kernel rs_code_kernel (device code only).
//
// Replaces klauspost/reedsolomon's codeSomeShards / galMulSlice[Xor] (AVX2 vpshufb nibble
// tables) that blb runs on the CPU at internal/tractserver/store.go:1099 (Encode),
// store.go:1133-1136 (Reconstruct + Verify) and client/blb/reconstruct.go:173
// (ReconstructData).  rs_kernels.hip instantiates it ahead of time for the table path and the
// compiled encode networks; rtc.hip compiles it with hipRTC for the decode network of one
// erasure pattern (NET = a generated struct), so this header is RTC-clean.
//
// Design (MI355X-first, byte-wise integer work -> HBM-bound, no MFMA):
//  * A block of 256 threads owns a column tile of one stripe; each lane moves U 16-byte
//    dwordx4 chunks per shard (U = 4 or 2), so every wave reads k*U coalesced 1 KiB
//    segments and writes rows*U.  One tile per block in dispatch order, and each XCD gets a
//    contiguous eighth of the (stripe, tile) space; loads and stores are nontemporal since
//    every byte is touched exactly once.  Nothing is re-read: PMC traffic = algorithmic
//    bytes (profiles/pmc_r03.json).
//  * GF multiply by a constant uses register lookup tables and v_perm_b32:
//    byte x = g0 | g1<<3 | g2<<6 (3+3+2 bits) and c*x = T0[g0]^T1[g1]^T2[g2]; each table
//    has <= 8 one-byte entries, so one v_perm_b32 byte-select over two dwords looks up 4
//    bytes at once.  Cost: 5 VALU per input dword for the bit groups (shared by every
//    output row) + 3 perms + 1.5 v_bitop3 XOR3 per (coefficient, dword).  LDS
//    log/antilog lookups would need k*m ds_read_u8 per byte with random bank conflicts and
//    cap well below the roofline (SURVEY.md §7 "Hard parts").
//  * With NET != void the rows are a fixed XOR network over bit planes (gf_bitslice.hpp):
//    the encode matrix compiled into the library, or a decode matrix generated at run time.
//  * Coefficient tables (5 dwords per coefficient) are wave-uniform, read through the
//    constant address space with scalar loads each tile (scalar-cache hits) instead of
//    being pinned for the whole launch, which would overflow the SGPR file.
//  * Every output byte is written, never accumulated into: callers hand in un-zeroed
//    pooled buffers (pkg/rpc/pool.go:28-43).
//  * A tile that is not entirely inside the shard, or whose shards are not 16-byte
//    aligned, takes a per-lane path (vector where a 16-byte chunk is whole, bytes for the
//    ragged end); results are identical because byte columns are independent.
#pragma once
#include "gf_bitslice.hpp"
#include "gf_device.hpp"
#include "rs_kernels.hpp"

// Network path A/B knobs (tools/ect_variants.sh builds):
// 1 = group-major loads and per-group stores in the network path; 0 = input-major loads and
// every store after the math, as the table path.
#ifndef BLBRS_CM_GROUP_LOADS
#define BLBRS_CM_GROUP_LOADS 1
#endif
// 1 = store mode writes each network row as soon as it is formed (NET::each); 0 = all rows, then
// the stores.
#ifndef BLBRS_CM_ROW_STORES
#define BLBRS_CM_ROW_STORES 1
#endif

namespace blbrs {
namespace code {

using namespace dev;

// Entry idx of stripe b's pointer-table row: the table in memory, or the inline one.
__device__ __forceinline__ uint64_t table_entry(const CodeArgs& a, uint32_t b, int idx) {
    const uint64_t pos = static_cast<uint64_t>(b) * a.nshards + idx;
    return a.ptrs ? as_const(a.ptrs)[pos] : a.inl[pos];
}

template <int ADDR>
__device__ __forceinline__ uint8_t* shard_ptr(const CodeArgs& a, uint32_t b, int idx) {
    if constexpr (ADDR == 0)
        return a.base + static_cast<uint64_t>(b) * a.stripe_stride +
               static_cast<uint64_t>(idx) * a.shard_stride;
    else
        return reinterpret_cast<uint8_t*>(table_entry(a, b, idx) & kPtrMask);
}

// Pointer-table addressing: every entry this pass reads or writes for stripe b must carry the
// table's tag (the host writes it into bits 48-63 of each entry, runtime.hpp TableFault).  An
// entry from another upload, or not from an upload at all, is never dereferenced: the stripe's
// tile is skipped and the entry recorded for the host, which fails the call naming the slot.
// Scalar loads of the entries the tile reads anyway; nothing for strided addressing.
template <int ADDR>
__device__ __forceinline__ bool stripe_table_ok(const CodeArgs& a, uint32_t b) {
    if constexpr (ADDR == 0) {
        return true;
    } else {
        const ci32 in_idx = as_const(a.in_idx), out_idx = as_const(a.out_idx);
        const int n = a.k + a.rows;
        for (int j = 0; j < n; ++j) {
            const int idx = j < a.k ? in_idx[j] : out_idx[j - a.k];
            const uint64_t e = table_entry(a, b, idx);
            if (static_cast<uint32_t>(e >> kPtrTagShift) != a.ptr_tag) {
                if (threadIdx.x == 0) {  // vector stores to the host-mapped record, header last
                    a.fault[1] = b;
                    a.fault[2] = static_cast<uint32_t>(idx);
                    a.fault[3] = a.ptr_tag;
                    a.fault[4] = static_cast<uint32_t>(e);
                    a.fault[5] = static_cast<uint32_t>(e >> 32);
                    __threadfence_system();
                    a.fault[0] = 1u;
                }
                return false;
            }
        }
        return true;
    }
}

// 16-byte global load/store; NT bit 0 = nontemporal loads, bit 1 = nontemporal stores
// (streamed data is touched exactly once).
template <int NT>
__device__ __forceinline__ V4 ld16(const uint8_t* p) {
    if constexpr (NT & 1) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return V4{v.x, v.y, v.z, v.w};
    } else {
        return *reinterpret_cast<const V4*>(p);
    }
}
template <int NT>
__device__ __forceinline__ void st16(uint8_t* p, const V4& v) {
    if constexpr (NT & 2) {
        const u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<V4*>(p) = v;
    }
}

__device__ __forceinline__ V4 load_bytes(const uint8_t* p, uint32_t n) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t j = 0; j < n; ++j) w[j >> 2] |= static_cast<uint32_t>(p[j]) << (8 * (j & 3));
    return V4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_bytes(uint8_t* p, const V4& v, uint32_t n) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t j = 0; j < n; ++j) p[j] = static_cast<uint8_t>(w[j >> 2] >> (8 * (j & 3)));
}

__device__ __forceinline__ bool neq(const V4& a, const V4& b) {
    return ((a.x ^ b.x) | (a.y ^ b.y) | (a.z ^ b.z) | (a.w ^ b.w)) != 0u;
}

// Verify: at most one atomic per wave (the lowest lane with a mismatch), so a batch of
// bad stripes does not serialise every lane on one flag word.
__device__ __forceinline__ void flag_mismatch(int32_t* flag, bool bad) {
    const unsigned long long m = __ballot(bad);
    if (m != 0ull && (threadIdx.x & 63u) == static_cast<unsigned>(__ffsll(static_cast<long long>(m)) - 1))
        atomicOr(flag, 1);
}

// Partial / unaligned tiles (runtime k, rows <= MR): 16-byte vector accesses where a
// chunk is whole and aligned, byte accesses for the shard's ragged end or unaligned shards.
//
// A small host call is all partial tile (a 4 KiB shard in a 16 KiB tile) and reads its shards
// over PCIe, ~1.5 us a round trip: the loads of an input group must all be in flight before
// the first one is waited for.  Chunks that every lane of the block holds whole and aligned
// (`all_vec`, uniform) take a branch-free group of kSlowBatch loads (the slots past k re-load
// input c0, valid and unused) -- with per-lane vector/byte choices the compiler waited for
// every load in turn (RS(6,3) 4 KiB: 11.9 us of kernel, RS(12,5) 21.7 us, profiles/r05).
constexpr int kSlowBatch = 8;

template <int MR, int MODE, int ADDR>
__device__ __forceinline__ void code_chunk_vec(const CodeArgs& a, uint32_t b, uint64_t off) {
    const int nr = a.rows;
    const ci32 in_idx = as_const(a.in_idx);
    uint32_t acc[MR][4] = {};
    for (int c0 = 0; c0 < a.k; c0 += kSlowBatch) {
        const int cn = a.k - c0 < kSlowBatch ? a.k - c0 : kSlowBatch;
        const uint8_t* p[kSlowBatch];
#pragma unroll
        for (int j = 0; j < kSlowBatch; ++j) p[j] = shard_ptr<ADDR>(a, b, in_idx[c0 + (j < cn ? j : 0)]) + off;
        V4 xin[kSlowBatch];
#pragma unroll
        for (int j = 0; j < kSlowBatch; ++j) xin[j] = ld16<0>(p[j]);
#pragma unroll
        for (int j = 0; j < kSlowBatch; ++j) {
            if (j >= cn) break;
            const int c = c0 + j;
            uint32_t x[4];
            unpack(xin[j], x);
            madd<MR, 4>(Groups<4>(x), [&](int r) { return as_const(a.tables) + (static_cast<uint32_t>(r) * a.k + c) * 5; },
                        acc, nr);
        }
    }
    if constexpr (MODE != 0) {
        V4 chk[MR];
#pragma unroll
        for (int r = 0; r < MR; ++r)
            if (r < nr && !(MODE == 2 && r < a.nstore)) chk[r] = ld16<0>(shard_ptr<ADDR>(a, b, as_const(a.out_idx)[r]) + off);
        bool bad = false;
#pragma unroll
        for (int r = 0; r < MR; ++r)
            if (r < nr && !(MODE == 2 && r < a.nstore)) bad |= neq(chk[r], pack(acc[r]));
        if (bad) atomicOr(&a.mismatch[b], 1);
    }
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r >= nr) break;
        if (MODE == 0 || (MODE == 2 && r < a.nstore)) st16<0>(shard_ptr<ADDR>(a, b, as_const(a.out_idx)[r]) + off, pack(acc[r]));
    }
}

template <int MR, int MODE, int ADDR, int U>
__device__ __forceinline__ void code_tile_slow(const CodeArgs& a, uint32_t b, uint64_t tile_off) {
    const int nr = a.rows;
    for (int u = 0; u < U; ++u) {
        const uint64_t chunk0 = tile_off + static_cast<uint64_t>(u) * kThreads * kBytesPerThread;
        if (chunk0 >= a.S) return;
        const uint64_t off = chunk0 + static_cast<uint64_t>(threadIdx.x) * kBytesPerThread;
        if (a.aligned && chunk0 + kThreads * kBytesPerThread <= a.S) {  // uniform over the block
            code_chunk_vec<MR, MODE, ADDR>(a, b, off);
            continue;
        }
        if (off >= a.S) return;
        const uint32_t nb = static_cast<uint32_t>(a.S - off < 16 ? a.S - off : 16);
        const bool vec = a.aligned && nb == 16;
        uint32_t acc[MR][4] = {};
        for (int c0 = 0; c0 < a.k; c0 += kSlowBatch) {
            const int cn = a.k - c0 < kSlowBatch ? a.k - c0 : kSlowBatch;
            V4 xin[kSlowBatch];
#pragma unroll
            for (int j = 0; j < kSlowBatch; ++j) {
                if (j >= cn) break;
                const uint8_t* p = shard_ptr<ADDR>(a, b, as_const(a.in_idx)[c0 + j]) + off;
                xin[j] = vec ? ld16<0>(p) : load_bytes(p, nb);
            }
#pragma unroll
            for (int j = 0; j < kSlowBatch; ++j) {
                if (j >= cn) break;
                const int c = c0 + j;
                uint32_t x[4];
                unpack(xin[j], x);
                madd<MR, 4>(Groups<4>(x),
                            [&](int r) { return as_const(a.tables) + (static_cast<uint32_t>(r) * a.k + c) * 5; }, acc, nr);
            }
        }
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            if (r >= nr) break;
            uint8_t* q = shard_ptr<ADDR>(a, b, as_const(a.out_idx)[r]) + off;
            if (MODE == 0 || (MODE == 2 && r < a.nstore)) {
                if (vec) st16<0>(q, pack(acc[r]));
                else store_bytes(q, pack(acc[r]), nb);
            } else if (neq(vec ? ld16<0>(q) : load_bytes(q, nb), pack(acc[r]))) {
                atomicOr(&a.mismatch[b], 1);
            }
        }
    }
}

// K > 0: compile-time input count (all K*U chunk loads issued before any math).
// K == 0: runtime k (loads issued per input, two inputs unrolled).
// MR: compile-time bound on output rows; a.rows <= MR honoured at runtime.
// MODE 0 = store outputs, 1 = compare against existing outputs (Verify), 2 = store rows
// [0, a.nstore) and compare the rest (reconstructAndVerify in one pass).
// ADDR 0 = strided stripes, 1 = pointer table.  U = 16-byte chunks per lane per tile.
// NET: void = v_perm tables; else the rows (a.rows == MR) are computed by NET's bit-plane XOR
// network (gf_bitslice.hpp: EncodeNet<K>, or a decode network generated by rtc.hip) on whole
// tiles (K > 0, U even); partial tiles keep the table path.
template <class T> struct is_void { static constexpr bool value = false; };
template <> struct is_void<void> { static constexpr bool value = true; };

// BLBRS_NET_WPE > 0: network kernels of k + rows <= 14 ask the compiler for that many waves per
// SIMD (RS(10,x) networks otherwise land at 129-130 VGPRs, one over the 4-wave budget).  Off in
// the library build; run-time networks take it from the knob BLBRS_RTC_WPE (rtc.hip).
#ifndef BLBRS_NET_WPE
#define BLBRS_NET_WPE 0
#endif
constexpr int net_wpe(int k, int rows, bool cm) { return cm && BLBRS_NET_WPE > 0 && k + rows <= 14 ? BLBRS_NET_WPE : 1; }

template <int K, int MR, int MODE, int ADDR, int U, int NT, class NET = void>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(net_wpe(K, MR, !is_void<NET>::value))))
void rs_code_kernel(CodeArgs a) {
    constexpr bool CM = !is_void<NET>::value;
    static_assert(!CM || (K > 0 && U % 2 == 0), "network shapes");
    constexpr uint32_t kTile = kTileBytes * U;
    const uint32_t total = a.B * a.tiles_per_stripe;
    const int nr = a.rows;
    const bool aligned = a.aligned != 0;

    // Blocks are dealt round-robin over the 8 XCDs; with xcd_remap each XCD streams its own
    // contiguous eighth of the (stripe, tile) space instead of every 8th tile.
    uint32_t first = blockIdx.x;
    if (a.xcd_remap) first = (first % 8u) * (gridDim.x / 8u) + first / 8u;
    for (uint32_t t = first; t < total; t += gridDim.x) {
        const uint32_t b = t / a.tiles_per_stripe;
        const uint64_t tile_off = static_cast<uint64_t>(t - b * a.tiles_per_stripe) * kTile;
        if (!stripe_table_ok<ADDR>(a, b)) continue;
        if (!aligned || tile_off + kTile > a.S) {
            code_tile_slow<MR, MODE, ADDR, U>(a, b, tile_off);
            continue;
        }
        // Opaque per-iteration copy of the table pointer: keeps the scalar table loads
        // inside the loop (no LICM -> no SGPR spill of K*MR*5 words).
        cu32 tables = as_const(a.tables);
        asm volatile("" : "+s"(tables));
        const ci32 in_idx = as_const(a.in_idx);
        const ci32 out_idx = as_const(a.out_idx);
        const uint64_t lane_off = tile_off + static_cast<uint64_t>(threadIdx.x) * kBytesPerThread;

        constexpr int NV = 4 * U;           // input dwords per lane per shard
        constexpr uint32_t kStep = kThreads * kBytesPerThread;
        uint32_t acc[MR][NV] = {};

        // Verify: the shards to check are loaded up front with the inputs, so the whole
        // tile's reads are in flight before any math.
        V4 chk[MODE != 0 ? MR : 1][U];
        if constexpr (MODE != 0) {
            const int first_chk = MODE == 2 ? a.nstore : 0;
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                if (r < nr && r >= first_chk) {
                    const uint8_t* q = shard_ptr<ADDR>(a, b, out_idx[r]) + lane_off;
#pragma unroll
                    for (int u = 0; u < U; ++u) chk[r][u] = ld16<NT>(q + u * kStep);
                }
            }
        }

        if constexpr (K > 0) {
            V4 x[K][U];
            if constexpr (CM) {
                // Group-major loads (chunks 2g, 2g+1 of every input, g = 0 first), so that group
                // 0's network starts while group 1 is still in flight; within a group the
                // network folds input pairs as they land.
#if BLBRS_CM_GROUP_LOADS
#pragma unroll
                for (int g = 0; g < U / 2; ++g)
#pragma unroll
                    for (int c = 0; c < K; ++c) {
                        const uint8_t* p = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
                        x[c][2 * g] = ld16<NT>(p + 2 * g * kStep);
                        x[c][2 * g + 1] = ld16<NT>(p + (2 * g + 1) * kStep);
                    }
#else
#pragma unroll
                for (int c = 0; c < K; ++c) {
                    const uint8_t* p = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
#pragma unroll
                    for (int u = 0; u < U; ++u) x[c][u] = ld16<NT>(p + u * kStep);
                }
#endif
                // Every load issued before any math: left alone, the scheduler sinks group 1's
                // loads into group 0's network (fewer registers, less in flight).
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int g = 0; g < U / 2; ++g) {
                    uint32_t xs[K][8], og[MR][8];
#pragma unroll
                    for (int c = 0; c < K; ++c) {
                        unpack(x[c][2 * g], xs[c]);
                        unpack(x[c][2 * g + 1], xs[c] + 4);
                    }
#pragma unroll
                    for (int c = 0; c < K; ++c) bs::transpose8(xs[c]);
                    if constexpr (MODE == 0 && BLBRS_CM_GROUP_LOADS && BLBRS_CM_ROW_STORES) {
                        // each row stored as soon as it is formed: 8 output registers live, not 8 * MR
                        auto put = [&](int r, const uint32_t (&o)[8]) {
                            uint8_t* q = shard_ptr<ADDR>(a, b, out_idx[r]) + lane_off;
                            st16<NT>(q + 2 * g * kStep, pack(o));
                            st16<NT>(q + (2 * g + 1) * kStep, pack(o + 4));
                        };
                        bs::NetRows<NET, K, MR>::each(xs, put);
                    } else {
                    bs::NetRows<NET, K, MR>::run(xs, og);
#pragma unroll
                    for (int r = 0; r < MR; ++r)
#pragma unroll
                        for (int d = 0; d < 8; ++d) acc[r][8 * g + d] = og[r][d];
                    if constexpr (MODE == 0 && BLBRS_CM_GROUP_LOADS) {  // this group's stores go out before the next group's math
#pragma unroll
                        for (int r = 0; r < MR; ++r) {
                            uint8_t* q = shard_ptr<ADDR>(a, b, out_idx[r]) + lane_off;
                            st16<NT>(q + 2 * g * kStep, pack(acc[r] + 8 * g));
                            st16<NT>(q + (2 * g + 1) * kStep, pack(acc[r] + 8 * g + 4));
                        }
                    }
                    }
                }
            } else {
#pragma unroll
            for (int c = 0; c < K; ++c) {
                const uint8_t* p = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
#pragma unroll
                for (int u = 0; u < U; ++u) x[c][u] = ld16<NT>(p + u * kStep);
            }
#pragma unroll
            for (int c = 0; c + 1 < K; c += 2) {
                uint32_t xa[NV], xb[NV];
#pragma unroll
                for (int u = 0; u < U; ++u) { unpack(x[c][u], xa + 4 * u); unpack(x[c + 1][u], xb + 4 * u); }
                madd2<MR, NV>(Groups<NV>(xa), [&](int r) { return tables + (r * K + c) * 5; },
                              Groups<NV>(xb), [&](int r) { return tables + (r * K + c + 1) * 5; }, acc, nr);
            }
            if constexpr (K & 1) {
                uint32_t xv[NV];
#pragma unroll
                for (int u = 0; u < U; ++u) unpack(x[K - 1][u], xv + 4 * u);
                madd<MR, NV>(Groups<NV>(xv), [&](int r) { return tables + (r * K + K - 1) * 5; }, acc, nr);
            }
            }
        } else {
            const int k = a.k;
            int c = 0;
            for (; c + 1 < k; c += 2) {
                const uint8_t* pa = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
                const uint8_t* pb = shard_ptr<ADDR>(a, b, in_idx[c + 1]) + lane_off;
                uint32_t xa[NV], xb[NV];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    unpack(ld16<NT>(pa + u * kStep), xa + 4 * u);
                    unpack(ld16<NT>(pb + u * kStep), xb + 4 * u);
                }
                madd2<MR, NV>(Groups<NV>(xa), [&](int r) { return tables + (static_cast<uint32_t>(r) * k + c) * 5; },
                              Groups<NV>(xb), [&](int r) { return tables + (static_cast<uint32_t>(r) * k + c + 1) * 5; },
                              acc, nr);
            }
            if (c < k) {
                const uint8_t* p = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
                uint32_t xv[NV];
#pragma unroll
                for (int u = 0; u < U; ++u) unpack(ld16<NT>(p + u * kStep), xv + 4 * u);
                madd<MR, NV>(Groups<NV>(xv), [&](int r) { return tables + (static_cast<uint32_t>(r) * k + c) * 5; },
                             acc, nr);
            }
        }

        bool bad = false;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            if (r >= nr) break;
            uint8_t* q = shard_ptr<ADDR>(a, b, out_idx[r]) + lane_off;
            if (CM && MODE == 0 && BLBRS_CM_GROUP_LOADS) {
                // stored per group above
            } else if (MODE == 0 || (MODE == 2 && r < a.nstore)) {
#pragma unroll
                for (int u = 0; u < U; ++u) st16<NT>(q + u * kStep, pack(acc[r] + 4 * u));
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) bad |= neq(chk[r][u], pack(acc[r] + 4 * u));
            }
        }
        if constexpr (MODE != 0) flag_mismatch(a.mismatch + b, bad);
    }
}

}  // namespace code
}  // namespace blbrs
