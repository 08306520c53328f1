// rs_kernels.hip -- CDNA4 (gfx950) GF(2^8) Reed-Solomon coding kernels.
//
// Replaces klauspost/reedsolomon's codeSomeShards / galMulSlice[Xor] (AVX2 vpshufb nibble
// tables) that blb runs on the CPU at internal/tractserver/store.go:1099 (Encode),
// store.go:1133-1136 (Reconstruct + Verify) and client/blb/reconstruct.go:173
// (ReconstructData).
//
// Design (MI355X-first, byte-wise integer work -> HBM-bound, no MFMA):
//  * A block of 256 threads owns a column tile of one stripe; each lane moves U 16-byte
//    dwordx4 chunks per shard (U = 4 or 2), so every wave reads k*U coalesced 1 KiB
//    segments and writes rows*U.  One tile per block in dispatch order, and each XCD gets a
//    contiguous eighth of the (stripe, tile) space; loads and stores are nontemporal since
//    every byte is touched exactly once.  Nothing is re-read: PMC traffic = algorithmic
//    bytes (profiles/pmc_r01_rs63_encode.json).
//  * GF multiply by a constant uses register lookup tables and v_perm_b32:
//    byte x = g0 | g1<<3 | g2<<6 (3+3+2 bits) and c*x = T0[g0]^T1[g1]^T2[g2]; each table
//    has <= 8 one-byte entries, so one v_perm_b32 byte-select over two dwords looks up 4
//    bytes at once.  Cost: 5 VALU per input dword for the bit groups (shared by every
//    output row) + 3 perms + 1.5 v_bitop3 XOR3 per (coefficient, dword).  RS(6,3) needs
//    ~19 VALU per 4 input bytes, well under the HBM time at full VALU rate.  LDS
//    log/antilog lookups would need k*m ds_read_u8 per byte with random bank conflicts and
//    cap well below the roofline (SURVEY.md §7 "Hard parts").
//  * Coefficient tables (5 dwords per coefficient) are wave-uniform, read through the
//    constant address space with scalar loads each tile (scalar-cache hits) instead of
//    being pinned for the whole launch, which would overflow the SGPR file.
//  * Every output byte is written, never accumulated into: callers hand in un-zeroed
//    pooled buffers (pkg/rpc/pool.go:28-43).
//  * A tile that is not entirely inside the shard, or whose shards are not 16-byte
//    aligned, takes a per-lane path (vector where a 16-byte chunk is whole, bytes for the
//    ragged end); results are identical because byte columns are independent.
#include "rs_kernels.hpp"

#include <algorithm>

#include "gf_bitslice.hpp"
#include "gf_device.hpp"

// Network path A/B knobs (tools/ect_variants.sh builds):
//  BLBRS_CM_PAIRS 1 = the network folds input pairs as their loads land (longer live ranges); 0 = one fold per 8-dword group after its loads.
#ifndef BLBRS_CM_PAIRS
#define BLBRS_CM_PAIRS 0
#endif
// 1 = group-major loads and per-group stores in the network path; 0 = input-major loads and
// every store after the math, as the table path.
#ifndef BLBRS_CM_GROUP_LOADS
#define BLBRS_CM_GROUP_LOADS 1
#endif

namespace blbrs {
namespace {

using namespace dev;

template <int ADDR>
__device__ __forceinline__ uint8_t* shard_ptr(const CodeArgs& a, uint32_t b, int idx) {
    if constexpr (ADDR == 0)
        return a.base + static_cast<uint64_t>(b) * a.stripe_stride +
               static_cast<uint64_t>(idx) * a.shard_stride;
    else
        return reinterpret_cast<uint8_t*>(as_const(a.ptrs)[static_cast<uint64_t>(b) * a.nshards + idx]);
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
template <int MR, int MODE, int ADDR, int U>
__device__ __forceinline__ void code_tile_slow(const CodeArgs& a, uint32_t b, uint64_t tile_off) {
    const int nr = a.rows;
    for (int u = 0; u < U; ++u) {
        const uint64_t off = tile_off + (static_cast<uint64_t>(u) * kThreads + threadIdx.x) * kBytesPerThread;
        if (off >= a.S) return;
        const uint32_t nb = static_cast<uint32_t>(a.S - off < 16 ? a.S - off : 16);
        const bool vec = a.aligned && nb == 16;
        uint32_t acc[MR][4] = {};
        for (int c = 0; c < a.k; ++c) {
            uint32_t x[4];
            const uint8_t* p = shard_ptr<ADDR>(a, b, as_const(a.in_idx)[c]) + off;
            unpack(vec ? ld16<0>(p) : load_bytes(p, nb), x);
            madd<MR, 4>(Groups<4>(x), [&](int r) { return as_const(a.tables) + (static_cast<uint32_t>(r) * a.k + c) * 5; },
                        acc, nr);
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
// CM: the rows are encode parity rows 0..MR-1 of K (a.rows == MR), computed by the compiled
// bit-plane XOR network of gf_bitslice.hpp on whole tiles (K > 0, U even).
template <int K, int MR, int MODE, int ADDR, int U, int NT, bool CM = false>
__global__ __launch_bounds__(kThreads) void rs_code_kernel(CodeArgs a) {
    static_assert(!CM || (K > 0 && U % 2 == 0 && MODE != 2), "compiled network shapes");
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
#if BLBRS_CM_PAIRS
                    bs::parity_rows_by_pairs<K, MR>(xs, og);
#else
#pragma unroll
                    for (int c = 0; c < K; ++c) bs::transpose8(xs[c]);
                    bs::parity_rows<K, MR>(xs, og);
#endif
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

using KernelFn = void (*)(CodeArgs);

// Compile-time input counts: blb's classes RS(6,3), RS(8,3), RS(10,3), RS(12,5)
// (internal/core/StorageClass.go:7-13), the bench's RS(10,4), the reference tests' RS(3,2)
// (store_test.go:750,818) and RS(4,2); rows 1..5 cover every encode and decode of those.
#define BLBRS_K_LIST(X) X(3) X(4) X(6) X(8) X(10) X(12)
constexpr int kMaxTemplRows = 5;

// Launch policy, measured on MI355X (tools/tune_kernels.hip, profiles/r01/tune*.txt):
//  * nontemporal loads and stores (every byte is touched once): +2-5 %;
//  * store mode: U = 4 chunks per lane (16 KiB tiles) when K + MR <= 9, else U = 2 -- wider
//    shapes at U = 4 drop to one wave per SIMD (RS(10,4) 4.6 vs 6.2 TB/s);
//  * verify mode (check shards prefetched with the inputs): U = 2 -- 6.8 TB/s, faster than
//    a plain 9-shard read stream; U = 4 needs too many VGPRs; U = 1 when K + MR > 13:
//    RS(12,5) at U = 2 holds 256 VGPRs (one wave per SIMD) and verified in 20.0 ms, at U = 1
//    147 VGPRs and 13.4 ms; RS(10,4) 10.45 -> 9.9-10.3 ms (tools/code_ab.py, r02);
//  * one tile per block in dispatch order (no persistent grid-stride), with each XCD given
//    a contiguous eighth of the tiles: +10-16 % over a resident persistent grid.
constexpr int kNT = 3;
#ifndef BLBRS_U_WIDE
#define BLBRS_U_WIDE 2         // store mode, K + MR > 9
#endif
#ifndef BLBRS_U_VERIFY_WIDE
#define BLBRS_U_VERIFY_WIDE 1  // verify mode, K + MR > 13
#endif
constexpr int pick_u(int K, int MR, int MODE) {
    return MODE == 0 ? ((K > 0 && K + MR <= 9) ? 4 : BLBRS_U_WIDE) : (K + MR > 13 ? BLBRS_U_VERIFY_WIDE : 2);  // MODE 1, 2
}

// The compiled network holds fewer registers than the table multiply (no bit groups, no
// table operands): verify keeps U = 2 on every shape (RS(12,5): 154 VGPRs), and encode may
// take BLBRS_CM_U_WIDE chunks on wide shapes (A/B builds; default as the table kernel).
#ifndef BLBRS_CM_U_WIDE
#define BLBRS_CM_U_WIDE BLBRS_U_WIDE
#endif
constexpr int pick_u_cm(int K, int MR, int MODE) {
    return MODE == 0 ? (K + MR <= 9 ? 4 : BLBRS_CM_U_WIDE) : 2;
}

template <int K, int MR, int MODE, int ADDR>
constexpr KernelFn fn_of() { return rs_code_kernel<K, MR, MODE, ADDR, pick_u(K, MR, MODE), kNT>; }

struct Choice {
    KernelFn fn = nullptr;
    int u = 0;
    bool fixed = false;
    bool cm = false;  // the compiled encode network
};

// Encode / Verify passes of parity rows: the compiled network where the shape has one.
template <int K, int MR, int MODE, int ADDR>
Choice choice_of(bool cm) {
    constexpr int UC = pick_u_cm(K, MR, MODE);
    if constexpr (K > 0 && UC % 2 == 0 && MODE != 2) {
        if (cm) return {rs_code_kernel<K, MR, MODE, ADDR, UC, kNT, true>, UC, true, true};
    }
    return {fn_of<K, MR, MODE, ADDR>(), pick_u(K, MR, MODE), K > 0, false};
}

template <int K, int MODE, int ADDR>
Choice pick_rows(int rows, bool cm = false) {
    switch (rows) {
        case 1: return choice_of<K, 1, MODE, ADDR>(cm);
        case 2: return choice_of<K, 2, MODE, ADDR>(cm);
        case 3: return choice_of<K, 3, MODE, ADDR>(cm);
        case 4: return choice_of<K, 4, MODE, ADDR>(cm);
        case 5: return choice_of<K, 5, MODE, ADDR>(cm);
        case 6: return {fn_of<0, 6, MODE, ADDR>(), pick_u(0, 6, MODE), false};
        case 7: return {fn_of<0, 7, MODE, ADDR>(), pick_u(0, 7, MODE), false};
        case 8: return {fn_of<0, 8, MODE, ADDR>(), pick_u(0, 8, MODE), false};
        default: return {};
    }
}

template <int MODE, int ADDR>
Choice pick_k(int k, int rows, bool cm) {
    if (rows <= kMaxTemplRows) {
        switch (k) {
#define BLBRS_CASE(KK) case KK: return pick_rows<KK, MODE, ADDR>(rows, cm);
            BLBRS_K_LIST(BLBRS_CASE)
#undef BLBRS_CASE
            default: break;
        }
    }
    return pick_rows<0, MODE, ADDR>(rows);
}

Choice pick(int k, int rows, Mode mode, bool strided, bool cm = false) {
    if (mode == Mode::kStore) return strided ? pick_k<0, 0>(k, rows, cm) : pick_k<0, 1>(k, rows, cm);
    if (mode == Mode::kVerify) return strided ? pick_k<1, 0>(k, rows, cm) : pick_k<1, 1>(k, rows, cm);
    return strided ? pick_k<2, 0>(k, rows, false) : pick_k<2, 1>(k, rows, false);
}

// A/B knob: BLBRS_OCC_LDS=<bytes> (<= 64 KiB, read per launch) reserves that much dynamic LDS
// per workgroup of the compiled-network launches, capping workgroups per CU (160 KiB / bytes).
unsigned occupancy_lds(bool cm) {
    if (!cm) return 0;
    const char* e = getenv("BLBRS_OCC_LDS");
    const long v = e ? atol(e) : 0;
    return v > 0 && v <= 65536 ? static_cast<unsigned>(v) : 0u;
}

}  // namespace

hipError_t launch_code(const CodeArgs& args, Mode mode, hipStream_t stream) {
    if (args.rows < 1 || args.rows > kMaxRows || args.k < 1) return hipErrorInvalidValue;
    if (mode != Mode::kStore && !args.mismatch) return hipErrorInvalidValue;
    if (mode == Mode::kStoreVerify && (args.nstore < 0 || args.nstore > args.rows)) return hipErrorInvalidValue;
    if (args.B == 0 || args.S == 0) return hipSuccess;
    const Choice ch = pick(args.k, args.rows, mode, args.base != nullptr, bs::use(args.parity, args.k, args.rows, bs::kWideCode));
    if (!ch.fn) return hipErrorInvalidValue;
    const uint64_t tile = static_cast<uint64_t>(kTileBytes) * ch.u;
    const uint64_t tps = (args.S + tile - 1) / tile;
    // Tiles are numbered with 32-bit ints: split huge batches.
    const uint64_t max_b = std::max<uint64_t>(1, 0x7FFFFFFFull / tps);
    for (uint64_t b0 = 0; b0 < args.B; b0 += max_b) {
        CodeArgs a = args;
        a.B = static_cast<uint32_t>(std::min<uint64_t>(max_b, args.B - b0));
        if (a.base) a.base += b0 * a.stripe_stride;
        else a.ptrs += b0 * a.nshards;
        if (a.mismatch) a.mismatch += b0;
        a.tiles_per_stripe = static_cast<uint32_t>(tps);
        const uint64_t total = static_cast<uint64_t>(a.B) * tps;
        uint64_t grid = total;
        a.xcd_remap = 0;
        if (total >= 64) {  // one tile per block; a multiple of 8 blocks for the XCD remap
            grid = total & ~uint64_t{7};
            a.xcd_remap = 1;
        }
        hipLaunchKernelGGL(ch.fn, dim3(static_cast<unsigned>(grid)), dim3(kThreads), occupancy_lds(ch.cm), stream, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

const char* kernel_name(int k, int rows, Mode mode, bool parity) {
    const Choice ch = pick(k, rows, mode, true, bs::use(parity, k, rows, bs::kWideCode));
    return ch.cm      ? "rs_code_kernel<K,MR,MODE,ADDR,U,NT,true>"
           : ch.fixed ? "rs_code_kernel<K,MR,MODE,ADDR,U,NT>"
                      : "rs_code_kernel<0,MR,MODE,ADDR,U,NT>";
}

}  // namespace blbrs
