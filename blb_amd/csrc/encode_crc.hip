// encode_crc.hip -- fused Reed-Solomon encode + CRC-32C of the parity, one pass over HBM.
// Persistent segment kernel: launch_encode_crc hands the shapes the tile-grid kernel covers
// (encode_crc_tile.hip, faster) to it and runs this one for the rest (rows = 5, lengths
// that are not whole 8 KiB tiles, blocks < 8 KiB, views not 16-byte aligned).
//
// On blb's RS path every parity shard the encoder writes is checksummed next: the
// tractserver ships each parity increment with CtlWrite, whose bulk RPC frame carries a
// CRC-32C of the whole buffer (pkg/rpc/bulk_codec.go:6-14,47; sent from
// internal/tractserver/store.go:1110-1120), and the receiving tractserver stores it in
// ChecksumFile blocks of 65532 bytes, each with its own CRC-32C
// (pkg/disk/checksum_block.go:18-34).  Run separately, the CRC re-reads all m parity shards
// from HBM (RS(6,3): a third of the encode's traffic again).  Here the parity bytes are
// checksummed while they are still in registers.
//
// Layout (one wave = one <= 64 KiB segment of one CRC block of one stripe, all m parity
// rows): the segment is R rows of 64*LC bytes; lane t owns the LC contiguous bytes at column
// t of every row.  Per row the lane loads its LC bytes of each of the k data shards, forms
// the m parity chunks with the v_perm GF multiply (gf_device.hpp), stores them, and runs
// one slicing-by-4 CRC chain per parity row over them (banked LDS tables, crc_device.hpp),
// jumping S_{64*LC-LC} to its next row's chunk.  Lanes then fold with S_{LC*2^j}, and a
// second tiny kernel folds the segments of each block (crc_combine).  Segments are laid out
// exactly as crc32c.hip's streaming kernel lays them out: aligned to END at the block's end,
// with a virtual zero prefix; the first row of such a segment is read and written through
// buffer resources bounded to the segment, so the prefix (which belongs to the previous
// block) reads as zero -- zero data gives zero parity, which leaves the raw CRC at 0 -- and
// its stores are dropped.  Every byte of every shard therefore belongs to exactly one wave.
//
// Occupancy: the 128 KiB of banked tables allow one workgroup per CU; 512 threads = 2 waves
// per SIMD with up to 256 VGPRs each -- the same occupancy at which the plain coding kernel
// (231 VGPRs) already runs at the read-k/write-m stream rate.  LC = 64 when the k data
// chunks plus m accumulators of a row fit (k + m <= 11), else LC = 32.
#include "encode_crc.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <set>

#include "crc_device.hpp"
#include "tuning.hpp"
#include "gf_device.hpp"

namespace blbrs {
namespace {

using namespace dev;

constexpr int kEcThreads = 512;               // 8 waves, one workgroup per CU
constexpr uint32_t kWaves = kEcThreads / 64;
#ifndef BLBRS_EC_SEG
#define BLBRS_EC_SEG 65536
#endif
constexpr uint32_t kSeg = BLBRS_EC_SEG;       // bytes per wave segment
constexpr size_t kEcLds = kBankedTableBytes;   // 128 KiB

struct KArgs {
    const uint32_t* tables;
    const int32_t* in_idx;
    const int32_t* out_idx;
    uint8_t* base;
    uint64_t shard_stride, stripe_stride;
    uint64_t S, block;
    uint32_t B, nblocks, segs_per_block;
    uint64_t total_segs;
    const CrcConsts* c;
    uint32_t* raw;            // [(j * B + b) * nblocks + blk] * segs_per_block + s
};

template <int LC>
struct Geo {
    static constexpr uint32_t kRow = 64u * LC;     // bytes per row
    static constexpr uint32_t kRows = kSeg / kRow;
    static constexpr int kDw = LC / 4;             // dwords per lane per row
    static constexpr int kQ = LC / 16;             // dwordx4 per lane per row
    static constexpr int kVar = LC == 64 ? 0 : 1;  // CrcConsts gap / wlvl variant
};

// Loads row r of the segment (plain dwordx4 per 16-byte piece, see lane_piece).
template <int K, int LC>
__device__ __forceinline__ void load_row(const KArgs& a, const uint8_t* stripe, ci32 in_idx, int64_t row_off,
                                         uint32_t lane, uint32_t (&x)[K][LC / 4]) {
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint8_t* p = stripe + static_cast<uint64_t>(in_idx[c]) * a.shard_stride + row_off + lane_piece<LC>(lane);
#pragma unroll
        for (int q = 0; q < LC / 16; ++q) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(p + 1024 * q);
            x[c][4 * q] = v.x;
            x[c][4 * q + 1] = v.y;
            x[c][4 * q + 2] = v.z;
            x[c][4 * q + 3] = v.w;
        }
    }
}

// Buffer offset of dword i of a lane's pieces (o = the lane's piece offset minus the prefix,
// negative before the segment start).  Opaque, so the constant part is not folded into the
// instruction offset: the range check must see the wrapped 32-bit sum, or a dword just past
// the start (voffset -4, offset +4) would test out of range and read as 0.
__device__ __forceinline__ int voff(int o, int i) {
    int v = o + 1024 * (i / 4) + 4 * (i % 4);
    asm volatile("" : "+v"(v));
    return v;
}

// The first row of an end-aligned segment: buffers bounded to [start, start + kRow - pad0);
// dwords before start have wrapped (huge) offsets and read as 0.
template <int K, int LC>
__device__ __forceinline__ void load_row_masked(const KArgs& a, const uint8_t* stripe, ci32 in_idx, uint64_t start,
                                                uint32_t pad0, uint32_t lane, uint32_t (&x)[K][LC / 4]) {
    const int o = static_cast<int>(lane_piece<LC>(lane)) - static_cast<int>(pad0);
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(stripe) + static_cast<uint64_t>(in_idx[c]) * a.shard_stride + start, 0,
            static_cast<int>(64 * LC - pad0), 0x00020000);
#pragma unroll
        for (int i = 0; i < LC / 4; ++i) x[c][i] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff(o, i), 0, 0);
    }
}

// One segment g (all m parity rows): encode its rows, CRC them, write the raw CRCs.
template <int K, int MR, int LC>
__device__ __forceinline__ void encode_crc_segment(const KArgs& a, uint64_t g, uint32_t lane, const LaneTabs& lt) {
    using G = Geo<LC>;
    const uint32_t s = static_cast<uint32_t>(g % a.segs_per_block);
    const uint32_t blk = static_cast<uint32_t>((g / a.segs_per_block) % a.nblocks);
    const uint32_t b = static_cast<uint32_t>(g / (static_cast<uint64_t>(a.segs_per_block) * a.nblocks));
    const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;
    const uint64_t blk_end = blk_start + a.block < a.S ? blk_start + a.block : a.S;
    const uint64_t start = blk_start + static_cast<uint64_t>(s) * kSeg;
    uint32_t* raw = a.raw + (static_cast<uint64_t>(b) * a.nblocks + blk) * a.segs_per_block + s;
    const uint64_t raw_row = static_cast<uint64_t>(a.B) * a.nblocks * a.segs_per_block;  // j -> j + 1
    if (start >= blk_end) {
        if (lane == 0)
#pragma unroll
            for (int j = 0; j < MR; ++j) raw[j * raw_row] = 0u;
        return;
    }
    const uint64_t end = start + kSeg < blk_end ? start + kSeg : blk_end;
    const uint32_t pad = static_cast<uint32_t>(kSeg - (end - start));  // virtual zero prefix
    const uint32_t r0 = pad / G::kRow, pad0 = pad % G::kRow;

    uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
    const ci32 in_idx = as_const(a.in_idx);
    const ci32 out_idx = as_const(a.out_idx);
    const int64_t seg_off = static_cast<int64_t>(end) - kSeg;  // row r at seg_off + r * kRow (>= start for r > r0)

    uint32_t crc[MR];
#pragma unroll
    for (int j = 0; j < MR; ++j) crc[j] = 0u;

    uint32_t x[K][G::kDw];
    if (pad0) load_row_masked<K, LC>(a, stripe, in_idx, start, pad0, lane, x);
    else load_row<K, LC>(a, stripe, in_idx, seg_off + static_cast<int64_t>(r0) * G::kRow, lane, x);

    // out[j] = sum_c coef[j][c] * x[c] for this lane's row pieces.
    auto compute = [&](uint32_t (&acc)[MR][G::kDw]) {
        // Opaque copies of the table pointer (per row, and per input pair): keep the scalar
        // table loads next to their use (no LICM -> no SGPR spill of K*MR*5 words).
        cu32 tables = as_const(a.tables);
        asm volatile("" : "+s"(tables));
#pragma unroll
        for (int c = 0; c + 1 < K; c += 2) {
            cu32 tp = tables;
            asm volatile("" : "+s"(tp));
            madd2_dw<MR, G::kDw>(x[c], [&](int rr) { return tp + (rr * K + c) * 5; }, x[c + 1],
                                 [&](int rr) { return tp + (rr * K + c + 1) * 5; }, acc);
        }
        if constexpr (K & 1)
            madd_dw<MR, G::kDw>(x[K - 1], [&](int rr) { return tables + (rr * K + K - 1) * 5; }, acc);
    };
    // Store row r's parity, then run it through the CRC chains.
    auto store_crc = [&](uint32_t r, uint32_t (&acc)[MR][G::kDw]) {
        const int64_t row_off = seg_off + static_cast<int64_t>(r) * G::kRow;
        if (r != r0 || pad0 == 0) {
#pragma unroll
            for (int j = 0; j < MR; ++j) {
                uint8_t* q = stripe + static_cast<uint64_t>(out_idx[j]) * a.shard_stride + row_off + lane_piece<LC>(lane);
#pragma unroll
                for (int u = 0; u < G::kQ; ++u) {
                    const u32x4 v = {acc[j][4 * u], acc[j][4 * u + 1], acc[j][4 * u + 2], acc[j][4 * u + 3]};
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(q + 1024 * u));
                }
            }
        } else {
            const int o = static_cast<int>(lane_piece<LC>(lane)) - static_cast<int>(pad0);
#pragma unroll
            for (int j = 0; j < MR; ++j) {
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    stripe + static_cast<uint64_t>(out_idx[j]) * a.shard_stride + start, 0,
                    static_cast<int>(G::kRow - pad0), 0x00020000);
#pragma unroll
                for (int i = 0; i < G::kDw; ++i) __builtin_amdgcn_raw_buffer_store_b32(acc[j][i], rs, voff(o, i), 0, 0);
            }
        }
        // CRC: each lane takes its LC contiguous parity bytes (register transpose), then one
        // slicing-by-4 chain per parity row, chains interleaved for LDS latency.
#pragma unroll
        for (int j = 0; j < MR; ++j) lane_contiguous<LC>(acc[j]);
        if (r > r0) {
            const cu32 gap = as_const(a.c->gap[G::kVar]);
#pragma unroll
            for (int j = 0; j < MR; ++j) crc[j] = apply(gap, crc[j]);
        }
#pragma unroll
        for (int d = 0; d < G::kDw; ++d)
#pragma unroll
            for (int j = 0; j < MR; ++j) crc[j] = slice4(lt, crc[j] ^ acc[j][d]);
    };

    // Rows r0 .. kRows-2: the next row's loads go out before this row's stores, so the wait
    // for them never includes the stores' completion, and the stores + CRC overlap the load
    // latency.  The sched barriers keep the loads after the math (hoisted into it they would
    // hold two rows of data at once).  The last row is peeled: a conditional load would keep
    // the consumed row alive through a phi.
    uint32_t r = r0;
    for (; r + 1 < G::kRows; ++r) {
        uint32_t acc[MR][G::kDw] = {};
        compute(acc);
        __builtin_amdgcn_sched_barrier(0);
        load_row<K, LC>(a, stripe, in_idx, seg_off + static_cast<int64_t>(r + 1) * G::kRow, lane, x);
        __builtin_amdgcn_sched_barrier(0);
        store_crc(r, acc);
    }
    {
        uint32_t acc[MR][G::kDw] = {};
        compute(acc);
        store_crc(r, acc);
    }

    // Lane chunks end at the row's lane*LC + LC; fold them to the segment end.
    const cu32 wlvl = as_const(&a.c->wlvl[G::kVar][0][0]);
#pragma unroll
    for (int l = 0; l < 6; ++l) {
#pragma unroll
        for (int j = 0; j < MR; ++j) {
            const uint32_t other = __shfl_down(crc[j], 1u << l, 64);
            if ((lane & ((2u << l) - 1u)) == 0) crc[j] = apply(wlvl + 32 * l, crc[j]) ^ other;
        }
    }
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < MR; ++j) raw[j * raw_row] = crc[j];
}

// Persistent: one workgroup per CU (the banked tables are built once), and its 8 waves walk
// segments independently with no further barrier.  The waves of XCD x (workgroups are
// dealt round-robin over the 8 XCDs) cover the x-th eighth of the segments, interleaved
// across the XCD's waves, so each XCD streams one contiguous region.
template <int K, int MR, int LC>
__global__ __launch_bounds__(kEcThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void encode_crc_kernel(
    KArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    init_banked_tables(tab, a.c, kEcThreads);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LaneTabs lt(lane);
    const uint32_t nxcd = gridDim.x >= 8 ? 8u : 1u;
    const uint32_t xcd = blockIdx.x % nxcd;
    const uint64_t xwaves = static_cast<uint64_t>(gridDim.x / nxcd) * kWaves;
    const uint64_t lo = a.total_segs * xcd / nxcd, hi = a.total_segs * (xcd + 1) / nxcd;
    for (uint64_t g = lo + (blockIdx.x / nxcd) * kWaves + wave; g < hi; g += xwaves)
        encode_crc_segment<K, MR, LC>(a, g, lane, lt);
}

using KernelFn = void (*)(KArgs);

constexpr int lc_for(int K, int MR) { return K + MR <= 11 ? 64 : 32; }

template <int K, int MR>
constexpr KernelFn fn_of() { return encode_crc_kernel<K, MR, lc_for(K, MR)>; }

template <int K>
KernelFn pick_rows(int rows) {
    switch (rows) {
        case 1: return fn_of<K, 1>();
        case 2: return fn_of<K, 2>();
        case 3: return fn_of<K, 3>();
        case 4: return fn_of<K, 4>();
        case 5: return fn_of<K, 5>();
        default: return nullptr;
    }
}

// blb's classes RS(6,3), RS(8,3), RS(10,3), RS(12,5) (internal/core/StorageClass.go:7-13),
// the bench's RS(10,4), the reference tests' RS(3,2) and RS(4,2).
KernelFn pick(int k, int rows) {
    switch (k) {
        case 3: return pick_rows<3>(rows);
        case 4: return pick_rows<4>(rows);
        case 6: return pick_rows<6>(rows);
        case 8: return pick_rows<8>(rows);
        case 10: return pick_rows<10>(rows);
        case 12: return pick_rows<12>(rows);
        default: return nullptr;
    }
}

std::mutex g_attr_mu;
std::set<std::pair<int, KernelFn>> g_attr_done;  // (device, kernel) with the LDS limit raised

}  // namespace

static bool segment_supported(const EncodeCrcArgs& a) {
    const bool aligned = (reinterpret_cast<uintptr_t>(a.base) & 3u) == 0 && (a.shard_stride & 3u) == 0 &&
                         (a.stripe_stride & 3u) == 0 && (a.S & 3u) == 0 && (a.block & 3u) == 0;
    return a.base && aligned && a.block > 0 && a.phase == 0 && pick(a.k, a.rows) != nullptr;
}

bool encode_crc_supported(const EncodeCrcArgs& a) { return encode_crc_tile_supported(a) || segment_supported(a); }

hipError_t launch_encode_crc(const EncodeCrcArgs& in, hipStream_t stream) {
    if (in.B == 0 || in.S == 0) return hipSuccess;
    if (!encode_crc_supported(in) || !in.crc) return hipErrorInvalidValue;
    const bool persistent = tune::get(tune::kEcPersistent) != 0;  // A/B in one process (tuning.hpp)
    if ((!persistent || !segment_supported(in)) && encode_crc_tile_supported(in))
        return launch_encode_crc_tile(in, stream);
    const KernelFn fn = pick(in.k, in.rows);
    const CrcConsts* c = nullptr;
    hipError_t e = crc_consts_for(kSeg, &c);
    if (e != hipSuccess) return e;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> g(g_attr_mu);
        if (g_attr_done.insert({dev, fn}).second) {
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    static_cast<int>(kEcLds));
            if (e != hipSuccess) {
                g_attr_done.erase({dev, fn});
                return e;
            }
        }
    }
    KArgs a{};
    a.tables = in.tables;
    a.in_idx = in.in_idx;
    a.out_idx = in.out_idx;
    a.base = in.base;
    a.shard_stride = in.shard_stride;
    a.stripe_stride = in.stripe_stride;
    a.S = in.S;
    a.block = std::min<uint64_t>(in.block, in.S);
    a.B = in.B;
    a.nblocks = static_cast<uint32_t>((in.S + a.block - 1) / a.block);
    a.segs_per_block = static_cast<uint32_t>((a.block + kSeg - 1) / kSeg);
    a.total_segs = static_cast<uint64_t>(in.B) * a.nblocks * a.segs_per_block;
    a.c = c;
    const uint64_t total_blocks = static_cast<uint64_t>(in.rows) * in.B * a.nblocks;
    if (a.total_segs * kWaves > 0x7FFFFFFFull || total_blocks * a.segs_per_block > 0x7FFFFFFFull)
        return hipErrorInvalidValue;
    if ((e = hipMallocAsync(reinterpret_cast<void**>(&a.raw), total_blocks * a.segs_per_block * 4, stream)) !=
        hipSuccess)
        return e;
    // Persistent grid: one workgroup per CU.
    static thread_local int cus = 0;
    if (!cus && (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0))
        cus = 256;
    uint64_t grid = std::min<uint64_t>((a.total_segs + kWaves - 1) / kWaves, static_cast<uint64_t>(cus));
    if (grid >= 8) grid = (grid + 7) & ~uint64_t{7};  // whole XCD rounds (the kernel splits by blockIdx % 8)
    hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(grid)), dim3(kEcThreads), kEcLds, stream, a);
    e = hipGetLastError();
    if (e == hipSuccess)
        e = crc_combine(c, a.raw, a.S, a.block, kSeg, a.nblocks, a.segs_per_block, total_blocks, in.crc, stream, 0,
                        in.seeds);
    const hipError_t f = hipFreeAsync(a.raw, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
