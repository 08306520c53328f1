// encode_crc_tile.hip -- fused Reed-Solomon encode + CRC-32C of the parity on the coding
// kernel's own tile grid (the layout rs_code_kernel streams at the read-k/write-m rate).
//
// Same job as encode_crc.hip (the tractserver checksums every parity increment it writes:
// pkg/disk/checksum_block.go:18-34 65532-byte ChecksumFile blocks, pkg/rpc/bulk_codec.go:47
// whole frames), different geometry.  encode_crc.hip walks end-aligned block segments with a
// persistent grid so that a segment never crosses a block boundary; that grid is what keeps
// it ~15 % behind the plain encode even with the CRC switched off.  Here:
//  * one workgroup = one tile of T = 256 * LC bytes of every shard of one stripe, one tile
//    per workgroup in dispatch order with each XCD streaming a contiguous eighth of the
//    tiles -- rs_code_kernel's grid.  Wave w owns the tile's w-th 64*LC-byte row, loaded
//    and stored with coalesced 1 KiB instructions (lane_piece) and transposed in registers
//    (lane_contiguous) so that lane L holds the LC contiguous bytes at tile offset LC * tid.
//  * CRC: each lane runs one slicing-by-4 chain per parity row over its LC bytes (tables in
//    LDS; C interleaved copies would spread bank conflicts but cost more to stage, so C = 1),
//    shifts it to its wave row's end with its own matrix S_{LC*(63-lane)} (64 matrices
//    staged in LDS), and the wave XORs its lanes; one lane per row shifts the 4 row values to the tile end (S_{64*LC*(3-w)}) and
//    XORs them.  Per workgroup that is 4*C + 8 KiB of constants from L2 -- kept small
//    because every workgroup stages them for one tile.
//  * Tiles ignore block boundaries.  A tile that contains one (at dword offset o) also runs
//    a second chain over its bytes at offsets >= o only (`hi`); by linearity the part before
//    the boundary is raw ^ hi.  A combine kernel then Horner-folds each block's tiles and
//    takes the block-end part of its last tile back by S_{-n} = S_{ord - n}, ord = 2^31 - 1
//    being the multiplicative order of x modulo the Castagnoli polynomial.
//  * Blocks are file-aligned: shard byte 0 sits `phase` bytes into block 0 (rsEncodeOne's
//    parity windows start at 4 MiB * i of the piece, store.go:1028-1037,1115), so the
//    boundaries are at offsets block * n - phase; block 0's CRC continues a caller seed
//    (crc32.Update, pkg/disk/checksum_block.go:80).  The last tile may be partial (S a
//    multiple of 16, e.g. the 4,128,704-byte last increment of a 67,043,264-byte piece): its
//    pieces past S are neither loaded nor stored and enter the CRC as zeros, which the
//    combine shifts back out like any block end inside a tile.
#include "encode_crc.hpp"

#include <map>
#include <mutex>

#include "crc_device.hpp"
#include "gf_device.hpp"

namespace blbrs {
namespace {

using namespace dev;

constexpr int kTThreads = 256;                     // 4 waves, one row each
constexpr uint64_t kOrd = 0x7FFFFFFFull;            // S_{kOrd} = I (checked on the host)
#ifndef BLBRS_ECT_COPIES
#define BLBRS_ECT_COPIES 1
#endif
constexpr int kCopies = BLBRS_ECT_COPIES;           // interleaved copies of the slicing tables

// Shift matrices (v = 0: LC 64, v = 1: LC 32): lanemat[v][i][l] = column i of S_{LC*(63-l)}
// (lane chunk end -> end of the wave's row; staged in LDS per workgroup, one conflict-free
// column read per lane) and wavemat[v][w] = S_{64*LC*(3-w)} (row end -> tile end).
struct TileConsts {
    uint32_t lanemat[2][32][64];
    uint32_t wavemat[2][4][32];
};

struct TArgs {
    const uint32_t* tables;
    const int32_t* in_idx;
    const int32_t* out_idx;
    uint8_t* base;
    uint64_t shard_stride, stripe_stride;
    uint64_t S, block, phase;
    const uint32_t* seeds;    // [j * B + b]: crc32.Update seed of block 0 (NULL = 0)
    uint32_t B, tps, xcd_remap, nblocks;
    const CrcConsts* c;
    const uint32_t* lanemat;  // [32][64] for this LC
    const uint32_t* wavemat;  // [4][32] for this LC
    uint32_t* raw;            // [(j * B + b) * tps + tile]: raw CRC of the tile's bytes
    uint32_t* hi;             // same index: raw CRC of the bytes past the tile's block boundary
};

// 32-byte lane chunks for every shape: 8 KiB tiles, <= 165 VGPRs for rows <= 4 (3-4 waves per
// SIMD); 64-byte chunks (16 KiB tiles, 2 waves per SIMD) measured slower.
constexpr int lc_for(int, int) { return 32; }

// One slicing-by-4 step over C-copy tables (table 3-k serves byte k).
template <int C>
__device__ __forceinline__ uint32_t slice4c(const uint32_t* tab, uint32_t copy, uint32_t x) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t e = __builtin_amdgcn_ubfe(x, 8 * k, 8);
        v[k] = tab[(3 - k) * 256 * C + e * C + copy];
    }
    return xor3(v[0], v[1], v[2]) ^ v[3];
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) v ^= __shfl_xor(v, s, 64);
    return v;
}

template <int K, int MR, int LC>
__global__ __launch_bounds__(kTThreads) void encode_crc_tile_kernel(TArgs a) {
    constexpr int NV = LC / 4;
    constexpr int NQ = LC / 16;
    constexpr uint32_t kRow = 64u * LC;
    constexpr uint32_t kTile = 4u * kRow;
    __shared__ uint32_t tab[4 * 256 * kCopies];
    __shared__ uint32_t lmat[32 * 64];
    __shared__ uint32_t red[2][4][MR];

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t t = blockIdx.x;
    if (a.xcd_remap) t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
    const uint32_t b = t / a.tps;
    const uint32_t tile = t - b * a.tps;
    const uint64_t tile_off = static_cast<uint64_t>(tile) * kTile;
    uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
    const uint32_t in_tile = wave * kRow + lane_piece<LC>(lane);  // tile offset of piece q = 0
    const uint64_t my_off = tile_off + in_tile;
    // Bytes of this tile inside the shard (kTile except in a partial last tile; uniform).
    const uint32_t lim = static_cast<uint32_t>(a.S - tile_off < kTile ? a.S - tile_off : kTile);
    const bool full = lim == kTile;
    const ci32 in_idx = as_const(a.in_idx);
    const ci32 out_idx = as_const(a.out_idx);

    constexpr int kFill = 4 * 256 * kCopies / kTThreads;  // table words per thread
    constexpr int kMFill = 32 * 64 / kTThreads;            // lane-matrix words per thread
    uint32_t tv[kFill], mv[kMFill];
    {
        const uint32_t* src = &a.c->table[0][0];
#pragma unroll
        for (int r = 0; r < kFill; ++r) tv[r] = src[(tid + r * kTThreads) / kCopies];
#pragma unroll
        for (int r = 0; r < kMFill; ++r) mv[r] = a.lanemat[tid + r * kTThreads];
    }
    // All K inputs in flight (nontemporal: every byte is read once).
    uint32_t x[K][NV];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint8_t* p = stripe + static_cast<uint64_t>(in_idx[c]) * a.shard_stride + my_off;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (full || in_tile + 1024u * q < lim) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 1024 * q));
            x[c][4 * q] = v.x;
            x[c][4 * q + 1] = v.y;
            x[c][4 * q + 2] = v.z;
            x[c][4 * q + 3] = v.w;
        }
    }
    // Slicing tables (L2 hits): written to LDS once their loads, issued before the data's,
    // have landed -- the in-order vmcnt lets that wait skip the data loads.
#pragma unroll
    for (int r = 0; r < kFill; ++r) tab[tid + r * kTThreads] = tv[r];
#pragma unroll
    for (int r = 0; r < kMFill; ++r) lmat[tid + r * kTThreads] = mv[r];

    uint32_t acc[MR][NV] = {};
    {
        cu32 tables = as_const(a.tables);
        asm volatile("" : "+s"(tables));
#pragma unroll
        for (int c = 0; c + 1 < K; c += 2)
            madd2<MR, NV>(Groups<NV>(x[c]), [&](int r) { return tables + (r * K + c) * 5; }, Groups<NV>(x[c + 1]),
                          [&](int r) { return tables + (r * K + c + 1) * 5; }, acc, MR);
        if constexpr (K & 1)
            madd<MR, NV>(Groups<NV>(x[K - 1]), [&](int r) { return tables + (r * K + K - 1) * 5; }, acc, MR);
    }
#pragma unroll
    for (int j = 0; j < MR; ++j) {
        uint8_t* q = stripe + static_cast<uint64_t>(out_idx[j]) * a.shard_stride + my_off;
#pragma unroll
        for (int u = 0; u < NQ; ++u)
            if (full || in_tile + 1024u * u < lim)
                __builtin_nontemporal_store(
                    u32x4{acc[j][4 * u], acc[j][4 * u + 1], acc[j][4 * u + 2], acc[j][4 * u + 3]},
                    reinterpret_cast<u32x4*>(q + 1024 * u));
    }

    // CRC of this lane's LC contiguous parity bytes (tile offset LC * tid) per row.
#pragma unroll
    for (int j = 0; j < MR; ++j) lane_contiguous<LC>(acc[j]);
    __syncthreads();  // tables
    const uint32_t copy = lane % kCopies;
    // The first block boundary after the tile start; inside the tile -> the bytes past it
    // get their own raw CRC (hi).  Only the wave whose row holds the boundary needs a masked
    // chain: in earlier waves hi = 0, in later ones hi = the full raw CRC.
    const uint64_t nb = ((tile_off + a.phase) / a.block + 1) * a.block - a.phase;
    const bool split = nb < tile_off + kTile;
    const uint32_t o = split ? static_cast<uint32_t>(nb - tile_off) : kTile;
    const uint32_t o_wave = o / kRow;
    const uint32_t mine = LC * tid;
    uint32_t crc[MR], chi[MR];
#pragma unroll
    for (int j = 0; j < MR; ++j) crc[j] = chi[j] = 0u;
    if (split && wave == o_wave) {
#pragma unroll
        for (int d = 0; d < NV; ++d) {
            const bool keep = mine + 4u * d >= o;
#pragma unroll
            for (int j = 0; j < MR; ++j) {
                crc[j] = slice4c<kCopies>(tab, copy, crc[j] ^ acc[j][d]);
                chi[j] = slice4c<kCopies>(tab, copy, chi[j] ^ (keep ? acc[j][d] : 0u));
            }
        }
    } else {
#pragma unroll
        for (int d = 0; d < NV; ++d)
#pragma unroll
            for (int j = 0; j < MR; ++j) crc[j] = slice4c<kCopies>(tab, copy, crc[j] ^ acc[j][d]);
    }

    // Shift each lane's chain to its row end (S_{LC*(63-lane)} from LDS) and XOR over the
    // wave; the row -> tile-end shift is applied once per row in the final reduction.
    uint32_t o_raw[MR], o_hi[MR];
#pragma unroll
    for (int j = 0; j < MR; ++j) o_raw[j] = o_hi[j] = 0u;
    if (split && wave == o_wave) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const uint32_t col = lmat[i * 64 + lane];
#pragma unroll
            for (int j = 0; j < MR; ++j) {
                o_raw[j] = __builtin_amdgcn_bitop3_b32(
                    o_raw[j], static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(crc[j]), i, 1)), col, 0x78);
                o_hi[j] = __builtin_amdgcn_bitop3_b32(
                    o_hi[j], static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(chi[j]), i, 1)), col, 0x78);
            }
        }
#pragma unroll
        for (int j = 0; j < MR; ++j) {
            o_raw[j] = wave_xor(o_raw[j]);
            o_hi[j] = wave_xor(o_hi[j]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const uint32_t col = lmat[i * 64 + lane];
#pragma unroll
            for (int j = 0; j < MR; ++j)
                o_raw[j] = __builtin_amdgcn_bitop3_b32(
                    o_raw[j], static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(crc[j]), i, 1)), col, 0x78);
        }
#pragma unroll
        for (int j = 0; j < MR; ++j) {
            o_raw[j] = wave_xor(o_raw[j]);
            o_hi[j] = split && wave > o_wave ? o_raw[j] : 0u;
        }
    }
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < MR; ++j) {
            red[0][wave][j] = o_raw[j];
            red[1][wave][j] = o_hi[j];
        }
    __syncthreads();
    if (tid < MR) {
        const uint32_t j = tid;
        const cu32 wm = as_const(a.wavemat);
        uint32_t r = red[0][3][j], h = red[1][3][j];
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            r ^= apply(wm + 32 * w, red[0][w][j]);
            h ^= apply(wm + 32 * w, red[1][w][j]);
        }
        const uint64_t at = (static_cast<uint64_t>(j) * a.B + b) * a.tps + tile;
        a.raw[at] = r;
        a.hi[at] = h;
    }
}

__device__ uint32_t shift_n(const CrcConsts* c, uint32_t r, uint64_t n) {
    const cu32 p = as_const(&c->pow2[0][0]);
    for (int i = 0; i < kCrcPow2 && n; ++i, n >>= 1)
        if (n & 1u) r = apply(p + 32 * i, r);
    return r;
}

// One thread per (row j, stripe b, block): Horner over the block's tiles (T = 2^log2t).
__global__ __launch_bounds__(256) void tile_combine_kernel(TArgs a, uint32_t log2t, uint64_t total, uint32_t* out) {
    const uint64_t id = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (id >= total) return;
    const uint32_t blk = static_cast<uint32_t>(id % a.nblocks);
    const uint64_t jb = id / a.nblocks;  // j * B + b
    const uint64_t vs = static_cast<uint64_t>(blk) * a.block;  // file-aligned block [vs, vs + block)
    const uint64_t bs = vs > a.phase ? vs - a.phase : 0;
    const uint64_t be = vs + a.block - a.phase < a.S ? vs + a.block - a.phase : a.S;
    const uint32_t* raw = a.raw + jb * a.tps;
    const uint32_t* hi = a.hi + jb * a.tps;
    const cu32 st = as_const(&a.c->pow2[log2t][0]);
    const uint64_t i0 = bs >> log2t, i1 = (be - 1) >> log2t;
    uint32_t acc = 0u;
    for (uint64_t i = i0; i <= i1; ++i) {
        uint32_t piece = (i << log2t) < bs ? hi[i] : raw[i];  // block starts inside tile i
        if (((i + 1) << log2t) > be && be < a.S) piece ^= hi[i];  // next block starts inside tile i
        acc = (i == i0 ? 0u : apply(st, acc)) ^ piece;
    }
    const uint64_t tail = ((i1 + 1) << log2t) - be;
    if (tail) acc = shift_n(a.c, acc, kOrd - tail);
    const uint32_t seed = blk == 0 && a.seeds ? a.seeds[jb] : 0u;
    out[id] = ~(shift_n(a.c, ~seed, be - bs) ^ acc);
}

using KernelFn = void (*)(TArgs);

template <int K>
KernelFn pick_rows(int rows) {
    constexpr int LC = lc_for(K, 0);
    switch (rows) {
        case 1: return encode_crc_tile_kernel<K, 1, LC>;
        case 2: return encode_crc_tile_kernel<K, 2, LC>;
        case 3: return encode_crc_tile_kernel<K, 3, LC>;
        case 4: return encode_crc_tile_kernel<K, 4, LC>;
        default: return nullptr;  // rows = 5 spills here; the segment kernel is faster (§4e)
    }
}

// Same instantiated shapes as encode_crc.hip (blb's classes, RS(10,4), RS(3,2), RS(4,2)).
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

std::mutex g_mu;
std::map<int, const TileConsts*> g_consts;  // per device, process lifetime

hipError_t tile_consts_for(const TileConsts** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(g_mu);
    auto& slot = g_consts[dev];
    if (!slot) {
        static TileConsts host;  // built under g_mu
        for (int v = 0; v < 2; ++v) {
            const uint64_t lc = v == 0 ? 64 : 32;
            uint32_t col[32];
            for (int l = 0; l < 64; ++l) {
                crc_shift_matrix(lc * static_cast<uint64_t>(63 - l), col);
                for (int i = 0; i < 32; ++i) host.lanemat[v][i][l] = col[i];
            }
            for (int w = 0; w < 4; ++w) {
                crc_shift_matrix(64 * lc * static_cast<uint64_t>(3 - w), col);
                for (int i = 0; i < 32; ++i) host.wavemat[v][w][i] = col[i];
            }
        }
        TileConsts* d = nullptr;
        if ((e = hipMalloc(&d, sizeof(TileConsts))) != hipSuccess) return e;
        if ((e = hipMemcpy(d, &host, sizeof(TileConsts), hipMemcpyHostToDevice)) != hipSuccess) {
            (void)hipFree(d);
            return e;
        }
        slot = d;
    }
    *out = slot;
    return hipSuccess;
}

// S_{kOrd} must be the identity for the combine's negative shifts.
bool order_ok() {
    static const bool ok = [] {
        uint32_t col[32];
        crc_shift_matrix(kOrd, col);
        for (int i = 0; i < 32; ++i)
            if (col[i] != (1u << i)) return false;
        return true;
    }();
    return ok;
}

}  // namespace

bool encode_crc_tile_supported(const EncodeCrcArgs& a) {
    if (!a.base || a.k <= 0 || a.rows <= 0 || pick(a.k, a.rows) == nullptr || !order_ok()) return false;
    const uint64_t T = 256ull * static_cast<uint64_t>(lc_for(a.k, a.rows));
    if (a.block == 0 || a.phase >= a.block) return false;
    const bool one_block = a.block >= a.S + a.phase;
    const bool aligned = (reinterpret_cast<uintptr_t>(a.base) & 15u) == 0 && (a.shard_stride & 15u) == 0 &&
                         (a.stripe_stride & 15u) == 0;
    // 16-byte pieces (the last tile may be partial), at most one block boundary per tile,
    // boundaries on dwords.
    return aligned && a.S % 16 == 0 && (one_block || (a.block >= T && (a.block & 3u) == 0 && (a.phase & 3u) == 0)) &&
           static_cast<uint64_t>(a.B) * ((a.S + T - 1) / T) <= 0x7FFFFFFFull;
}

hipError_t launch_encode_crc_tile(const EncodeCrcArgs& in, hipStream_t stream) {
    if (in.B == 0 || in.S == 0) return hipSuccess;
    if (!encode_crc_tile_supported(in) || !in.crc) return hipErrorInvalidValue;
    const int lc = lc_for(in.k, in.rows);
    const KernelFn fn = pick(in.k, in.rows);
    const CrcConsts* c = nullptr;
    hipError_t e = crc_consts_for(65536, &c);  // tables + pow2 (the segment size is irrelevant here)
    if (e != hipSuccess) return e;
    const TileConsts* tc = nullptr;
    if ((e = tile_consts_for(&tc)) != hipSuccess) return e;
    TArgs a{};
    a.tables = in.tables;
    a.in_idx = in.in_idx;
    a.out_idx = in.out_idx;
    a.base = in.base;
    a.shard_stride = in.shard_stride;
    a.stripe_stride = in.stripe_stride;
    a.S = in.S;
    a.phase = in.phase;
    a.block = in.block < in.S + in.phase ? in.block : in.S + in.phase;
    a.seeds = in.seeds;
    a.B = in.B;
    const uint32_t log2t = lc == 64 ? 14u : 13u;
    a.tps = static_cast<uint32_t>((in.S + (uint64_t{1} << log2t) - 1) >> log2t);
    a.nblocks = static_cast<uint32_t>((in.S + a.phase + a.block - 1) / a.block);
    a.c = c;
    a.lanemat = &tc->lanemat[lc == 64 ? 0 : 1][0][0];
    a.wavemat = &tc->wavemat[lc == 64 ? 0 : 1][0][0];
    const uint64_t tiles = static_cast<uint64_t>(in.B) * a.tps;
    a.xcd_remap = tiles % 8 == 0 ? 1u : 0u;
    const uint64_t nraw = static_cast<uint64_t>(in.rows) * tiles;
    uint32_t* buf = nullptr;
    if ((e = hipMallocAsync(reinterpret_cast<void**>(&buf), nraw * 8, stream)) != hipSuccess) return e;
    a.raw = buf;
    a.hi = buf + nraw;
    hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(tiles)), dim3(kTThreads), 0, stream, a);
    e = hipGetLastError();
    if (e == hipSuccess) {
        const uint64_t total = static_cast<uint64_t>(in.rows) * in.B * a.nblocks;
        hipLaunchKernelGGL(tile_combine_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                           stream, a, log2t, total, in.crc);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(buf, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
