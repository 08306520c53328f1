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
//  * CRC: each lane runs one slicing-by-8 chain per parity row over its LC bytes (8 KiB of
//    tables in LDS).  The lane's chains are shifted to the row end by S_{LC*(63-lane)} in two
//    nibble-table factors (8.5 KiB in LDS), the first on every row, the second on one row
//    per lane after an 8-lane XOR (row_totals); the row totals are then folded to the tile
//    end with S_{64*LC*(3-w)}, spread over the lanes of waves 0 and 1.  Every workgroup
//    stages 17 KiB of constants from L2 for its one tile.
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

#include <algorithm>
#include <map>
#include <mutex>

#include "crc_device.hpp"
#include "gf_bitslice.hpp"
#include "gf_device.hpp"
#include "tuning.hpp"

namespace blbrs {
namespace rt {
hipError_t upload_pinned(void* dev, const void* src, size_t n);  // runtime.hpp
}  // namespace rt
namespace {

using namespace dev;

constexpr int kTThreads = 256;                     // 4 waves, one row each
constexpr uint64_t kOrd = 0x7FFFFFFFull;            // S_{kOrd} = I (checked on the host)
// Tuning builds only (tools/ect_variants.sh; the cost split in profiles/r02/ect_ab): 1 = skip
// the constant staging, 2 = skip the slicing chains, 4 = skip the lane shifts, 16 = the slicing
// lookups made bank-conflict-free (index = the byte's top 3 bits * 32 + lane % 32: the same
// instructions and data dependence, one bank per lane of a 32-lane group; profiles/r04/crc_lds).
// Results are wrong with any bit set.
#ifndef BLBRS_ECT_FLAGS
#define BLBRS_ECT_FLAGS 0
#endif
constexpr int kFlags = BLBRS_ECT_FLAGS;

// Lane chunks: LC = 32 bytes (8 KiB tiles) for every instantiated shape.  16-byte chunks
// (4 KiB tiles) halve the input registers at twice the lane shifts per byte; RS(12,5) needed
// them while its 32-byte form took 256 VGPRs, and since the shift work moved to row_totals
// and the coefficient loads were sequenced it fits 168 and runs 14.10-14.15 vs 15.06-15.11 ms
// (r2u_lc32).  k + rows >= BLBRS_ECT_LC16_MIN selects 16 (A/B builds).  64-byte chunks (16
// KiB tiles, 2 waves per SIMD) were slower.
#ifndef BLBRS_ECT_LC16_MIN
#define BLBRS_ECT_LC16_MIN 18
#endif
constexpr int lc_for(int k, int rows) { return k + rows >= BLBRS_ECT_LC16_MIN ? 16 : 32; }
constexpr int lc_index(int lc) { return lc == 32 ? 0 : 1; }

// Per LC: the nibble tables of the lane shifts and the row-end -> tile-end matrices.
//   nib: S_{LC*e} (e = 63 - lane: lane chunk end -> end of the wave's row) in two factors,
//        S_{LC*e} = A_{e>>3} B_{e&7} with B_b = S_{LC*b} (tables 0..7) and A_a = S_{8*LC*a}
//        (tables 8..15); table t, nibble k, value v at [t * kNibStride + 16 * k + v] is the
//        matrix applied to v << 4k.  16 lookups per value instead of 32 columns x 2 VALU.
//   wavemat[w] = S_{64*LC*(3-w)} (row end -> tile end), column-major.
// tab[k][i] = CRC of byte i followed by k zero bytes (slicing-by-kSlice uses tables 0..kSlice-1).
constexpr uint32_t kNibStride = 136;  // 128 + 8 words: the 16 tables start on 8 different banks
constexpr uint32_t kNibWords = 16 * kNibStride;
struct TileConsts {
    uint32_t nib[2][kNibWords];
    uint32_t wavemat[2][4][32];
    uint32_t tab[32][256];
};

// Slicing width of the chains: 8 (4 dependent steps per 32-byte lane chunk, 8 KiB of tables
// per workgroup), 16 (2 steps, 16 KiB) or 32 (no dependent step, 32 KiB).
#ifndef BLBRS_ECT_SLICE
#define BLBRS_ECT_SLICE 8
#endif
constexpr int kSlice = BLBRS_ECT_SLICE;
static_assert(kSlice == 8 || kSlice == 16 || kSlice == 32, "slicing width");

// Coefficient loads one input pair behind the accumulators (0 = unconstrained): without it
// all K*MR*5 table words are loaded up front and spill SGPRs (RS(12,5): 300 words, 70
// spills); with it RS(12,5) 15.82 vs 16.18 ms, RS(10,4) 11.12 vs 11.22 (r2r_tabseq).
#ifndef BLBRS_ECT_TABSEQ
#define BLBRS_ECT_TABSEQ 1
#endif
constexpr int kTabSeq = BLBRS_ECT_TABSEQ;

// 1 = the split wave's second pass zeroes the acc dwords before the boundary in place, so the
// chain loop carries no per-dword masks: RS(12,5) 14.15-14.41 vs 14.25-14.43 ms, RS(6,3)
// 12.60-12.97 vs 12.68-12.95 (profiles/r03/ect_ab).  0 = the masked loop (A/B builds).
#ifndef BLBRS_ECT_MASKACC
#define BLBRS_ECT_MASKACC 1
#endif
constexpr int kMaskAcc = BLBRS_ECT_MASKACC;
// N > 0 = persistent grid of N workgroups per CU, each walking its XCD's tiles in a loop with
// the constants staged once (A/B builds).
#ifndef BLBRS_ECT_PERSIST
#define BLBRS_ECT_PERSIST 0
#endif
[[maybe_unused]] constexpr int kPersist = BLBRS_ECT_PERSIST;

struct TArgs {
    const uint32_t* tables;
    const int32_t* in_idx;
    const int32_t* out_idx;
    uint8_t* base;
    uint64_t shard_stride, stripe_stride;
    uint64_t S, block, phase;
    const uint32_t* seeds;    // [j * B + b]: crc32.Update seed of block 0 (NULL = 0)
    uint32_t B, tps, xcd_remap, nblocks;
    uint32_t tps_full;        // whole tiles per stripe (the main grid); tps - 1 when S % T != 0
    const CrcConsts* c;
    const uint32_t* nib;      // [kNibWords] for this LC
    const uint32_t* tab8;     // [kSlice][256] (the first kSlice tables of TileConsts::tab)
    const uint32_t* wavemat;  // [4][32] for this LC
    uint32_t* raw;            // [(j * B + b) * tps + tile]: raw CRC of the tile's bytes
    uint32_t* hi;             // same index: raw CRC of the bytes past the tile's block boundary
};

// XOR over the 64 lanes, result in every lane, all on the VALU: DPP inside each 16-lane row
// (swap neighbours, swap pairs, half-row mirror, row mirror), then permlane16/32 swaps across
// rows -- no ds_bpermute through the LDS pipe the slicing lookups need.  (Cost-split builds
// only: the shipped path reduces through row_totals.)
[[maybe_unused]] __device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x141, 0xF, 0xF, false));  // half-row mirror
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x140, 0xF, 0xF, false));  // row mirror
    auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = r16[0] ^ r16[1];
    auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return r32[0] ^ r32[1];
}

// 1 = each nibble-table address is v_bfe + v_lshl_add (the nibble is made opaque so the
// compiler does not rewrite it as shift + and + add, 3 VALU).
#ifndef BLBRS_ECT_NIB2
#define BLBRS_ECT_NIB2 0
#endif

__device__ __forceinline__ uint32_t apply_nib(const uint32_t* t, uint32_t c) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint32_t nb = __builtin_amdgcn_ubfe(c, 4 * k, 4);
        if constexpr (BLBRS_ECT_NIB2) asm volatile("" : "+v"(nb));
        v[k] = t[16 * k + nb];
    }
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
}

// The wave's row totals: row j's sum over lanes of S_{LC*(63-lane)} crc_lane[j].  B factor on
// every row, XOR over the lane's 8-lane group (whose values then agree), lane h = lane & 7
// takes row h for the A factor (one apply instead of MR), XOR over the 8 groups.  Lane h
// returns row h's total (h < MR).  Per lane: MR + 1 factor applies instead of 2 MR, one
// 8-group reduction instead of MR wave reductions (RS(12,5) 16.6 -> 15.6 ms, r2q_spread).
template <int MR>
__device__ __forceinline__ uint32_t row_totals(const uint32_t* nt, uint32_t lane, const uint32_t (&crc)[MR]) {
    static_assert(MR <= 8, "one row per lane of an 8-lane group");
    const uint32_t e = 63u - lane;
    const uint32_t* tb = nt + (e & 7u) * kNibStride;
    const uint32_t* ta = nt + (8u + (e >> 3)) * kNibStride;
    uint32_t row = 0u;
#pragma unroll
    for (int j = 0; j < MR; ++j) {
        uint32_t t = apply_nib(tb, crc[j]);
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0xB1, 0xF, 0xF, false));
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0x4E, 0xF, 0xF, false));
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0x141, 0xF, 0xF, false));
        row = (lane & 7u) == static_cast<uint32_t>(j) ? t : row;
    }
    row = apply_nib(ta, row);
    row ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(row), 0x128, 0xF, 0xF, false));  // row_ror:8
    auto r16 = __builtin_amdgcn_permlane16_swap(row, row, false, false);
    row = r16[0] ^ r16[1];
    auto r32 = __builtin_amdgcn_permlane32_swap(row, row, false, false);
    return r32[0] ^ r32[1];
}

// One slicing-by-8 step: x = crc ^ first dword, y = second dword (byte k of x: table 7-k,
// byte k of y: table 3-k).  The y lookups do not depend on the chain, and a 32-byte lane
// chunk takes 4 dependent LDS round trips instead of 8 (slicing-by-4: +1.5 % at RS(6,3)).
__device__ __forceinline__ uint32_t slice8(const uint32_t* tab, uint32_t x, uint32_t y) {
    uint32_t v[8];
    if constexpr (kFlags & 16) {
        const uint32_t l32 = threadIdx.x & 31u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = tab[(7 - k) * 256 + ((__builtin_amdgcn_ubfe(x, 8 * k + 5, 3) << 5) | l32)];
            v[4 + k] = tab[(3 - k) * 256 + ((__builtin_amdgcn_ubfe(y, 8 * k + 5, 3) << 5) | l32)];
        }
        return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = tab[(7 - k) * 256 + __builtin_amdgcn_ubfe(x, 8 * k, 8)];
        v[4 + k] = tab[(3 - k) * 256 + __builtin_amdgcn_ubfe(y, 8 * k, 8)];
    }
    return xor3(xor3(v[0], v[1], v[2]), xor3(v[3], v[4], v[5]), v[6]) ^ v[7];
}

// XOR of N values, three at a time (v_bitop3).
template <int N>
__device__ __forceinline__ uint32_t xor_tree(const uint32_t* v) {
    if constexpr (N == 1) return v[0];
    else if constexpr (N == 2) return v[0] ^ v[1];
    else return xor3(xor_tree<N / 3>(v), xor_tree<N / 3>(v + N / 3), xor_tree<N - 2 * (N / 3)>(v + 2 * (N / 3)));
}

// One slicing-by-SL step over SL / 4 dwords: d[0] already holds crc ^ first dword.  Byte k of
// dword q uses table SL-1-4q-k; the lookups are independent of one another.
template <int SL>
__device__ __forceinline__ uint32_t slice_n(const uint32_t* tab, const uint32_t* d) {
    uint32_t v[SL];
#pragma unroll
    for (int q = 0; q < SL / 4; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) v[4 * q + k] = tab[(SL - 1 - 4 * q - k) * 256 + __builtin_amdgcn_ubfe(d[q], 8 * k, 8)];
    return xor_tree<SL>(v);
}

// The CRC part of one tile: this lane's LC contiguous parity bytes per row (acc, already in
// lane_contiguous order) -> raw / hi of the tile, written by waves 0 and 1.  `red` is the
// workgroup's reduction buffer (2 x 4 x MR words); one __syncthreads inside.
template <int MR, int LC>
__device__ __forceinline__ void crc_tile(const TArgs& a, uint32_t (&acc)[MR][LC / 4], const uint32_t* tab,
                                         const uint32_t* nib, const uint32_t* wm, uint32_t (*red)[4][MR],
                                         uint64_t tile_off, uint64_t at0, uint32_t tid, uint32_t lane, uint32_t wave) {
    constexpr int NV = LC / 4;
    constexpr uint32_t kRow = 64u * LC;
    constexpr uint32_t kTile = 4u * kRow;
    // The first block boundary after the tile start; inside the tile -> the bytes past it
    // get their own raw CRC (hi).  Only the wave whose row holds the boundary needs a masked
    // chain: in earlier waves hi = 0, in later ones hi = the full raw CRC.
    const uint64_t nb = ((tile_off + a.phase) / a.block + 1) * a.block - a.phase;
    const bool split = nb < tile_off + kTile;
    const uint32_t o = split ? static_cast<uint32_t>(nb - tile_off) : kTile;
    const uint32_t o_wave = o / kRow;
    const uint32_t mine = LC * tid;
    // Pass 0: every byte (raw).  Pass 1, only in the wave whose row holds the boundary: the
    // bytes past it (hi).  One masked code path for both keeps the register footprint of the
    // rare split wave at that of the others; separate unmasked pass-0 chains let the compiler
    // hoist every lookup (165 instead of 112 VGPRs at RS(6,3)).
    uint32_t r_raw = 0u, r_hi = 0u;  // this lane's row (lane & 7) of the wave totals
    uint32_t f_raw[MR], f_hi[MR];    // BLBRS_ECT_FLAGS & 4 only: per-row wave XORs
    const uint32_t passes = split && wave == o_wave ? 2u : 1u;
#pragma unroll 1
    for (uint32_t pass = 0; pass < passes; ++pass) {
        uint32_t crc[MR];
#pragma unroll
        for (int j = 0; j < MR; ++j) crc[j] = 0u;
        if constexpr (kMaskAcc) {
            if (pass == 1)
#pragma unroll
                for (int d = 0; d < NV; ++d)
#pragma unroll
                    for (int j = 0; j < MR; ++j) acc[j][d] = mine + 4u * d >= o ? acc[j][d] : 0u;
        }
        if constexpr (kSlice == 8) {
#pragma unroll
            for (int d = 0; d < NV; d += 2) {
                const bool keep0 = kMaskAcc || pass == 0 || mine + 4u * d >= o;
                const bool keep1 = kMaskAcc || pass == 0 || mine + 4u * d + 4u >= o;
#pragma unroll
                for (int j = 0; j < MR; ++j) {
                    const uint32_t x = crc[j] ^ (keep0 ? acc[j][d] : 0u), y = keep1 ? acc[j][d + 1] : 0u;
                    crc[j] = (kFlags & 2) ? x ^ y : slice8(tab, x, y);
                }
            }
        } else {
            static_assert(kMaskAcc, "wide slicing needs the in-place mask");
            constexpr int W = kSlice / 4 < NV ? kSlice / 4 : NV;
#pragma unroll
            for (int d = 0; d < NV; d += W) {
#pragma unroll
                for (int j = 0; j < MR; ++j) {
                    uint32_t w[W];
#pragma unroll
                    for (int q = 0; q < W; ++q) w[q] = acc[j][d + q];
                    w[0] ^= crc[j];
                    crc[j] = (kFlags & 2) ? w[0] ^ w[W - 1] : slice_n<4 * W>(tab, w);
                }
            }
        }
        if constexpr (kFlags & 4) {
#pragma unroll
            for (int j = 0; j < MR; ++j) (pass == 0 ? f_raw : f_hi)[j] = wave_xor(crc[j]);
        } else {
            const uint32_t t = row_totals<MR>(nib, lane, crc);
            if (pass == 0) r_raw = t;
            else r_hi = t;
        }
    }
    if constexpr (kFlags & 4) {
        if (passes == 1)
#pragma unroll
            for (int j = 0; j < MR; ++j) f_hi[j] = split && wave > o_wave ? f_raw[j] : 0u;
        if (lane == 0)
#pragma unroll
            for (int j = 0; j < MR; ++j) {
                red[0][wave][j] = f_raw[j];
                red[1][wave][j] = f_hi[j];
            }
    } else {
        if (passes == 1) r_hi = split && wave > o_wave ? r_raw : 0u;
        if (lane < static_cast<uint32_t>(MR)) {
            red[0][wave][lane] = r_raw;
            red[1][wave][lane] = r_hi;
        }
    }
    __syncthreads();
    // Row ends -> tile end, spread over lanes: wave 0 folds the raw values, wave 1 the hi
    // values; lane 8j + s takes half s&1 of S_{64*LC*(3-w)} (w = s>>1, 16 columns) on row j's
    // wave-w value (s = 6: wave 3's value unshifted, s = 7: nothing), and the 8-lane group
    // XORs -- 32 VALU per lane instead of six serial 32-column applies in one wave.
    if (wave < 2 && lane < 8u * MR) {
        const uint32_t j = lane >> 3, sl = lane & 7u;
        uint32_t t = 0u;
        if (sl < 6u) {
            const uint32_t w = sl >> 1, h16 = (sl & 1u) * 16u;
            const uint32_t v = red[wave][w][j];
            const uint32_t* col = wm + 32u * w + h16;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                t = __builtin_amdgcn_bitop3_b32(
                    t, static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(v), static_cast<int>(h16) + i, 1)),
                    col[i], 0x78);
        } else if (sl == 6u) {
            t = red[wave][3][j];
        }
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
        t ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(t), 0x141, 0xF, 0xF, false));  // half-row mirror
        if (sl == 0u) {
            const uint64_t at = at0 + static_cast<uint64_t>(j) * a.B * a.tps;
            (wave == 0 ? a.raw : a.hi)[at] = t;
        }
    }
}

// All K inputs of the tile in flight (nontemporal: every byte is read once).
template <int K, int LC, bool PARTIAL>
__device__ __forceinline__ void load_tile(const TArgs& a, const uint8_t* stripe, uint64_t tile_off, uint32_t in_tile,
                                          uint32_t lim, uint32_t (&x)[K][LC / 4]) {
    constexpr int NQ = LC / 16;
    const ci32 in_idx = as_const(a.in_idx);
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const uint8_t* p = stripe + static_cast<uint64_t>(in_idx[c]) * a.shard_stride + tile_off + in_tile;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (!PARTIAL || in_tile + 1024u * q < lim)
                v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 1024 * q));
            x[c][4 * q] = v.x;
            x[c][4 * q + 1] = v.y;
            x[c][4 * q + 2] = v.z;
            x[c][4 * q + 3] = v.w;
        }
    }
}

// The parity rows of the tile, stored nontemporal; acc keeps them.  CM: the plan's rows are
// encode parity rows 0..MR-1 of K, computed by the compiled bit-plane XOR network (the
// inputs are transposed in place); otherwise the v_perm multiply with the plan's tables.
template <int K, int MR, int LC, bool PARTIAL, bool CM>
__device__ __forceinline__ void code_tile(const TArgs& a, uint8_t* stripe, uint64_t tile_off, uint32_t in_tile,
                                          uint32_t lim, uint32_t (&x)[K][LC / 4], uint32_t (&acc)[MR][LC / 4]) {
    constexpr int NV = LC / 4;
    constexpr int NQ = LC / 16;
    const ci32 out_idx = as_const(a.out_idx);
    if constexpr (CM) {
        static_assert(NV == 8, "bit planes of 8 dwords");
#ifdef BLBRS_ECT_CM_PAIRS  // A/B: fold input pairs as their loads land
        bs::parity_rows_by_pairs<K, MR>(x, acc);
#else
#pragma unroll
        for (int c = 0; c < K; ++c) bs::transpose8(x[c]);
        bs::parity_rows<K, MR>(x, acc);
#endif
    } else {
        cu32 tables = as_const(a.tables);
        asm volatile("" : "+s"(tables));
#pragma unroll
        for (int c = 0; c + 1 < K; c += 2) {
            if constexpr (kTabSeq > 0)
                if (c >= 2 * kTabSeq) asm volatile("" : "+s"(tables) : "v"(acc[0][0]));
            madd2<MR, NV>(Groups<NV>(x[c]), [&](int r) { return tables + (r * K + c) * 5; }, Groups<NV>(x[c + 1]),
                          [&](int r) { return tables + (r * K + c + 1) * 5; }, acc, MR);
        }
        if constexpr (K & 1)
            madd<MR, NV>(Groups<NV>(x[K - 1]), [&](int r) { return tables + (r * K + K - 1) * 5; }, acc, MR);
    }
#pragma unroll
    for (int j = 0; j < MR; ++j) {
        uint8_t* q = stripe + static_cast<uint64_t>(out_idx[j]) * a.shard_stride + tile_off + in_tile;
#pragma unroll
        for (int u = 0; u < NQ; ++u)
            if (!PARTIAL || in_tile + 1024u * u < lim)
                __builtin_nontemporal_store(u32x4{acc[j][4 * u], acc[j][4 * u + 1], acc[j][4 * u + 2], acc[j][4 * u + 3]},
                                            reinterpret_cast<u32x4*>(q + 1024 * u));
    }
}

// One workgroup = one tile of one stripe (PARTIAL: the stripe's partial last tile, in a
// second B-workgroup launch so that the masking never touches the main kernel).  Several
// tiles per workgroup (constants staged once, the next tile's loads issued under this
// tile's CRC) held 149-197 VGPRs and lost 5-7 % (r2g).
// Wide-slicing builds hold the main instantiations to 3 waves per SIMD (RS(12,5) lands one
// VGPR past 168 otherwise); the partial-tile launch (B workgroups) is left unconstrained.
template <int K, int MR, int LC, bool PARTIAL, bool CM>
__global__ __launch_bounds__(kTThreads) __attribute__((amdgpu_waves_per_eu((PARTIAL || kSlice == 8) ? 1 : 3)))
void encode_crc_tile_kernel(TArgs a) {
    constexpr int NV = LC / 4;
    constexpr uint32_t kRow = 64u * LC;
    constexpr uint32_t kTile = 4u * kRow;
    __shared__ __attribute__((aligned(16))) uint32_t tab[kSlice * 256];
    __shared__ __attribute__((aligned(16))) uint32_t nib[kNibWords];
    __shared__ uint32_t red[2][4][MR];
    __shared__ uint32_t wm[96];  // S_{64*LC*(3-w)}, w < 3

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t b, tile;
    if constexpr (PARTIAL) {
        b = blockIdx.x;
        tile = a.tps - 1;
    } else {
        uint32_t t = blockIdx.x;
        if (a.xcd_remap) t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
        b = t / a.tps_full;
        tile = t - b * a.tps_full;
    }
    const uint64_t tile_off = static_cast<uint64_t>(tile) * kTile;
    uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
    const uint32_t in_tile = wave * kRow + lane_piece<LC>(lane);  // tile offset of piece q = 0
    // Bytes of the partial tile inside the shard (a multiple of 16).
    const uint32_t lim = PARTIAL ? static_cast<uint32_t>(a.S - tile_off) : kTile;

    // Constants (L2 hits) into registers first, then the data loads: the LDS writes below
    // wait for the constants only (in-order vmcnt).  Wide slicing tables (16-32 KiB, 16-byte
    // vectors) are loaded after the data, so their registers are not held while the inputs
    // are in flight.
    constexpr int kFill = kSlice == 8 ? 8 * 256 / kTThreads : 1;            // slicing-by-8 words
    constexpr int kFillV = kSlice == 8 ? 1 : kSlice * 256 / 4 / kTThreads;  // wide: vectors
    constexpr int kNFill = (kNibWords + kTThreads - 1) / kTThreads;         // nibble-table words
    uint32_t tv[kFill], nv[kNFill];
    if constexpr (kSlice == 8)
#pragma unroll
        for (int r = 0; r < kFill; ++r) tv[r] = (kFlags & 1) ? tid * 3u + r : a.tab8[tid + r * kTThreads];
#pragma unroll
    for (int r = 0; r < kNFill; ++r) {
        const uint32_t i = tid + r * kTThreads;
        nv[r] = (kFlags & 1) ? tid * 5u + r : i < kNibWords ? a.nib[i] : 0u;
    }
    const uint32_t wmv = tid < 96u ? a.wavemat[tid] : 0u;
    uint32_t x[K][NV];
    load_tile<K, LC, PARTIAL>(a, stripe, tile_off, in_tile, lim, x);
    if constexpr (kSlice == 8) {
#pragma unroll
        for (int r = 0; r < kFill; ++r) tab[tid + r * kTThreads] = tv[r];
    } else {
        const u32x4* tsrc = reinterpret_cast<const u32x4*>(a.tab8);
        u32x4 tw[kFillV];
#pragma unroll
        for (int r = 0; r < kFillV; ++r)
            tw[r] = (kFlags & 1) ? u32x4{tid, 3u, 5u, static_cast<uint32_t>(r)} : tsrc[tid + r * kTThreads];
#pragma unroll
        for (int r = 0; r < kFillV; ++r) reinterpret_cast<u32x4*>(tab)[tid + r * kTThreads] = tw[r];
    }
#pragma unroll
    for (int r = 0; r < kNFill; ++r) {
        const uint32_t i = tid + r * kTThreads;
        if (i < kNibWords) nib[i] = nv[r];
    }
    if (tid < 96u) wm[tid] = wmv;

    uint32_t acc[MR][NV] = {};
    code_tile<K, MR, LC, PARTIAL, CM>(a, stripe, tile_off, in_tile, lim, x, acc);
    // CRC of this lane's LC contiguous parity bytes (tile offset LC * tid) per row.
#pragma unroll
    for (int j = 0; j < MR; ++j) lane_contiguous<LC>(acc[j]);
    __syncthreads();  // tables
    crc_tile<MR, LC>(a, acc, tab, nib, wm, red, tile_off, static_cast<uint64_t>(b) * a.tps + tile, tid, lane, wave);
}

#if BLBRS_ECT_PERSIST
// Persistent form (BLBRS_ECT_PERSIST workgroups per CU): constants staged once per workgroup,
// then the workgroup walks tiles of its XCD's contiguous share in a loop.  The reduction
// buffer alternates between two halves: crc_tile's barrier keeps the waves within one tile
// of each other, so a wave writing tile i+1's row totals never meets the fold of tile i-1.
template <int K, int MR, int LC>
__global__ __launch_bounds__(kTThreads) __attribute__((amdgpu_waves_per_eu(kPersist > 3 ? kPersist : 3)))
void encode_crc_tile_persist_kernel(TArgs a) {
    constexpr int NV = LC / 4;
    constexpr uint32_t kRow = 64u * LC;
    constexpr uint32_t kTile = 4u * kRow;
    __shared__ uint32_t tab[kSlice * 256];
    __shared__ uint32_t nib[kNibWords];
    __shared__ uint32_t red[2][2][4][MR];
    __shared__ uint32_t wm[96];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (uint32_t i = tid; i < kSlice * 256u; i += kTThreads) tab[i] = a.tab8[i];
    for (uint32_t i = tid; i < kNibWords; i += kTThreads) nib[i] = a.nib[i];
    if (tid < 96u) wm[tid] = a.wavemat[tid];
    __syncthreads();
    const uint32_t groups = a.B * a.tps_full;
    // XCD x = blockIdx % 8 takes tiles [x * groups / 8, (x + 1) * groups / 8); its workgroups
    // interleave over that range in dispatch order.
    const uint32_t xcd = blockIdx.x % 8u, per_xcd = gridDim.x / 8u, local = blockIdx.x / 8u;
    const uint32_t t0 = static_cast<uint32_t>(static_cast<uint64_t>(groups) * xcd / 8u);
    const uint32_t t1 = static_cast<uint32_t>(static_cast<uint64_t>(groups) * (xcd + 1u) / 8u);
    const uint32_t in_tile = wave * kRow + lane_piece<LC>(lane);
    uint32_t it = 0;
#pragma unroll 1
    for (uint32_t t = t0 + local; t < t1; t += per_xcd, ++it) {
        const uint32_t b = t / a.tps_full, tile = t - b * a.tps_full;
        const uint64_t tile_off = static_cast<uint64_t>(tile) * kTile;
        uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
        uint32_t x[K][NV];
        load_tile<K, LC, false>(a, stripe, tile_off, in_tile, kTile, x);
        uint32_t acc[MR][NV] = {};
        code_tile<K, MR, LC, false, false>(a, stripe, tile_off, in_tile, kTile, x, acc);
#pragma unroll
        for (int j = 0; j < MR; ++j) lane_contiguous<LC>(acc[j]);
        crc_tile<MR, LC>(a, acc, tab, nib, wm, red[it & 1u], tile_off, static_cast<uint64_t>(b) * a.tps + tile, tid,
                         lane, wave);
    }
}
#endif

__device__ uint32_t shift_n(const CrcConsts* c, uint32_t r, uint64_t n) {
    const cu32 p = as_const(&c->pow2[0][0]);
    for (int i = 0; i < kCrcPow2 && n; ++i, n >>= 1)
        if (n & 1u) r = apply(p + 32 * i, r);
    return r;
}

// Block `blk` of row-stripe jb in shard coordinates: [bs, be) (file-aligned, phase).
__device__ __forceinline__ void block_range(const TArgs& a, uint32_t blk, uint64_t* bs, uint64_t* be) {
    const uint64_t vs = static_cast<uint64_t>(blk) * a.block;  // file-aligned block [vs, vs + block)
    *bs = vs > a.phase ? vs - a.phase : 0;
    *be = vs + a.block - a.phase < a.S ? vs + a.block - a.phase : a.S;
}

// Horner over tiles [f, l] of the block [bs, be): the raw CRC of the block's bytes in them,
// as if ending at tile l's end.
__device__ __forceinline__ uint32_t fold_tiles(const TArgs& a, uint64_t jb, uint64_t bs, uint64_t be, uint32_t log2t,
                                               uint64_t f, uint64_t l) {
    const uint32_t* raw = a.raw + jb * a.tps;
    const uint32_t* hi = a.hi + jb * a.tps;
    const cu32 st = as_const(&a.c->pow2[log2t][0]);
    uint32_t acc = 0u;
    for (uint64_t i = f; i <= l; ++i) {
        uint32_t piece = (i << log2t) < bs ? hi[i] : raw[i];  // block starts inside tile i
        if (((i + 1) << log2t) > be && be < a.S) piece ^= hi[i];  // next block starts inside tile i
        acc = (i == f ? 0u : apply(st, acc)) ^ piece;
    }
    return acc;
}

// Whole-shard frames span 512-2048 tiles: folding them in one thread per (row, stripe)
// serialises ~1-2k matrix applies on a few thousand threads.  Blocks of more than
// kChunk tiles fold in two levels: this kernel, one thread per (row, stripe, block, chunk of
// kChunk tiles), then tile_combine_kernel over the chunks.
constexpr uint32_t kChunkLog2 = 5;
constexpr uint32_t kChunk = 1u << kChunkLog2;

__global__ __launch_bounds__(256) void tile_chunk_kernel(TArgs a, uint32_t log2t, uint32_t nchunk, uint64_t total,
                                                         uint32_t* part) {
    const uint64_t id = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (id >= total) return;
    const uint32_t c = static_cast<uint32_t>(id % nchunk);
    const uint64_t rest = id / nchunk;
    const uint32_t blk = static_cast<uint32_t>(rest % a.nblocks);
    const uint64_t jb = rest / a.nblocks;
    uint64_t bs, be;
    block_range(a, blk, &bs, &be);
    const uint64_t i0 = bs >> log2t, i1 = (be - 1) >> log2t;
    const uint64_t f = i0 + (static_cast<uint64_t>(c) << kChunkLog2);
    part[id] = f > i1 ? 0u : fold_tiles(a, jb, bs, be, log2t, f, f + kChunk - 1 < i1 ? f + kChunk - 1 : i1);
}

// One thread per (row j, stripe b, block): Horner over the block's tiles (T = 2^log2t), or
// over its chunk partials when `part` is set.
__global__ __launch_bounds__(256) void tile_combine_kernel(TArgs a, uint32_t log2t, uint64_t total, uint32_t* out,
                                                           uint32_t nchunk, const uint32_t* part) {
    const uint64_t id = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    if (id >= total) return;
    const uint32_t blk = static_cast<uint32_t>(id % a.nblocks);
    const uint64_t jb = id / a.nblocks;  // j * B + b
    uint64_t bs, be;
    block_range(a, blk, &bs, &be);
    const uint64_t i0 = bs >> log2t, i1 = (be - 1) >> log2t;
    uint32_t acc;
    if (part) {
        const cu32 sc = as_const(&a.c->pow2[log2t + kChunkLog2][0]);  // S_{kChunk * T}
        const uint32_t* p = part + id * nchunk;
        acc = 0u;
        for (uint32_t c = 0; c < nchunk; ++c) {
            const uint64_t f = i0 + (static_cast<uint64_t>(c) << kChunkLog2);
            if (f > i1) break;
            const uint64_t n = i1 - f + 1 < kChunk ? i1 - f + 1 : kChunk;  // tiles in chunk c
            if (c > 0) acc = n == kChunk ? apply(sc, acc) : shift_n(a.c, acc, n << log2t);
            acc ^= p[c];
        }
    } else {
        acc = fold_tiles(a, jb, bs, be, log2t, i0, i1);
    }
    const uint64_t tail = ((i1 + 1) << log2t) - be;
    if (tail) acc = shift_n(a.c, acc, kOrd - tail);
    const uint32_t seed = blk == 0 && a.seeds ? a.seeds[jb] : 0u;
    out[id] = ~(shift_n(a.c, ~seed, be - bs) ^ acc);
}

using KernelFn = void (*)(TArgs);

template <int K, int MR, bool P>
KernelFn pick_cm(bool cm) {
    constexpr int LC = lc_for(K, MR);
    if constexpr (LC == 32) {
        if (cm) return encode_crc_tile_kernel<K, MR, LC, P, true>;
    }
    return encode_crc_tile_kernel<K, MR, LC, P, false>;
}

template <int K, bool P>
KernelFn pick_rows(int rows, bool cm) {
    switch (rows) {
        case 1: return pick_cm<K, 1, P>(cm);
        case 2: return pick_cm<K, 2, P>(cm);
        case 3: return pick_cm<K, 3, P>(cm);
        case 4: return pick_cm<K, 4, P>(cm);
        case 5: return pick_cm<K, 5, P>(cm);
        default: return nullptr;
    }
}

// Same instantiated shapes as encode_crc.hip (blb's classes, RS(10,4), RS(3,2), RS(4,2)).
// cm: the pass computes encode parity rows (the compiled bit-plane network).
KernelFn pick(int k, int rows, bool partial = false, bool cm = false) {
    switch (k) {
        case 3: return partial ? pick_rows<3, true>(rows, cm) : pick_rows<3, false>(rows, cm);
        case 4: return partial ? pick_rows<4, true>(rows, cm) : pick_rows<4, false>(rows, cm);
        case 6: return partial ? pick_rows<6, true>(rows, cm) : pick_rows<6, false>(rows, cm);
        case 8: return partial ? pick_rows<8, true>(rows, cm) : pick_rows<8, false>(rows, cm);
        case 10: return partial ? pick_rows<10, true>(rows, cm) : pick_rows<10, false>(rows, cm);
        case 12: return partial ? pick_rows<12, true>(rows, cm) : pick_rows<12, false>(rows, cm);
        default: return nullptr;
    }
}

#if BLBRS_ECT_PERSIST
template <int K>
KernelFn pick_persist_rows(int rows) {
    switch (rows) {
        case 1: return encode_crc_tile_persist_kernel<K, 1, lc_for(K, 1)>;
        case 2: return encode_crc_tile_persist_kernel<K, 2, lc_for(K, 2)>;
        case 3: return encode_crc_tile_persist_kernel<K, 3, lc_for(K, 3)>;
        case 4: return encode_crc_tile_persist_kernel<K, 4, lc_for(K, 4)>;
        case 5: return encode_crc_tile_persist_kernel<K, 5, lc_for(K, 5)>;
        default: return nullptr;
    }
}

KernelFn pick_persist(int k, int rows) {
    switch (k) {
        case 3: return pick_persist_rows<3>(rows);
        case 4: return pick_persist_rows<4>(rows);
        case 6: return pick_persist_rows<6>(rows);
        case 8: return pick_persist_rows<8>(rows);
        case 10: return pick_persist_rows<10>(rows);
        case 12: return pick_persist_rows<12>(rows);
        default: return nullptr;
    }
}
#endif

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
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int j = 0; j < 8; ++j) v = (v & 1u) ? (v >> 1) ^ kCrcPoly : v >> 1;
            host.tab[0][i] = v;
        }
        for (int k = 1; k < 32; ++k)
            for (uint32_t i = 0; i < 256; ++i)
                host.tab[k][i] = (host.tab[k - 1][i] >> 8) ^ host.tab[0][host.tab[k - 1][i] & 255u];
        for (int v = 0; v < 2; ++v) {
            const uint64_t lc = v == 0 ? 32 : 16;
            uint32_t col[32];
            for (int w = 0; w < 4; ++w) {
                crc_shift_matrix(64 * lc * static_cast<uint64_t>(3 - w), col);
                for (int i = 0; i < 32; ++i) host.wavemat[v][w][i] = col[i];
            }
            for (int t = 0; t < 16; ++t) {
                crc_shift_matrix(t < 8 ? lc * static_cast<uint64_t>(t) : 8 * lc * static_cast<uint64_t>(t - 8), col);
                for (int k = 0; k < 8; ++k)
                    for (uint32_t x = 0; x < 16; ++x) {
                        uint32_t o = 0;
                        for (int bit = 0; bit < 4; ++bit)
                            if ((x >> bit) & 1u) o ^= col[4 * k + bit];
                        host.nib[v][t * kNibStride + 16 * k + x] = o;
                    }
            }
        }
        TileConsts* d = nullptr;
        if ((e = hipMalloc(&d, sizeof(TileConsts))) != hipSuccess) return e;
        if ((e = rt::upload_pinned(d, &host, sizeof(TileConsts))) != hipSuccess) {
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
    const bool cm = bs::use(in.parity, in.k, in.rows, bs::kWideTile);
    const KernelFn fn = pick(in.k, in.rows, false, cm);
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
    const uint32_t log2t = lc == 32 ? 13u : 12u;
    a.tps = static_cast<uint32_t>((in.S + (uint64_t{1} << log2t) - 1) >> log2t);
    a.tps_full = static_cast<uint32_t>(in.S >> log2t);
    a.nblocks = static_cast<uint32_t>((in.S + a.phase + a.block - 1) / a.block);
    a.c = c;
    a.nib = &tc->nib[lc_index(lc)][0];
    a.wavemat = &tc->wavemat[lc_index(lc)][0][0];
    a.tab8 = &tc->tab[0][0];
    const uint64_t tiles = static_cast<uint64_t>(in.B) * a.tps;
    const uint64_t groups = static_cast<uint64_t>(in.B) * a.tps_full;  // one tile per workgroup
    a.xcd_remap = groups % 8 == 0 ? 1u : 0u;
    const uint64_t nraw = static_cast<uint64_t>(in.rows) * tiles;
    uint32_t* buf = nullptr;
    if ((e = hipMallocAsync(reinterpret_cast<void**>(&buf), nraw * 8, stream)) != hipSuccess) return e;
    a.raw = buf;
    a.hi = buf + nraw;
#if BLBRS_ECT_PERSIST
    if constexpr (kPersist > 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint64_t grid = std::min<uint64_t>(groups, static_cast<uint64_t>(cus) * kPersist) / 8u * 8u;
        if (groups && grid >= 8)
            hipLaunchKernelGGL(pick_persist(in.k, in.rows), dim3(static_cast<unsigned>(grid)), dim3(kTThreads), 0, stream, a);
        else if (groups)
            hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(groups)), dim3(kTThreads), 0, stream, a);
    }
#else
    if (groups) hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(groups)), dim3(kTThreads), 0, stream, a);
#endif
    e = hipGetLastError();
    if (e == hipSuccess && a.tps != a.tps_full) {
        hipLaunchKernelGGL(pick(in.k, in.rows, true, cm), dim3(in.B), dim3(kTThreads), 0, stream, a);
        e = hipGetLastError();
    }
    const uint64_t total = static_cast<uint64_t>(in.rows) * in.B * a.nblocks;
    // Tiles a block can touch: ceil(block / T) + 1 (an unaligned block straddles one more).
    const uint64_t max_tiles = ((a.block + (uint64_t{1} << log2t) - 1) >> log2t) + 1;
    const uint32_t nchunk = max_tiles > 2 * kChunk ? static_cast<uint32_t>((max_tiles + kChunk - 1) >> kChunkLog2) : 0u;
    uint32_t* part = nullptr;
    if (e == hipSuccess && nchunk) {
        e = hipMallocAsync(reinterpret_cast<void**>(&part), total * nchunk * sizeof(uint32_t), stream);
        if (e == hipSuccess) {
            const uint64_t nthreads = total * nchunk;
            hipLaunchKernelGGL(tile_chunk_kernel, dim3(static_cast<unsigned>((nthreads + 255) / 256)), dim3(256), 0,
                               stream, a, log2t, nchunk, nthreads, part);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(tile_combine_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                           stream, a, log2t, total, in.crc, nchunk, part);
        e = hipGetLastError();
    }
    hipError_t f = hipSuccess;
    if (part) f = hipFreeAsync(part, stream);
    const hipError_t g = hipFreeAsync(buf, stream);
    if (f == hipSuccess) f = g;
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
