// crc_device.hpp -- CRC-32C (Castagnoli) building blocks shared by the CRC kernels
// (crc32c.hip) and the fused encode+CRC kernel (encode_crc.hip).
//
// CRC is linear over GF(2).  With raw(M) = the register after feeding M into a zero
// register (no init, no final xor):
//     raw(A || B) = S_{|B|} raw(A)  ^  raw(B)          S_n = "feed n zero bytes", a 32x32
//     crc(M)      = ~( S_{|M|} 0xFFFFFFFF ^ raw(M) )   GF(2) matrix (host-precomputed).
#pragma once
#include "dev_common.hpp"

namespace blbrs {

constexpr uint32_t kCrcPoly = 0x82F63B78u;  // reflected Castagnoli
constexpr int kCrcPow2 = 48;                // S_{2^i}, i < 48

// Device constants for one segment size (host-built once per (device, seg)).
struct CrcConsts {
    uint32_t table[4][256];        // slicing-by-4 tables
    uint32_t chain[3][32];         // S_{(3-j) * Lc}: chain j -> end of the lane's region
    uint32_t lvl[8][32];           // S_{L * 2^j}, columns
    uint32_t seg[32];              // S_SEG
    uint32_t pow2[kCrcPow2][32];   // S_{2^i}
    // streaming kernels: lane chunks of LC bytes at column lane of 64*LC-byte rows
    uint32_t gap[2][32];           // S_{64*LC - LC} for LC = 64, 32: chunk end -> next chunk
    uint32_t wlvl[2][6][32];       // S_{LC * 2^j} for LC = 64, 32: lane folds inside a wave
};

// Per-segment raw CRCs -> per-block CRCs: block id of `total_blocks` (= rows * nblocks; row
// r's block j is id r * nblocks + j) folds its raw[id * segs_per_block + s] with S_seg
// (Horner, virtual coordinates: row bytes start `phase` into block 0) and applies the init
// term with block 0's real length and seed.  out[id] = crc32.Update(seed, block bytes).
hipError_t crc_consts_for(uint64_t seg, const CrcConsts** out);
// Host: the column-major matrix S_n (feed n zero bytes), for kernels' constant tables.
void crc_shift_matrix(uint64_t n, uint32_t col[32]);

hipError_t crc_combine(const CrcConsts* c, const uint32_t* raw, uint64_t len, uint64_t block, uint64_t seg,
                       uint32_t nblocks, uint32_t segs_per_block, uint64_t total_blocks, uint32_t* out,
                       hipStream_t stream, uint64_t phase = 0, const uint32_t* seeds = nullptr);

namespace dev {

// r -> S r for a column-major 32x32 GF(2) matrix held in constant memory (scalar loads):
// per bit, a 1-bit sign-extract and one v_bitop3 (out ^ (mask & col), truth table 0x78).
__device__ __forceinline__ uint32_t apply(cu32 col, uint32_t r) {
    uint32_t out = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t mask = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(r), i, 1));
        out = __builtin_amdgcn_bitop3_b32(out, mask, col[i], 0x78);
    }
    return out;
}

// Banked slicing tables in LDS (128 KiB): a private copy of the four tables per bank, laid
// out so table j, entry e, bank l lives at byte (j>>1)<<16 | e<<8 | (j&1)<<7 | l<<2.  A
// 32-lane group then always hits 32 distinct banks and each lookup address is ONE v_perm_b32
// of (x, base_j).  The kernel must have no static LDS, so its dynamic LDS starts at address
// 0 and a perm result IS the LDS address.
constexpr size_t kBankedTableBytes = 4u * 256u * 32u * 4u;

__device__ __forceinline__ void init_banked_tables(uint32_t* tab, const CrcConsts* c, uint32_t nthreads) {
    for (uint32_t i = threadIdx.x; i < 4u * 256u * 32u; i += nthreads) {
        const uint32_t j = ((i >> 14) << 1) | ((i >> 5) & 1u), e = (i >> 6) & 255u;
        tab[i] = c->table[j][e];
    }
}

struct LaneTabs {
    uint32_t b[4];  // LDS address of this lane's bank in the table serving byte k
    __device__ __forceinline__ explicit LaneTabs(uint32_t lane) {
        const uint32_t lb = (lane & 31u) << 2;
        b[0] = (1u << 16) | (1u << 7) | lb;  // table 3
        b[1] = (1u << 16) | lb;              // table 2
        b[2] = (1u << 7) | lb;               // table 1
        b[3] = lb;                           // table 0
    }
};

typedef const __attribute__((address_space(3))) uint32_t* lds_u32;

// Table lookups for byte k of x: table 3-k (crc32c_le slicing order).
template <uint32_t K>
__device__ __forceinline__ uint32_t lookup(const LaneTabs& t, uint32_t x) {
    constexpr uint32_t sel = 0x03020000u | ((4u + K) << 8);  // [base.b0, x.bK, base.b2, base.b3]
    return *reinterpret_cast<lds_u32>(static_cast<size_t>(__builtin_amdgcn_perm(x, t.b[K], sel)));
}

// raw(c || w) for one dword w: slicing-by-4 (4 perms + 4 LDS reads + 2 XOR).
__device__ __forceinline__ uint32_t slice4(const LaneTabs& t, uint32_t x) {
    return xor3(lookup<0>(t, x), lookup<1>(t, x), lookup<2>(t, x)) ^ lookup<3>(t, x);
}

// Coalesced loads and stores, ordered for the CRC: instruction q of a row covers its 1 KiB
// sub-row q (64 pieces of 16 B), and within it lane (h, j) -- h = lane / (64 / P), P =
// LC / 16 pieces per lane -- takes piece P*j + h.  Lane L's LC contiguous CRC bytes
// (pieces P*L .. P*L + P-1) then sit in register q = L / (64 / P) of the P lanes (i, L %
// (64 / P)): a P x P transpose over (lane group, register) that v_permlane{16,32}_swap do
// in registers (lane_contiguous below), instead of a round trip through LDS.
template <int LC>
__device__ __forceinline__ uint32_t lane_piece(uint32_t lane) {
    if constexpr (LC == 64) return 16u * (4u * (lane & 15u) + (lane >> 4));
    else if constexpr (LC == 32) return 16u * (2u * (lane & 31u) + (lane >> 5));
    else return 16u * lane;  // LC 16: one piece per lane, already contiguous
}

// v[q][0..3] = this lane's piece of sub-row q -> v[i][0..3] = piece i of the lane's own
// LC-byte chunk.  E[row][q] -> E[q][row] with rows = 16-lane (LC 64) or 32-lane (LC 32)
// lane groups: permlane32_swap(a, b) swaps a's upper-half lanes with b's lower-half lanes,
// permlane16_swap(a, b) a's odd 16-lane rows with b's even rows.
template <int LC>
__device__ __forceinline__ void lane_contiguous(uint32_t (&v)[LC / 4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        if constexpr (LC == 64) {
            auto s02 = __builtin_amdgcn_permlane32_swap(v[d], v[8 + d], false, false);
            auto s13 = __builtin_amdgcn_permlane32_swap(v[4 + d], v[12 + d], false, false);
            auto s01 = __builtin_amdgcn_permlane16_swap(s02[0], s13[0], false, false);
            auto s23 = __builtin_amdgcn_permlane16_swap(s02[1], s13[1], false, false);
            v[d] = s01[0];
            v[4 + d] = s01[1];
            v[8 + d] = s23[0];
            v[12 + d] = s23[1];
        } else if constexpr (LC == 32) {
            auto s01 = __builtin_amdgcn_permlane32_swap(v[d], v[4 + d], false, false);
            v[d] = s01[0];
            v[4 + d] = s01[1];
        }
    }
}

}  // namespace dev
}  // namespace blbrs
