// gf_device.hpp -- GF(2^8) multiply-accumulate by constants on gfx950 (v_perm_b32 tables),
// shared by the coding kernel (rs_kernels.hip) and the fused encode+CRC kernel
// (encode_crc.hip).
//
// byte x = g0 | g1<<3 | g2<<6 (3+3+2 bits) and c*x = T0[g0]^T1[g1]^T2[g2]; each table has
// <= 8 one-byte entries, so one v_perm_b32 byte-select over two dwords looks up 4 bytes at
// once.  A coefficient is 5 table dwords (gf256.hpp builds them on the host).  Cost: 5 VALU
// per input dword for the bit groups (shared by every output row) + 3 perms + 1.5
// v_bitop3 XOR3 per (coefficient, dword).
#pragma once
#include "dev_common.hpp"

namespace blbrs {
namespace dev {

struct alignas(16) V4 { uint32_t x, y, z, w; };

__device__ __forceinline__ void unpack(const V4& q, uint32_t* w) { w[0] = q.x; w[1] = q.y; w[2] = q.z; w[3] = q.w; }
__device__ __forceinline__ V4 pack(const uint32_t* w) { return V4{w[0], w[1], w[2], w[3]}; }

// Bit groups of NV input dwords: g0 = x[2:0], g1 = x[5:3], g2 = x[7:6] of every byte
// (5 VALU per dword, shared by every output row).
template <int NV>
struct Groups {
    uint32_t g0[NV], g1[NV], g2[NV];
    __device__ __forceinline__ explicit Groups(const uint32_t (&x)[NV]) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            g0[v] = x[v] & 0x07070707u;
            g1[v] = (x[v] >> 3) & 0x07070707u;
            g2[v] = (x[v] >> 6) & 0x03030303u;
        }
    }
};

template <typename TP>
__device__ __forceinline__ void load_tab(TP tp, uint32_t (&t)[5]) {
#pragma unroll
    for (int w = 0; w < 5; ++w) t[w] = tp[w];
}

// acc[r] ^= coef(r, c) * x over NV input dwords of ONE input shard c: 3 v_perm + 2 xor3
// per (row, dword).  Each row's 5 table words are fetched once and applied to all NV
// dwords (amortises the SGPR->VGPR moves v_perm needs for its second table operand under
// gfx9's one-SGPR constant-bus limit).
template <int MR, int NV, typename Tab>
__device__ __forceinline__ void madd(const Groups<NV>& g, Tab tab, uint32_t (&acc)[MR][NV], int nr) {
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r < nr) {
            uint32_t t[5];
            load_tab(tab(r), t);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const uint32_t p0 = __builtin_amdgcn_perm(t[1], t[0], g.g0[v]);
                const uint32_t p1 = __builtin_amdgcn_perm(t[3], t[2], g.g1[v]);
                const uint32_t p2 = __builtin_amdgcn_perm(0u, t[4], g.g2[v]);
                acc[r][v] = xor3(xor3(acc[r][v], p0, p1), p2, 0u);
            }
        }
    }
}

// Two input shards at once: 6 perm terms + acc folded by 3 xor3 (1.5 VALU per coefficient
// and dword instead of 3 plain XORs).
template <int MR, int NV, typename TabA, typename TabB>
__device__ __forceinline__ void madd2(const Groups<NV>& ga, TabA taba, const Groups<NV>& gb, TabB tabb,
                                      uint32_t (&acc)[MR][NV], int nr) {
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r < nr) {
            uint32_t a[5], b[5];
            load_tab(taba(r), a);
            load_tab(tabb(r), b);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const uint32_t a0 = __builtin_amdgcn_perm(a[1], a[0], ga.g0[v]);
                const uint32_t a1 = __builtin_amdgcn_perm(a[3], a[2], ga.g1[v]);
                const uint32_t a2 = __builtin_amdgcn_perm(0u, a[4], ga.g2[v]);
                const uint32_t b0 = __builtin_amdgcn_perm(b[1], b[0], gb.g0[v]);
                const uint32_t b1 = __builtin_amdgcn_perm(b[3], b[2], gb.g1[v]);
                const uint32_t b2 = __builtin_amdgcn_perm(0u, b[4], gb.g2[v]);
                acc[r][v] = xor3(xor3(xor3(acc[r][v], a0, a1), a2, b0), b1, b2);
            }
        }
    }
}


// Dword-outer forms for wide rows (NV = 16): the coefficient tables of an input pair for all
// rows stay in registers across the NV dwords and the bit groups of one dword are formed at
// a time, so only one dword's groups are live instead of NV of them (the row-outer forms
// above hold 3*NV group registers per input through all rows).
template <int MR, int NV, typename TabA, typename TabB>
__device__ __forceinline__ void madd2_dw(const uint32_t (&xa)[NV], TabA taba, const uint32_t (&xb)[NV], TabB tabb,
                                         uint32_t (&acc)[MR][NV]) {
    uint32_t ta[MR][5], tb[MR][5];
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        load_tab(taba(r), ta[r]);
        load_tab(tabb(r), tb[r]);
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const uint32_t a0g = xa[v] & 0x07070707u, a1g = (xa[v] >> 3) & 0x07070707u, a2g = (xa[v] >> 6) & 0x03030303u;
        const uint32_t b0g = xb[v] & 0x07070707u, b1g = (xb[v] >> 3) & 0x07070707u, b2g = (xb[v] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const uint32_t a0 = __builtin_amdgcn_perm(ta[r][1], ta[r][0], a0g);
            const uint32_t a1 = __builtin_amdgcn_perm(ta[r][3], ta[r][2], a1g);
            const uint32_t a2 = __builtin_amdgcn_perm(0u, ta[r][4], a2g);
            const uint32_t b0 = __builtin_amdgcn_perm(tb[r][1], tb[r][0], b0g);
            const uint32_t b1 = __builtin_amdgcn_perm(tb[r][3], tb[r][2], b1g);
            const uint32_t b2 = __builtin_amdgcn_perm(0u, tb[r][4], b2g);
            acc[r][v] = xor3(xor3(xor3(acc[r][v], a0, a1), a2, b0), b1, b2);
        }
    }
}

template <int MR, int NV, typename Tab>
__device__ __forceinline__ void madd_dw(const uint32_t (&x)[NV], Tab tab, uint32_t (&acc)[MR][NV]) {
    uint32_t t[MR][5];
#pragma unroll
    for (int r = 0; r < MR; ++r) load_tab(tab(r), t[r]);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const uint32_t g0 = x[v] & 0x07070707u, g1 = (x[v] >> 3) & 0x07070707u, g2 = (x[v] >> 6) & 0x03030303u;
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            const uint32_t p0 = __builtin_amdgcn_perm(t[r][1], t[r][0], g0);
            const uint32_t p1 = __builtin_amdgcn_perm(t[r][3], t[r][2], g1);
            const uint32_t p2 = __builtin_amdgcn_perm(0u, t[r][4], g2);
            acc[r][v] = xor3(xor3(acc[r][v], p0, p1), p2, 0u);
        }
    }
}

}  // namespace dev
}  // namespace blbrs
