// rs_rbs.hpp -- wide decode passes on bit planes with the coefficients read at run time
// (measurement only: built by tools/rbs_ab.hip, not part of libblbrs).
//
// The v_perm table kernel (rs_code.hpp) spends 3 perms + 1.5 XOR3 per (row, input, dword):
// at RS(12,5)'s recovery shape it keeps the SIMD's VALU ~97 % busy at 2 waves per SIMD
// (profiles/pmc_r06.json), so any drop in clock or rise in HBM rate leaves it behind the
// stream.  The compiled bit-plane networks need the coefficients at
// compile time (the encode matrix, or hipRTC per erasure pattern).  This kernel keeps the bit
// planes but takes the coefficients from memory:
//   * input c's 32 bytes per lane are bit-transposed (gf_bitslice.hpp transpose8) into 8
//     planes x; its multiples Y_i = 2^i x (i = 0..7) follow from x by the field's doubling,
//     3 XORs per step on planes;
//   * coef * x = XOR of Y_i over the set bits i of coef, so each (row, input) adds the Y_i
//     selected by the coefficient's low nibble (Y_0..3) and by its high nibble (Y_4..7):
//     a 16-way branch on a wave-uniform value into straight-line XOR3 code, 10 VALU per
//     nibble on average (8 planes x ceil(popcount / 2));
//   * inputs stream through a runtime loop with two inputs in flight ahead of the one being
//     multiplied (any k, no per-k code), the row accumulators stay in planes, and each row is
//     transposed back once at the end.
// Store mode only (the recovery RPC and the client's ReconstructData); partial or unaligned
// tiles take the table kernel's per-lane path.
#pragma once
#include "rs_code.hpp"

namespace blbrs {
namespace code {

// y = 2 * x on bit planes: GF(2^8) modulo x^8 + x^4 + x^3 + x^2 + 1 (0x11d).
__device__ __forceinline__ void times2(const uint32_t (&x)[8], uint32_t (&y)[8]) {
    y[0] = x[7];
    y[1] = x[0];
    y[2] = x[1] ^ x[7];
    y[3] = x[2] ^ x[7];
    y[4] = x[3] ^ x[7];
    y[5] = x[4];
    y[6] = x[5];
    y[7] = x[6];
}

constexpr int nth_bit(int m, int n) {
    for (int i = 0; i < 4; ++i)
        if ((m >> i) & 1) {
            if (n == 0) return i;
            --n;
        }
    return -1;
}
constexpr int popcount4(int m) { return (m & 1) + ((m >> 1) & 1) + ((m >> 2) & 1) + ((m >> 3) & 1); }

// acc ^= XOR of Y[i] over the set bits i of M, folded three at a time.
template <int M>
__device__ __forceinline__ void add_set(uint32_t (&acc)[8], const uint32_t (&Y)[4][8]) {
    constexpr int n = popcount4(M);
    constexpr int b0 = nth_bit(M, 0), b1 = nth_bit(M, 1), b2 = nth_bit(M, 2), b3 = nth_bit(M, 3);
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        if constexpr (n == 1) {
            acc[p] ^= Y[b0][p];
        } else if constexpr (n == 2) {
            acc[p] = dev::xor3(acc[p], Y[b0][p], Y[b1][p]);
        } else if constexpr (n == 3) {
            acc[p] = dev::xor3(acc[p] ^ Y[b2][p], Y[b0][p], Y[b1][p]);
        } else if constexpr (n == 4) {
            acc[p] = dev::xor3(dev::xor3(acc[p], Y[b0][p], Y[b1][p]), Y[b2][p], Y[b3][p]);
        }
    }
}

// The nibble's branch: n is wave-uniform (a scalar value), so this is a scalar branch tree.
__device__ __forceinline__ void add_nibble(uint32_t n, uint32_t (&acc)[8], const uint32_t (&Y)[4][8]) {
    switch (n) {
        case 1: add_set<1>(acc, Y); break;
        case 2: add_set<2>(acc, Y); break;
        case 3: add_set<3>(acc, Y); break;
        case 4: add_set<4>(acc, Y); break;
        case 5: add_set<5>(acc, Y); break;
        case 6: add_set<6>(acc, Y); break;
        case 7: add_set<7>(acc, Y); break;
        case 8: add_set<8>(acc, Y); break;
        case 9: add_set<9>(acc, Y); break;
        case 10: add_set<10>(acc, Y); break;
        case 11: add_set<11>(acc, Y); break;
        case 12: add_set<12>(acc, Y); break;
        case 13: add_set<13>(acc, Y); break;
        case 14: add_set<14>(acc, Y); break;
        case 15: add_set<15>(acc, Y); break;
        default: break;
    }
}

// Coefficients of a pass for this kernel: [k][2] dwords, byte r of the pair = coef[r][c]
// (rows <= 8).  rbs_coef_words() builds them on the host.
template <int MR, int ADDR>
__global__ __launch_bounds__(kThreads) void rs_rbs_kernel(CodeArgs a, const uint32_t* coef8) {
    constexpr int U = 2;  // 32 bytes per lane per shard: one group of 8 planes
    constexpr uint32_t kTile = kTileBytes * U;
    constexpr uint32_t kStep = kThreads * kBytesPerThread;
    const uint32_t total = a.B * a.tiles_per_stripe;
    uint32_t first = blockIdx.x;
    if (a.xcd_remap) first = (first % 8u) * (gridDim.x / 8u) + first / 8u;
    for (uint32_t t = first; t < total; t += gridDim.x) {
        const uint32_t b = t / a.tiles_per_stripe;
        const uint64_t tile_off = static_cast<uint64_t>(t - b * a.tiles_per_stripe) * kTile;
        if (!stripe_table_ok<ADDR>(a, b)) continue;
        if (!a.aligned || tile_off + kTile > a.S) {
            code_tile_slow<MR, 0, ADDR, U>(a, b, tile_off);
            continue;
        }
        const ci32 in_idx = as_const(a.in_idx);
        const ci32 out_idx = as_const(a.out_idx);
        const cu32 cw = as_const(coef8);
        const uint64_t lane_off = tile_off + static_cast<uint64_t>(threadIdx.x) * kBytesPerThread;
        const int k = a.k;
        auto load = [&](int c, V4 (&v)[2]) {
            const uint8_t* p = shard_ptr<ADDR>(a, b, in_idx[c]) + lane_off;
            v[0] = ld16<3>(p);
            v[1] = ld16<3>(p + kStep);
        };
        uint32_t acc[MR][8];
#pragma unroll
        for (int r = 0; r < MR; ++r)
#pragma unroll
            for (int p = 0; p < 8; ++p) acc[r][p] = 0u;
        V4 cur[2], n1[2], n2[2];
        load(0, cur);
        if (k > 1) load(1, n1);
        for (int c = 0; c < k; ++c) {
            if (c + 2 < k) load(c + 2, n2);
            uint32_t Y[4][8];
            unpack(cur[0], Y[0]);
            unpack(cur[1], Y[0] + 4);
            bs::transpose8(Y[0]);
            times2(Y[0], Y[1]);
            times2(Y[1], Y[2]);
            times2(Y[2], Y[3]);
            const uint32_t w0 = cw[2 * c], w1 = cw[2 * c + 1];
#pragma unroll
            for (int r = 0; r < MR; ++r) add_nibble(((r < 4 ? w0 : w1) >> (8 * (r & 3))) & 15u, acc[r], Y);
            uint32_t Z[4][8];
            times2(Y[3], Z[0]);
            times2(Z[0], Z[1]);
            times2(Z[1], Z[2]);
            times2(Z[2], Z[3]);
#pragma unroll
            for (int r = 0; r < MR; ++r) add_nibble(((r < 4 ? w0 : w1) >> (8 * (r & 3) + 4)) & 15u, acc[r], Z);
            cur[0] = n1[0];
            cur[1] = n1[1];
            n1[0] = n2[0];
            n1[1] = n2[1];
        }
#pragma unroll
        for (int r = 0; r < MR; ++r) {
            if (r >= a.rows) break;
            bs::transpose8(acc[r]);
            uint8_t* q = shard_ptr<ADDR>(a, b, out_idx[r]) + lane_off;
            st16<3>(q, pack(acc[r]));
            st16<3>(q + kStep, pack(acc[r] + 4));
        }
    }
}

}  // namespace code
}  // namespace blbrs
