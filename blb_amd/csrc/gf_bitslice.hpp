// gf_bitslice.hpp -- GF(2^8) encode with the coding matrix known at compile time: bit planes
// and a fixed XOR network instead of v_perm table lookups.
//
// Multiplying a byte by a constant c is GF(2)-linear: bit p of c*x is the XOR of the bits q
// of x for which bit p of c*2^q is set (an 8x8 bit matrix per coefficient).  Encode's
// coefficients are the parity rows P_j = V[k+j] * inv(V[0:k]) of reedsolomon.go buildMatrix
// (klauspost @925cb01d6510), fixed per k -- and independent of m, since V's rows do not
// depend on it -- so for blb's shapes the whole row of bit matrices is known when the kernel
// is compiled.  Then:
//   * 8 dwords of a shard (32 bytes per lane) are bit-transposed in place (transpose8: byte
//     lane b of dword i <-> bit i of byte lane b, three SWAR stages, 4 VALU per dword pair
//     per stage = 6 VALU per dword), so dword q holds bit q of all 32 bytes -- a "plane";
//   * parity plane (j, p) = XOR of the input planes (c, q) with bit p of P_j[c]*2^q set,
//     a fixed list of terms folded three at a time with v_bitop3 (XOR3); no table operand, no
//     constant-bus move, no bit-group split;
//   * the 8 parity planes of a row are transposed back (the transpose is an involution).
// VALU per 4 bytes of every shard (one dword column): RS(6,3) 81 vs 115 with v_perm tables,
// RS(10,4) 159 vs 240, RS(12,5) 211 vs 345 (tools/bitslice_count.py).  Decode matrices
// depend on the erasure pattern and stay on the v_perm path (gf_device.hpp).
//
// The same kernels run decode networks too: rtc.hip generates a network for the rows of one
// erasure pattern at run time and compiles it with hipRTC against these headers, so the device
// parts below are RTC-clean (no standard headers).
#pragma once
#include "dev_common.hpp"

namespace blbrs {
namespace bs {

constexpr int kMaxParity = 5;  // parity rows compiled per k (blb's classes need m <= 5)

// --- compile-time field and parity rows (same construction as gf256.hpp, constexpr) -------
struct CField {
    uint8_t exp[512] = {};
    uint8_t log[256] = {};
};
constexpr CField make_field() {
    CField f{};
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        f.exp[i] = f.exp[i + 255] = static_cast<uint8_t>(x);
        f.log[x] = static_cast<uint8_t>(i);
        x <<= 1;
        if (x & 0x100) x ^= 0x11d;
    }
    f.exp[510] = f.exp[511] = f.exp[0];
    return f;
}
constexpr CField kField = make_field();
constexpr uint8_t cmul(uint8_t a, uint8_t b) {
    return (a == 0 || b == 0) ? 0 : kField.exp[kField.log[a] + kField.log[b]];
}
constexpr uint8_t cinv(uint8_t a) { return kField.exp[(255 - kField.log[a]) % 255]; }
constexpr uint8_t cpow(uint8_t a, int n) {
    return n == 0 ? 1 : a == 0 ? 0 : kField.exp[(static_cast<int>(kField.log[a]) * n) % 255];
}

template <int K>
struct ParityRows {
    uint8_t c[kMaxParity][K] = {};
};

// P_j = V[K+j] * inv(V[0:K]), V[r][c] = r^c (matrix.go vandermonde, reedsolomon.go buildMatrix).
template <int K>
constexpr ParityRows<K> make_parity_rows() {
    uint8_t t[K][2 * K] = {};
    for (int r = 0; r < K; ++r) {
        for (int c = 0; c < K; ++c) t[r][c] = cpow(static_cast<uint8_t>(r), c);
        t[r][K + r] = 1;
    }
    for (int col = 0; col < K; ++col) {  // Gauss-Jordan, as gf256.hpp invert()
        int piv = col;
        while (t[piv][col] == 0) ++piv;  // V[0:K] is invertible
        if (piv != col)
            for (int j = 0; j < 2 * K; ++j) {
                const uint8_t s = t[col][j];
                t[col][j] = t[piv][j];
                t[piv][j] = s;
            }
        const uint8_t s = cinv(t[col][col]);
        for (int j = 0; j < 2 * K; ++j) t[col][j] = cmul(t[col][j], s);
        for (int r = 0; r < K; ++r) {
            const uint8_t f = t[r][col];
            if (r == col || f == 0) continue;
            for (int j = 0; j < 2 * K; ++j) t[r][j] ^= cmul(f, t[col][j]);
        }
    }
    ParityRows<K> p{};
    for (int j = 0; j < kMaxParity; ++j)
        for (int c = 0; c < K; ++c) {
            uint8_t v = 0;
            for (int i = 0; i < K; ++i) v ^= cmul(cpow(static_cast<uint8_t>(K + j), i), t[i][K + c]);
            p.c[j][c] = v;
        }
    return p;
}

template <int K>
constexpr ParityRows<K> kParity = make_parity_rows<K>();

// The XOR network: for parity row j and output bit p, the input planes (c, q) to fold.
template <int K>
struct Terms {
    int n[kMaxParity][8] = {};
    uint8_t c[kMaxParity][8][8 * K] = {};
    uint8_t q[kMaxParity][8][8 * K] = {};
};
template <int K>
constexpr Terms<K> make_terms() {
    Terms<K> t{};
    for (int j = 0; j < kMaxParity; ++j)
        for (int c = 0; c < K; ++c)
            for (int q = 0; q < 8; ++q) {
                const uint8_t col = cmul(kParity<K>.c[j][c], static_cast<uint8_t>(1u << q));
                for (int p = 0; p < 8; ++p)
                    if ((col >> p) & 1u) {
                        const int i = t.n[j][p]++;
                        t.c[j][p][i] = static_cast<uint8_t>(c);
                        t.q[j][p][i] = static_cast<uint8_t>(q);
                    }
            }
    return t;
}
template <int K>
constexpr Terms<K> kTerms = make_terms<K>();

// The same network grouped by inputs: for parity row j, output bit p and input group g
// (inputs [G*g, G*g + G)), the planes (c, q) to fold.  Kernels that fold inputs as their loads
// arrive (G = 2: the coding kernels, one pair at a time) or one at a time (G = 1: PackTracts
// + Encode, which assembles pieces sequentially).
template <int K, int G>
struct GroupTerms {
    static constexpr int kGroups = (K + G - 1) / G;
    int n[kMaxParity][8][kGroups] = {};
    uint8_t c[kMaxParity][8][kGroups][8 * G] = {};
    uint8_t q[kMaxParity][8][kGroups][8 * G] = {};
};
template <int K, int G>
constexpr GroupTerms<K, G> make_group_terms() {
    GroupTerms<K, G> t{};
    for (int j = 0; j < kMaxParity; ++j)
        for (int c = 0; c < K; ++c)
            for (int q = 0; q < 8; ++q) {
                const uint8_t col = cmul(kParity<K>.c[j][c], static_cast<uint8_t>(1u << q));
                for (int p = 0; p < 8; ++p)
                    if ((col >> p) & 1u) {
                        const int g = c / G, i = t.n[j][p][g]++;
                        t.c[j][p][g][i] = static_cast<uint8_t>(c);
                        t.q[j][p][g][i] = static_cast<uint8_t>(q);
                    }
            }
    return t;
}
template <int K, int G>
constexpr GroupTerms<K, G> kGroupTerms = make_group_terms<K, G>();

#ifndef __HIPCC_RTC__
}  // namespace bs
}  // namespace blbrs
#include "tuning.hpp"
namespace blbrs {
namespace bs {

// Host side: true when `rows` (nrows x k, row-major) are parity rows 0..nrows-1 of k, i.e.
// a pass the compiled network computes.
template <int K>
bool is_parity_rows_k(const uint8_t* rows, int nrows) {
    if (nrows < 1 || nrows > kMaxParity) return false;
    for (int j = 0; j < nrows; ++j)
        for (int c = 0; c < K; ++c)
            if (rows[j * K + c] != kParity<K>.c[j][c]) return false;
    return true;
}
inline bool is_parity_rows(const uint8_t* rows, int nrows, int k) {
    switch (k) {
        case 3: return is_parity_rows_k<3>(rows, nrows);
        case 4: return is_parity_rows_k<4>(rows, nrows);
        case 6: return is_parity_rows_k<6>(rows, nrows);
        case 8: return is_parity_rows_k<8>(rows, nrows);
        case 10: return is_parity_rows_k<10>(rows, nrows);
        case 12: return is_parity_rows_k<12>(rows, nrows);
        default: return false;
    }
}

// Which encode passes take the network (tools/bitslice_ab.py): the shapes where
// the table multiply is VALU-bound, k + rows > `wide` (each kernel passes its own measured
// threshold).  Where the table kernel already runs at the access pattern's speed (RS(6,3)) it
// folds each input pair as its loads land and stays 2-5 % ahead of the network.
// Knob BLBRS_BITSLICE (tuning.hpp; A/B runs): 0 = never, 2 = every compiled shape.
// 0 and 2 as set; any other value is the default 1 (a stray value must not switch the compiled
// encode networks off, which only the m == 1 / m == 2 branches of use() would notice).
inline int mode() {
    const long v = tune::get(tune::kBitslice);
    return v == 0 || v == 2 ? static_cast<int>(v) : 1;
}
inline bool use(bool parity, int k, int rows, int wide) {
    if (!parity) return false;
    const int m = mode();
    return m == 2 || (m == 1 && k + rows > wide);
}
// Thresholds per kernel: rs_code_kernel (k + rows > 9 is also where it drops to U = 2), the
// fused encode+CRC tile kernel, PackTracts + Encode.
constexpr int kWideCode = 9, kWideTile = 11, kWidePack = 9;
#endif  // __HIPCC_RTC__

// --- device ----------------------------------------------------------------------------

// 8x8 bit transpose inside every byte lane of 8 dwords: afterwards bit i of byte b of d[q]
// is what bit q of byte b of d[i] was.  Stage s swaps element (i, q + s) with (i + s, q) for
// q with bit s clear; v_bfi_b32 merges, so each pair costs 2 shifts + 2 bfi.
template <int S>
__device__ __forceinline__ void transpose_stage(uint32_t* d) {
    constexpr uint32_t m = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        const int i = (h / S) * 2 * S + h % S;  // the four rows with bit S clear
        const uint32_t a = d[i], b = d[i + S];
        d[i] = (a & m) | ((b << S) & ~m);
        d[i + S] = ((a >> S) & m) | (b & ~m);
    }
}
__device__ __forceinline__ void transpose8(uint32_t* d) {
    transpose_stage<4>(d);
    transpose_stage<2>(d);
    transpose_stage<1>(d);
}

// XOR of terms [J, n) of parity row R, output bit P, three at a time.
template <int K, int R, int P, int J>
__device__ __forceinline__ uint32_t fold(const uint32_t (&x)[K][8]) {
    constexpr int n = kTerms<K>.n[R][P];
    if constexpr (J >= n) {
        return 0u;
    } else if constexpr (J + 1 == n) {
        constexpr int c0 = kTerms<K>.c[R][P][J], q0 = kTerms<K>.q[R][P][J];
        return x[c0][q0];
    } else if constexpr (J + 2 == n) {
        constexpr int c0 = kTerms<K>.c[R][P][J], q0 = kTerms<K>.q[R][P][J];
        constexpr int c1 = kTerms<K>.c[R][P][J + 1], q1 = kTerms<K>.q[R][P][J + 1];
        return x[c0][q0] ^ x[c1][q1];
    } else {
        constexpr int c0 = kTerms<K>.c[R][P][J], q0 = kTerms<K>.q[R][P][J];
        constexpr int c1 = kTerms<K>.c[R][P][J + 1], q1 = kTerms<K>.q[R][P][J + 1];
        return dev::xor3(x[c0][q0], x[c1][q1], fold<K, R, P, J + 2>(x));
    }
}

template <int K, int R, int P>
__device__ __forceinline__ void row_planes(const uint32_t (&x)[K][8], uint32_t* out) {
    if constexpr (P < 8) {
        out[P] = fold<K, R, P, 0>(x);
        row_planes<K, R, P + 1>(x, out);
    }
}

// Parity rows 0..MR-1 (x transposed in place by the caller), rows in byte form.
template <int K, int MR, int R = 0>
__device__ __forceinline__ void parity_rows(const uint32_t (&x)[K][8], uint32_t (&out)[MR][8]) {
    if constexpr (R < MR) {
        row_planes<K, R, 0>(x, out[R]);
        transpose8(out[R]);
        parity_rows<K, MR, R + 1>(x, out);
    }
}

// The network the coding kernel runs (rs_code_kernel's NET parameter): NET::rows<MR>(x, out)
// takes every input's planes (x, transposed by the caller) and returns rows 0..MR-1 in byte
// form.  EncodeNet<K> is the encode matrix compiled into the library; rtc.hip generates the
// same interface for decode rows.
// NET::each<MR>(x, f) does the same one row at a time, calling f(r, row) as soon as row r is in
// byte form, so a store-only caller keeps 8 output registers live instead of 8 * MR.
template <int K, int R, int MR, class F>
__device__ __forceinline__ void parity_each(const uint32_t (&x)[K][8], F& f) {
    if constexpr (R < MR) {
        uint32_t o[8];
        row_planes<K, R, 0>(x, o);
        transpose8(o);
        f(R, o);
        parity_each<K, R + 1, MR>(x, f);
    }
}

template <int K>
struct EncodeNet {
    template <int MR>
    __device__ static __forceinline__ void rows(const uint32_t (&x)[K][8], uint32_t (&out)[MR][8]) {
        parity_rows<K, MR>(x, out);
    }
    template <int MR, class F>
    __device__ static __forceinline__ void each(const uint32_t (&x)[K][8], F& f) {
        parity_each<K, 0, MR>(x, f);
    }
};

// rs_code_kernel's call into its NET (void: the table path, never called).
template <class NET, int K, int MR>
struct NetRows {
    __device__ static __forceinline__ void run(const uint32_t (&x)[K][8], uint32_t (&out)[MR][8]) {
        NET::template rows<MR>(x, out);
    }
    template <class F>
    __device__ static __forceinline__ void each(const uint32_t (&x)[K][8], F& f) {
        NET::template each<MR>(x, f);
    }
};
template <int K, int MR>
struct NetRows<void, K, MR> {
    __device__ static __forceinline__ void run(const uint32_t (&)[K][8], uint32_t (&)[MR][8]) {}
    template <class F>
    __device__ static __forceinline__ void each(const uint32_t (&)[K][8], F&) {}
};

// acc ^ the terms [J, n) of input group GI for parity row R, output bit P (x: every input's
// planes, those of group GI transposed).  Every index is bound to a constexpr int first:
// used directly as a subscript, a member of the constexpr table may be read from memory at
// run time, and x then lives in scratch.
template <int K, int G, int R, int P, int GI, int J>
__device__ __forceinline__ uint32_t fold_group(const uint32_t (&x)[K][8], uint32_t acc) {
    constexpr int n = kGroupTerms<K, G>.n[R][P][GI];
    if constexpr (J >= n) {
        return acc;
    } else if constexpr (J + 1 == n) {
        constexpr int c0 = kGroupTerms<K, G>.c[R][P][GI][J], q0 = kGroupTerms<K, G>.q[R][P][GI][J];
        return acc ^ x[c0][q0];
    } else {
        constexpr int c0 = kGroupTerms<K, G>.c[R][P][GI][J], q0 = kGroupTerms<K, G>.q[R][P][GI][J];
        constexpr int c1 = kGroupTerms<K, G>.c[R][P][GI][J + 1], q1 = kGroupTerms<K, G>.q[R][P][GI][J + 1];
        return fold_group<K, G, R, P, GI, J + 2>(x, dev::xor3(acc, x[c0][q0], x[c1][q1]));
    }
}

// Input group GI's contribution to the planes of parity rows R.. < MR (acc in plane form).
template <int K, int G, int MR, int GI, int R = 0, int P = 0>
__device__ __forceinline__ void add_group(const uint32_t (&x)[K][8], uint32_t (&acc)[MR][8]) {
    if constexpr (R < MR) {
        if constexpr (P < 8) {
            acc[R][P] = fold_group<K, G, R, P, GI, 0>(x, acc[R][P]);
            add_group<K, G, MR, GI, R, P + 1>(x, acc);
        } else {
            add_group<K, G, MR, GI, R + 1, 0>(x, acc);
        }
    }
}

// One input C at a time (G = 1 terms; x = input C's planes only).
template <int K, int R, int P, int C, int J>
__device__ __forceinline__ uint32_t fold_one(const uint32_t (&x)[8], uint32_t acc) {
    constexpr int n = kGroupTerms<K, 1>.n[R][P][C];
    if constexpr (J >= n) {
        return acc;
    } else if constexpr (J + 1 == n) {
        constexpr int q0 = kGroupTerms<K, 1>.q[R][P][C][J];
        return acc ^ x[q0];
    } else {
        constexpr int q0 = kGroupTerms<K, 1>.q[R][P][C][J], q1 = kGroupTerms<K, 1>.q[R][P][C][J + 1];
        return fold_one<K, R, P, C, J + 2>(x, dev::xor3(acc, x[q0], x[q1]));
    }
}
template <int K, int MR, int C, int R = 0, int P = 0>
__device__ __forceinline__ void add_one(const uint32_t (&x)[8], uint32_t (&acc)[MR][8]) {
    if constexpr (R < MR) {
        if constexpr (P < 8) {
            acc[R][P] = fold_one<K, R, P, C, 0>(x, acc[R][P]);
            add_one<K, MR, C, R, P + 1>(x, acc);
        } else {
            add_one<K, MR, C, R + 1, 0>(x, acc);
        }
    }
}

// Parity rows 0..MR-1 of 8 dwords per input, folding input pairs in order so that the work
// on a pair can start as soon as its loads land: x holds the inputs in byte form and is
// transposed in place pair by pair; acc gets the rows in byte form.
template <int K, int MR, int GI = 0>
__device__ __forceinline__ void parity_rows_by_pairs(uint32_t (&x)[K][8], uint32_t (&acc)[MR][8]) {
    constexpr int kPairs = (K + 1) / 2;
    if constexpr (GI == 0) {
#pragma unroll
        for (int r = 0; r < MR; ++r)
#pragma unroll
            for (int d = 0; d < 8; ++d) acc[r][d] = 0u;
    }
    if constexpr (GI < kPairs) {
        transpose8(x[2 * GI]);
        if constexpr (2 * GI + 1 < K) transpose8(x[2 * GI + 1]);
        add_group<K, 2, MR, GI>(x, acc);
        parity_rows_by_pairs<K, MR, GI + 1>(x, acc);
    } else {
#pragma unroll
        for (int r = 0; r < MR; ++r) transpose8(acc[r]);
    }
}

}  // namespace bs
}  // namespace blbrs
