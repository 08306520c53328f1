// gf256.hpp -- host-side GF(2^8) field and coding-matrix construction for the engine.
//
// Field and matrices follow klauspost/reedsolomon @925cb01d6510 (go.mod:20), the library
// blb calls at internal/tractserver/store.go:1022 and client/blb/reconstruct.go:166:
//   polynomial 0x11D, generator 2 (galois.go); V[r][c] = r^c (matrix.go vandermonde);
//   M = V * inv(V[0:k]) (reedsolomon.go buildMatrix); decode = inv(M[first k present rows]).
// These are tiny k x k computations done once per (k, m) / erasure pattern and cached by
// the caller (the GPU never sees anything but the per-coefficient lookup tables built by
// perm_tables()).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace blbrs {

struct GF {
    uint8_t exp[512];
    uint8_t log[256];
    GF() {
        unsigned x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = exp[i + 255] = static_cast<uint8_t>(x);
            log[x] = static_cast<uint8_t>(i);
            x <<= 1;
            if (x & 0x100) x ^= 0x11d;
        }
        exp[510] = exp[511] = exp[0];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        return (a == 0 || b == 0) ? 0 : exp[log[a] + log[b]];
    }
    uint8_t inv(uint8_t a) const { return exp[(255 - log[a]) % 255]; }
    // galExp(a, n): 1 for n == 0, 0 for a == 0, else a^n.
    uint8_t pow(uint8_t a, int n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(static_cast<int>(log[a]) * n) % 255];
    }
};

inline const GF& gf() {
    static const GF g;
    return g;
}

using Mat = std::vector<uint8_t>;  // row-major

// Gauss-Jordan inverse of an n x n matrix; false when singular.
inline bool invert(const Mat& a, int n, Mat& out) {
    const GF& g = gf();
    const int w = 2 * n;
    Mat t(static_cast<size_t>(n) * w, 0);
    for (int r = 0; r < n; ++r) {
        std::memcpy(&t[r * w], &a[r * n], n);
        t[r * w + n + r] = 1;
    }
    for (int col = 0; col < n; ++col) {
        int piv = col;
        while (piv < n && t[piv * w + col] == 0) ++piv;
        if (piv == n) return false;
        if (piv != col)
            for (int j = 0; j < w; ++j) std::swap(t[col * w + j], t[piv * w + j]);
        const uint8_t s = g.inv(t[col * w + col]);
        for (int j = 0; j < w; ++j) t[col * w + j] = g.mul(t[col * w + j], s);
        for (int r = 0; r < n; ++r) {
            const uint8_t f = t[r * w + col];
            if (r == col || f == 0) continue;
            for (int j = 0; j < w; ++j) t[r * w + j] ^= g.mul(f, t[col * w + j]);
        }
    }
    out.assign(static_cast<size_t>(n) * n, 0);
    for (int r = 0; r < n; ++r) std::memcpy(&out[r * n], &t[r * w + n], n);
    return true;
}

// (ar x ac) * (ac x bc)
inline Mat matmul(const Mat& a, int ar, int ac, const Mat& b, int bc) {
    const GF& g = gf();
    Mat o(static_cast<size_t>(ar) * bc, 0);
    for (int r = 0; r < ar; ++r)
        for (int c = 0; c < bc; ++c) {
            uint8_t v = 0;
            for (int i = 0; i < ac; ++i) v ^= g.mul(a[r * ac + i], b[i * bc + c]);
            o[r * bc + c] = v;
        }
    return o;
}

// reedsolomon.go buildMatrix(k, k+m): systematic (k+m) x k encoding matrix.
inline bool build_matrix(int k, int m, Mat& out) {
    const GF& g = gf();
    const int n = k + m;
    Mat v(static_cast<size_t>(n) * k);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c) v[r * k + c] = g.pow(static_cast<uint8_t>(r), c);
    Mat top(v.begin(), v.begin() + static_cast<size_t>(k) * k), top_inv;
    if (!invert(top, k, top_inv)) return false;
    out = matmul(v, n, k, top_inv, k);
    return true;
}

// Per-coefficient v_perm_b32 lookup tables consumed by the HIP kernels.
// A byte x splits into bit groups g0 = x[2:0], g1 = x[5:3], g2 = x[7:6]; since GF
// multiplication distributes over XOR, c*x = c*g0 ^ c*(g1<<3) ^ c*(g2<<6).  Each group's
// products fit in <= 8 bytes, i.e. one v_perm_b32 byte-select:
//   word0/1 = c*{0..7}        (lo dword = entries 0..3, hi dword = entries 4..7)
//   word2/3 = c*({0..7} << 3)
//   word4   = c*({0..3} << 6)
constexpr int kWordsPerCoef = 5;

inline void perm_table(uint8_t c, uint32_t out[kWordsPerCoef]) {
    const GF& g = gf();
    uint8_t b[20];
    for (int i = 0; i < 8; ++i) b[i] = g.mul(c, static_cast<uint8_t>(i));
    for (int i = 0; i < 8; ++i) b[8 + i] = g.mul(c, static_cast<uint8_t>(i << 3));
    for (int i = 0; i < 4; ++i) b[16 + i] = g.mul(c, static_cast<uint8_t>(i << 6));
    for (int w = 0; w < kWordsPerCoef; ++w)
        out[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) |
                 (static_cast<uint32_t>(b[4 * w + 3]) << 24);
}

// rows: nrows x k coefficient matrix -> nrows*k*5 words, layout [row][input][word].
inline std::vector<uint32_t> perm_tables(const Mat& rows, int nrows, int k) {
    std::vector<uint32_t> t(static_cast<size_t>(nrows) * k * kWordsPerCoef);
    for (int r = 0; r < nrows; ++r)
        for (int c = 0; c < k; ++c)
            perm_table(rows[r * k + c], &t[(static_cast<size_t>(r) * k + c) * kWordsPerCoef]);
    return t;
}

}  // namespace blbrs
