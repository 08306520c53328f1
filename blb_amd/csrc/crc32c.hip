// crc32c.hip -- CRC-32C (Castagnoli) of shard blocks on gfx950 (see crc32c.hpp).
//
// CRC is linear over GF(2).  With raw(M) = the register after feeding M into a zero
// register (no init, no final xor):
//     raw(A || B) = S_{|B|} raw(A)  ^  raw(B)          S_n = "feed n zero bytes", a 32x32
//     crc(M)      = ~( S_{|M|} 0xFFFFFFFF ^ raw(M) )   GF(2) matrix (host-precomputed).
// Kernel 1 (one workgroup per <= 64 KiB segment): the segment is staged in LDS behind a
// zero prefix so that 256 lanes each own exactly L = C*Lc bytes (leading zeros do not
// change raw).  Each lane runs C = 4 independent slicing-by-4 chains over its C adjacent
// Lc-byte sub-chunks (4x the LDS-latency tolerance of one chain), with the four 1 KiB
// tables in LDS and one pad dword per lane region so every chain read hits 64 distinct
// banks.  Chains fold with S_{3Lc}, S_{2Lc}, S_{Lc}; lanes fold pairwise with S_L, S_2L,
// ..., S_128L -- shuffles inside a wave, LDS across the four waves.
// Kernel 2 (one lane per block): folds the block's segments with S_SEG (Horner) and applies
// the init term.  CRC is computed byte-serially per lane, so this is LDS/VALU work, not
// a streaming HBM kernel; it runs beside the coding kernel on the data it just wrote.
#include "crc32c.hpp"

#include <map>
#include <mutex>
#include <vector>

namespace blbrs {
namespace {

constexpr int kThreads = 256;
constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli
constexpr int kPow2 = 48;                // S_{2^i}, i < 48

// Device constants for one (L, SEG) configuration.
struct CrcConsts {
    uint32_t table[4][256];     // slicing-by-4 tables
    uint32_t chain[3][32];      // S_{(3-j) * Lc}: chain j -> end of the lane's region
    uint32_t lvl[8][32];        // S_{L * 2^j}, columns
    uint32_t seg[32];           // S_SEG
    uint32_t pow2[kPow2][32];   // S_{2^i}
};

using cu32 = const uint32_t __attribute__((address_space(4)))*;
__device__ __forceinline__ cu32 as_const(const uint32_t* p) { return (cu32)(uintptr_t)p; }

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

struct SegArgs {
    const uint8_t* data;
    uint64_t stride, len, block, seg;
    uint32_t nblocks, segs_per_block;
    const CrcConsts* c;
    uint32_t* raw;                        // [batch][nblocks][segs_per_block]
};

constexpr int kChains = 4;                        // independent CRC chains per lane
constexpr uint32_t kChainDw = 16;                 // dwords per chain (Lc = 64 bytes)
constexpr uint32_t kLaneDw = kChains * kChainDw;  // 64 dwords = L = 256 bytes per lane
constexpr uint32_t kLanePitch = kLaneDw + 1;      // +1 pad dword: conflict-free chain reads
constexpr uint32_t kSegMax = kThreads * kLaneDw * 4;  // 64 KiB
constexpr size_t kLdsBytes = (1024 + kThreads * kLanePitch + 4) * 4;

__device__ __forceinline__ uint32_t lds_dw(uint32_t v4) { return (v4 / kLaneDw) * kLanePitch + v4 % kLaneDw; }

__global__ __launch_bounds__(kThreads) void crc_segment_kernel(SegArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    uint32_t* tab = lds;                          // 4 x 256
    uint32_t* buf = lds + 1024;                   // 256 lane regions of kLanePitch dwords
    uint32_t* wave_v = buf + kThreads * kLanePitch;
    const uint32_t tid = threadIdx.x;

    const uint32_t g = blockIdx.x;
    const uint32_t s = g % a.segs_per_block;
    const uint32_t blk = (g / a.segs_per_block) % a.nblocks;
    const uint64_t b = g / (static_cast<uint64_t>(a.segs_per_block) * a.nblocks);
    const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;
    const uint64_t blk_end = blk_start + a.block < a.len ? blk_start + a.block : a.len;
    const uint64_t start = blk_start + static_cast<uint64_t>(s) * a.seg;
    if (start >= blk_end) {
        if (tid == 0) a.raw[g] = 0u;
        return;
    }
    const uint32_t seglen = static_cast<uint32_t>(blk_end - start < a.seg ? blk_end - start : a.seg);
    const uint32_t pad = kSegMax - seglen;        // virtual zero prefix
    const uint8_t* src = a.data + b * a.stride + start;

    for (uint32_t i = tid; i < 1024; i += kThreads) tab[i] = a.c->table[i >> 8][i & 255];
    for (uint32_t v4 = tid; v4 < (pad + 3) / 4; v4 += kThreads) buf[lds_dw(v4)] = 0u;
    if ((reinterpret_cast<uintptr_t>(src) & 3u) == 0 && (seglen & 3u) == 0) {
        // 16 loads in flight per lane before any LDS store (a plain loop waits on each).
        const uint32_t* src32 = reinterpret_cast<const uint32_t*>(src);
        const uint32_t nd = seglen / 4, base = pad / 4;
        for (uint32_t i0 = tid; i0 < nd; i0 += kThreads * 16) {
            uint32_t v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint32_t i = i0 + u * kThreads;
                v[u] = i < nd ? __builtin_nontemporal_load(src32 + i) : 0u;
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint32_t i = i0 + u * kThreads;
                if (i < nd) buf[lds_dw(base + i)] = v[u];
            }
        }
    } else {
        __syncthreads();  // the zeroed dword holding the prefix's last bytes is shared
        uint8_t* buf8 = reinterpret_cast<uint8_t*>(buf);
        for (uint32_t i = tid; i < seglen; i += kThreads) {
            const uint32_t v = pad + i;
            buf8[lds_dw(v / 4) * 4 + (v & 3u)] = src[i];
        }
    }
    __syncthreads();

    // C independent chains per lane (slicing-by-4; leading virtual zeros keep raw 0).
    uint32_t c[kChains] = {0u, 0u, 0u, 0u};
    const uint32_t* mine = buf + tid * kLanePitch;
#pragma unroll 4
    for (uint32_t w = 0; w < kChainDw; ++w) {
#pragma unroll
        for (int j = 0; j < kChains; ++j) {
            uint32_t x = c[j] ^ mine[j * kChainDw + w];
            c[j] = tab[768 + (x & 255u)] ^ tab[512 + ((x >> 8) & 255u)] ^ tab[256 + ((x >> 16) & 255u)] ^ tab[x >> 24];
        }
    }
    const cu32 chain = as_const(&a.c->chain[0][0]);
    uint32_t r = c[3] ^ apply(chain, c[0]);
    r ^= apply(chain + 32, c[1]);
    r ^= apply(chain + 64, c[2]);

    // Fold lanes: within a wave (6 levels), then the four waves (2 levels).
    const uint32_t lane = tid & 63u;
    const cu32 lvl = as_const(&a.c->lvl[0][0]);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t other = __shfl_down(r, 1u << j, 64);
        if ((lane & ((2u << j) - 1u)) == 0) r = apply(lvl + 32 * j, r) ^ other;
    }
    if (lane == 0) wave_v[tid >> 6] = r;
    __syncthreads();
    if (tid == 0) {
        const uint32_t v01 = apply(lvl + 32 * 6, wave_v[0]) ^ wave_v[1];
        const uint32_t v23 = apply(lvl + 32 * 6, wave_v[2]) ^ wave_v[3];
        a.raw[g] = apply(lvl + 32 * 7, v01) ^ v23;
    }
}

__device__ uint32_t shift_n(const CrcConsts* c, uint32_t r, uint64_t n) {
    const cu32 p = as_const(&c->pow2[0][0]);
    for (int i = 0; i < kPow2 && n; ++i, n >>= 1)
        if (n & 1u) r = apply(p + 32 * i, r);
    return r;
}

__global__ __launch_bounds__(kThreads) void crc_combine_kernel(SegArgs a, uint64_t total_blocks, uint32_t* out) {
    const uint64_t id = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    if (id >= total_blocks) return;
    const uint32_t blk = static_cast<uint32_t>(id % a.nblocks);
    const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;
    const uint64_t blk_len = (blk_start + a.block < a.len ? blk_start + a.block : a.len) - blk_start;
    const uint32_t nseg = static_cast<uint32_t>((blk_len + a.seg - 1) / a.seg);
    const uint32_t* raw = a.raw + id * a.segs_per_block;
    const cu32 segm = as_const(a.c->seg);
    uint32_t acc = raw[0];
    for (uint32_t s = 1; s < nseg; ++s) {
        const uint64_t sl = s + 1 < nseg ? a.seg : blk_len - static_cast<uint64_t>(s) * a.seg;
        acc = (sl == a.seg ? apply(segm, acc) : shift_n(a.c, acc, sl)) ^ raw[s];
    }
    out[id] = ~(shift_n(a.c, 0xFFFFFFFFu, blk_len) ^ acc);
}

// ---- host-side constants ----

struct Mat32 {
    uint32_t col[32];
};

uint32_t mat_apply(const Mat32& m, uint32_t r) {
    uint32_t o = 0;
    for (int i = 0; i < 32; ++i)
        if ((r >> i) & 1u) o ^= m.col[i];
    return o;
}

Mat32 mat_mul(const Mat32& a, const Mat32& b) {  // a after b
    Mat32 o;
    for (int i = 0; i < 32; ++i) o.col[i] = mat_apply(a, b.col[i]);
    return o;
}

Mat32 shift_one_byte(const uint32_t* t0) {
    Mat32 m;
    for (int i = 0; i < 32; ++i) {
        const uint32_t r = 1u << i;
        m.col[i] = t0[r & 255u] ^ (r >> 8);
    }
    return m;
}

Mat32 mat_pow(const Mat32* pow2, uint64_t n) {
    Mat32 r;
    for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
    for (int i = 0; i < kPow2 && n; ++i, n >>= 1)
        if (n & 1u) r = mat_mul(pow2[i], r);
    return r;
}

void build_consts(uint64_t seg, CrcConsts* c) {
    const uint32_t L = kLaneDw * 4, Lc = kChainDw * 4;
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t v = i;
        for (int j = 0; j < 8; ++j) v = (v & 1u) ? (v >> 1) ^ kPoly : v >> 1;
        c->table[0][i] = v;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i) c->table[k][i] = (c->table[k - 1][i] >> 8) ^ c->table[0][c->table[k - 1][i] & 255u];
    Mat32 p[kPow2];
    p[0] = shift_one_byte(c->table[0]);
    for (int i = 1; i < kPow2; ++i) p[i] = mat_mul(p[i - 1], p[i - 1]);
    for (int i = 0; i < kPow2; ++i)
        for (int j = 0; j < 32; ++j) c->pow2[i][j] = p[i].col[j];
    for (int j = 0; j < 3; ++j) {
        const Mat32 m = mat_pow(p, static_cast<uint64_t>(3 - j) * Lc);
        for (int i = 0; i < 32; ++i) c->chain[j][i] = m.col[i];
    }
    for (int l = 0; l < 8; ++l) {
        const Mat32 m = mat_pow(p, static_cast<uint64_t>(L) << l);
        for (int j = 0; j < 32; ++j) c->lvl[l][j] = m.col[j];
    }
    const Mat32 ms = mat_pow(p, seg);
    for (int j = 0; j < 32; ++j) c->seg[j] = ms.col[j];
}

std::mutex g_mu;
std::map<std::pair<int, uint64_t>, CrcConsts*> g_consts;  // device copies, process lifetime

hipError_t consts_for(uint64_t seg, const CrcConsts** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(g_mu);
    auto& slot = g_consts[{dev, seg}];
    if (!slot) {
        CrcConsts host;
        build_consts(seg, &host);
        CrcConsts* d = nullptr;
        if ((e = hipMalloc(&d, sizeof(CrcConsts))) != hipSuccess) return e;
        if ((e = hipMemcpy(d, &host, sizeof(CrcConsts), hipMemcpyHostToDevice)) != hipSuccess) {
            (void)hipFree(d);
            return e;
        }
        slot = d;
    }
    *out = slot;
    return hipSuccess;
}

}  // namespace

hipError_t crc32c_blocks(const uint8_t* data, uint64_t stride, uint64_t batch, uint64_t len, uint64_t block,
                         uint32_t* out, hipStream_t stream) {
    if (batch == 0 || len == 0) return hipSuccess;
    if (block == 0 || !data || !out) return hipErrorInvalidValue;
    if (block > len) block = len;
    const uint64_t seg = block < kSegMax ? block : kSegMax;
    const CrcConsts* c = nullptr;
    hipError_t e = consts_for(seg, &c);
    if (e != hipSuccess) return e;
    SegArgs a{};
    a.data = data;
    a.stride = stride;
    a.len = len;
    a.block = block;
    a.seg = seg;
    a.nblocks = static_cast<uint32_t>((len + block - 1) / block);
    a.segs_per_block = static_cast<uint32_t>((block + seg - 1) / seg);
    a.c = c;
    const uint64_t total_blocks = batch * a.nblocks;
    const uint64_t total_segs = total_blocks * a.segs_per_block;
    if (total_segs > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if ((e = hipMallocAsync(reinterpret_cast<void**>(&a.raw), total_segs * 4, stream)) != hipSuccess) return e;
    hipLaunchKernelGGL(crc_segment_kernel, dim3(static_cast<unsigned>(total_segs)), dim3(kThreads), kLdsBytes, stream,
                       a);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(crc_combine_kernel, dim3(static_cast<unsigned>((total_blocks + kThreads - 1) / kThreads)),
                           dim3(kThreads), 0, stream, a, total_blocks, out);
        e = hipGetLastError();
    }
    hipError_t f = hipFreeAsync(a.raw, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
