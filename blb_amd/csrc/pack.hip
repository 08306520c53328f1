// pack.hip -- device PackTracts (see pack.hpp).
//
// One workgroup per 64 KiB destination tile, each XCD streaming a contiguous eighth of the
// tiles, every chunk of the tile in flight at once.  The workgroup finds the first extent of its
// piece that ends inside or after the tile (binary search over the sorted extents), then
// walks the tile as a list of uniform regions: "copy from extent e" or "zero".  Inside a
// region the destination is written as 16-byte aligned dwordx4 stores; the source, which
// can have any alignment (tract lengths are arbitrary, so are offsets inside a source), is
// read as ALIGNED 16-byte blocks and realigned with v_alignbyte_b32.  An aligned block that
// holds at least one wanted byte never crosses a page the buffer does not own, so no read
// leaves the source buffer's pages.  Region heads/tails (< 16 bytes) go byte by byte.
#include "pack.hpp"

namespace blbrs {
namespace {

typedef uint32_t V4 __attribute__((ext_vector_type(4)));

struct PackArgs {
    uint8_t* dst;
    uint64_t dst_stride, piece_len;
    uint32_t npieces, tiles_per_piece;
    const uint64_t* table;
    uint32_t per_group;    // pieces per group: piece p at dst + (p / per_group) * group_stride
    uint64_t group_stride; //   + (p % per_group) * dst_stride
};

// Lane i receives lane (i + 1) mod 64's dword (DPP wave_rol:1, no LDS).
__device__ __forceinline__ uint32_t rol1(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x134, 0xF, 0xF, false));
}
__device__ __forceinline__ V4 rol1(const V4& v) { return V4{rol1(v.x), rol1(v.y), rol1(v.z), rol1(v.w)}; }

// out = bytes [s, s+16) of the 32-byte window a||b, s = 4q + r (q wave-uniform).
__device__ __forceinline__ V4 funnel(const V4& a, const V4& b, uint32_t q, uint32_t r) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    V4 o;
    switch (q) {
        case 0:
            o = V4{__builtin_amdgcn_alignbyte(w[1], w[0], r), __builtin_amdgcn_alignbyte(w[2], w[1], r),
                   __builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r)};
            break;
        case 1:
            o = V4{__builtin_amdgcn_alignbyte(w[2], w[1], r), __builtin_amdgcn_alignbyte(w[3], w[2], r),
                   __builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r)};
            break;
        case 2:
            o = V4{__builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r),
                   __builtin_amdgcn_alignbyte(w[5], w[4], r), __builtin_amdgcn_alignbyte(w[6], w[5], r)};
            break;
        default:
            o = V4{__builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r),
                   __builtin_amdgcn_alignbyte(w[6], w[5], r), __builtin_amdgcn_alignbyte(w[7], w[6], r)};
            break;
    }
    return o;
}

// Copy n bytes src -> dst with the whole workgroup (n, src, dst uniform).  Chunk i (16
// destination bytes) is lane i % 256's, kUnr chunks per lane in flight (the whole 64 KiB tile).
// Loads stay cached: nontemporal loads were 3-28 % slower box to box (profiles/r03/pack/).  A
// misaligned source is read as aligned blocks: lane i loads block i and takes block i + 1 from
// the next lane (DPP) -- one load per chunk -- except lane 63 of each wave, whose next block is
// another wave's and is loaded.  (Round 2 loaded both blocks in every lane: 15.8 vs 13.6 ms.)
constexpr int kUnr = 16;

__device__ void copy_region(uint8_t* dst, const uint8_t* src, uint64_t n) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const uint64_t head = ((16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u) < n
                              ? ((16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u)
                              : n;
    if (tid < head) dst[tid] = src[tid];
    const uint64_t nb = (n - head) >> 4, tail = (n - head) & 15u;
    V4* d = reinterpret_cast<V4*>(dst + head);
    const uint8_t* s = src + head;
    const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(s) & 15u);
    const V4* sa = reinterpret_cast<const V4*>(s - mis);  // aligned block holding s[0]
    if (mis == 0) {
        for (uint64_t c = tid; c < nb; c += kUnr * kPackThreads) {
            V4 v[kUnr];
#pragma unroll
            for (int u = 0; u < kUnr; ++u)
                if (c + u * kPackThreads < nb) v[u] = sa[c + u * kPackThreads];
#pragma unroll
            for (int u = 0; u < kUnr; ++u)
                if (c + u * kPackThreads < nb) __builtin_nontemporal_store(v[u], d + c + u * kPackThreads);
        }
    } else {
        const uint32_t q = mis >> 2, r = mis & 3u;
        // Every block up to nb holds wanted bytes (mis > 0: the last wanted byte lies in block
        // nb), so no read leaves them.
        for (uint64_t c = tid; c < nb + (nb > 0 ? 1 : 0); c += kUnr * kPackThreads) {
            V4 v[kUnr], h[kUnr];
#pragma unroll
            for (int u = 0; u < kUnr; ++u) v[u] = h[u] = V4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int u = 0; u < kUnr; ++u) {
                const uint64_t i = c + u * kPackThreads;
                if (i <= nb) v[u] = sa[i];
                if (lane == 63u && i < nb) h[u] = sa[i + 1];
            }
#pragma unroll
            for (int u = 0; u < kUnr; ++u) {
                const uint64_t i = c + u * kPackThreads;
                const V4 nx = rol1(v[u]);
                const V4 hb = lane != 63u ? nx : h[u];
                if (i < nb) __builtin_nontemporal_store(funnel(v[u], hb, q, r), d + i);
            }
        }
    }
    if (tid < tail) {
        const uint64_t o = head + (nb << 4) + tid;
        dst[o] = src[o];
    }
}

__device__ void zero_region(uint8_t* dst, uint64_t n) {
    const uint32_t tid = threadIdx.x;
    const uint64_t a = (16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u;
    const uint64_t head = a < n ? a : n;
    if (tid < head) dst[tid] = 0;
    const uint64_t nb = (n - head) >> 4, tail = (n - head) & 15u;
    V4* d = reinterpret_cast<V4*>(dst + head);
    for (uint64_t c = tid; c < nb; c += kPackThreads) __builtin_nontemporal_store(V4{0u, 0u, 0u, 0u}, d + c);
    if (tid < tail) dst[head + (nb << 4) + tid] = 0;
}

// Each XCD takes a contiguous eighth of the tiles (blocks are dealt round-robin over the 8
// XCDs), so the workgroups resident on one XCD stream neighbouring tiles.
__global__ __launch_bounds__(kPackThreads) void pack_kernel(PackArgs a) {
    uint32_t t = blockIdx.x;
    t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
    if (t >= a.npieces * a.tiles_per_piece) return;
    const uint32_t piece = t / a.tiles_per_piece;
    const uint64_t t0 = static_cast<uint64_t>(t % a.tiles_per_piece) * kPackTile;
    const uint64_t t1 = t0 + kPackTile < a.piece_len ? t0 + kPackTile : a.piece_len;
    const uint64_t* ex = a.table + a.npieces + 1;
    uint64_t lo = a.table[piece];
    const uint64_t hi = a.table[piece + 1];
    // First extent whose end is past t0 (ends are non-decreasing inside a piece).
    for (uint64_t n = hi - lo; n > 0;) {
        const uint64_t half = n >> 1, m = lo + half;
        if (ex[4 * m + 1] + ex[4 * m + 2] <= t0) {
            lo = m + 1;
            n -= half + 1;
        } else {
            n = half;
        }
    }
    uint8_t* d = a.dst + static_cast<uint64_t>(piece / a.per_group) * a.group_stride +
                 static_cast<uint64_t>(piece % a.per_group) * a.dst_stride;
    uint64_t cur = t0;
    for (uint64_t e = lo; cur < t1;) {
        const uint64_t off = e < hi ? ex[4 * e + 1] : t1;
        if (off <= cur) {  // inside extent e
            const uint64_t end = off + ex[4 * e + 2] < t1 ? off + ex[4 * e + 2] : t1;
            const uint8_t* src = reinterpret_cast<const uint8_t*>(ex[4 * e]);
            copy_region(d + cur, src + (cur - off), end - cur);
            cur = end > cur ? end : cur;
            ++e;
        } else {  // hole or pad up to the next extent / tile end
            const uint64_t end = off < t1 ? off : t1;
            zero_region(d + cur, end - cur);
            cur = end;
        }
    }
}

}  // namespace

hipError_t pack_pieces(uint8_t* dst, uint64_t dst_stride, uint64_t npieces, uint64_t piece_len,
                       const uint64_t* table_dev, hipStream_t stream, uint32_t per_group, uint64_t group_stride) {
    if (npieces == 0 || piece_len == 0) return hipSuccess;
    const uint64_t tpp = (piece_len + kPackTile - 1) / kPackTile;
    if (npieces > 0xFFFFFFFFull || tpp * npieces > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if (per_group == 0) {
        per_group = 1;
        group_stride = dst_stride;
    }
    PackArgs a{dst, dst_stride, piece_len, static_cast<uint32_t>(npieces), static_cast<uint32_t>(tpp), table_dev,
               per_group, group_stride};
    const uint64_t grid = (tpp * npieces + 7) & ~uint64_t{7};  // a multiple of 8 blocks; the extra ones exit
    hipLaunchKernelGGL(pack_kernel, dim3(static_cast<unsigned>(grid)), dim3(kPackThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace blbrs
