// pack_encode.hip -- PackTracts fused with Encode (see pack.hpp).
//
// The curator's RS transition packs tracts into data pieces (encPack -> Store.PackTracts,
// internal/curator/pack_tracts.go:244-275, internal/tractserver/store.go:922-994) and then
// encodes them (encEncode -> Store.RSEncode, pack_tracts.go:277-292).  Run as two device
// passes, the encode re-reads all k*S bytes the pack has just written.  Here one workgroup
// owns one column tile (4 KiB * U) of one stripe: it assembles the tile of each of the k data
// pieces from the extent table straight into registers, stores it (the packed piece), and
// multiplies the same registers into the m parity rows -- HBM traffic = tract bytes read +
// k*S + m*S written.
//
// Per (tile, piece) the extent layout is uniform over the workgroup:
//  * ZERO  -- no extent overlaps the tile (a hole or the pad, store.go:974-980);
//  * COPY  -- one extent covers the whole tile: each lane reads the aligned 16-byte source
//    block(s) holding its 16 bytes and realigns them with v_alignbyte (the source
//    misalignment is uniform: tile offsets step by 16), every load issued before any use;
//  * MIXED -- an extent starts or ends inside the tile (tract boundaries, a partial last
//    tile): the tile is assembled byte by byte in LDS, then read back.  Rare: about two
//    tiles per piece for multi-MiB tracts.
// Reads of a source never leave the bytes of its extent's 16-byte blocks that hold wanted
// bytes (pack.hip's rule), so no read touches a page the source does not own.
#include "pack.hpp"

#include "gf_device.hpp"


namespace blbrs {
namespace {

using namespace dev;

constexpr int kPEThreads = 256;

struct PEArgs {
    const uint32_t* tables;
    const int32_t* out_idx;
    uint8_t* base;
    uint64_t shard_stride, stripe_stride, S;
    uint32_t B, tps, xcd_remap, rows;
    const uint64_t* table;
    const u32x4* desc;  // [piece][tile]: {sbase lo, sbase hi, first extent, kind}
    uint32_t tile;      // bytes per tile
};

enum : uint32_t { kZero = 0, kCopy = 1, kMixed = 2 };

// Pre-pass: one thread per (piece, tile) finds the tile's first extent and its layout, so
// the main kernel reads one descriptor per piece instead of running K binary searches
// (dependent scalar loads) before it can issue a single data load.
__global__ __launch_bounds__(256) void pe_classify_kernel(PEArgs a, uint32_t k, u32x4* desc) {
    const uint64_t id = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
    const uint64_t npieces = static_cast<uint64_t>(a.B) * k;
    if (id >= npieces * a.tps) return;
    const uint64_t piece = id / a.tps;
    const uint64_t t0 = (id - piece * a.tps) * a.tile;
    const uint64_t t1 = t0 + a.tile < a.S ? t0 + a.tile : a.S;
    const bool full = t1 - t0 == a.tile;
    const uint64_t* ex = a.table + npieces + 1;
    uint64_t lo = a.table[piece];
    const uint64_t hi = a.table[piece + 1];
    for (uint64_t n = hi - lo; n > 0;) {
        const uint64_t half = n >> 1, m = lo + half;
        if (ex[4 * m + 1] + ex[4 * m + 2] <= t0) {
            lo = m + 1;
            n -= half + 1;
        } else {
            n = half;
        }
    }
    uint32_t kind = kZero;
    uint64_t sbase = 0;
    if (lo != hi) {
        const uint64_t off = ex[4 * lo + 1], len = ex[4 * lo + 2];
        if (off < t1) {
            if (full && off <= t0 && off + len >= t1) {
                kind = kCopy;
                sbase = ex[4 * lo] - off;
            } else {
                kind = kMixed;
            }
        }
    }
    desc[id] = u32x4{static_cast<uint32_t>(sbase), static_cast<uint32_t>(sbase >> 32), static_cast<uint32_t>(lo), kind};
}

// out = bytes [s, s+16) of the 32-byte window lo||hi, s = 4q + r (q, r uniform).
__device__ __forceinline__ V4 funnel(const V4& a, const V4& b, uint32_t q, uint32_t r) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    switch (q) {
        case 0:
            return V4{__builtin_amdgcn_alignbyte(w[1], w[0], r), __builtin_amdgcn_alignbyte(w[2], w[1], r),
                      __builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r)};
        case 1:
            return V4{__builtin_amdgcn_alignbyte(w[2], w[1], r), __builtin_amdgcn_alignbyte(w[3], w[2], r),
                      __builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r)};
        case 2:
            return V4{__builtin_amdgcn_alignbyte(w[3], w[2], r), __builtin_amdgcn_alignbyte(w[4], w[3], r),
                      __builtin_amdgcn_alignbyte(w[5], w[4], r), __builtin_amdgcn_alignbyte(w[6], w[5], r)};
        default:
            return V4{__builtin_amdgcn_alignbyte(w[4], w[3], r), __builtin_amdgcn_alignbyte(w[5], w[4], r),
                      __builtin_amdgcn_alignbyte(w[6], w[5], r), __builtin_amdgcn_alignbyte(w[7], w[6], r)};
    }
}

__device__ __forceinline__ V4 ldnt(const uint8_t* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return V4{v.x, v.y, v.z, v.w};
}

__device__ __forceinline__ void stnt(uint8_t* p, const V4& v) {
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
}

// Store n <= 16 bytes of v at p (a partial last tile).
__device__ __forceinline__ void store_part(uint8_t* p, const V4& v, uint32_t n) {
    if (n >= 16) {
        stnt(p, v);
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t j = 0; j < n; ++j) p[j] = static_cast<uint8_t>(w[j >> 2] >> (8 * (j & 3)));
}

template <int K, int MR, int U>
__global__ __launch_bounds__(kPEThreads) void pack_encode_kernel(PEArgs a) {
    constexpr uint32_t kStep = kPEThreads * 16u;  // 4 KiB per chunk row
    constexpr uint32_t kTile = kStep * U;
    constexpr int NV = 4 * U;
    __shared__ __attribute__((aligned(16))) uint8_t stage[kTile];

    const uint32_t tid = threadIdx.x;
    uint32_t t = blockIdx.x;
    if (a.xcd_remap) t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
    const uint32_t b = t / a.tps;
    const uint64_t t0 = static_cast<uint64_t>(t - b * a.tps) * kTile;
    const uint64_t t1 = t0 + kTile < a.S ? t0 + kTile : a.S;
    const bool full = t1 - t0 == kTile;
    uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
    const uint64_t* ex = a.table + static_cast<uint64_t>(a.B) * K + 1;

    // Per piece, the tile's extent layout (uniform, from the pre-pass): lane p of every
    // wave loads piece p's descriptor -- K loads in parallel -- and the values are read back
    // per piece with v_readlane.
    const uint32_t lane = tid & 63u;
    uint32_t my_kind = kZero;
    uint64_t my_first = 0, my_sbase = 0;
    if (lane < static_cast<uint32_t>(K)) {
        const u32x4 d = a.desc[(static_cast<uint64_t>(b) * K + lane) * a.tps + (t0 / kTile)];
        my_sbase = (static_cast<uint64_t>(d.y) << 32) | d.x;
        my_first = d.z;
        my_kind = d.w;
    }
    auto rl64 = [](uint64_t v, int l) -> uint64_t {
        const uint32_t lo32 = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
        const uint32_t hi32 = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
        return (static_cast<uint64_t>(hi32) << 32) | lo32;
    };
    uint32_t copy_mask = 0, zero_mask = 0;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        const uint32_t kd = __builtin_amdgcn_readlane(my_kind, p);
        copy_mask |= (kd == kCopy ? 1u : 0u) << p;
        zero_mask |= (kd == kZero ? 1u : 0u) << p;
    }
    uint32_t acc[MR][NV] = {};
    cu32 tables = as_const(a.tables);
    asm volatile("" : "+s"(tables));
    // Store the packed data piece p (every byte written: PackTracts zero-fills,
    // store.go:974-980) and multiply it into the parity rows.
    auto consume = [&](int p, const V4 (&x)[U]) {
        uint8_t* dp = stripe + static_cast<uint64_t>(p) * a.shard_stride + t0 + 16u * tid;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c0 = t0 + u * kStep + 16u * tid;
            if (full) stnt(dp + u * kStep, x[u]);
            else if (c0 < t1) store_part(dp + u * kStep, x[u], static_cast<uint32_t>(t1 - c0));
        }
        uint32_t xv[NV];
#pragma unroll
        for (int u = 0; u < U; ++u) unpack(x[u], xv + 4 * u);
        madd<MR, NV>(Groups<NV>(xv), [&](int r) { return tables + (r * K + p) * 5; }, acc, static_cast<int>(a.rows));
    };
    const bool any_mixed = (copy_mask | zero_mask) != (1u << K) - 1u;

    if (!any_mixed) {
        // Fast path: COPY loads of every piece in flight before any use.
        V4 lo_blk[K][U], hi_blk[K][U];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            if (!((copy_mask >> p) & 1u)) continue;
            const uint64_t sb = rl64(my_sbase, p) + t0 + 16u * tid;
            const uint32_t mis = static_cast<uint32_t>(sb & 15u);
            const uint8_t* sa = reinterpret_cast<const uint8_t*>(sb - mis);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                lo_blk[p][u] = ldnt(sa + u * kStep);
                hi_blk[p][u] = mis ? ldnt(sa + u * kStep + 16) : lo_blk[p][u];  // holds wanted bytes
            }
        }
#pragma unroll
        for (int p = 0; p < K; ++p) {
            V4 x[U];
            const uint32_t mis = static_cast<uint32_t>((rl64(my_sbase, p) + t0) & 15u);
#pragma unroll
            for (int u = 0; u < U; ++u)
                x[u] = ((zero_mask >> p) & 1u) ? V4{0u, 0u, 0u, 0u}
                       : mis            ? funnel(lo_blk[p][u], hi_blk[p][u], mis >> 2, mis & 3u)
                                        : lo_blk[p][u];
            consume(p, x);
        }
    } else {
        // Slow path (an extent starts or ends inside the tile, or a partial last tile): each
        // piece's [t0, t1) assembled byte by byte in LDS from its extents, then read back.
        // The barriers are unconditional here: every thread runs every piece.
#pragma unroll 1
        for (int p = 0; p < K; ++p) {
            __syncthreads();  // the previous piece's reads of `stage` are done
            const uint64_t piece = static_cast<uint64_t>(b) * K + p;
            const uint64_t hi = a.table[piece + 1];
            const uint64_t first = rl64(my_first, p);
            uint64_t cur = t0;
            for (uint64_t e = first; cur < t1;) {
                const uint64_t off = e < hi ? ex[4 * e + 1] : t1;
                uint64_t end;
                if (off <= cur) {  // inside extent e
                    end = off + ex[4 * e + 2] < t1 ? off + ex[4 * e + 2] : t1;
                    const uint8_t* src = reinterpret_cast<const uint8_t*>(ex[4 * e]) + (cur - off);
                    for (uint64_t i = tid; i < end - cur; i += kPEThreads) stage[cur - t0 + i] = src[i];
                    ++e;
                } else {  // hole or pad up to the next extent / tile end
                    end = off < t1 ? off : t1;
                    for (uint64_t i = tid; i < end - cur; i += kPEThreads) stage[cur - t0 + i] = 0;
                }
                cur = end > cur ? end : cur;
            }
            for (uint64_t i = t1 - t0 + tid; i < kTile; i += kPEThreads) stage[i] = 0;
            __syncthreads();
            V4 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = *reinterpret_cast<const V4*>(stage + u * kStep + 16u * tid);
            // consume() with a runtime p: the table index is the only p-dependent part.
            uint8_t* dp = stripe + static_cast<uint64_t>(p) * a.shard_stride + t0 + 16u * tid;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t c0 = t0 + u * kStep + 16u * tid;
                if (full) stnt(dp + u * kStep, x[u]);
                else if (c0 < t1) store_part(dp + u * kStep, x[u], static_cast<uint32_t>(t1 - c0));
            }
            uint32_t xv[NV];
#pragma unroll
            for (int u = 0; u < U; ++u) unpack(x[u], xv + 4 * u);
            madd<MR, NV>(Groups<NV>(xv), [&](int r) { return tables + (r * K + p) * 5; }, acc,
                         static_cast<int>(a.rows));
        }
    }
    const ci32 out_idx = as_const(a.out_idx);
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r >= static_cast<int>(a.rows)) break;
        uint8_t* q = stripe + static_cast<uint64_t>(out_idx[r]) * a.shard_stride + t0 + 16u * tid;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c0 = t0 + u * kStep + 16u * tid;
            if (full) stnt(q + u * kStep, pack(acc[r] + 4 * u));
            else if (c0 < t1) store_part(q + u * kStep, pack(acc[r] + 4 * u), static_cast<uint32_t>(t1 - c0));
        }
    }
}

using KernelFn = void (*)(PEArgs);

#ifndef BLBRS_PE_U
#define BLBRS_PE_U 1
#endif
constexpr int kU = BLBRS_PE_U;  // 16-byte chunks per lane per piece (tile = 4 KiB * kU)

template <int K>
KernelFn pick_rows(uint32_t rows) {
    switch (rows) {
        case 1: return pack_encode_kernel<K, 1, kU>;
        case 2: return pack_encode_kernel<K, 2, kU>;
        case 3: return pack_encode_kernel<K, 3, kU>;
        case 4: return pack_encode_kernel<K, 4, kU>;
        case 5: return pack_encode_kernel<K, 5, kU>;
        default: return nullptr;
    }
}

// blb's classes RS(6,3), RS(8,3), RS(10,3), RS(12,5), the bench's RS(10,4), the reference
// tests' RS(3,2) and RS(4,2).
KernelFn pick(uint32_t k, uint32_t rows) {
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

}  // namespace

bool pack_encode_supported(const PackEncodeArgs& a) {
    const bool aligned = (reinterpret_cast<uintptr_t>(a.base) & 15u) == 0 && (a.shard_stride & 15u) == 0 &&
                         (a.stripe_stride & 15u) == 0;
    const uint64_t tile = 4096ull * kU;
    return a.base && aligned && pick(a.k, a.rows) != nullptr && a.nextents <= 0xFFFFFFFFull &&
           static_cast<uint64_t>(a.B) * ((a.S + tile - 1) / tile) <= 0x7FFFFFFFull;
}

hipError_t launch_pack_encode(const PackEncodeArgs& in, hipStream_t stream) {
    if (in.B == 0 || in.S == 0) return hipSuccess;
    if (!pack_encode_supported(in)) return hipErrorInvalidValue;
    const uint64_t tile = 4096ull * kU;
    const uint64_t ndesc = static_cast<uint64_t>(in.B) * in.k * ((in.S + tile - 1) / tile);
    if (ndesc > 0xFFFFFFFFull * 256) return hipErrorInvalidValue;
    PEArgs a{};
    a.tables = in.tables;
    a.out_idx = in.out_idx;
    a.base = in.base;
    a.shard_stride = in.shard_stride;
    a.stripe_stride = in.stripe_stride;
    a.S = in.S;
    a.B = in.B;
    a.rows = in.rows;
    a.tps = static_cast<uint32_t>((in.S + tile - 1) / tile);
    a.table = in.table;
    a.tile = static_cast<uint32_t>(tile);
    const uint64_t total = static_cast<uint64_t>(in.B) * a.tps;
    uint64_t grid = total;
    a.xcd_remap = 0;
    if (total >= 64 && total % 8 == 0) a.xcd_remap = 1;
    u32x4* desc = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&desc), ndesc * sizeof(u32x4), stream);
    if (e != hipSuccess) return e;
    a.desc = desc;
    hipLaunchKernelGGL(pe_classify_kernel, dim3(static_cast<unsigned>((ndesc + 255) / 256)), dim3(256), 0, stream, a,
                       in.k, desc);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(pick(in.k, in.rows), dim3(static_cast<unsigned>(grid)), dim3(kPEThreads), 0, stream, a);
        e = hipGetLastError();
    }
    const hipError_t f = hipFreeAsync(desc, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
