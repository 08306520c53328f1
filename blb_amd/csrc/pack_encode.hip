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
//  * COPY  -- one extent covers the whole tile: each lane reads the aligned 16-byte block
//    holding the start of its 16 bytes, takes the following block from the next lane (DPP
//    rotate) and realigns the pair with v_alignbyte (the source misalignment is uniform: tile
//    offsets step by 16); every load of every COPY piece is issued before any use;
//  * MIXED -- an extent starts or ends inside the tile (tract boundaries, a partial last
//    tile): each lane resolves its own 16 bytes from the extents (one extent: funnel with a
//    per-lane shift; a hole: zero; cut by a boundary: bytes).  Other pieces of the same tile
//    stay COPY / ZERO.  Rare: about two tiles per piece for multi-MiB tracts.
// Reads of a source never leave the bytes of its extent's 16-byte blocks that hold wanted
// bytes (pack.hip's rule), so no read touches a page the source does not own.
#include "pack.hpp"

#include <type_traits>

#include "gf_bitslice.hpp"
#include "gf_device.hpp"
#include "tuning.hpp"


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

// The same with a per-lane shift s (MIXED pieces): dword select by q, then v_alignbyte by r.
__device__ __forceinline__ V4 funnel_lane(const V4& a, const V4& b, uint32_t s) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t q = s >> 2, r = s & 3u;
    uint32_t d[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) d[i] = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
    return V4{__builtin_amdgcn_alignbyte(d[1], d[0], r), __builtin_amdgcn_alignbyte(d[2], d[1], r),
              __builtin_amdgcn_alignbyte(d[3], d[2], r), __builtin_amdgcn_alignbyte(d[4], d[3], r)};
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

// Lane i receives lane (i + 1) mod 64's dword (DPP wave_rol:1, no LDS).
__device__ __forceinline__ uint32_t rol1(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x134, 0xF, 0xF, false));
}
__device__ __forceinline__ V4 rol1(const V4& v) { return V4{rol1(v.x), rol1(v.y), rol1(v.z), rol1(v.w)}; }

// Bytes [c0, c0 + 16) of a piece whose tile is MIXED, resolved by this lane alone from the
// piece's extents (e = the tile's first extent ending past the tile start, hi = the piece's
// end in the table).  A chunk inside one extent is two aligned loads and a per-lane funnel, a
// chunk inside a hole or past t1 is zero (bytes past t1 are never stored), and a chunk that
// an extent boundary cuts is assembled byte by byte.  Reads stay within wanted 16-byte blocks.
__device__ V4 mixed_chunk(const uint64_t* ex, uint64_t e, uint64_t hi, uint64_t c0, uint64_t t1) {
    while (e < hi && ex[4 * e + 1] + ex[4 * e + 2] <= c0) ++e;
    const uint64_t c1 = c0 + 16 < t1 ? c0 + 16 : t1;
    if (c0 >= t1 || e >= hi || ex[4 * e + 1] >= c1) return V4{0u, 0u, 0u, 0u};
    const uint64_t off = ex[4 * e + 1], len = ex[4 * e + 2];
    if (off <= c0 && off + len >= c0 + 16) {
        const uint64_t s = ex[4 * e] + (c0 - off);
        const uint32_t mis = static_cast<uint32_t>(s & 15u);
        const uint8_t* sa = reinterpret_cast<const uint8_t*>(s - mis);
        const V4 lo = ldnt(sa);
        if (mis == 0) return lo;
        return funnel_lane(lo, ldnt(sa + 16), mis);
    }
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t j = 0; j < 16; ++j) {
        const uint64_t pos = c0 + j;
        if (pos >= t1) break;
        while (e < hi && ex[4 * e + 1] + ex[4 * e + 2] <= pos) ++e;
        if (e < hi && ex[4 * e + 1] <= pos) {
            const uint8_t* src = reinterpret_cast<const uint8_t*>(ex[4 * e]);
            w[j >> 2] |= static_cast<uint32_t>(src[pos - ex[4 * e + 1]]) << (8 * (j & 3));
        }
    }
    return V4{w[0], w[1], w[2], w[3]};
}

// One workgroup per (stripe, tile); wave w owns the tile's bytes [w*U KiB, (w+1)*U KiB) of
// every piece, chunk u of lane l at w*U KiB + u KiB + 16 l, so the 16-byte block after lane
// 63's chunk u is lane 0's chunk u + 1 (a DPP rotate away) except after the last chunk.
// f(integral_constant<int, I>) for I = 0..N-1 (compile-time piece indices for the network).
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// CM: the parity rows are encode parity rows 0..MR-1 of K, accumulated in bit-plane form by
// the compiled network (gf_bitslice.hpp) one piece at a time (U = 2: 8 dwords per lane).
template <int K, int MR, int U, bool CM>
__global__ __launch_bounds__(kPEThreads) void pack_encode_kernel(PEArgs a) {
    static_assert(!CM || U == 2, "bit planes of 8 dwords");
    constexpr uint32_t kWaveRow = 64u * 16u;             // 1 KiB per wave instruction
    constexpr uint32_t kWaveRun = kWaveRow * U;          // contiguous bytes per wave
    constexpr uint32_t kTile = kWaveRun * (kPEThreads / 64u);
    constexpr int NV = 4 * U;

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    uint32_t t = blockIdx.x;
    if (a.xcd_remap) t = (t % 8u) * (gridDim.x / 8u) + t / 8u;
    const uint32_t b = t / a.tps;
    const uint64_t t0 = static_cast<uint64_t>(t - b * a.tps) * kTile;
    const uint64_t t1 = t0 + kTile < a.S ? t0 + kTile : a.S;
    const bool full = t1 - t0 == kTile;
    const uint64_t lane_off = t0 + (tid >> 6) * kWaveRun + 16u * lane;  // + u KiB
    uint8_t* stripe = a.base + static_cast<uint64_t>(b) * a.stripe_stride;
    const uint64_t* ex = a.table + static_cast<uint64_t>(a.B) * K + 1;

    // Per piece, the tile's extent layout (uniform, from the pre-pass): lane p of every
    // wave loads piece p's descriptor -- K loads in parallel -- and the values are read back
    // per piece with v_readlane.
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
    uint32_t kinds = 0;  // 2 bits per piece
#pragma unroll
    for (int p = 0; p < K; ++p) kinds |= __builtin_amdgcn_readlane(my_kind, p) << (2 * p);
    auto kind = [&](int p) { return (kinds >> (2 * p)) & 3u; };

    // COPY loads of every piece in flight before any use: the aligned 16-byte blocks of the
    // wave's run, plus (lane 63 only, misaligned sources only) the block just past it.
    V4 lo_blk[K][U], tail[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (kind(p) != kCopy) continue;
        const uint64_t sb = rl64(my_sbase, p) + lane_off;
        const uint32_t mis = static_cast<uint32_t>(sb & 15u);
        const uint8_t* sa = reinterpret_cast<const uint8_t*>(sb - mis);
#pragma unroll
        for (int u = 0; u < U; ++u) lo_blk[p][u] = ldnt(sa + u * kWaveRow);
        if (mis != 0 && lane == 63u) tail[p] = ldnt(sa + (U - 1) * kWaveRow + 16);
    }

    uint32_t acc[MR][NV] = {};
    cu32 tables = as_const(a.tables);
    asm volatile("" : "+s"(tables));
    static_for<K>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        V4 x[U];
        const uint32_t kd = kind(p);
        if (kd == kZero) {
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = V4{0u, 0u, 0u, 0u};
        } else if (kd == kCopy) {
            const uint32_t mis = static_cast<uint32_t>((rl64(my_sbase, p) + lane_off) & 15u);
            if (mis == 0) {
#pragma unroll
                for (int u = 0; u < U; ++u) x[u] = lo_blk[p][u];
            } else {
                V4 nb[U];  // lane l: the block after lane l's chunk u (lane 63: chunk u+1 of lane 0)
#pragma unroll
                for (int u = 0; u < U; ++u) nb[u] = rol1(lo_blk[p][u]);
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const V4 h63 = u + 1 < U ? nb[u + 1] : tail[p];
                    const V4 hb = lane == 63u ? h63 : nb[u];
                    x[u] = funnel(lo_blk[p][u], hb, mis >> 2, mis & 3u);
                }
            }
        } else {
            const uint64_t piece = static_cast<uint64_t>(b) * K + p;
            const uint64_t hi = a.table[piece + 1];
            const uint64_t first = rl64(my_first, p);
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = mixed_chunk(ex, first, hi, lane_off + u * kWaveRow, t1);
        }
        // Store the packed data piece p (every byte written: PackTracts zero-fills,
        // store.go:974-980) and multiply it into the parity rows.
        uint8_t* dp = stripe + static_cast<uint64_t>(p) * a.shard_stride + lane_off;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c0 = lane_off + u * kWaveRow;
            if (full) stnt(dp + u * kWaveRow, x[u]);
            else if (c0 < t1) store_part(dp + u * kWaveRow, x[u], static_cast<uint32_t>(t1 - c0));
        }
        uint32_t xv[NV];
#pragma unroll
        for (int u = 0; u < U; ++u) unpack(x[u], xv + 4 * u);
        if constexpr (CM) {
            bs::transpose8(xv);
            bs::add_one<K, MR, p>(xv, acc);
        } else {
            madd<MR, NV>(Groups<NV>(xv), [&](int r) { return tables + (r * K + p) * 5; }, acc,
                         static_cast<int>(a.rows));
        }
    });
    if constexpr (CM)
#pragma unroll
        for (int r = 0; r < MR; ++r) bs::transpose8(acc[r]);
    const ci32 out_idx = as_const(a.out_idx);
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        if (r >= static_cast<int>(a.rows)) break;
        uint8_t* q = stripe + static_cast<uint64_t>(out_idx[r]) * a.shard_stride + lane_off;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c0 = lane_off + u * kWaveRow;
            if (full) stnt(q + u * kWaveRow, pack(acc[r] + 4 * u));
            else if (c0 < t1) store_part(q + u * kWaveRow, pack(acc[r] + 4 * u), static_cast<uint32_t>(t1 - c0));
        }
    }
}

using KernelFn = void (*)(PEArgs);

// 16-byte chunks per lane per piece (tile = 4 KiB * U), measured (tools/pe_variants.sh,
// profiles/r02/pack_encode_ab/): RS(6,3) B=1024 U=1/2/4 20.2/19.8/20.4 ms (22.3 ms for the
// previous LDS-assembly kernel at U=1); RS(12,5) B=512 U=1/2/4 23.7/24.0/46.6 ms.
#ifndef BLBRS_PE_U_NARROW
#define BLBRS_PE_U_NARROW 2
#endif
#ifndef BLBRS_PE_U_WIDE
#define BLBRS_PE_U_WIDE 1
#endif
constexpr int pe_u(uint32_t k) { return k <= 6 ? BLBRS_PE_U_NARROW : BLBRS_PE_U_WIDE; }

// The network runs at U = 2 for every k: it holds fewer registers than the table multiply
// (RS(12,5) 141 at U = 1 with tables).
int tile_u(uint32_t k, bool cm) { return cm ? 2 : pe_u(k); }

template <int K, int MR>
KernelFn pick_cm(bool cm) {
    if (cm && tile_u(K, cm) == 2) return pack_encode_kernel<K, MR, 2, true>;
    return pack_encode_kernel<K, MR, pe_u(K), false>;
}

template <int K>
KernelFn pick_rows(uint32_t rows, bool cm) {
    switch (rows) {
        case 1: return pick_cm<K, 1>(cm);
        case 2: return pick_cm<K, 2>(cm);
        case 3: return pick_cm<K, 3>(cm);
        case 4: return pick_cm<K, 4>(cm);
        case 5: return pick_cm<K, 5>(cm);
        default: return nullptr;
    }
}

// blb's classes RS(6,3), RS(8,3), RS(10,3), RS(12,5), the bench's RS(10,4), the reference
// tests' RS(3,2) and RS(4,2).  cm: the compiled encode network (parity-row tables).
KernelFn pick(uint32_t k, uint32_t rows, bool cm = false) {
    switch (k) {
        case 3: return pick_rows<3>(rows, cm);
        case 4: return pick_rows<4>(rows, cm);
        case 6: return pick_rows<6>(rows, cm);
        case 8: return pick_rows<8>(rows, cm);
        case 10: return pick_rows<10>(rows, cm);
        case 12: return pick_rows<12>(rows, cm);
        default: return nullptr;
    }
}

}  // namespace

bool pack_encode_supported(const PackEncodeArgs& a) {
    const bool aligned = (reinterpret_cast<uintptr_t>(a.base) & 15u) == 0 && (a.shard_stride & 15u) == 0 &&
                         (a.stripe_stride & 15u) == 0;
    const uint64_t tile = 4096ull * tile_u(a.k, bs::use(a.parity, static_cast<int>(a.k), static_cast<int>(a.rows), bs::kWidePack));
    return a.base && aligned && pick(a.k, a.rows) != nullptr && a.nextents <= 0xFFFFFFFFull &&
           static_cast<uint64_t>(a.B) * ((a.S + tile - 1) / tile) <= 0x7FFFFFFFull;
}

hipError_t launch_pack_encode(const PackEncodeArgs& in, hipStream_t stream) {
    if (in.B == 0 || in.S == 0) return hipSuccess;
    if (!pack_encode_supported(in)) return hipErrorInvalidValue;
    const bool cm = bs::use(in.parity, static_cast<int>(in.k), static_cast<int>(in.rows), bs::kWidePack);
    const uint64_t tile = 4096ull * tile_u(in.k, cm);
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
    // Descriptors live in the caller's scratch (the extent table's slot, PtrLease): a per-launch
    // hipMallocAsync / hipFreeAsync of 100-134 MB cost 0.7-1.1 ms per call at blb's shapes.
    if (!in.scratch) return hipErrorInvalidValue;
    u32x4* desc = static_cast<u32x4*>(in.scratch);
    a.desc = desc;
    hipError_t e = hipSuccess;
    hipLaunchKernelGGL(pe_classify_kernel, dim3(static_cast<unsigned>((ndesc + 255) / 256)), dim3(256), 0, stream, a,
                       in.k, desc);
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(pick(in.k, in.rows, cm), dim3(static_cast<unsigned>(grid)),
                           dim3(kPEThreads), 0, stream, a);
        e = hipGetLastError();
    }
    return e;
}

size_t pack_encode_scratch_bytes(const PackEncodeArgs& in) {
    const bool cm = bs::use(in.parity, static_cast<int>(in.k), static_cast<int>(in.rows), bs::kWidePack);
    const uint64_t tile = 4096ull * tile_u(in.k, cm);
    return static_cast<size_t>(in.B) * in.k * ((in.S + tile - 1) / tile) * sizeof(u32x4);
}

}  // namespace blbrs
