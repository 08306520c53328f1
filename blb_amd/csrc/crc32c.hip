// crc32c.hip -- CRC-32C (Castagnoli) of shard blocks on gfx950 (see crc32c.hpp; the raw-CRC
// algebra, S_n shift matrices and banked LDS tables are in crc_device.hpp).
//
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
//
// Blocks are FILE-aligned: a buffer starts `phase` bytes into its first block (the file
// offset of its byte 0, mod block -- rsEncodeOne writes parity windows at 4 MiB * i,
// internal/tractserver/store.go:1028-1037,1115, and the receiver checksums 65532-byte
// ChecksumFile blocks, pkg/disk/checksum_block.go:18-34).  All kernels work in VIRTUAL
// coordinates v = phase + offset: the `phase` bytes before the buffer are virtual zeros,
// which leave a raw CRC unchanged, so segment layout and folding are those of a buffer
// starting at a block boundary; only the init term of the first block uses its real length
// and its seed (crc32.Update(seed, ...), checksum_block.go:80 chains appends that way).
#include "crc32c.hpp"
#include "crc_device.hpp"

#include <map>
#include <mutex>
#include <vector>

namespace blbrs {
namespace rt {
hipError_t upload_pinned(void* dev, const void* src, size_t n);  // runtime.hpp
}  // namespace rt
namespace {

using namespace dev;
using V4x = u32x4;

constexpr int kThreads = 256;
constexpr int kPow2 = kCrcPow2;

struct SegArgs {
    const uint8_t* data;
    uint64_t stride, len, block, seg;
    uint32_t nblocks, segs_per_block;
    const CrcConsts* c;
    uint32_t* raw;                        // [batch][nblocks][segs_per_block]
    uint64_t phase;                       // virtual offset of byte 0 (see top)
    const uint32_t* seeds;                // per row: crc32.Update seed of block 0 (NULL = 0)
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
    const uint64_t len_v = a.len + a.phase;
    const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;  // virtual
    const uint64_t blk_end = blk_start + a.block < len_v ? blk_start + a.block : len_v;
    const uint64_t seg_start = blk_start + static_cast<uint64_t>(s) * a.seg;
    const uint64_t seg_end = seg_start + a.seg < blk_end ? seg_start + a.seg : blk_end;
    const uint64_t start = seg_start > a.phase ? seg_start : a.phase;  // first real byte
    if (start >= seg_end) {
        if (tid == 0) a.raw[g] = 0u;
        return;
    }
    const uint32_t seglen = static_cast<uint32_t>(seg_end - start);
    const uint32_t pad = kSegMax - seglen;        // virtual zero prefix
    const uint8_t* src = a.data + b * a.stride + (start - a.phase);

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

// ---- streaming kernel: coalesced HBM reads, conflict-free banked tables ----
// One 1024-thread workgroup per CU keeps the four slicing tables in LDS with a private copy
// per bank: table j, entry e, bank l lives at byte (j>>1)<<16 | e<<8 | (j&1)<<7 | l<<2, so a
// 32-lane group always hits 32 distinct banks and each lookup address is ONE v_perm_b32 of
// (x, base_j).  Each WAVE owns a 64 KiB segment = 16 rows of 4 KiB; lane t owns the 64
// contiguous bytes at column t of every row (4 dwordx4 loads; the wave's loads cover each
// row contiguously), runs slicing-by-4 over them and jumps the 4032 bytes to its next chunk
// with one S_4032 matrix.  Lanes then fold with S_{64*2^j}.  A segment is aligned to END at
// its real end; the bytes before its start are virtual zeros: rows wholly inside that prefix
// are skipped (a zero prefix leaves the raw CRC at 0), the row holding the start is loaded
// dword by dword, and the rest run through a branch-free loop that loads one row ahead.
// Rows of the register ring: loads run kRing - 1 rows ahead of the row being checksummed.
#ifndef BLBRS_CRC_RING
#define BLBRS_CRC_RING 3
#endif
constexpr int kRing = BLBRS_CRC_RING;
// 2 = each wave runs two chains at once, over rows 0-7 and 8-15 of its segment (joined with
// S_{32 KiB}), halving the dependent LDS steps per row consumed (A/B builds).
#ifndef BLBRS_CRC_ILP
#define BLBRS_CRC_ILP 1
#endif
constexpr int kIlp = BLBRS_CRC_ILP;
#ifndef BLBRS_CRC_XCD
#define BLBRS_CRC_XCD 0
#endif
constexpr bool kXcdMap = BLBRS_CRC_XCD != 0;
constexpr int kStreamThreads = 1024;
constexpr uint32_t kChunk = 64, kRowBytes = kChunk * 64, kRows = 16;  // 4 KiB rows
constexpr uint32_t kWaveSeg = kRowBytes * kRows;                      // 64 KiB per wave
// 1 = the row jump S_4032 and the six lane-fold matrices are applied through byte tables in
// LDS (T_b[v] = the matrix applied to v << 8b: 4 lookups + 2 XOR, about 7 VALU) instead of
// 32 columns of v_bfe + v_bitop3 (64 VALU on the chain, 15 jumps + 6 folds per 64 KiB).
#ifndef BLBRS_CRC_TABAPPLY
#define BLBRS_CRC_TABAPPLY 1
#endif
constexpr bool kTabApply = BLBRS_CRC_TABAPPLY != 0;
constexpr uint32_t kApplyMats = 7;                                     // gap, then wlvl levels 0..5
constexpr size_t kApplyTabBytes = kApplyMats * 4 * 256 * 4;            // 28 KiB
constexpr size_t kStreamLds = kBankedTableBytes + (kTabApply ? kApplyTabBytes : 0);  // 156 KiB
static_assert(kStreamLds <= 160 * 1024, "one workgroup per CU");

// Byte tables of the stream kernel's matrices, after the banked slicing tables.
__device__ __forceinline__ void init_apply_tables(uint32_t* at, const CrcConsts* c) {
    for (uint32_t i = threadIdx.x; i < kApplyMats * 1024u; i += kStreamThreads) {
        const uint32_t mat = i >> 10, b = (i >> 8) & 3u, v = i & 255u;
        const uint32_t* col = mat == 0 ? c->gap[0] : c->wlvl[0][mat - 1];
        uint32_t o = 0;
        for (uint32_t t = 0; t < 8; ++t)
            if ((v >> t) & 1u) o ^= col[8 * b + t];
        at[i] = o;
    }
}
__device__ __forceinline__ uint32_t apply_tab(const uint32_t* T, uint32_t r) {
    return xor3(T[r & 255u], T[256u + ((r >> 8) & 255u)], T[512u + ((r >> 16) & 255u)]) ^ T[768u + (r >> 24)];
}

struct StreamArgs {
    const uint8_t* data;
    uint64_t stride, len, block;
    uint32_t nblocks, segs_per_block;
    uint64_t total_segs;
    const CrcConsts* c;
    uint32_t* raw;
    uint64_t phase;  // virtual offset of byte 0 (multiple of 4)
};

struct Chunk {
    V4x q[4];
};

__device__ __forceinline__ uint32_t crc_chunk(const LaneTabs& t, uint32_t c, const Chunk& ch) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        c = slice4(t, c ^ ch.q[i].x);
        c = slice4(t, c ^ ch.q[i].y);
        c = slice4(t, c ^ ch.q[i].z);
        c = slice4(t, c ^ ch.q[i].w);
    }
    return c;
}

// Per-lane layout (BLBRS_CRC_COAL=0): plain (L1-allocating) loads, because each 128-byte
// line is split over the four dwordx4 instructions of two lanes and the L1 merges them;
// nontemporal loads bypass that merge and measured 1.6x slower (3.3 vs 5.3 TB/s).  The
// coalesced layout below has no split lines, so it can stream nontemporal.
[[maybe_unused]] __device__ __forceinline__ Chunk load_row(const uint8_t* p) {
    Chunk ch;
#pragma unroll
    for (int i = 0; i < 4; ++i) ch.q[i] = *reinterpret_cast<const V4x*>(p + 16 * i);
    return ch;
}

// Row loads.  0 = lane t loads its own 64 contiguous bytes (four dwordx4 64 bytes apart: each
// instruction touches 64 partial lines that the L1 merges); 1 = each wave instruction loads a
// contiguous 1 KiB sub-row (lane_piece order) and v_permlane swaps give every lane its 64
// contiguous bytes at use; 2 (default) = 1 with nontemporal loads.  3072 x 8 MiB rows:
// 65532-byte blocks 4.40-4.49 ms (2) vs 4.69 (1) vs 4.78-4.89 (0), whole rows 4.28-4.37 vs
// 4.68-4.71 vs 4.52-4.57 (profiles/r03/crc_ab).
#ifndef BLBRS_CRC_COAL
#define BLBRS_CRC_COAL 2
#endif
constexpr int kCoal = BLBRS_CRC_COAL;

__device__ __forceinline__ Chunk load_row_at(const uint8_t* lane_chunk, const uint8_t* row, uint32_t lane) {
    if constexpr (kCoal == 0) {
        return load_row(lane_chunk);
    } else {
        Chunk ch;
        const uint8_t* p = row + lane_piece<64>(lane);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            ch.q[q] = kCoal == 2 ? __builtin_nontemporal_load(reinterpret_cast<const V4x*>(p + 1024 * q))
                                 : *reinterpret_cast<const V4x*>(p + 1024 * q);
        return ch;
    }
}

// A coalesced row into lane-contiguous order (no-op for the per-lane layout).
__device__ __forceinline__ Chunk to_lane(const Chunk& in) {
    if constexpr (kCoal == 0) {
        return in;
    } else {
        uint32_t v[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            v[4 * q] = in.q[q].x;
            v[4 * q + 1] = in.q[q].y;
            v[4 * q + 2] = in.q[q].z;
            v[4 * q + 3] = in.q[q].w;
        }
        lane_contiguous<64>(v);
        Chunk out;
#pragma unroll
        for (int i = 0; i < 4; ++i) out.q[i] = V4x{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
        return out;
    }
}

// 4 waves per SIMD is fixed by the 1024-thread workgroup + 128 KiB LDS; saying so lets the
// scheduler spend VGPRs on load-ahead instead of sinking loads next to their uses.
__global__ __launch_bounds__(kStreamThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void crc_stream_kernel(
    StreamArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab[];
    uint32_t* const atab = tab + kBankedTableBytes / 4;
    init_banked_tables(tab, a.c, kStreamThreads);
    if constexpr (kTabApply) init_apply_tables(atab, a.c);
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const LaneTabs t(lane);
    // S_4032 (chunk end -> the lane's next chunk) and the lane folds S_{64 * 2^j}.
    auto jump = [&](uint32_t r) { return kTabApply ? apply_tab(atab, r) : apply(as_const(a.c->gap[0]), r); };
    auto fold = [&](int j, uint32_t r) {
        return kTabApply ? apply_tab(atab + 1024u * (1 + j), r) : apply(as_const(&a.c->wlvl[0][j][0]), r);
    };
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (kStreamThreads / 64);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // Segments in dispatch order, or (BLBRS_CRC_XCD) each XCD's workgroups walking one
    // contiguous eighth of them.
    uint64_t g_lo = blockIdx.x * (kStreamThreads / 64) + wave, g_hi = a.total_segs, g_step = waves;
    if (kXcdMap && gridDim.x % 8u == 0) {
        const uint32_t x = blockIdx.x % 8u;
        g_lo = a.total_segs * x / 8u + (blockIdx.x / 8u) * (kStreamThreads / 64) + wave;
        g_hi = a.total_segs * (x + 1u) / 8u;
        g_step = waves / 8u;
    }
    for (uint64_t g = g_lo; g < g_hi; g += g_step) {
        const uint32_t s = static_cast<uint32_t>(g % a.segs_per_block);
        const uint32_t blk = static_cast<uint32_t>((g / a.segs_per_block) % a.nblocks);
        const uint64_t b = g / (static_cast<uint64_t>(a.segs_per_block) * a.nblocks);
        // Virtual coordinates (phase + offset); `data_v` is never dereferenced below byte 0.
        const uint64_t len_v = a.len + a.phase;
        const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;
        const uint64_t blk_end = blk_start + a.block < len_v ? blk_start + a.block : len_v;
        const uint64_t seg_start = blk_start + static_cast<uint64_t>(s) * kWaveSeg;
        const uint64_t start = seg_start > a.phase ? seg_start : a.phase;  // first real byte
        const uint64_t end = seg_start + kWaveSeg < blk_end ? seg_start + kWaveSeg : blk_end;
        if (start >= end) {
            if (lane == 0) a.raw[g] = 0u;
            continue;
        }
        const uint32_t pad = static_cast<uint32_t>(kWaveSeg - (end - start));  // multiple of 4
        const uint8_t* row_data = a.data + b * a.stride - a.phase;  // virtual origin
        const uint8_t* lane_base = row_data + end - kWaveSeg + lane * kChunk;  // row 0 chunk

        uint32_t c = 0;
        if (pad < kRowBytes) {
            // Common case (every segment of 65532-byte blocks and of whole dword frames): only
            // row 0 can hold virtual zeros.  Straight-line code, loads two rows ahead.
            Chunk ring[kRing];
            if (pad == 0) {
                if constexpr (!kCoal) ring[0] = load_row(lane_base);
            } else {
                // Row 0 through a buffer resource based at the segment start and bounded to
                // row 0's real bytes: dwords before the start have negative (wrapped) offsets,
                // fail the range check and read as 0 -- no branches, no access before start.
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<uint8_t*>(row_data + start), 0, static_cast<int>(kRowBytes - pad), 0x00020000);
                const uint32_t o = lane * kChunk - pad;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t w[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        w[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(o + 16u * i + 4u * k), 0, 0);
                    ring[0].q[i] = V4x{w[0], w[1], w[2], w[3]};
                }
            }
            if constexpr (kIlp == 2) {
                // Chain A over rows 0..7, chain B over rows 8..15, a ring per chain.
                constexpr uint32_t kHalf = kRows / 2;
                Chunk rb[kRing];
                const uint8_t* row0 = lane_base - lane * kChunk;
                auto ld = [&](uint32_t r) { return load_row_at(lane_base + r * kRowBytes, row0 + r * kRowBytes, lane); };
                if (kCoal && pad == 0) ring[0] = ld(0);
#pragma unroll
                for (int r = 1; r < kRing; ++r) ring[r] = ld(r);
#pragma unroll
                for (int r = 0; r < kRing; ++r) rb[r] = ld(kHalf + r);
                __builtin_amdgcn_sched_barrier(0);
                uint32_t cb = 0;
#pragma unroll
                for (uint32_t r = 0; r < kHalf; ++r) {
                    const Chunk ca_cur = (r == 0 && pad != 0) ? ring[0] : to_lane(ring[r % kRing]);
                    const Chunk cb_cur = to_lane(rb[r % kRing]);
                    if (r + kRing < kHalf) {
                        ring[r % kRing] = ld(r + kRing);
                        rb[r % kRing] = ld(kHalf + r + kRing);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (r) {
                        c = jump(c);
                        cb = jump(cb);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        c = slice4(t, c ^ ca_cur.q[i].x);
                        cb = slice4(t, cb ^ cb_cur.q[i].x);
                        c = slice4(t, c ^ ca_cur.q[i].y);
                        cb = slice4(t, cb ^ cb_cur.q[i].y);
                        c = slice4(t, c ^ ca_cur.q[i].z);
                        cb = slice4(t, cb ^ cb_cur.q[i].z);
                        c = slice4(t, c ^ ca_cur.q[i].w);
                        cb = slice4(t, cb ^ cb_cur.q[i].w);
                    }
                }
                c = apply(as_const(&a.c->pow2[15][0]), c) ^ cb;  // S_{8 rows = 32 KiB}
            } else {
            const uint8_t* row0 = lane_base - lane * kChunk;
            if (kCoal && pad == 0) ring[0] = load_row_at(lane_base, row0, lane);
#pragma unroll
            for (int r = 1; r < kRing; ++r) ring[r] = load_row_at(lane_base + r * kRowBytes, row0 + r * kRowBytes, lane);
            // sched_barrier pins each row's loads where they are issued; left alone the
            // scheduler sinks them next to their first use and every row waits on HBM.
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (uint32_t r = 0; r < kRows; ++r) {
                const Chunk cur = (r == 0 && pad != 0) ? ring[0] : to_lane(ring[r % kRing]);
                if (r + kRing < kRows)
                    ring[r % kRing] = load_row_at(lane_base + (r + kRing) * kRowBytes, row0 + (r + kRing) * kRowBytes, lane);
                __builtin_amdgcn_sched_barrier(0);
                if (r) c = jump(c);
                c = crc_chunk(t, c, cur);
            }
            }
        } else {
            // Short tail segment: rows before the start are all zeros (raw CRC stays 0).
            for (uint32_t r = pad / kRowBytes; r < kRows; ++r) {
                uint32_t w[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t off = r * kRowBytes + lane * kChunk + 4u * i;
                    w[i] = off >= pad ? *reinterpret_cast<const uint32_t*>(lane_base + r * kRowBytes + 4 * i) : 0u;
                }
                c = jump(c);  // no-op on the first row, whose c is 0
#pragma unroll
                for (int i = 0; i < 16; ++i) c = slice4(t, c ^ w[i]);
            }
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const uint32_t other = __shfl_down(c, 1u << j, 64);
            if ((lane & ((2u << j) - 1u)) == 0) c = fold(j, c) ^ other;
        }
        if (lane == 0) a.raw[g] = c;
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
    const uint64_t len_v = a.len + a.phase;
    const uint64_t blk_start = static_cast<uint64_t>(blk) * a.block;  // virtual
    const uint64_t blk_end = blk_start + a.block < len_v ? blk_start + a.block : len_v;
    const uint64_t blk_len = blk_end - blk_start;
    const uint64_t real_len = blk_end - (blk_start > a.phase ? blk_start : a.phase);
    const uint32_t seed = blk == 0 && a.seeds ? a.seeds[id / a.nblocks] : 0u;
    const uint32_t nseg = static_cast<uint32_t>((blk_len + a.seg - 1) / a.seg);
    const uint32_t* raw = a.raw + id * a.segs_per_block;
    const cu32 segm = as_const(a.c->seg);
    uint32_t acc = raw[0];
    for (uint32_t s = 1; s < nseg; ++s) {
        const uint64_t sl = s + 1 < nseg ? a.seg : blk_len - static_cast<uint64_t>(s) * a.seg;
        acc = (sl == a.seg ? apply(segm, acc) : shift_n(a.c, acc, sl)) ^ raw[s];
    }
    out[id] = ~(shift_n(a.c, ~seed, real_len) ^ acc);
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
        for (int j = 0; j < 8; ++j) v = (v & 1u) ? (v >> 1) ^ kCrcPoly : v >> 1;
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
    for (int v = 0; v < 2; ++v) {  // lane chunks of LC = 64 (v = 0) and 32 (v = 1) bytes
        const uint64_t lc = v == 0 ? 64 : 32;
        const Mat32 mg = mat_pow(p, 64 * lc - lc);
        for (int j = 0; j < 32; ++j) c->gap[v][j] = mg.col[j];
        for (int l = 0; l < 6; ++l) {
            const Mat32 m = mat_pow(p, lc << l);
            for (int j = 0; j < 32; ++j) c->wlvl[v][l][j] = m.col[j];
        }
    }
}

std::mutex g_mu;
std::map<std::pair<int, uint64_t>, CrcConsts*> g_consts;  // device copies, process lifetime

}  // namespace

void crc_shift_matrix(uint64_t n, uint32_t col[32]) {
    uint32_t t0[256];
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t v = i;
        for (int j = 0; j < 8; ++j) v = (v & 1u) ? (v >> 1) ^ kCrcPoly : v >> 1;
        t0[i] = v;
    }
    Mat32 p[kPow2];
    p[0] = shift_one_byte(t0);
    for (int i = 1; i < kPow2; ++i) p[i] = mat_mul(p[i - 1], p[i - 1]);
    const Mat32 m = mat_pow(p, n);
    for (int i = 0; i < 32; ++i) col[i] = m.col[i];
}

hipError_t crc_consts_for(uint64_t seg, const CrcConsts** out) {
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
        if ((e = rt::upload_pinned(d, &host, sizeof(CrcConsts))) != hipSuccess) {
            (void)hipFree(d);
            return e;
        }
        slot = d;
    }
    *out = slot;
    return hipSuccess;
}

hipError_t crc_combine(const CrcConsts* c, const uint32_t* raw, uint64_t len, uint64_t block, uint64_t seg,
                       uint32_t nblocks, uint32_t segs_per_block, uint64_t total_blocks, uint32_t* out,
                       hipStream_t stream, uint64_t phase, const uint32_t* seeds) {
    SegArgs a{};
    a.len = len;
    a.phase = phase;
    a.seeds = seeds;
    a.block = block;
    a.seg = seg;
    a.nblocks = nblocks;
    a.segs_per_block = segs_per_block;
    a.c = c;
    a.raw = const_cast<uint32_t*>(raw);
    hipLaunchKernelGGL(crc_combine_kernel, dim3(static_cast<unsigned>((total_blocks + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, stream, a, total_blocks, out);
    return hipGetLastError();
}

hipError_t crc32c_blocks(const uint8_t* data, uint64_t stride, uint64_t batch, uint64_t len, uint64_t block,
                         uint64_t phase, const uint32_t* seeds, uint32_t* out, hipStream_t stream) {
    if (batch == 0 || len == 0) return hipSuccess;
    if (block == 0 || !data || !out || phase >= block) return hipErrorInvalidValue;
    if (block > len + phase) block = len + phase;  // one block; only its real length matters
    // Streaming kernel when every dwordx4 row load is 4-byte aligned (segments end at block
    // ends): blb's 65532-byte blocks and whole-shard frames of dword-multiple shards.
    const bool stream_ok = (reinterpret_cast<uintptr_t>(data) & 3u) == 0 && (stride & 3u) == 0 &&
                           (block & 3u) == 0 && (len & 3u) == 0 && (phase & 3u) == 0;
    const uint64_t seg = stream_ok ? kWaveSeg : (block < kSegMax ? block : kSegMax);
    const CrcConsts* c = nullptr;
    hipError_t e = crc_consts_for(seg, &c);
    if (e != hipSuccess) return e;
    SegArgs a{};
    a.data = data;
    a.stride = stride;
    a.len = len;
    a.block = block;
    a.seg = seg;
    a.nblocks = static_cast<uint32_t>((len + phase + block - 1) / block);
    a.segs_per_block = static_cast<uint32_t>((block + seg - 1) / seg);
    a.c = c;
    a.phase = phase;
    a.seeds = seeds;
    const uint64_t total_blocks = batch * a.nblocks;
    const uint64_t total_segs = total_blocks * a.segs_per_block;
    if (total_segs > 0x7FFFFFFFull) return hipErrorInvalidValue;
    if ((e = hipMallocAsync(reinterpret_cast<void**>(&a.raw), total_segs * 4, stream)) != hipSuccess) return e;
    if (stream_ok) {
        static thread_local int cus = 0;
        if (!cus) {
            int dev = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
                cus = 256;
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(crc_stream_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kStreamLds));
        }
        StreamArgs sa{data, stride, len, block, a.nblocks, a.segs_per_block, total_segs, c, a.raw, phase};
        const uint64_t waves_needed = (total_segs + 15) / 16;  // 16 waves per workgroup
        const unsigned grid = static_cast<unsigned>(waves_needed < static_cast<uint64_t>(cus) ? waves_needed : cus);
        hipLaunchKernelGGL(crc_stream_kernel, dim3(grid), dim3(kStreamThreads), kStreamLds, stream, sa);
    } else {
        hipLaunchKernelGGL(crc_segment_kernel, dim3(static_cast<unsigned>(total_segs)), dim3(kThreads), kLdsBytes,
                           stream, a);
    }
    e = hipGetLastError();
    if (e == hipSuccess)
        e = crc_combine(c, a.raw, len, block, seg, a.nblocks, a.segs_per_block, total_blocks, out, stream, phase,
                        seeds);
    hipError_t f = hipFreeAsync(a.raw, stream);
    return e != hipSuccess ? e : f;
}

}  // namespace blbrs
