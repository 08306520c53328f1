// encode_crc.hpp -- fused RS encode + CRC-32C of the parity it writes (encode_crc.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace blbrs {

// One pass over HBM: parity rows out[j] = XOR_c coef[j][c] * in[c] of every stripe are
// stored, and CRC-32C of every `block`-byte block of every parity shard is written to
// crc[(j * B + b) * nblocks + i] (Go's crc32.Checksum with the Castagnoli table).
struct EncodeCrcArgs {
    const uint32_t* tables;   // device: [rows][k][5] v_perm words (the encode pass)
    const int32_t* in_idx;    // device: [k]
    const int32_t* out_idx;   // device: [rows]
    uint8_t* base;            // strided stripes: shard i of stripe b at base + b*stripe_stride + i*shard_stride
    uint64_t shard_stride, stripe_stride;
    uint32_t B;
    uint64_t S;               // shard length
    uint64_t block;           // CRC block length
    int32_t k, rows;
    uint32_t* crc;            // device: [rows][B][nblocks], nblocks = ceil((phase + S) / block)
    uint64_t phase = 0;       // file offset of byte 0 of each shard, mod block (< block)
    const uint32_t* seeds = nullptr;  // device [rows][B]: crc32.Update seed of block 0, or NULL
    bool parity = false;      // rows are encode parity rows 0..rows-1 of k (gf_bitslice.hpp)
};

// True when a fused kernel covers this shape: the tile-grid kernel (below), or the segment
// kernel for an instantiated (k, rows) with 4-byte aligned base/strides/length/block and
// phase 0.  Otherwise the caller runs the coding pass and crc32c_blocks.
bool encode_crc_supported(const EncodeCrcArgs& a);

// Launches the fused kernel plus the per-block combine on `stream`: the tile-grid kernel
// (encode_crc_tile.hip) when it covers the shape, else the persistent segment kernel.
// knob BLBRS_EC_PERSISTENT=1 (tuning.hpp) forces the segment kernel (A/B measurements).
hipError_t launch_encode_crc(const EncodeCrcArgs& a, hipStream_t stream);

// The tile-grid form: k in {3, 4, 6, 8, 10, 12} and rows <= 5, 16-byte aligned base and
// strides, S a multiple of 16 (the last tile may be partial), block >= the tile (4 or 8 KiB),
// block and phase multiples of 4.
bool encode_crc_tile_supported(const EncodeCrcArgs& a);
hipError_t launch_encode_crc_tile(const EncodeCrcArgs& a, hipStream_t stream);

}  // namespace blbrs
