// pack.hpp -- device assembly of packed RS data pieces, the byte work of blb's
// Store.PackTracts (internal/tractserver/store.go:922-994): every source tract lands at its
// offset in the piece, and every byte not covered by a tract (the holes before/between
// tracts, and the pad up to the piece length, store.go:974-980) is zero -- exactly the
// contents of the packed chunk file that RSEncode later reads.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace blbrs {

// Extent table layout (device, uint64 words):
//   [0, npieces]            first extent index of each piece (piece p owns [t[p], t[p+1]))
//   then 4 words per extent {src address, dst offset, length, piece}, sorted by
//   (piece, offset), non-overlapping and inside piece_len (validated on the host).
constexpr uint32_t kPackTile = 64u * 1024u;  // destination bytes per workgroup
constexpr int kPackThreads = 256;

// Piece p is written at dst + p * dst_stride, piece_len bytes (per_group > 0: at
// dst + (p / per_group) * group_stride + (p % per_group) * dst_stride -- data shard j of
// stripe b for per_group = k).  Asynchronous on `stream`.
hipError_t pack_pieces(uint8_t* dst, uint64_t dst_stride, uint64_t npieces, uint64_t piece_len,
                       const uint64_t* table_dev, hipStream_t stream, uint32_t per_group = 0,
                       uint64_t group_stride = 0);

// PackTracts fused with Encode (pack_encode.hip): the k data shards of each of B strided
// stripes are assembled from the extent table (piece b * k + j = data shard j of stripe b,
// same table layout as above) and, in the same pass, the m parity shards are encoded from
// the assembled bytes -- the data pieces are written once and never read back.
struct PackEncodeArgs {
    const uint32_t* tables;   // device: encode pass v_perm tables [rows][k][5]
    const int32_t* out_idx;   // device: [rows] parity shard indices
    uint8_t* base;            // shard i of stripe b at base + b * stripe_stride + i * shard_stride
    uint64_t shard_stride, stripe_stride, S;
    uint32_t B, k, rows;
    const uint64_t* table;    // device extent table (pieces = B * k)
    uint64_t nextents;        // extents in the table
    bool parity = false;      // tables are encode parity rows 0..rows-1 of k (gf_bitslice.hpp)
    void* scratch = nullptr;  // device: >= pack_encode_scratch_bytes(*this), free for this launch
};
// Device scratch the launch needs (the per-(piece, tile) layout descriptors of its pre-pass).
size_t pack_encode_scratch_bytes(const PackEncodeArgs& a);
// True when a fused instantiation covers the shape (k in blb's list, rows <= 5, 16-byte
// aligned base and strides); otherwise the caller packs, then encodes.
bool pack_encode_supported(const PackEncodeArgs& a);
hipError_t launch_pack_encode(const PackEncodeArgs& a, hipStream_t stream);

}  // namespace blbrs
