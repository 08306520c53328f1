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

// Piece p is written at dst + p * dst_stride, piece_len bytes.  Asynchronous on `stream`.
hipError_t pack_pieces(uint8_t* dst, uint64_t dst_stride, uint64_t npieces, uint64_t piece_len,
                       const uint64_t* table_dev, hipStream_t stream);

}  // namespace blbrs
