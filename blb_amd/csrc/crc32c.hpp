// crc32c.hpp -- GPU CRC-32C (Castagnoli) of shard blocks, the checksum blb computes over
// every shard written on the RS path: 64 KiB ChecksumFile blocks of 65532 data bytes
// (pkg/disk/checksum_block.go:18-34,70-80) and bulk RPC frames (pkg/rpc/bulk_codec.go:47).
// Results equal Go's crc32.Checksum(block, crc32.MakeTable(crc32.Castagnoli)).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace blbrs {

// CRC of the file-aligned blocks of each of `batch` buffers (buffer b at data + b * stride,
// `len` bytes, starting `phase` < block bytes into its first block): nblocks =
// ceil((phase + len) / block), out[b * nblocks + j] = crc32.Update(j == 0 && seeds ?
// seeds[b] : 0, the buffer's bytes in block j).  All pointers are device pointers (seeds may
// be NULL); asynchronous on `stream`.  Returns hipSuccess or the first failure.
hipError_t crc32c_blocks(const uint8_t* data, uint64_t stride, uint64_t batch, uint64_t len, uint64_t block,
                         uint64_t phase, const uint32_t* seeds, uint32_t* out, hipStream_t stream);

}  // namespace blbrs
