// rpc.hpp -- rpc.GetBuffer (pkg/rpc/pool.go:28-43) for the C++ mirror, over the engine's
// pinned buffer pool (blbrs_buffer_get): pooled, NOT zeroed, capacity classes of 1, 4 and
// 8 MiB + 64 KiB.  Shards on such buffers are coded in place by the GPU (zero-copy).  The
// buffer goes back to the pool when the last Bytes holding it is dropped -- the
// PutBuffer(b, true) of store.go:1048-1052, and a Bytes that is simply dropped releases it
// too (the GC semantics blb relies on: reconstruct.go:126-152 drops straggling replies).
// Without a usable GPU, or past the engine's pinned live limit (BLBRS_ERR_LIMIT), it falls
// back to make(): pageable memory, which the engine stages.
#pragma once
#include <cstring>

#include "../../include/blb_rs.h"
#include "bytes.hpp"

namespace rpc {

inline blb::Bytes GetBuffer(size_t n) {
    uint8_t* p = nullptr;
    size_t cap = 0;
    if (n == 0 || blbrs_buffer_get(n, &p, &cap) != BLBRS_OK) return blb::Bytes::make(n);
    return blb::Bytes::adopt(p, n, cap, [](uint8_t* q) { (void)blbrs_buffer_put(q); });
}

}  // namespace rpc
