// reedsolomon.cpp -- the Encoder mirror over include/blb_rs.h (see reedsolomon.hpp).
#include "reedsolomon.hpp"

#include <atomic>
#include <vector>

#include "../../include/blb_rs.h"

namespace reedsolomon {

namespace {

Err map_rc(int rc) {
    switch (rc) {
        case BLBRS_OK: return Err::None;
        case BLBRS_ERR_INV_SHARD_NUM: return Err::ErrInvShardNum;
        case BLBRS_ERR_MAX_SHARD_NUM: return Err::ErrMaxShardNum;
        case BLBRS_ERR_TOO_FEW_SHARDS: return Err::ErrTooFewShards;
        case BLBRS_ERR_SHARD_NO_DATA: return Err::ErrShardNoData;
        case BLBRS_ERR_SHARD_SIZE: return Err::ErrShardSize;
        case BLBRS_ERR_SINGULAR: return Err::ErrSingular;
        default: return Err::ErrEngine;
    }
}

// reedsolomon.go shardSize: first non-zero length.
size_t shard_size(const Shards& shards) {
    for (const auto& s : shards)
        if (s.len() != 0) return s.len();
    return 0;
}

}  // namespace

const char* ErrString(Err e) {
    switch (e) {
        case Err::None: return "<nil>";
        case Err::ErrInvShardNum: return "cannot create Encoder with zero or less data/parity shards";
        case Err::ErrMaxShardNum: return "cannot create Encoder with more than 256 data+parity shards";
        case Err::ErrTooFewShards: return "too few shards given";
        case Err::ErrShardNoData: return "no shard data";
        case Err::ErrShardSize: return "shard sizes do not match";
        case Err::ErrSingular: return "matrix is singular";
        case Err::ErrEngine: return "engine error";
    }
    return "unknown";
}

std::string Encoder::LastEngineError() { return blbrs_last_error(); }

namespace {
std::atomic<blbrs_batcher*> g_batcher{nullptr};
}

Err EnableBatching(int maxBatch, int windowMicros) {
    blbrs_batcher* b = nullptr;
    const int rc = blbrs_batcher_new(maxBatch, windowMicros, &b);
    if (rc != BLBRS_OK) return map_rc(rc);
    blbrs_batcher* none = nullptr;
    if (!g_batcher.compare_exchange_strong(none, b)) {  // already on: keep the first
        blbrs_batcher_free(b);
    }
    return Err::None;
}

void DisableBatching() {
    if (blbrs_batcher* b = g_batcher.exchange(nullptr)) blbrs_batcher_free(b);
}

void BatchingStats(uint64_t* requests, uint64_t* launches) {
    *requests = *launches = 0;
    if (blbrs_batcher* b = g_batcher.load()) blbrs_batcher_stats(b, requests, launches);
}

std::pair<std::unique_ptr<Encoder>, Err> New(int dataShards, int parityShards) {
    blbrs_encoder* h = nullptr;
    const int rc = blbrs_new(dataShards, parityShards, &h);
    if (rc != BLBRS_OK) return {nullptr, map_rc(rc)};
    if (blbrs_batcher* b = g_batcher.load()) blbrs_encoder_set_batcher(h, b);
    return {std::unique_ptr<Encoder>(new Encoder(h, dataShards, parityShards)), Err::None};
}

Encoder::~Encoder() { blbrs_free(h_); }

Err Encoder::Encode(Shards& shards) {
    if (static_cast<int>(shards.size()) != TotalShards()) return Err::ErrTooFewShards;
    std::vector<uint8_t*> ptrs(shards.size());
    std::vector<size_t> lens(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
        ptrs[i] = shards[i].data();
        lens[i] = shards[i].len();
    }
    return map_rc(blbrs_encode(h_, ptrs.data(), lens.data()));
}

std::pair<bool, Err> Encoder::Verify(const Shards& shards) {
    if (static_cast<int>(shards.size()) != TotalShards()) return {false, Err::ErrTooFewShards};
    std::vector<const uint8_t*> ptrs(shards.size());
    std::vector<size_t> lens(shards.size());
    for (size_t i = 0; i < shards.size(); ++i) {
        ptrs[i] = shards[i].data();
        lens[i] = shards[i].len();
    }
    int ok = 0;
    const int rc = blbrs_verify(h_, ptrs.data(), lens.data(), &ok);
    if (rc != BLBRS_OK) return {false, map_rc(rc)};
    return {ok != 0, Err::None};
}

Err Encoder::reconstruct(Shards& shards, bool data_only, bool* verify_ok) {
    const int n = TotalShards();
    if (static_cast<int>(shards.size()) != n) return Err::ErrTooFewShards;
    const size_t size = shard_size(shards);
    int present = 0;
    for (const auto& s : shards) present += s.len() != 0;
    // Outputs exist only once the argument checks would pass (klauspost allocates after
    // them); error cases are left to the engine, which reports the same error value.
    if (size != 0 && present >= k_ && present < n) {
        for (int i = 0; i < n; ++i) {
            if (shards[i].len() != 0 || !(i < k_ || !data_only)) continue;
            if (shards[i].cap() >= size) shards[i] = shards[i].slice(0, 0);  // keep backing array
            else shards[i] = blb::Bytes::make(0, size);
        }
    }
    std::vector<uint8_t*> ptrs(n);
    std::vector<size_t> lens(n);
    for (int i = 0; i < n; ++i) {
        ptrs[i] = shards[i].data();
        lens[i] = shards[i].len();
    }
    int ok = 0;
    const int rc = verify_ok ? blbrs_reconstruct_verify(h_, ptrs.data(), lens.data(), &ok)
                   : data_only ? blbrs_reconstruct_data(h_, ptrs.data(), lens.data())
                               : blbrs_reconstruct(h_, ptrs.data(), lens.data());
    if (rc != BLBRS_OK) return map_rc(rc);
    if (verify_ok) *verify_ok = ok != 0;
    for (int i = 0; i < n; ++i)
        if (shards[i].len() == 0 && lens[i] != 0) shards[i] = shards[i].slice(0, size);
    return Err::None;
}

Err Encoder::Reconstruct(Shards& shards) { return reconstruct(shards, false, nullptr); }
Err Encoder::ReconstructData(Shards& shards) { return reconstruct(shards, true, nullptr); }
Err Encoder::ReconstructAndVerify(Shards& shards, bool* ok) {
    *ok = false;
    return reconstruct(shards, false, ok);
}

}  // namespace reedsolomon
