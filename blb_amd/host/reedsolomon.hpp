// reedsolomon.hpp -- C++ mirror of github.com/klauspost/reedsolomon's Encoder (the
// interface blb binds, /root/reference/go.mod:20) over the MI355X engine's C ABI
// (include/blb_rs.h).  Same names, argument meaning and error values:
//
//   auto [enc, err] = reedsolomon::New(N, M);      // internal/tractserver/store.go:1022
//   err = enc->Encode(shards);                     // store.go:1099
//   err = enc->Reconstruct(shards);                // store.go:1133
//   auto [ok, verr] = enc->Verify(shards);         // store.go:1136
//   err = enc->ReconstructData(shards);            // client/blb/reconstruct.go:173
//
// shards is a std::vector<blb::Bytes> (Go [][]byte): len 0 = missing; a missing shard with
// cap >= size is resliced in place, otherwise a new buffer is made -- exactly klauspost.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "bytes.hpp"

struct blbrs_encoder;

namespace reedsolomon {

enum class Err {
    None = 0,
    ErrInvShardNum,   // "cannot create Encoder with zero or less data/parity shards"
    ErrMaxShardNum,   // "cannot create Encoder with more than 256 data+parity shards"
    ErrTooFewShards,  // "too few shards given"
    ErrShardNoData,   // "no shard data"
    ErrShardSize,     // "shard sizes do not match"
    ErrSingular,      // "matrix is singular"
    ErrEngine,        // HIP / device failure (no GPU, launch error, ...)
};

const char* ErrString(Err e);

using Shards = std::vector<blb::Bytes>;

class Encoder {
 public:
    ~Encoder();
    Encoder(const Encoder&) = delete;
    Encoder& operator=(const Encoder&) = delete;

    Err Encode(Shards& shards);
    std::pair<bool, Err> Verify(const Shards& shards);
    Err Reconstruct(Shards& shards);
    Err ReconstructData(Shards& shards);
    // Extension: reconstructAndVerify (internal/tractserver/store.go:1132-1142) in one
    // device round trip.  *ok = false is errVerifyFailed.
    Err ReconstructAndVerify(Shards& shards, bool* ok);

    int DataShards() const { return k_; }
    int ParityShards() const { return m_; }
    int TotalShards() const { return k_ + m_; }
    // Detail of the last ErrEngine on this thread.
    static std::string LastEngineError();

 private:
    friend std::pair<std::unique_ptr<Encoder>, Err> New(int, int);
    Encoder(blbrs_encoder* h, int k, int m) : h_(h), k_(k), m_(m) {}
    Err reconstruct(Shards& shards, bool data_only, bool* verify_ok);
    blbrs_encoder* h_;
    int k_, m_;
};

// reedsolomon.New(dataShards, parityShards)
std::pair<std::unique_ptr<Encoder>, Err> New(int dataShards, int parityShards);

// Extension (the Go shim's rsgpu.EnableBatching): every encoder New returns afterwards routes
// its Encode / Verify / Reconstruct / ReconstructData through one process-wide batcher
// (blbrs_batcher_new), so concurrent RSEncode RPCs and degraded reads share kernel
// launches.  windowMicros = 0 batches naturally.  DisableBatching frees it: call it only once
// every encoder made while batching was on has been destroyed.
Err EnableBatching(int maxBatch, int windowMicros);
void DisableBatching();
// Calls served and kernel launches issued by the batcher so far (0, 0 when off).
void BatchingStats(uint64_t* requests, uint64_t* launches);

}  // namespace reedsolomon
