// client.hpp -- C++ mirror of blb's client-side degraded read over the MI355X engine:
// readOneTractRS (client/blb/client.go:1158-1205), shouldReconstruct and
// reconstructOneTract (client/blb/reconstruct.go:47-195).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "bytes.hpp"
#include "core.hpp"
#include "reedsolomon.hpp"

namespace client {

// core.TractPointer (internal/core/messages.go:54-68)
struct TractPointer {
    core::RSChunkID Chunk;
    std::string Host;
    uint64_t TSID = 0;
    uint32_t Offset = 0;
    uint32_t Length = 0;
    core::StorageClass Class = core::StorageClass::REPLICATED;
    core::RSChunkID BaseChunk;
    std::vector<std::string> OtherHosts;
    std::vector<uint64_t> OtherTSIDs;
};

// tractResult{len, read, err}
struct TractResult {
    int len = 0;
    int read = 0;
    core::Error err = core::Error::NoError;
};

// The two TractserverTalker calls of the RS read path (client/blb/tractserver_talker.go).
// ctx is cancelled once a reconstruct has the n pieces it needs (reconstruct.go:154); a
// talker may return early then.
class TractserverTalker {
 public:
    virtual ~TractserverTalker() = default;
    virtual std::pair<blb::Bytes, core::Error> Read(const core::ContextPtr& ctx, const std::string& addr,
                                                    core::TractID id, int version, int length, int64_t off) = 0;
    virtual std::pair<int, core::Error> ReadInto(const core::ContextPtr& ctx, const std::string& addr,
                                                 core::TractID id, int version, blb::Bytes b, int64_t off) = 0;
};

// reconstruct.go:24-28
struct ReconstructBehavior {
    bool Enabled = true;
    int MaxInFlight = 0;  // 0 -> defaultMaxReconstructInFlight = 1
};

class Client {
 public:
    Client(TractserverTalker* ts, ReconstructBehavior rb);
    // Waits for straggler piece reads still running (they were cancelled when their
    // reconstruct returned), so none outlives the client or its talker.
    ~Client();
    bool shouldReconstruct(const TractPointer& tract) const;
    TractResult readOneTractRS(const core::ContextPtr& ctx, const TractPointer& tract, blb::Bytes thisB,
                               int64_t thisOffset);
    TractResult reconstructOneTract(const core::ContextPtr& ctx, const TractPointer& tract, blb::Bytes thisB,
                                    int64_t offset, int length);
    int Reconstructs() const { return reconstructs_; }
    // Piece reads started by reconstructs and not finished yet.
    int OutstandingReads() const;

 private:
    struct Readers {
        std::mutex mu;
        std::condition_variable cv;
        int running = 0;
    };
    std::shared_ptr<Readers> readers_ = std::make_shared<Readers>();
    reedsolomon::Encoder* encoder(int n, int m);
    TractserverTalker* ts_;
    ReconstructBehavior rb_;
    // server.Semaphore(MaxInFlight)
    std::mutex sem_mu_;
    std::condition_variable sem_cv_;
    int sem_free_;
    std::mutex enc_mu_;
    std::map<std::pair<int, int>, std::unique_ptr<reedsolomon::Encoder>> encoders_;
    int reconstructs_ = 0;
};

}  // namespace client
