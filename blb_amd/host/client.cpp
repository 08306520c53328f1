// client.cpp -- degraded read with client-side RS reconstruction (see client.hpp).
#include "client.hpp"

#include <algorithm>
#include <cstring>
#include <thread>

namespace client {

using core::Error;

Client::Client(TractserverTalker* ts, ReconstructBehavior rb)
    : ts_(ts), rb_(rb), sem_free_(rb.MaxInFlight > 0 ? rb.MaxInFlight : 1) {}

// reconstruct.go:166 makes a fresh encoder per call; the GPU encoder caches its device
// plans, so one per (n, m) is kept.
reedsolomon::Encoder* Client::encoder(int n, int m) {
    std::lock_guard<std::mutex> g(enc_mu_);
    auto& slot = encoders_[{n, m}];
    if (!slot) {
        auto [enc, err] = reedsolomon::New(n, m);
        if (err != reedsolomon::Err::None) return nullptr;
        slot = std::move(enc);
    }
    return slot.get();
}

// reconstruct.go:47-63
bool Client::shouldReconstruct(const TractPointer& tract) const {
    if (!rb_.Enabled) return false;
    int n = 0, m = 0;
    if (!core::RSParams(tract.Class, &n, &m)) return false;
    return static_cast<int>(tract.OtherHosts.size()) == n + m;
}

// client.go:1158-1205
TractResult Client::readOneTractRS(const TractPointer& tract, blb::Bytes thisB, int64_t thisOffset) {
    const core::TractID rsTract = tract.Chunk.ToTractID();
    const int length = std::min(static_cast<int>(thisB.len()), static_cast<int>(tract.Length));
    const int64_t offset = static_cast<int64_t>(tract.Offset) + thisOffset;
    auto [read, err] = ts_->ReadInto(tract.Host, rsTract, core::RSChunkVersion, thisB.slice(0, length), offset);
    if (err != Error::NoError && err != Error::ErrEOF) {
        if (!shouldReconstruct(tract)) return {static_cast<int>(thisB.len()), 0, err};
        return reconstructOneTract(tract, thisB, offset, length);
    }
    for (size_t i = read; i < thisB.len(); ++i) thisB[i] = 0;  // pad with zeros
    if (static_cast<int>(tract.Length) < static_cast<int>(thisB.len())) err = Error::ErrEOF;
    return {static_cast<int>(thisB.len()), read, err};
}

// reconstruct.go:65-195
TractResult Client::reconstructOneTract(const TractPointer& tract, blb::Bytes thisB, int64_t offset, int length) {
    {
        std::unique_lock<std::mutex> g(sem_mu_);
        sem_cv_.wait(g, [&] { return sem_free_ > 0; });
        --sem_free_;
    }
    struct Release {
        Client* c;
        ~Release() {
            std::lock_guard<std::mutex> g(c->sem_mu_);
            ++c->sem_free_;
            c->sem_cv_.notify_one();
        }
    } release{this};

    const int L = static_cast<int>(thisB.len());
    int n = 0, m = 0;
    core::RSParams(tract.Class, &n, &m);

    int targetIdx = -1;
    std::vector<int> requests;
    for (size_t i = 0; i < tract.OtherHosts.size(); ++i) {
        if (tract.OtherTSIDs[i] == tract.TSID) {
            targetIdx = static_cast<int>(i);
            continue;
        }
        if (tract.OtherHosts[i].empty()) continue;
        requests.push_back(static_cast<int>(i));
    }
    if (targetIdx < 0) return {L, 0, Error::ErrInvalidArgument};
    if (static_cast<int>(requests.size()) < n) return {L, 0, Error::ErrHostNotExist};

    // Fan out reads of all other pieces; the first n good replies win.  Go cancels the
    // context for the stragglers; here they finish and are dropped, and are joined before
    // returning so no read outlives the call.
    struct Piece {
        int idx;
        blb::Bytes res;
        Error err;
    };
    auto shared = std::make_shared<std::pair<std::mutex, std::vector<Piece>>>();
    auto cv = std::make_shared<std::condition_variable>();
    struct Joiner {
        std::vector<std::thread> t;
        ~Joiner() {
            for (auto& x : t) x.join();
        }
    } readers;
    for (int i : requests) {
        const core::TractID id = tract.BaseChunk.Add(i).ToTractID();
        const std::string host = tract.OtherHosts[i];
        readers.t.emplace_back([this, i, id, host, offset, length, shared, cv]() {
            auto [res, err] = ts_->Read(host, id, core::RSChunkVersion, length, offset);
            if ((err == Error::NoError || err == Error::ErrEOF) && static_cast<int>(res.len()) != length)
                err = Error::ErrShortRead;
            {
                std::lock_guard<std::mutex> g(shared->first);
                shared->second.push_back(Piece{i, res, err});
            }
            cv->notify_all();
        });
    }
    reedsolomon::Shards data(n + m);
    Error lastErr = Error::NoError;
    int inFlight = static_cast<int>(requests.size()), good = 0;
    size_t consumed = 0;
    while (good < n && inFlight > 0) {
        Piece p;
        {
            std::unique_lock<std::mutex> g(shared->first);
            cv->wait(g, [&] { return shared->second.size() > consumed; });
            p = shared->second[consumed++];
        }
        --inFlight;
        if (p.err != Error::NoError && p.err != Error::ErrEOF) {
            lastErr = p.err;
            continue;
        }
        ++good;
        data[p.idx] = p.res;
    }
    if (good < n) return {L, 0, lastErr};

    reedsolomon::Encoder* enc = encoder(n, m);
    if (!enc) return {L, 0, Error::ErrInvalidArgument};
    // Reconstruct into our destination: data[targetIdx] = thisB[0:0:length].
    data[targetIdx] = thisB.slice3(0, 0, length);
    const reedsolomon::Err e = enc->ReconstructData(data);
    const blb::Bytes& out = data[targetIdx];
    if (e != reedsolomon::Err::None || static_cast<int>(out.len()) != length || out.data() != thisB.data())
        return {L, 0, Error::ErrCorruptData};
    for (int i = length; i < L; ++i) thisB[i] = 0;
    {
        std::lock_guard<std::mutex> g(sem_mu_);
        ++reconstructs_;
    }
    return {L, length, length < L ? Error::ErrEOF : Error::NoError};
}

}  // namespace client
