// client.cpp -- degraded read with client-side RS reconstruction (see client.hpp).
#include "client.hpp"

#include <algorithm>
#include <cstring>
#include <thread>

namespace client {

using core::Error;

Client::Client(TractserverTalker* ts, ReconstructBehavior rb)
    : ts_(ts), rb_(rb), sem_free_(rb.MaxInFlight > 0 ? rb.MaxInFlight : 1) {}

Client::~Client() {
    std::unique_lock<std::mutex> g(readers_->mu);
    readers_->cv.wait(g, [&] { return readers_->running == 0; });
}

int Client::OutstandingReads() const {
    std::lock_guard<std::mutex> g(readers_->mu);
    return readers_->running;
}

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
TractResult Client::readOneTractRS(const core::ContextPtr& ctx, const TractPointer& tract, blb::Bytes thisB,
                                   int64_t thisOffset) {
    const core::TractID rsTract = tract.Chunk.ToTractID();
    const int length = std::min(static_cast<int>(thisB.len()), static_cast<int>(tract.Length));
    const int64_t offset = static_cast<int64_t>(tract.Offset) + thisOffset;
    auto [read, err] = ts_->ReadInto(ctx, tract.Host, rsTract, core::RSChunkVersion, thisB.slice(0, length), offset);
    if (err != Error::NoError && err != Error::ErrEOF) {
        if (!shouldReconstruct(tract)) return {static_cast<int>(thisB.len()), 0, err};
        return reconstructOneTract(ctx, tract, thisB, offset, length);
    }
    for (size_t i = read; i < thisB.len(); ++i) thisB[i] = 0;  // pad with zeros
    if (static_cast<int>(tract.Length) < static_cast<int>(thisB.len())) err = Error::ErrEOF;
    return {static_cast<int>(thisB.len()), read, err};
}

// reconstruct.go:65-195
TractResult Client::reconstructOneTract(const core::ContextPtr& ctx, const TractPointer& tract, blb::Bytes thisB,
                                        int64_t offset, int length) {
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

    // Fan out reads of all other pieces; the first n good replies win.  As in Go
    // (reconstruct.go:119,154) the reads get a child context that is cancelled as soon as
    // n good pieces are in, and the call returns without waiting for the stragglers; their
    // replies land in the shared mailbox and are dropped with it.  ~Client waits for any
    // still running, so none outlives the client or its talker.
    struct Piece {
        int idx;
        blb::Bytes res;
        Error err;
    };
    struct Mailbox {
        std::mutex mu;
        std::condition_variable cv;
        std::vector<Piece> pieces;
    };
    auto box = std::make_shared<Mailbox>();
    auto nctx = core::Background();  // context.WithCancel(ctx)
    if (ctx && ctx->Done()) nctx->Cancel();
    struct CancelOnReturn {
        core::ContextPtr c;
        ~CancelOnReturn() { c->Cancel(); }
    } cancel{nctx};
    for (int i : requests) {
        const core::TractID id = tract.BaseChunk.Add(i).ToTractID();
        const std::string host = tract.OtherHosts[i];
        {
            std::lock_guard<std::mutex> g(readers_->mu);
            ++readers_->running;
        }
        std::thread([ts = ts_, readers = readers_, i, id, host, offset, length, box, nctx]() {
            auto [res, err] = ts->Read(nctx, host, id, core::RSChunkVersion, length, offset);
            if ((err == Error::NoError || err == Error::ErrEOF) && static_cast<int>(res.len()) != length)
                err = Error::ErrShortRead;
            {
                std::lock_guard<std::mutex> g(box->mu);
                box->pieces.push_back(Piece{i, res, err});
            }
            box->cv.notify_all();
            std::lock_guard<std::mutex> g(readers->mu);
            if (--readers->running == 0) readers->cv.notify_all();
        }).detach();
    }
    reedsolomon::Shards data(n + m);
    Error lastErr = Error::NoError;
    int inFlight = static_cast<int>(requests.size()), good = 0;
    size_t consumed = 0;
    while (good < n && inFlight > 0) {
        Piece p;
        {
            std::unique_lock<std::mutex> g(box->mu);
            box->cv.wait(g, [&] { return box->pieces.size() > consumed; });
            p = box->pieces[consumed++];
        }
        --inFlight;
        if (p.err != Error::NoError && p.err != Error::ErrEOF) {
            lastErr = p.err;
            continue;
        }
        ++good;
        data[p.idx] = p.res;
    }
    nctx->Cancel();  // reconstruct.go:154
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
