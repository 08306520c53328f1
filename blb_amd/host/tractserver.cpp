// tractserver.cpp -- Store::RSEncode over the GPU engine (see tractserver.hpp).
#include "tractserver.hpp"

#include "rpc.hpp"

#include <algorithm>
#include <future>
#include <thread>

namespace tractserver {

using core::Error;

// store.go:1132-1142 -- Reconstruct then Verify, fused into one device round trip.
reedsolomon::Err reconstructAndVerify(reedsolomon::Encoder& enc, reedsolomon::Shards& data, bool* verified) {
    return enc.ReconstructAndVerify(data, verified);
}

Error Store::RSEncode(core::RSChunkID baseid, int length, const std::vector<core::TSAddr>& srcs,
                      const std::vector<core::TSAddr>& dests, const std::vector<int>& indexMap) {
    const int N = static_cast<int>(srcs.size()), M = static_cast<int>(dests.size());
    const int increment = cfg_.EncodeIncrementSize;
    if (!baseid.IsValid() || !baseid.Add(N + M - 1).IsValid()) return Error::ErrInvalidArgument;
    auto [enc, e] = reedsolomon::New(N, M);
    if (e != reedsolomon::Err::None) return Error::ErrInvalidArgument;  // store.go:1023-1026

    bool encode = false;
    std::vector<int> imap = indexMap;
    if (imap.empty()) {
        encode = true;  // identity map (store.go:1054-1061)
        imap.resize(N + M);
        for (int i = 0; i < N + M; ++i) imap[i] = i;
    } else if (static_cast<int>(imap.size()) != N + M) {
        return Error::ErrInvalidArgument;
    }

    std::vector<std::pair<int64_t, int>> windows;
    for (int64_t off = 0; length > 0;) {
        const int l = std::min(length, increment);
        windows.emplace_back(off, l);
        length -= l;
        off += l;
    }
    if (!cfg_.Pipeline) {
        for (auto [off, l] : windows) {
            Error err = rsEncodeOne(baseid, off, l, srcs, dests, imap, encode, *enc);
            if (err != Error::NoError) return err;
        }
        return Error::NoError;
    }

    // Pipelined: window i+1's reads run while window i's writes are in flight, and window
    // i's coding overlaps window i-1's writes.  Window i+1's reads start only once window i
    // has been coded AND window i-1's writes have succeeded, so a failing read or coding
    // step issues exactly the reference's calls (store.go:1029-1036 stops at the first
    // failing window).  The one difference: when a CtlWrite of window i-1 fails, window i's
    // reads have already been issued (side-effect free); no write of window i is ever sent.
    if (windows.empty()) return Error::NoError;
    auto start_gather = [&](size_t i) {
        auto w = std::make_shared<Window>();
        w->offset = windows[i].first;
        w->length = windows[i].second;
        return std::async(std::launch::async, [this, w, baseid, &srcs, &imap, N, M]() {
            w->err = gather(baseid, srcs, imap, N, M, *w);
            return w;
        });
    };
    auto next = start_gather(0);
    std::future<Error> pending_write;
    Error result = Error::NoError;
    for (size_t i = 0; i < windows.size(); ++i) {
        std::shared_ptr<Window> w = next.get();
        if (w->err != Error::NoError) { result = w->err; break; }
        Error err = code(*enc, encode, imap, N, *w);
        if (err != Error::NoError) { result = err; break; }
        if (pending_write.valid()) {
            err = pending_write.get();
            if (err != Error::NoError) { result = err; break; }
        }
        if (i + 1 < windows.size()) next = start_gather(i + 1);
        pending_write = std::async(std::launch::async, [this, w, baseid, &dests, &imap, N]() {
            return scatter(baseid, dests, imap, N, *w);
        });
    }
    if (next.valid()) next.wait();
    if (pending_write.valid()) {
        Error err = pending_write.get();
        if (result == Error::NoError) result = err;
    }
    return result;
}

// store.go:1066-1090: N concurrent CtlReads into data[indexMap[i]].
Error Store::gather(core::RSChunkID baseid, const std::vector<core::TSAddr>& srcs, const std::vector<int>& imap,
                    int N, int M, Window& w) {
    w.data.assign(N + M, blb::Bytes());
    std::vector<Error> errs(N, Error::NoError);
    std::vector<std::thread> th;
    th.reserve(N);
    for (int srcI = 0; srcI < N; ++srcI) {
        th.emplace_back([&, srcI]() {
            const int dataI = imap[srcI];
            const core::TractID id = baseid.Add(dataI).ToTractID();
            auto [b, err] = tt_->CtlRead(srcs[srcI].Host, id, core::RSChunkVersion, w.length, w.offset);
            if (err != Error::NoError && err != Error::ErrEOF) {
                errs[srcI] = err;
            } else if (static_cast<int>(b.len()) != w.length) {
                errs[srcI] = Error::ErrVersionMismatch;
            } else {
                w.data[dataI] = b;
            }
        });
    }
    for (auto& t : th) t.join();
    for (Error e : errs)
        if (e != Error::NoError) return e;
    return Error::NoError;
}

// store.go:1092-1108: Encode into fresh (pooled, un-zeroed) parity buffers, or
// reconstructAndVerify; any coding error is ErrUnknown.  The parity buffers come from
// rpc::GetBuffer (pinned pool), so the GPU writes them in place.
Error Store::code(reedsolomon::Encoder& enc, bool encode, const std::vector<int>& imap, int N, Window& w) {
    if (encode) {
        for (size_t j = N; j < imap.size(); ++j) {
            blb::Bytes b = rpc::GetBuffer(w.length);
            std::fill(b.data(), b.data() + b.len(), uint8_t{0xA5});  // rpc.GetBuffer: stale contents
            w.data[imap[j]] = b;
        }
        return enc.Encode(w.data) == reedsolomon::Err::None ? Error::NoError : Error::ErrUnknown;
    }
    bool verified = false;
    if (reconstructAndVerify(enc, w.data, &verified) != reedsolomon::Err::None || !verified)
        return Error::ErrUnknown;
    return Error::NoError;
}

// store.go:1110-1127: CtlWrite data[dataI] for every dest with dataI >= 0 and ID != 0.
Error Store::scatter(core::RSChunkID baseid, const std::vector<core::TSAddr>& dests, const std::vector<int>& imap,
                     int N, Window& w) {
    const int M = static_cast<int>(dests.size());
    std::vector<Error> errs(M, Error::NoError);
    std::vector<std::thread> th;
    for (int destI = 0; destI < M; ++destI) {
        const int dataI = imap[N + destI];
        if (dataI < 0 || dests[destI].ID == 0) continue;
        th.emplace_back([&, destI, dataI]() {
            const core::TractID id = baseid.Add(dataI).ToTractID();
            errs[destI] = tt_->CtlWrite(dests[destI].Host, id, core::RSChunkVersion, w.offset, w.data[dataI]);
        });
    }
    for (auto& t : th) t.join();
    for (Error e : errs)
        if (e != Error::NoError) return e;
    return Error::NoError;
}

Error Store::rsEncodeOne(core::RSChunkID baseid, int64_t offset, int length, const std::vector<core::TSAddr>& srcs,
                         const std::vector<core::TSAddr>& dests, const std::vector<int>& imap, bool encode,
                         reedsolomon::Encoder& enc) {
    const int N = static_cast<int>(srcs.size()), M = static_cast<int>(dests.size());
    Window w;
    w.offset = offset;
    w.length = length;
    if (Error e = gather(baseid, srcs, imap, N, M, w); e != Error::NoError) return e;
    if (Error e = code(enc, encode, imap, N, w); e != Error::NoError) return e;
    return scatter(baseid, dests, imap, N, w);
}

}  // namespace tractserver
