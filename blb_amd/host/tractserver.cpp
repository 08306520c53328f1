// tractserver.cpp -- Store::RSEncode over the GPU engine (see tractserver.hpp).
#include "tractserver.hpp"

#include "rpc.hpp"

#include <algorithm>
#include <cstring>
#include <future>
#include <thread>

namespace tractserver {

using core::Error;

// store.go:1132-1142 -- Reconstruct then Verify, fused into one device round trip.
reedsolomon::Err reconstructAndVerify(reedsolomon::Encoder& enc, reedsolomon::Shards& data, bool* verified) {
    return enc.ReconstructAndVerify(data, verified);
}

bool checkTractSpec(const std::vector<core::PackTractSpec>& srcs, int length) {
    int end = 0;
    for (const auto& src : srcs) {
        if (!src.ID.IsValid() || src.From.empty() || src.Offset < end) return false;
        end = src.Offset + src.Length;
    }
    return length >= end;
}

Error Store::PackTracts(int length, const std::vector<core::PackTractSpec>& srcs, core::RSChunkID dest) {
    if (!dest.IsValid() || !checkTractSpec(srcs, length)) return Error::ErrInvalidArgument;
    const core::TractID destTract = dest.ToTractID();
    {
        std::lock_guard<std::mutex> g(mu_);
        tracts_.erase(destTract);  // removeTract
    }
    // The file ends at `length` when there are sources (the pad, store.go:974-980) and is
    // empty otherwise.  Its bytes come from the pinned pool (not zeroed), so every hole is
    // written explicitly, as the sparse file reads them: zeros.
    const size_t size = srcs.empty() ? 0 : static_cast<size_t>(length);
    blb::Bytes piece = size ? rpc::GetBuffer(size) : blb::Bytes::make(0);
    size_t cursor = 0;
    for (const auto& src : srcs) {
        bool pulled = false;
        for (const auto& from : src.From) {
            // Ask for TractLength and compare with src.Length, so that a tract of an
            // unexpected length is caught (store.go:953-962).
            auto [b, err] = tt_->CtlRead(from.Host, src.ID, src.Version, static_cast<int>(core::TractLength), 0);
            if ((err == Error::NoError || err == Error::ErrEOF) && static_cast<int>(b.len()) == src.Length) {
                std::memset(piece.data() + cursor, 0, static_cast<size_t>(src.Offset) - cursor);
                if (src.Length) std::memcpy(piece.data() + src.Offset, b.data(), static_cast<size_t>(src.Length));
                cursor = static_cast<size_t>(src.Offset + src.Length);
                pulled = true;
                break;
            }
        }
        if (!pulled) return Error::ErrRPC;  // the half-written file is deleted
    }
    if (size > cursor) std::memset(piece.data() + cursor, 0, size - cursor);
    std::lock_guard<std::mutex> g(mu_);
    tracts_[destTract] = Local{piece, core::RSChunkVersion};
    return Error::NoError;
}

std::pair<blb::Bytes, Error> Store::Read(core::TractID id, int version, int length, int64_t off) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = tracts_.find(id);
    if (it == tracts_.end()) return {blb::Bytes(), Error::ErrNoSuchTract};
    if (it->second.version != version) return {blb::Bytes(), Error::ErrVersionMismatch};
    const blb::Bytes& d = it->second.data;
    const size_t start = std::min(static_cast<size_t>(std::max<int64_t>(off, 0)), d.len());
    const size_t n = std::min(static_cast<size_t>(std::max(length, 0)), d.len() - start);
    blb::Bytes out = rpc::GetBuffer(n);
    if (n) std::memcpy(out.data(), d.data() + start, n);
    return {out, static_cast<int>(n) < length ? Error::ErrEOF : Error::NoError};
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
