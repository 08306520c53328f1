// rs_test.cpp -- blb's RS tests, ported to the C++ mirror over the MI355X engine.
//
// TestPackTractsInvalid / TestPackTractsRPCError / TestPackTracts follow
// store_test.go:647-746 (golden bytes of the packed piece included); TestPackThenRSEncode
// runs the curator's encPack -> encEncode flow (internal/curator/pack_tracts.go:244-292):
// three data tractservers pack tracts into their pieces, a fourth RSEncodes them.
//
// TestRSEncode / TestRSReconstruct follow internal/tractserver/store_test.go:749-879 line
// for line (memTractserverTalker with scripted replies, RS(3,2), B=12000 in 5000-byte
// increments / B=20000 with pieces 1 and 3 missing and indexMap [0,2,4,1,3]), checked with
// the engine's Verify exactly as the Go test uses enc.Verify.  TestClientRecovery follows
// internal/testblb/test_rs_recovery.go's reads after a tractserver dies.
//
// usage: rs_test [--cpu]   (--cpu: only the tests that need no GPU)
#include <execinfo.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <csignal>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/blb_rs.h"
#include "../../blb_amd/host/client.hpp"
#include "../../blb_amd/host/reedsolomon.hpp"
#include "../../blb_amd/host/tractserver.hpp"

using blb::Bytes;
using core::Error;

// ---- a minimal testing.T ----
struct T {
    std::string name;
    bool failed = false;
    void Errorf(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
};
void T::Errorf(const char* fmt, ...) {
    failed = true;
    va_list ap;
    va_start(ap, fmt);
    std::fprintf(stderr, "    %s: ", name.c_str());
    std::vfprintf(stderr, fmt, ap);
    std::fprintf(stderr, "\n");
    va_end(ap);
}
#define Fatalf(...) do { t->Errorf(__VA_ARGS__); return; } while (0)

static Bytes randBytes(std::mt19937_64& rng, size_t n) {
    Bytes b = Bytes::make(n);
    for (size_t i = 0; i < n; ++i) b[i] = static_cast<uint8_t>(rng());
    return b;
}

static Bytes concat(const Bytes& a, const Bytes& b) {
    Bytes c = Bytes::make(a.len() + b.len());
    if (a.len()) std::memcpy(c.data(), a.data(), a.len());
    if (b.len()) std::memcpy(c.data() + a.len(), b.data(), b.len());
    return c;
}

// store_test.go:21-81
struct ReadReply { Bytes B; Error Err; };
struct WriteReq { core::TractID ID; int Version; Bytes B; int64_t Off; };

class memTractserverTalker : public tractserver::TractserverTalker {
 public:
    std::mutex mu;
    std::map<std::string, std::vector<ReadReply>> ctlReadReplies;
    std::map<std::string, std::vector<Error>> ctlWriteReplies;
    std::map<std::string, std::vector<WriteReq>> ctlWriteCalls;
    std::map<std::string, int> ctlReadCalls;

    void addCtlReadReply(const std::string& addr, const Bytes& origB, Error err) {
        std::lock_guard<std::mutex> g(mu);
        ctlReadReplies[addr].push_back({Bytes::copy_of(origB.data(), origB.len()), err});
    }
    void addCtlWriteReply(const std::string& addr, Error err) {
        std::lock_guard<std::mutex> g(mu);
        ctlWriteReplies[addr].push_back(err);
    }
    std::pair<Bytes, Error> CtlRead(const std::string& addr, core::TractID, int, int, int64_t) override {
        std::lock_guard<std::mutex> g(mu);
        ctlReadCalls[addr]++;
        auto& q = ctlReadReplies[addr];
        if (q.empty()) return {Bytes(), Error::ErrRPC};
        ReadReply r = q.front();
        q.erase(q.begin());
        return {r.B, r.Err};
    }
    Error CtlWrite(const std::string& addr, core::TractID id, int v, int64_t off, const Bytes& b) override {
        std::lock_guard<std::mutex> g(mu);
        ctlWriteCalls[addr].push_back({id, v, Bytes::copy_of(b.data(), b.len()), off});
        auto& q = ctlWriteReplies[addr];
        if (q.empty()) return Error::ErrRPC;
        Error e = q.front();
        q.erase(q.begin());
        return e;
    }
};

static std::vector<core::TSAddr> makeAddrs(int n) {
    std::vector<core::TSAddr> a(n);
    for (int i = 0; i < n; ++i) a[i] = core::TSAddr{static_cast<uint64_t>(i), "addr" + std::to_string(i)};
    return a;
}

static const core::RSChunkID cid{0x80000005u, 5000};

// ---------------------------------------------------------------- CPU-only tests

static void TestNewErrors(T* t) {
    auto [e0, err0] = reedsolomon::New(0, 3);
    if (e0 || err0 != reedsolomon::Err::ErrInvShardNum) Fatalf("New(0,3): %s", reedsolomon::ErrString(err0));
    auto [e1, err1] = reedsolomon::New(6, 0);
    if (e1 || err1 != reedsolomon::Err::ErrInvShardNum) Fatalf("New(6,0): %s", reedsolomon::ErrString(err1));
    auto [e2, err2] = reedsolomon::New(250, 7);
    if (e2 || err2 != reedsolomon::Err::ErrMaxShardNum) Fatalf("New(250,7): %s", reedsolomon::ErrString(err2));
    auto [e3, err3] = reedsolomon::New(250, 6);
    if (!e3 || err3 != reedsolomon::Err::None) Fatalf("New(250,6) failed");
}

static void TestShardChecks(T* t) {
    auto [enc, err] = reedsolomon::New(3, 2);
    reedsolomon::Shards four(4, Bytes::make(10));
    if (enc->Encode(four) != reedsolomon::Err::ErrTooFewShards) Fatalf("want ErrTooFewShards");
    reedsolomon::Shards empty(5);
    if (enc->Encode(empty) != reedsolomon::Err::ErrShardNoData) Fatalf("want ErrShardNoData");
    reedsolomon::Shards ragged{Bytes::make(10), Bytes::make(10), Bytes::make(9), Bytes::make(10), Bytes::make(10)};
    if (enc->Encode(ragged) != reedsolomon::Err::ErrShardSize) Fatalf("want ErrShardSize");
    reedsolomon::Shards few{Bytes::make(10), Bytes(), Bytes(), Bytes(), Bytes::make(10)};
    if (enc->Reconstruct(few) != reedsolomon::Err::ErrTooFewShards) Fatalf("want ErrTooFewShards");
    reedsolomon::Shards all(5, Bytes::make(10));
    if (enc->Reconstruct(all) != reedsolomon::Err::None) Fatalf("all present must be a no-op");
}

static void TestRSEncodeArgErrors(T* t) {
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{5000, false});
    auto addrs = makeAddrs(5);
    std::vector<core::TSAddr> srcs(addrs.begin(), addrs.begin() + 3), dests(addrs.begin() + 3, addrs.end());
    if (s.RSEncode(core::RSChunkID{5, 5000}, 12000, srcs, dests, {}) != Error::ErrInvalidArgument)
        Fatalf("non-RS partition accepted");
    if (s.RSEncode(cid, 12000, srcs, dests, {0, 1, 2}) != Error::ErrInvalidArgument) Fatalf("bad indexMap accepted");
    // no replies scripted: the first CtlRead fails with ErrRPC before any coding
    if (s.RSEncode(cid, 12000, srcs, dests, {}) != Error::ErrRPC) Fatalf("want ErrRPC");
}

// ---------------------------------------------------------------- GPU tests

// store_test.go:749-815
static void TestRSEncode(T* t, bool pipeline) {
    const int N = 3, M = 2, B = 12000;
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{5000, pipeline});
    auto addrs = makeAddrs(N + M);
    std::mt19937_64 rng(97531);
    std::vector<Bytes> data(N + M);
    for (int i = 0; i < N; ++i) data[i] = randBytes(rng, B);

    const int cuts[4] = {0, 5000, 10000, 12000};  // 0..5000, 5000..10000, 10000..12000
    for (int w = 0; w < 3; ++w) {
        for (int i = 0; i < N; ++i) tt.addCtlReadReply(addrs[i].Host, data[i].slice(cuts[w], cuts[w + 1]), Error::ErrEOF);
        for (int i = N; i < N + M; ++i) tt.addCtlWriteReply(addrs[i].Host, Error::NoError);
    }
    std::vector<core::TSAddr> srcs(addrs.begin(), addrs.begin() + N), dests(addrs.begin() + N, addrs.end());
    Error err = s.RSEncode(cid, B, srcs, dests, {});
    if (err != Error::NoError) Fatalf("error from RSEncode: %s", core::String(err));

    for (int i = N; i < N + M; ++i) {
        int j = 0;
        for (const auto& reply : tt.ctlWriteCalls[addrs[i].Host]) {
            if (!(reply.ID == cid.Add(i).ToTractID())) t->Errorf("bad tract id for reply %d from %d", j, i);
            if (reply.Off != static_cast<int64_t>(data[i].len()))
                t->Errorf("bad offset for reply %d from %d: %lld != %zu", j, i, (long long)reply.Off, data[i].len());
            data[i] = concat(data[i], reply.B);
            ++j;
        }
    }
    auto [enc, e] = reedsolomon::New(N, M);
    auto [ok, verr] = enc->Verify(data);
    if (verr != reedsolomon::Err::None || !ok) Fatalf("RS verify failed: %s, %d", reedsolomon::ErrString(verr), ok);
}

// store_test.go:817-879
static void TestRSReconstruct(T* t, bool pipeline) {
    const int N = 3, M = 2, B = 20000;
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{1 << 20, pipeline});
    auto addrs = makeAddrs(N + M);
    std::mt19937_64 rng(97532);
    std::vector<Bytes> data(N + M);
    for (int i = 0; i < N + M; ++i) data[i] = randBytes(rng, B);

    auto [enc, e] = reedsolomon::New(N, M);
    if (enc->Encode(data) != reedsolomon::Err::None) Fatalf("RS encode failed");
    std::vector<Bytes> want = data;

    // We're missing 1 (data) and 3 (parity): 0_2_4
    data[1] = Bytes();
    data[3] = Bytes();
    tt.addCtlReadReply(addrs[0].Host, data[0], Error::ErrEOF);
    tt.addCtlReadReply(addrs[2].Host, data[2], Error::ErrEOF);
    tt.addCtlReadReply(addrs[4].Host, data[4], Error::ErrEOF);
    tt.addCtlWriteReply(addrs[1].Host, Error::NoError);
    tt.addCtlWriteReply(addrs[3].Host, Error::NoError);

    Error err = s.RSEncode(cid, B, {addrs[0], addrs[2], addrs[4]}, {addrs[1], addrs[3]}, {0, 2, 4, 1, 3});
    if (err != Error::NoError) Fatalf("error from RSEncode: %s", core::String(err));
    for (int i : {1, 3}) {
        for (const auto& reply : tt.ctlWriteCalls[addrs[i].Host]) {
            if (!(reply.ID == cid.Add(i).ToTractID())) t->Errorf("bad tract id from %d", i);
            if (reply.Off != static_cast<int64_t>(data[i].len())) t->Errorf("bad offset from %d", i);
            data[i] = concat(data[i], reply.B);
        }
    }
    auto [ok, verr] = enc->Verify(data);
    if (verr != reedsolomon::Err::None || !ok) Fatalf("RS verify failed");
    for (int i = 0; i < N + M; ++i)
        if (!data[i].equal(want[i])) Fatalf("piece %d differs from the original", i);
}

// Cap reuse: a missing shard with room gets the output in its own backing array
// (client/blb/reconstruct.go:172-175).
static void TestReconstructDataIntoCallerBuffer(T* t) {
    const int n = 6, m = 3, L = 98765;
    std::mt19937_64 rng(5);
    auto [enc, e] = reedsolomon::New(n, m);
    reedsolomon::Shards sh(n + m);
    for (int i = 0; i < n; ++i) sh[i] = randBytes(rng, L);
    for (int i = n; i < n + m; ++i) sh[i] = Bytes::make(L);
    if (enc->Encode(sh) != reedsolomon::Err::None) Fatalf("encode");
    Bytes truth = Bytes::copy_of(sh[2].data(), L);
    Bytes thisB = Bytes::make(L + 5);
    sh[2] = thisB.slice3(0, 0, L);
    sh[7] = Bytes();
    if (enc->ReconstructData(sh) != reedsolomon::Err::None) Fatalf("ReconstructData");
    if (sh[2].data() != thisB.data() || sh[2].len() != static_cast<size_t>(L)) Fatalf("output not in caller buffer");
    if (!sh[2].equal(truth)) Fatalf("wrong bytes");
    if (sh[7].len() != 0) Fatalf("ReconstructData rebuilt parity");
}

// test_rs_recovery.go: a tractserver holding a piece dies; reads of that piece are
// reconstructed from n others into the caller's buffer.
class memPieces : public client::TractserverTalker {
 public:
    std::map<std::string, Bytes> pieces;
    std::map<std::string, bool> down;
    std::atomic<int> reads{0};
    std::map<std::string, bool> slow;      // blocks until its context is cancelled (or 20 s)
    std::atomic<int> cancelled_reads{0};
    std::pair<Bytes, Error> Read(const core::ContextPtr& ctx, const std::string& addr, core::TractID, int, int length,
                                 int64_t off) override {
        ++reads;
        if (slow.count(addr) && slow.at(addr)) {
            for (int i = 0; i < 20000 && !ctx->Done(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
            if (ctx->Done()) {
                ++cancelled_reads;
                return {Bytes(), Error::ErrRPC};  // context canceled
            }
        }
        if (down.count(addr) && down.at(addr)) return {Bytes(), Error::ErrRPC};
        const Bytes& p = pieces.at(addr);
        const size_t end = std::min<size_t>(p.len(), off + length);
        return {Bytes::copy_of(p.data() + off, end - off), end == p.len() ? Error::ErrEOF : Error::NoError};
    }
    std::pair<int, Error> ReadInto(const core::ContextPtr&, const std::string& addr, core::TractID, int, Bytes b,
                                   int64_t off) override {
        if (down[addr]) return {0, Error::ErrRPC};
        const Bytes& p = pieces[addr];
        const size_t n = std::min<size_t>(b.len(), p.len() - off);
        std::memcpy(b.data(), p.data() + off, n);
        return {static_cast<int>(n), Error::NoError};
    }
};

static void TestClientRecovery(T* t) {
    const int n = 6, m = 3, target = 2;
    const size_t S = core::TractLength + 65536;
    std::mt19937_64 rng(97531);
    auto [enc, e] = reedsolomon::New(n, m);
    reedsolomon::Shards sh(n + m);
    for (int i = 0; i < n; ++i) sh[i] = randBytes(rng, S);
    for (int i = n; i < n + m; ++i) sh[i] = Bytes::make(S);
    if (enc->Encode(sh) != reedsolomon::Err::None) Fatalf("encode");
    memPieces ts;
    client::TractPointer tr;
    tr.Chunk = cid.Add(target);
    tr.Host = "ts2";
    tr.TSID = 100 + target;
    tr.Length = static_cast<uint32_t>(core::TractLength);
    tr.Class = core::StorageClass::RS_6_3;
    tr.BaseChunk = cid;
    for (int i = 0; i < n + m; ++i) {
        const std::string h = "ts" + std::to_string(i);
        ts.pieces[h] = sh[i];
        tr.OtherHosts.push_back(h);
        tr.OtherTSIDs.push_back(100 + i);
    }
    ts.down["ts2"] = true;  // the piece we want
    ts.down["ts5"] = true;  // and one more
    client::Client cli(&ts, client::ReconstructBehavior{});
    // test_rs_recovery.go's windows; the caller (readAt) clips each read to the tract, and
    // a tract shorter than the buffer reads as EOF with zero padding (client.go:1193-1202).
    struct Case { int64_t off; int buf; uint32_t tractLen; int want; Error err; };
    const Case cases[] = {
        {4000, 123000, static_cast<uint32_t>(core::TractLength), 123000, Error::NoError},
        {core::TractLength - 56789, 56789, static_cast<uint32_t>(core::TractLength), 56789, Error::NoError},
        {0, 6000, 5000, 5000, Error::ErrEOF},
    };
    for (const Case& c : cases) {
        Bytes buf = Bytes::make(c.buf);
        std::memset(buf.data(), 0xEE, c.buf);
        client::TractPointer tc = tr;
        tc.Length = c.tractLen;
        client::TractResult r = cli.readOneTractRS(core::Background(), tc, buf, c.off);
        if (r.err != c.err || r.read != c.want)
            Fatalf("read at %lld: %s, %d bytes", (long long)c.off, core::String(r.err), r.read);
        if (std::memcmp(buf.data(), sh[target].data() + c.off, c.want) != 0) Fatalf("wrong reconstructed bytes");
        for (int i = c.want; i < c.buf; ++i)
            if (buf[i] != 0) Fatalf("not zero padded at %d", i);
    }
    if (cli.Reconstructs() != 3) Fatalf("want 3 reconstructs, got %d", cli.Reconstructs());
}

// reconstruct.go:119,154: once n good pieces are in, the straggler reads are cancelled
// and the reconstruct returns without waiting for them.
static void TestClientCancelsStragglers(T* t) {
    const int n = 6, m = 3, target = 0;
    const size_t S = 1 << 20;
    std::mt19937_64 rng(4242);
    auto [enc, e] = reedsolomon::New(n, m);
    reedsolomon::Shards sh(n + m);
    for (int i = 0; i < n; ++i) sh[i] = randBytes(rng, S);
    for (int i = n; i < n + m; ++i) sh[i] = Bytes::make(S);
    if (enc->Encode(sh) != reedsolomon::Err::None) Fatalf("encode");
    memPieces ts;
    client::TractPointer tr;
    tr.Chunk = cid.Add(target);
    tr.Host = "ts0";
    tr.TSID = 100 + target;
    tr.Length = static_cast<uint32_t>(S);
    tr.Class = core::StorageClass::RS_6_3;
    tr.BaseChunk = cid;
    for (int i = 0; i < n + m; ++i) {
        const std::string h = "ts" + std::to_string(i);
        ts.pieces[h] = sh[i];
        tr.OtherHosts.push_back(h);
        tr.OtherTSIDs.push_back(100 + i);
    }
    ts.down["ts0"] = true;  // the piece we want
    ts.slow["ts7"] = true;  // a straggler: 8 others are asked, 6 needed
    ts.slow["ts8"] = true;
    {
        client::Client cli(&ts, client::ReconstructBehavior{});
        Bytes buf = Bytes::make(S);
        const auto t0 = std::chrono::steady_clock::now();
        client::TractResult r = cli.readOneTractRS(core::Background(), tr, buf, 0);
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (r.err != Error::NoError || r.read != static_cast<int>(S)) Fatalf("read: %s, %d", core::String(r.err), r.read);
        if (!buf.equal(sh[target])) Fatalf("wrong reconstructed bytes");
        if (secs > 10.0) Fatalf("reconstruct waited for the stragglers (%.1f s)", secs);
        for (int i = 0; i < 10000 && cli.OutstandingReads() > 0; ++i)
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        if (cli.OutstandingReads() != 0) Fatalf("straggler reads still running");
    }
    if (ts.cancelled_reads.load() != 2) Fatalf("want 2 cancelled straggler reads, got %d", ts.cancelled_reads.load());
}

// store.go:1029-1036: the increment loop stops at the first failing window.  A failing read
// (here a short one: ErrVersionMismatch, store.go:1076-1077) must not be followed by any
// read or write of a later window, pipelined or not.
static void TestRSEncodeStopsAtFailingRead(T* t, bool pipeline) {
    const int N = 3, M = 2, B = 12000;
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{5000, pipeline});
    auto addrs = makeAddrs(N + M);
    std::mt19937_64 rng(7);
    std::vector<Bytes> data(N);
    for (int i = 0; i < N; ++i) data[i] = randBytes(rng, B);
    const int cuts[4] = {0, 5000, 10000, 12000};
    for (int w = 0; w < 3; ++w) {
        for (int i = 0; i < N; ++i) {
            Bytes b = data[i].slice(cuts[w], cuts[w + 1]);
            if (w == 1 && i == 1) b = b.slice(0, b.len() - 1);  // short read in window 1
            tt.addCtlReadReply(addrs[i].Host, b, Error::ErrEOF);
        }
        for (int i = N; i < N + M; ++i) tt.addCtlWriteReply(addrs[i].Host, Error::NoError);
    }
    std::vector<core::TSAddr> srcs(addrs.begin(), addrs.begin() + N), dests(addrs.begin() + N, addrs.end());
    Error err = s.RSEncode(cid, B, srcs, dests, {});
    if (err != Error::ErrVersionMismatch) Fatalf("want ErrVersionMismatch, got %s", core::String(err));
    for (int i = 0; i < N; ++i)
        if (tt.ctlReadCalls[addrs[i].Host] != 2) Fatalf("src %d: %d reads, want 2", i, tt.ctlReadCalls[addrs[i].Host]);
    for (int i = N; i < N + M; ++i)
        if (tt.ctlWriteCalls[addrs[i].Host].size() != 1) Fatalf("dest %d: %zu writes, want 1", i, tt.ctlWriteCalls[addrs[i].Host].size());
}

// A failing CtlWrite in window 1: no write of window 2 is ever sent.  Sequential: exactly
// the reference's reads (windows 0 and 1); pipelined: window 2's reads may already have
// been issued (documented difference; reads have no side effects).
static void TestRSEncodeStopsAtFailingWrite(T* t, bool pipeline) {
    const int N = 3, M = 2, B = 12000;
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{5000, pipeline});
    auto addrs = makeAddrs(N + M);
    std::mt19937_64 rng(8);
    std::vector<Bytes> data(N);
    for (int i = 0; i < N; ++i) data[i] = randBytes(rng, B);
    const int cuts[4] = {0, 5000, 10000, 12000};
    for (int w = 0; w < 3; ++w) {
        for (int i = 0; i < N; ++i) tt.addCtlReadReply(addrs[i].Host, data[i].slice(cuts[w], cuts[w + 1]), Error::ErrEOF);
        tt.addCtlWriteReply(addrs[N].Host, w == 1 ? Error::ErrUnknown : Error::NoError);
        tt.addCtlWriteReply(addrs[N + 1].Host, Error::NoError);
    }
    std::vector<core::TSAddr> srcs(addrs.begin(), addrs.begin() + N), dests(addrs.begin() + N, addrs.end());
    Error err = s.RSEncode(cid, B, srcs, dests, {});
    if (err != Error::ErrUnknown) Fatalf("want ErrUnknown, got %s", core::String(err));
    for (int i = N; i < N + M; ++i) {
        const auto& w = tt.ctlWriteCalls[addrs[i].Host];
        if (w.size() != 2) Fatalf("dest %d: %zu writes, want 2", i, w.size());
        for (const auto& x : w)
            if (x.Off >= 10000) Fatalf("dest %d: write of window 2 sent", i);
    }
    for (int i = 0; i < N; ++i) {
        const int r = tt.ctlReadCalls[addrs[i].Host];
        if (pipeline ? (r < 2 || r > 3) : r != 2) Fatalf("src %d: %d reads", i, r);
    }
}

// ---------------------------------------------------------------- PackTracts (store_test.go:647-746)

static const core::RSChunkID packCid{0x80000555u, 5555};

static std::vector<core::TSAddr> packAddrs() {
    return {core::TSAddr{1, "a1"}, core::TSAddr{2, "a2"}, core::TSAddr{3, "a3"}};
}

static core::PackTractSpec spec(core::TractID id, std::vector<core::TSAddr> from, int version, int off, int len) {
    core::PackTractSpec s;
    s.ID = id;
    s.From = std::move(from);
    s.Version = version;
    s.Offset = off;
    s.Length = len;
    return s;
}

static void TestPackTractsInvalid(T* t) {
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{});
    auto addrs = packAddrs();
    const core::TractID tid = core::TractIDFromParts(core::BlobIDFromParts(1, 1), 0);
    auto check = [&](int length, const std::vector<core::PackTractSpec>& srcs, const char* what) {
        if (s.PackTracts(length, srcs, packCid) != Error::ErrInvalidArgument)
            t->Errorf("PackTracts should have returned an error for %s", what);
    };
    check(-100, {}, "negative length");
    check(1000, {spec(core::TractID{}, addrs, 1, 0, 500)}, "invalid tract id");
    check(1000, {spec(tid, {}, 1, 0, 500)}, "no from");
    check(1000, {spec(tid, addrs, 1, 0, 1500)}, "too long");
    check(1000, {spec(tid, addrs, 1, 1500, 500)}, "starting too high");
    check(1000, {spec(tid, addrs, 1, 700, 200), spec(tid, addrs, 1, 100, 200)}, "out of order");
    if (s.PackTracts(1000, {}, core::RSChunkID{5, 5}) != Error::ErrInvalidArgument) t->Errorf("bad dest accepted");
}

static void TestPackTractsRPCError(T* t) {
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{});
    auto addrs = packAddrs();
    const core::TractID tid1 = core::TractIDFromParts(core::BlobIDFromParts(1, 2), 0);
    const core::TractID tid2 = core::TractIDFromParts(core::BlobIDFromParts(1, 7), 0);
    // no read replies, should fail
    Error err = s.PackTracts(1000, {spec(tid1, addrs, 1, 100, 200), spec(tid2, addrs, 1, 700, 200)}, packCid);
    if (err != Error::ErrRPC) Fatalf("error from PackTracts: %s", core::String(err));
    auto [b, rerr] = s.Read(packCid.ToTractID(), core::RSChunkVersion, 1000, 0);
    if (rerr != Error::ErrNoSuchTract) t->Errorf("a failed pack must leave no tract (%s)", core::String(rerr));
}

static Bytes str(const char* p, size_t n) { return Bytes::copy_of(reinterpret_cast<const uint8_t*>(p), n); }

static void TestPackTracts(T* t) {
    memTractserverTalker tt;
    tractserver::Store s(&tt, tractserver::Config{});
    auto addrs = packAddrs();
    const core::TractID tid1 = core::TractIDFromParts(core::BlobIDFromParts(1, 2), 0);
    const core::TractID tid2 = core::TractIDFromParts(core::BlobIDFromParts(1, 7), 0);
    const std::string data1 = "this is some data", data2 = "this is some more data";
    // tract 1: first one fails, should fall back to second
    tt.addCtlReadReply(addrs[0].Host, str("oops", 4), Error::ErrRPC);
    tt.addCtlReadReply(addrs[1].Host, str(data1.data(), data1.size()), Error::ErrEOF);
    // tract 2: first one has wrong length, second is corrupt, third is ok
    tt.addCtlReadReply(addrs[0].Host, str("wrong length", 12), Error::ErrEOF);
    tt.addCtlReadReply(addrs[1].Host, Bytes(), Error::ErrCorruptData);
    tt.addCtlReadReply(addrs[2].Host, str(data2.data(), data2.size()), Error::ErrEOF);
    const int n1 = static_cast<int>(data1.size()), n2 = static_cast<int>(data2.size());
    Error err = s.PackTracts(n1 + n2 + 10, {spec(tid1, addrs, 1, 2, n1), spec(tid2, addrs, 1, n1 + 5, n2)}, packCid);
    if (err != Error::NoError) Fatalf("error from PackTracts: %s", core::String(err));
    // read it back
    auto [b, rerr] = s.Read(packCid.ToTractID(), core::RSChunkVersion, 1000, 0);
    if (rerr != Error::ErrEOF) Fatalf("error reading back packed tract: %s", core::String(rerr));
    static const char want[] = "\x00\x00this is some data\x00\x00\x00this is some more data\x00\x00\x00\x00\x00";
    const size_t wn = sizeof(want) - 1;
    if (b.len() != wn || std::memcmp(b.data(), want, wn) != 0) t->Errorf("wrong data (len %zu, want %zu)", b.len(), wn);
}

// Routes CtlReads to the data tractservers' Stores (their packed pieces) or to a source
// host holding whole tracts; records CtlWrites (the parity windows).
class ClusterTalker : public tractserver::TractserverTalker {
 public:
    std::map<std::string, tractserver::Store*> stores;
    std::map<std::string, std::map<core::TractID, Bytes>> tracts;
    std::mutex mu;
    std::map<std::string, std::vector<WriteReq>> writes;
    std::pair<Bytes, Error> CtlRead(const std::string& addr, core::TractID id, int version, int length,
                                    int64_t off) override {
        if (auto it = stores.find(addr); it != stores.end()) return it->second->Read(id, version, length, off);
        std::lock_guard<std::mutex> g(mu);
        auto& host = tracts[addr];
        auto it = host.find(id);
        if (it == host.end()) return {Bytes(), Error::ErrNoSuchTract};
        const Bytes& b = it->second;  // CtlRead of TractLength at 0: the whole tract, ErrEOF
        return {Bytes::copy_of(b.data(), b.len()), static_cast<int64_t>(b.len()) < length ? Error::ErrEOF : Error::NoError};
    }
    Error CtlWrite(const std::string& addr, core::TractID id, int v, int64_t off, const Bytes& b) override {
        std::lock_guard<std::mutex> g(mu);
        writes[addr].push_back({id, v, Bytes::copy_of(b.data(), b.len()), off});
        return Error::NoError;
    }
};

static void TestPackThenRSEncode(T* t) {
    const int N = 3, M = 2;
    const int pad = 65532;             // padToLength (internal/curator/pack_tracts.go)
    const int length = 3 * pad + 4000;
    ClusterTalker ct;
    std::vector<std::unique_ptr<tractserver::Store>> data;
    for (int i = 0; i < N; ++i) {
        data.emplace_back(new tractserver::Store(&ct, tractserver::Config{}));
        ct.stores["d" + std::to_string(i)] = data.back().get();
    }
    std::mt19937_64 rng(4242);
    std::vector<Bytes> want(N);
    for (int i = 0; i < N; ++i) {
        // tracts at padToLength multiples; piece i gets i + 1 tracts, the last piece a hole
        want[i] = Bytes::make(length);
        std::vector<core::PackTractSpec> specs;
        for (int j = 0; j <= i; ++j) {
            if (i == 2 && j == 1) continue;  // hole
            const int len = 1 + static_cast<int>(rng() % (j == 3 ? 4000 : pad));
            const core::TractID id = core::TractIDFromParts(core::BlobIDFromParts(7, 100 + 10 * i + j), 0);
            Bytes b = randBytes(rng, len);
            ct.tracts["src"][id] = b;
            std::memcpy(want[i].data() + j * pad, b.data(), len);
            specs.push_back(spec(id, {core::TSAddr{9, "gone"}, core::TSAddr{10, "src"}}, 1, j * pad, len));
        }
        Error err = data[i]->PackTracts(length, specs, cid.Add(i));
        if (err != Error::NoError) Fatalf("PackTracts piece %d: %s", i, core::String(err));
        auto [b, rerr] = data[i]->Read(cid.Add(i).ToTractID(), core::RSChunkVersion, length, 0);
        if (rerr != Error::NoError || b.len() != static_cast<size_t>(length) ||
            std::memcmp(b.data(), want[i].data(), length) != 0)
            Fatalf("piece %d does not hold its tracts at their offsets", i);
    }
    // encEncode: the parity tractserver reads the packed pieces in increments and writes
    // the parity to the M destinations.
    tractserver::Store enc_ts(&ct, tractserver::Config{65536, true});
    std::vector<core::TSAddr> srcs, dests;
    for (int i = 0; i < N; ++i) srcs.push_back(core::TSAddr{static_cast<uint64_t>(i + 1), "d" + std::to_string(i)});
    for (int j = 0; j < M; ++j) dests.push_back(core::TSAddr{static_cast<uint64_t>(N + j + 1), "p" + std::to_string(j)});
    Error err = enc_ts.RSEncode(cid, length, srcs, dests, {});
    if (err != Error::NoError) Fatalf("RSEncode: %s", core::String(err));
    reedsolomon::Shards shards(want.begin(), want.end());
    for (int j = 0; j < M; ++j) {
        Bytes par = Bytes::make(length);
        size_t got = 0;
        for (const auto& w : ct.writes["p" + std::to_string(j)]) {
            if (!(w.ID == cid.Add(N + j).ToTractID())) t->Errorf("parity %d written to the wrong tract", j);
            std::memcpy(par.data() + w.Off, w.B.data(), w.B.len());
            got += w.B.len();
        }
        if (got != static_cast<size_t>(length)) Fatalf("parity %d: %zu of %d bytes written", j, got, length);
        shards.push_back(par);
    }
    auto [enc, e] = reedsolomon::New(N, M);
    auto [ok, verr] = enc->Verify(shards);
    if (verr != reedsolomon::Err::None || !ok) Fatalf("packed stripe does not verify");
    shards[N].data()[12345] ^= 1;
    auto [ok2, verr2] = enc->Verify(shards);
    if (verr2 != reedsolomon::Err::None || ok2) t->Errorf("corrupted parity verified");
}

// The tractserver under load: concurrent RSEncode RPCs (internal/tractserver/server.go:553-582,
// up to RejectCtlReqThreshold at once) with batching on (reedsolomon::EnableBatching, the Go
// shim's rsgpu.EnableBatching).  Every RPC's parity must verify, and the increments of
// different RPCs must have shared launches.
static void TestRSEncodeConcurrentBatched(T* t) {
    const int N = 6, M = 3, B = 200000, inc = 65536, R = 12;
    // A 1 ms window so that the RPCs' increments reliably meet (sharing is checked below).
    if (reedsolomon::EnableBatching(64, 1000) != reedsolomon::Err::None) Fatalf("EnableBatching failed");
    std::vector<std::vector<Bytes>> data(R);
    std::vector<std::unique_ptr<memTractserverTalker>> talkers;
    std::vector<std::vector<core::TSAddr>> addrs(R);
    for (int r = 0; r < R; ++r) {
        talkers.push_back(std::make_unique<memTractserverTalker>());
        addrs[r] = makeAddrs(N + M);
        std::mt19937_64 rng(97531 * (r + 1));
        data[r].resize(N + M);
        for (int i = 0; i < N; ++i) data[r][i] = randBytes(rng, B);
        for (int64_t off = 0; off < B; off += inc) {
            const int64_t end = std::min<int64_t>(off + inc, B);
            for (int i = 0; i < N; ++i)
                talkers[r]->addCtlReadReply(addrs[r][i].Host, data[r][i].slice(off, end), Error::ErrEOF);
            for (int i = N; i < N + M; ++i) talkers[r]->addCtlWriteReply(addrs[r][i].Host, Error::NoError);
        }
    }
    std::vector<Error> errs(R, Error::NoError);
    std::vector<std::thread> th;
    for (int r = 0; r < R; ++r)
        th.emplace_back([&, r] {
            tractserver::Store s(talkers[r].get(), tractserver::Config{inc, r % 2 == 1});
            std::vector<core::TSAddr> srcs(addrs[r].begin(), addrs[r].begin() + N), dests(addrs[r].begin() + N, addrs[r].end());
            errs[r] = s.RSEncode(cid, B, srcs, dests, {});
        });
    for (auto& x : th) x.join();
    uint64_t requests = 0, launches = 0;
    reedsolomon::BatchingStats(&requests, &launches);
    reedsolomon::DisableBatching();  // every RPC's encoder is gone
    auto [enc, e] = reedsolomon::New(N, M);
    for (int r = 0; r < R; ++r) {
        if (errs[r] != Error::NoError) t->Errorf("RPC %d: %s", r, core::String(errs[r]));
        for (int i = N; i < N + M; ++i)
            for (const auto& w : talkers[r]->ctlWriteCalls[addrs[r][i].Host]) data[r][i] = concat(data[r][i], w.B);
        auto [ok, verr] = enc->Verify(data[r]);
        if (verr != reedsolomon::Err::None || !ok) t->Errorf("RPC %d: parity does not verify", r);
    }
    const uint64_t calls = static_cast<uint64_t>(R) * ((B + inc - 1) / inc);
    if (requests != calls) t->Errorf("batcher served %llu calls, want %llu", (unsigned long long)requests, (unsigned long long)calls);
    if (launches >= requests) t->Errorf("no launch was shared (%llu launches)", (unsigned long long)launches);
}

// crc32.Update(crc, crc32.MakeTable(crc32.Castagnoli), p), bitwise: this test's own checker.
static uint32_t crc32cUpdate(uint32_t crc, const uint8_t* p, size_t n) {
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int b = 0; b < 8; ++b) crc = (crc & 1u) ? (crc >> 1) ^ 0x82F63B78u : crc >> 1;
    }
    return ~crc;
}

extern "C" int hipDeviceSynchronize(void);  // the *_dev calls are asynchronous on the null stream

// The recovery write path (curator reconstructChunk -> RSEncode with an indexMap, store.go:
// 1102-1120): the missing pieces are rebuilt and CtlWrite'n to new hosts whose ChecksumFile
// checksums them in 65532-byte blocks (pkg/disk/checksum_block.go:76-81).
// blbrs_reconstruct_crc_dev_at does both in one pass; here on a window at file offset 4 MiB
// (phase 256) continuing per-shard seeds, for fused shapes (RS(6,3) data-only and mixed,
// RS(12,5) three erasures) and the (5,5) fallback (decode, then the CRC kernel).  Stripes live
// in pinned host memory (device-accessible), checked against the bytes they held and this
// file's bitwise CRC-32C.
static void TestRecoveryWriteCRC(T* t) {
    struct Case { int k, m; std::vector<int> lost; int data_only; };
    const Case cases[] = {{6, 3, {1}, 1}, {6, 3, {0, 7}, 0}, {12, 5, {3, 9, 13}, 0}, {5, 5, {2, 6}, 0}, {6, 3, {2, 8}, 1}};
    const size_t S = 200000, block = 65532, phase = 256, B = 2;
    const size_t nblocks = (phase + S + block - 1) / block;
    std::mt19937_64 rng(2024);
    for (const Case& c : cases) {
        const int n = c.k + c.m;
        const size_t shard_stride = S + 64, stripe_stride = static_cast<size_t>(n) * shard_stride;
        blbrs_encoder* enc = nullptr;
        if (blbrs_new(c.k, c.m, &enc) != BLBRS_OK) Fatalf("New(%d,%d): %s", c.k, c.m, blbrs_last_error());
        std::vector<int> rows;
        for (int i : c.lost)
            if (i < c.k) rows.push_back(i);
        if (!c.data_only)
            for (int i : c.lost)
                if (i >= c.k) rows.push_back(i);
        std::sort(rows.begin(), rows.begin() + std::count_if(rows.begin(), rows.end(), [&](int i) { return i < c.k; }));
        void *mem = nullptr, *seed_mem = nullptr, *crc_mem = nullptr;
        if (blbrs_host_alloc(B * stripe_stride, &mem) != BLBRS_OK ||
            blbrs_host_alloc(rows.size() * B * 4, &seed_mem) != BLBRS_OK ||
            blbrs_host_alloc(rows.size() * B * nblocks * 4, &crc_mem) != BLBRS_OK)
            Fatalf("host_alloc: %s", blbrs_last_error());
        uint8_t* st = static_cast<uint8_t*>(mem);
        auto* seeds = static_cast<uint32_t*>(seed_mem);
        auto* crc = static_cast<uint32_t*>(crc_mem);
        std::vector<Bytes> truth;
        for (size_t b = 0; b < B; ++b) {
            std::vector<uint8_t*> ptrs(n);
            std::vector<size_t> lens(n, S);
            for (int i = 0; i < n; ++i) ptrs[i] = st + b * stripe_stride + i * shard_stride;
            for (int i = 0; i < c.k; ++i) {
                Bytes r = randBytes(rng, S);
                std::memcpy(ptrs[i], r.data(), S);
            }
            if (blbrs_encode(enc, ptrs.data(), lens.data()) != BLBRS_OK) Fatalf("Encode: %s", blbrs_last_error());
            for (int i = 0; i < n; ++i) truth.push_back(Bytes::copy_of(ptrs[i], S));
        }
        for (size_t j = 0; j < rows.size() * B; ++j) seeds[j] = static_cast<uint32_t>(rng());
        std::vector<uint8_t> present(n, 1);
        for (int i : c.lost) present[i] = 0;
        for (size_t b = 0; b < B; ++b)
            for (int i : c.lost) std::memset(st + b * stripe_stride + i * shard_stride, 0xA5, S);
        int rc = blbrs_reconstruct_crc_dev_at(enc, st, shard_stride, stripe_stride, B, S, present.data(), c.data_only,
                                              block, phase, seeds, crc, nullptr);
        if (rc != BLBRS_OK) Fatalf("RS(%d,%d): reconstruct_crc: %s", c.k, c.m, blbrs_last_error());
        if (hipDeviceSynchronize() != 0) Fatalf("hipDeviceSynchronize failed");
        for (size_t b = 0; b < B; ++b)
            for (int i : c.lost) {
                const uint8_t* got = st + b * stripe_stride + i * shard_stride;
                const bool rebuilt = std::find(rows.begin(), rows.end(), i) != rows.end();
                if (rebuilt && std::memcmp(got, truth[b * n + i].data(), S) != 0)
                    t->Errorf("RS(%d,%d) stripe %zu shard %d: wrong bytes", c.k, c.m, b, i);
                if (!rebuilt && (got[0] != 0xA5 || got[S - 1] != 0xA5))
                    t->Errorf("RS(%d,%d) stripe %zu: data-only call touched parity %d", c.k, c.m, b, i);
            }
        for (size_t j = 0; j < rows.size(); ++j)
            for (size_t b = 0; b < B; ++b) {
                const uint8_t* shard = truth[b * n + rows[j]].data();
                for (size_t blk = 0; blk < nblocks; ++blk) {
                    const size_t lo = blk * block > phase ? blk * block - phase : 0;
                    const size_t hi = std::min(S, (blk + 1) * block - phase);
                    const uint32_t want = crc32cUpdate(blk == 0 ? seeds[j * B + b] : 0u, shard + lo, hi - lo);
                    const uint32_t got = crc[(j * B + b) * nblocks + blk];
                    if (got != want)
                        t->Errorf("RS(%d,%d) row %zu stripe %zu block %zu: crc %08x want %08x", c.k, c.m, j, b, blk, got, want);
                }
            }
        blbrs_host_free(mem);
        blbrs_host_free(seed_mem);
        blbrs_host_free(crc_mem);
        blbrs_free(enc);
    }
}

// GF(2^8)/0x11D products for this file's own parity check (the library's matrix, this
// file's arithmetic).
struct GfTable {
    uint8_t mul[256][256];
    GfTable() {
        for (int a = 0; a < 256; ++a)
            for (int b = 0; b < 256; ++b) {
                uint8_t p = 0, x = static_cast<uint8_t>(a);
                for (int y = b; y; y >>= 1) {
                    if (y & 1) p ^= x;
                    x = static_cast<uint8_t>((x << 1) ^ ((x & 0x80) ? 0x1D : 0));
                }
                mul[a][b] = p;
            }
    }
};

// Host calls from many threads over the round-3 host runtime at once: two lanes on GPU 0
// (device list [0, 0], routed by bytes in flight), per-slot addressing (pageable, pool and
// registered slots mixed in one call), registrations refused by a small live limit (those
// buffers stay pageable and are staged), the batcher's mixed path, and the one-pass
// reconstructAndVerify with and without a corrupted shard.  Every output is checked against
// parity computed here from the library's matrix.  The ThreadSanitizer build runs it
// (profiles/r03/tsan).
static void TestConcurrentHostSlots(T* t) {
    const int k = 6, m = 3, n = k + m, threads = 8, iters = 10;
    static const GfTable gf;
    blbrs_pool_stats ps0{};
    blbrs_get_pool_stats(&ps0);
    // Room for a few registered shards beyond what is pinned now: the rest are refused.
    if (blbrs_pool_set_live_limit(ps0.live_bytes + ps0.registered_bytes + (12u << 20)) != BLBRS_OK)
        Fatalf("set_live_limit: %s", blbrs_last_error());
    const int devs[2] = {0, 0};
    blbrs_encoder *lanes = nullptr, *batched = nullptr;
    blbrs_batcher* bat = nullptr;
    if (blbrs_new_on(k, m, devs, 2, &lanes) != BLBRS_OK || blbrs_new_on(k, m, devs, 2, &batched) != BLBRS_OK ||
        blbrs_batcher_new_on(16, 200, devs, 2, &bat) != BLBRS_OK || blbrs_encoder_set_batcher(batched, bat) != BLBRS_OK)
        Fatalf("setup: %s", blbrs_last_error());
    uint8_t mat[n * k];
    blbrs_matrix(lanes, mat, sizeof(mat));

    std::mutex emu;
    std::vector<std::string> errors;
    auto report = [&](const std::string& s) {
        std::lock_guard<std::mutex> g(emu);
        if (errors.size() < 20) errors.push_back(s);
    };
    std::atomic<int> refused{0}, mixed_calls{0};
    std::vector<std::thread> th;
    for (int w = 0; w < threads; ++w)
        th.emplace_back([&, w] {
            std::mt19937_64 rng(4242 + w);
            for (int it = 0; it < iters; ++it) {
                const size_t sizes[] = {4096, 65536 + 16 * (rng() % 512), 1 + rng() % (1u << 20), 1u << 20};
                const size_t S = sizes[rng() % 4];
                const size_t alloc = (S + 4095) / 4096 * 4096;
                enum Kind { Pageable, Pool, Registered };
                Kind kind[n];
                uint8_t* p[n];
                bool pinned_reg[n];
                for (int i = 0; i < n; ++i) {
                    kind[i] = static_cast<Kind>(rng() % 3);
                    pinned_reg[i] = false;
                    if (kind[i] == Pool) {
                        size_t cap = 0;
                        if (blbrs_buffer_get(S, &p[i], &cap) != BLBRS_OK) kind[i] = Pageable;  // over the limit
                    }
                    if (kind[i] == Registered) {
                        p[i] = static_cast<uint8_t*>(std::aligned_alloc(4096, alloc));
                        const int rc = blbrs_buffer_register(p[i], alloc);
                        if (rc == BLBRS_OK) pinned_reg[i] = true;
                        else if (rc == BLBRS_ERR_LIMIT) ++refused;
                        else report(std::string("register: ") + blbrs_last_error());
                    }
                    if (kind[i] == Pageable) p[i] = static_cast<uint8_t*>(std::malloc(S));
                }
                int kinds_seen = 0;
                for (int i = 0; i < n; ++i) kinds_seen |= 1 << kind[i];
                if (__builtin_popcount(kinds_seen) > 1) ++mixed_calls;
                std::vector<uint8_t> truth(n * S);
                for (int i = 0; i < k; ++i)
                    for (size_t b = 0; b < S; ++b) truth[i * S + b] = static_cast<uint8_t>(rng());
                for (int r = k; r < n; ++r)
                    for (int i = 0; i < k; ++i) {
                        const uint8_t* row = gf.mul[mat[r * k + i]];
                        for (size_t b = 0; b < S; ++b) truth[r * S + b] ^= row[truth[i * S + b]];
                    }
                for (int i = 0; i < k; ++i) std::memcpy(p[i], truth.data() + i * S, S);
                for (int i = k; i < n; ++i) std::memset(p[i], 0x5A, S);
                blbrs_encoder* enc = (it + w) % 2 ? batched : lanes;
                const std::string where = "thread " + std::to_string(w) + " iter " + std::to_string(it) +
                                          " S=" + std::to_string(S) + (enc == batched ? " batched" : " lanes");
                std::vector<size_t> lens(n, S);
                if (blbrs_encode(enc, p, lens.data()) != BLBRS_OK) report(where + ": Encode: " + blbrs_last_error());
                for (int i = k; i < n; ++i)
                    if (std::memcmp(p[i], truth.data() + i * S, S) != 0) report(where + ": parity " + std::to_string(i));
                // Lose 1-3 shards, then one of Reconstruct / ReconstructData / reconstructAndVerify.
                std::vector<int> idx(n);
                for (int i = 0; i < n; ++i) idx[i] = i;
                std::shuffle(idx.begin(), idx.end(), rng);
                const int e = 1 + static_cast<int>(rng() % m);
                for (int j = 0; j < e; ++j) {
                    lens[idx[j]] = 0;
                    std::memset(p[idx[j]], 0xA5, S);
                }
                const int op = static_cast<int>(rng() % 3);
                // reconstructAndVerify: corrupt a present shard the decode does not read (the last
                // present one, if it is not among the first k present) in every other call.
                int corrupt = -1;
                if (op == 2 && rng() % 2) {
                    int present = 0, last = -1;
                    for (int i = 0; i < n; ++i)
                        if (lens[i]) { ++present; last = i; }
                    if (present > k) {
                        corrupt = last;
                        p[last][S / 2] ^= 0x01;
                    }
                }
                int rc, ok = 1;
                if (op == 0) rc = blbrs_reconstruct(enc, p, lens.data());
                else if (op == 1) rc = blbrs_reconstruct_data(enc, p, lens.data());
                else rc = blbrs_reconstruct_verify(enc, p, lens.data(), &ok);
                if (rc != BLBRS_OK) report(where + ": reconstruct op " + std::to_string(op) + ": " + blbrs_last_error());
                if (op == 2 && ok != (corrupt < 0 ? 1 : 0))
                    report(where + ": reconstructAndVerify ok=" + std::to_string(ok) + " corrupt=" + std::to_string(corrupt));
                for (int j = 0; j < e; ++j) {
                    const int i = idx[j];
                    const bool want = op != 1 || i < k;
                    if (want && std::memcmp(p[i], truth.data() + i * S, S) != 0)
                        report(where + ": op " + std::to_string(op) + " shard " + std::to_string(i) + " wrong");
                    if (!want && (p[i][0] != 0xA5 || p[i][S - 1] != 0xA5))
                        report(where + ": ReconstructData touched parity " + std::to_string(i));
                }
                for (int i = 0; i < n; ++i) {
                    if (kind[i] == Pool) blbrs_buffer_put(p[i]);
                    else {
                        if (pinned_reg[i] && blbrs_buffer_unregister(p[i]) != BLBRS_OK)
                            report(where + ": unregister: " + blbrs_last_error());
                        std::free(p[i]);
                    }
                }
            }
        });
    for (auto& x : th) x.join();
    blbrs_lane_stats l0{}, l1{};
    blbrs_encoder_lane_stats(lanes, 0, &l0);
    blbrs_encoder_lane_stats(lanes, 1, &l1);
    blbrs_pool_stats ps1{};
    blbrs_get_pool_stats(&ps1);
    blbrs_encoder_set_batcher(batched, nullptr);
    blbrs_batcher_free(bat);
    blbrs_free(batched);
    blbrs_free(lanes);
    blbrs_pool_set_live_limit(ps0.live_limit);
    for (const auto& s : errors) t->Errorf("%s", s.c_str());
    if (ps1.registered_bytes != ps0.registered_bytes)
        t->Errorf("registered bytes %llu after the test, %llu before", (unsigned long long)ps1.registered_bytes,
                  (unsigned long long)ps0.registered_bytes);
    if (l0.inflight_calls != 0 || l1.inflight_calls != 0) t->Errorf("lanes still report calls in flight");
    std::printf("    lanes: %llu / %llu calls, %llu / %llu bytes; %d registrations refused by the limit; %d mixed calls\n",
                (unsigned long long)l0.calls, (unsigned long long)l1.calls, (unsigned long long)l0.bytes,
                (unsigned long long)l1.bytes, refused.load(), mixed_calls.load());
}

// Wide recovery from many threads at once (RS(12,5), 2..5 erasures from a small set of
// patterns), run-time networks opted in: every pass with k + rows > 13 requests a network, the background thread
// compiles it (no HIP call there), and whichever launching thread next finds it compiled loads
// it while the others keep launching -- the interleaving rtc.hpp describes.  Shards are pool
// buffers or pageable memory.  Every rebuilt shard is compared with the truth.
static void TestConcurrentWideRecovery(T* t) {
    const int k = 12, m = 5, n = k + m, threads = 8, iters = 12;
    static const GfTable gf;
    blbrs_encoder* enc = nullptr;
    if (blbrs_new(k, m, &enc) != BLBRS_OK) Fatalf("New: %s", blbrs_last_error());
    uint8_t mat[n * k];
    blbrs_matrix(enc, mat, sizeof(mat));
    long rtc0 = 0;
    blbrs_get_tuning("BLBRS_RTC", &rtc0);
    blbrs_set_tuning("BLBRS_RTC", 1);  // opt in: background compiles, loads by the launching threads
    blbrs_rtc_stats st0{};
    blbrs_rtc_get_stats(&st0);
    const std::vector<std::vector<int>> patterns = {{1, 3}, {0, 5, 11}, {2, 4, 6, 8}, {1, 3, 5, 8, 10}, {12, 14}, {0, 13, 16}};
    std::mutex emu;
    std::vector<std::string> errors;
    auto report = [&](const std::string& s) {
        std::lock_guard<std::mutex> g(emu);
        if (errors.size() < 20) errors.push_back(s);
    };
    std::vector<std::thread> th;
    for (int w = 0; w < threads; ++w)
        th.emplace_back([&, w] {
            std::mt19937_64 rng(977 + w);
            for (int it = 0; it < iters; ++it) {
                const size_t sizes[] = {3 * 16384 + 123, 1u << 20, 65536};
                const size_t S = sizes[rng() % 3];
                const bool pool = rng() % 2;
                uint8_t* p[n];
                bool from_pool[n];
                for (int i = 0; i < n; ++i) {
                    size_t cap = 0;
                    from_pool[i] = pool && blbrs_buffer_get(S, &p[i], &cap) == BLBRS_OK;
                    if (!from_pool[i]) p[i] = static_cast<uint8_t*>(std::malloc(S));
                }
                std::vector<uint8_t> truth(n * S, 0);
                for (int i = 0; i < k; ++i)
                    for (size_t b = 0; b < S; ++b) truth[i * S + b] = static_cast<uint8_t>(rng());
                for (int r = k; r < n; ++r)
                    for (int i = 0; i < k; ++i) {
                        const uint8_t* row = gf.mul[mat[r * k + i]];
                        for (size_t b = 0; b < S; ++b) truth[r * S + b] ^= row[truth[i * S + b]];
                    }
                for (int i = 0; i < n; ++i) std::memcpy(p[i], truth.data() + i * S, S);
                const std::vector<int>& bad = patterns[(w + it) % patterns.size()];
                std::vector<size_t> lens(n, S);
                for (int i : bad) {
                    lens[i] = 0;
                    std::memset(p[i], 0xA5, S);
                }
                const std::string where = "thread " + std::to_string(w) + " iter " + std::to_string(it) +
                                          " S=" + std::to_string(S);
                if (blbrs_reconstruct(enc, p, lens.data()) != BLBRS_OK) report(where + ": " + blbrs_last_error());
                for (int i : bad)
                    if (std::memcmp(p[i], truth.data() + i * S, S) != 0) report(where + ": shard " + std::to_string(i));
                for (int i = 0; i < n; ++i) {
                    if (from_pool[i]) blbrs_buffer_put(p[i]);
                    else std::free(p[i]);
                }
            }
        });
    for (auto& x : th) x.join();
    blbrs_rtc_stats st1{};
    blbrs_rtc_get_stats(&st1);
    blbrs_set_tuning("BLBRS_RTC", rtc0);
    blbrs_free(enc);
    for (const auto& s : errors) t->Errorf("%s", s.c_str());
    if (st1.failed != st0.failed) t->Errorf("run-time network failures: %llu", (unsigned long long)(st1.failed - st0.failed));
    std::printf("    run-time networks: %llu requested, %llu compiled, %llu loaded\n",
                (unsigned long long)(st1.requested - st0.requested), (unsigned long long)(st1.compiled - st0.compiled),
                (unsigned long long)(st1.loaded - st0.loaded));
}

// A crash (also one at exit, after the last test) prints the faulting thread's stack: frames in
// the library are "libblbrs.so(+offset)", resolved with addr2line against the same build.
static void crash_handler(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    const char msg[] = "rs_test: fatal signal, backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(frames, n, 2);
    std::signal(sig, SIG_DFL);
    std::raise(sig);
}

int main(int argc, char** argv) {
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // each test's line survives an abort
    std::signal(SIGSEGV, crash_handler);
    std::signal(SIGABRT, crash_handler);
    std::signal(SIGBUS, crash_handler);
    const bool cpu_only = argc > 1 && std::string(argv[1]) == "--cpu";
    struct Test { const char* name; void (*fn)(T*); bool gpu; };
    const Test tests[] = {
        {"TestNewErrors", TestNewErrors, false},
        {"TestShardChecks", TestShardChecks, false},
        {"TestRSEncodeArgErrors", TestRSEncodeArgErrors, false},
        {"TestPackTractsInvalid", TestPackTractsInvalid, false},
        {"TestPackTractsRPCError", TestPackTractsRPCError, false},
        {"TestPackTracts", TestPackTracts, false},
        {"TestPackThenRSEncode", TestPackThenRSEncode, true},
        {"TestRSEncode", [](T* t) { TestRSEncode(t, false); }, true},
        {"TestRSEncode/pipelined", [](T* t) { TestRSEncode(t, true); }, true},
        {"TestRSReconstruct", [](T* t) { TestRSReconstruct(t, false); }, true},
        {"TestRSReconstruct/pipelined", [](T* t) { TestRSReconstruct(t, true); }, true},
        {"TestReconstructDataIntoCallerBuffer", TestReconstructDataIntoCallerBuffer, true},
        {"TestClientRecovery", TestClientRecovery, true},
        {"TestClientCancelsStragglers", TestClientCancelsStragglers, true},
        {"TestRSEncodeStopsAtFailingRead", [](T* t) { TestRSEncodeStopsAtFailingRead(t, false); }, true},
        {"TestRSEncodeStopsAtFailingRead/pipelined", [](T* t) { TestRSEncodeStopsAtFailingRead(t, true); }, true},
        {"TestRSEncodeStopsAtFailingWrite", [](T* t) { TestRSEncodeStopsAtFailingWrite(t, false); }, true},
        {"TestRSEncodeStopsAtFailingWrite/pipelined", [](T* t) { TestRSEncodeStopsAtFailingWrite(t, true); }, true},
        {"TestRSEncodeConcurrentBatched", TestRSEncodeConcurrentBatched, true},
        {"TestRecoveryWriteCRC", TestRecoveryWriteCRC, true},
        {"TestConcurrentHostSlots", TestConcurrentHostSlots, true},
        {"TestConcurrentWideRecovery", TestConcurrentWideRecovery, true},
    };
    int failed = 0, ran = 0;
    for (const Test& tc : tests) {
        if (cpu_only && tc.gpu) continue;
        T t{tc.name};
        tc.fn(&t);
        ++ran;
        std::printf("--- %s: %s\n", t.failed ? "FAIL" : "PASS", tc.name);
        failed += t.failed;
    }
    std::printf("%s (%d tests, %d failed)\n", failed ? "FAIL" : "PASS", ran, failed);
    return failed ? 1 : 0;
}
