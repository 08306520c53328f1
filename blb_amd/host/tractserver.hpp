// tractserver.hpp -- C++ mirror of blb's tractserver RS path over the MI355X engine:
// Store::RSEncode / rsEncodeOne / reconstructAndVerify (internal/tractserver/store.go:1012-1144).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "bytes.hpp"
#include "core.hpp"
#include "reedsolomon.hpp"

namespace tractserver {

// The two TractserverTalker calls rsEncodeOne makes (internal/tractserver/repl.go:26-32).
class TractserverTalker {
 public:
    virtual ~TractserverTalker() = default;
    virtual std::pair<blb::Bytes, core::Error> CtlRead(const std::string& addr, core::TractID id, int version,
                                                       int length, int64_t off) = 0;
    virtual core::Error CtlWrite(const std::string& addr, core::TractID id, int version, int64_t off,
                                 const blb::Bytes& b) = 0;
};

struct Config {
    int EncodeIncrementSize = 4 << 20;  // config.go:117 (prod); 1 MiB in the test config
    // Overlap window i's coding with window i+1's reads and window i-1's writes (SURVEY.md
    // §8f row 1).  Off = the reference's strictly sequential loop; bytes written are equal.
    bool Pipeline = false;
};

class Store {
 public:
    Store(TractserverTalker* tt, Config cfg) : tt_(tt), cfg_(cfg) {}

    // store.go:1014 -- srcs[N] data pieces, dests[M]; indexMap empty = encode, else
    // N+M entries mapping sources then destinations to piece indexes (-1 = skip).
    core::Error RSEncode(core::RSChunkID baseid, int length, const std::vector<core::TSAddr>& srcs,
                         const std::vector<core::TSAddr>& dests, const std::vector<int>& indexMap);

    // store.go:921-994 -- pull every source tract (sequentially, from the first replica that
    // returns exactly src.Length bytes) into a local RS data piece of `length` bytes: tracts
    // at their offsets, holes and the tail zero.  ErrInvalidArgument for a bad dest or spec,
    // ErrRPC when a source cannot be pulled (nothing is kept).
    core::Error PackTracts(int length, const std::vector<core::PackTractSpec>& srcs, core::RSChunkID dest);

    // Store.Read of a local tract: [off, off + length) of it; a short read is ErrEOF.
    std::pair<blb::Bytes, core::Error> Read(core::TractID id, int version, int length, int64_t off);

 private:
    struct Window {
        int64_t offset;
        int length;
        std::vector<blb::Bytes> data;
        core::Error err = core::Error::NoError;
    };
    core::Error gather(core::RSChunkID baseid, const std::vector<core::TSAddr>& srcs, const std::vector<int>& imap,
                       int N, int M, Window& w);
    core::Error code(reedsolomon::Encoder& enc, bool encode, const std::vector<int>& imap, int N, Window& w);
    core::Error scatter(core::RSChunkID baseid, const std::vector<core::TSAddr>& dests, const std::vector<int>& imap,
                        int N, Window& w);
    core::Error rsEncodeOne(core::RSChunkID baseid, int64_t offset, int length, const std::vector<core::TSAddr>& srcs,
                            const std::vector<core::TSAddr>& dests, const std::vector<int>& imap, bool encode,
                            reedsolomon::Encoder& enc);

    TractserverTalker* tt_;
    Config cfg_;
    struct Local {
        blb::Bytes data;  // pinned pool memory: the GPU codes it in place when read for RSEncode
        int version;
    };
    std::mutex mu_;
    std::map<core::TractID, Local> tracts_;
};

// store.go:998-1009: sources in order, non-overlapping, each from >= 1 host with a valid ID,
// all inside `length`.
bool checkTractSpec(const std::vector<core::PackTractSpec>& srcs, int length);

// store.go:1132-1142; false with Err::None means errVerifyFailed.
reedsolomon::Err reconstructAndVerify(reedsolomon::Encoder& enc, reedsolomon::Shards& data, bool* verified);

}  // namespace tractserver
