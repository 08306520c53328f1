// core.hpp -- the slice of blb's internal/core the RS path touches (C++ restatement).
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace core {

constexpr int64_t TractLength = 8 * 1024 * 1024;                   // constants.go:15
constexpr int RSChunkVersion = -317866832;                         // constants.go:36
constexpr int64_t RSPieceLength = 64 * 1024 * 1024 - 64 * 1024 - 64;  // curator/storage_class_loop.go:22
constexpr uint64_t MaxRSChunkKey = (uint64_t{1} << 48) - 1;        // ids.go

// core.Error values on the RS path (internal/core/errors.go).
enum class Error {
    NoError,
    ErrVersionMismatch,
    ErrShortRead,
    ErrCorruptData,
    ErrEOF,
    ErrInvalidArgument,
    ErrHostNotExist,
    ErrRPC,
    ErrUnknown,
    ErrAllocHost,
    ErrNoSuchTract,
};

inline const char* String(Error e) {
    switch (e) {
        case Error::NoError: return "no error";
        case Error::ErrVersionMismatch: return "version mismatch";
        case Error::ErrShortRead: return "short read";
        case Error::ErrCorruptData: return "corrupt data";
        case Error::ErrEOF: return "EOF";
        case Error::ErrInvalidArgument: return "invalid argument";
        case Error::ErrHostNotExist: return "host does not exist";
        case Error::ErrRPC: return "rpc error";
        case Error::ErrUnknown: return "unknown error";
        case Error::ErrAllocHost: return "could not allocate host";
        case Error::ErrNoSuchTract: return "no such tract";
    }
    return "?";
}

struct TractID {
    uint64_t Blob = 0;
    uint16_t Index = 0;
    bool operator==(const TractID& o) const { return Blob == o.Blob && Index == o.Index; }
    bool operator<(const TractID& o) const { return Blob != o.Blob ? Blob < o.Blob : Index < o.Index; }
    // ids.go:237-239: a valid regular blob (partition type 0, key > 0) or any blob of a
    // valid RS partition (type 2).
    bool IsValid() const {
        const uint32_t p = static_cast<uint32_t>(Blob >> 32);
        const bool part = (p & 0x3fffffffu) != 0;
        return (part && (p >> 30) == 0 && static_cast<uint32_t>(Blob) > 0) || (part && (p >> 30) == 2);
    }
};

// ids.go:196-198, 242-244
inline uint64_t BlobIDFromParts(uint32_t partition, uint32_t key) {
    return (static_cast<uint64_t>(partition) << 32) | key;
}
inline TractID TractIDFromParts(uint64_t blob, uint16_t index) { return TractID{blob, index}; }

// ids.go:113 -- RS partitions have upper two bits 10.
struct RSChunkID {
    uint32_t Partition = 0;
    uint64_t ID = 0;
    bool IsValid() const {
        return (Partition & 0x3fffffffu) != 0 && (Partition >> 30) == 2 && ID != 0 && ID <= MaxRSChunkKey;
    }
    RSChunkID Add(int i) const { return RSChunkID{Partition, ID + static_cast<uint64_t>(i)}; }
    TractID ToTractID() const {
        return TractID{(static_cast<uint64_t>(Partition) << 32) | ((ID >> 16) & 0xffffffffull),
                       static_cast<uint16_t>(ID & 0xffff)};
    }
};

// context.Context, as far as the RS path uses it: cancellation of the client's straggler
// piece reads (client/blb/reconstruct.go:119,154).
struct Context {
    std::atomic<bool> cancelled{false};
    bool Done() const { return cancelled.load(); }
    void Cancel() { cancelled.store(true); }
};
using ContextPtr = std::shared_ptr<Context>;
inline ContextPtr Background() { return std::make_shared<Context>(); }

struct TSAddr {
    uint64_t ID = 0;
    std::string Host;
};

// core.PackTractSpec (internal/core/types.go): tract ID at Offset of the packed piece,
// pulled from any of From.
struct PackTractSpec {
    TractID ID;
    std::vector<TSAddr> From;
    int Version = 0;
    int Offset = 0;
    int Length = 0;
};

// internal/core/StorageClass.go:7-13 and storageclass.go RSParams.
enum class StorageClass : int32_t { REPLICATED = 0, RS_6_3 = 1, RS_8_3 = 2, RS_10_3 = 3, RS_12_5 = 4 };

inline bool RSParams(StorageClass c, int* n, int* m) {
    switch (c) {
        case StorageClass::RS_6_3: *n = 6; *m = 3; return true;
        case StorageClass::RS_8_3: *n = 8; *m = 3; return true;
        case StorageClass::RS_10_3: *n = 10; *m = 3; return true;
        case StorageClass::RS_12_5: *n = 12; *m = 5; return true;
        default: return false;
    }
}

}  // namespace core
