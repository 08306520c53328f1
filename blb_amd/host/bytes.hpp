// bytes.hpp -- a Go []byte for the C++ mirror of blb's RS callers.
//
// The RS call surface depends on Go slice semantics: a missing shard is len 0, and
// klauspost reuses its backing array when cap >= size (client/blb/reconstruct.go:172-175
// hands in thisB[0:0:length] and asserts the output landed there).  Bytes models
// (pointer, len, cap) over a shared backing store, or over caller-owned memory.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace blb {

class Bytes {
 public:
    Bytes() = default;

    // make([]byte, len, cap): zeroed, owned.
    static Bytes make(size_t len, size_t cap = 0) {
        if (cap < len) cap = len;
        Bytes b;
        b.store_ = std::shared_ptr<uint8_t[]>(new uint8_t[cap ? cap : 1]());
        b.base_ = b.store_.get();
        b.len_ = len;
        b.cap_ = cap;
        return b;
    }
    // A view of caller-owned memory (not freed by Bytes).
    static Bytes wrap(uint8_t* p, size_t len, size_t cap = 0) {
        Bytes b;
        b.base_ = p;
        b.len_ = len;
        b.cap_ = cap < len ? len : cap;
        return b;
    }
    // A buffer whose last holder releases it through `release` (pooled memory).
    template <class Release>
    static Bytes adopt(uint8_t* p, size_t len, size_t cap, Release release) {
        Bytes b;
        b.store_ = std::shared_ptr<uint8_t[]>(p, release);
        b.base_ = p;
        b.len_ = len;
        b.cap_ = cap < len ? len : cap;
        return b;
    }
    // Copy of a byte range (like append([]byte(nil), p...)).
    static Bytes copy_of(const uint8_t* p, size_t n) {
        Bytes b = make(n);
        if (n) std::memcpy(b.data(), p, n);
        return b;
    }

    uint8_t* data() const { return base_; }
    size_t len() const { return len_; }
    size_t cap() const { return cap_; }
    bool nil() const { return base_ == nullptr; }
    uint8_t& operator[](size_t i) const { return base_[i]; }

    // s[lo:hi] and s[lo:hi:max]
    Bytes slice(size_t lo, size_t hi) const { return slice3(lo, hi, cap_); }
    Bytes slice3(size_t lo, size_t hi, size_t max) const {
        if (lo > hi || hi > max || max > cap_) throw std::out_of_range("slice bounds out of range");
        Bytes b = *this;
        b.base_ = base_ ? base_ + lo : nullptr;
        b.len_ = hi - lo;
        b.cap_ = max - lo;
        return b;
    }
    bool equal(const Bytes& o) const {
        return len_ == o.len_ && (len_ == 0 || std::memcmp(base_, o.base_, len_) == 0);
    }

 private:
    std::shared_ptr<uint8_t[]> store_;
    uint8_t* base_ = nullptr;
    size_t len_ = 0, cap_ = 0;
};

}  // namespace blb
