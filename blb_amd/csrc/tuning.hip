// tuning.hip -- the knob store of tuning.hpp and its C ABI (blbrs_set_tuning / _get_tuning).
#include "tuning.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "../../include/blb_rs.h"

namespace blbrs {
namespace tune {
namespace {

struct Def {
    const char* name;
    long dflt;
};
// Order = enum Knob.
constexpr Def kDefs[kCount] = {
    {"BLBRS_BITSLICE", 1}, {"BLBRS_EC_PERSISTENT", 0}, {"BLBRS_RTC", 1}, {"BLBRS_RTC_WIDE", 13}, {"BLBRS_DONE_WORD", 1},
};

// The environment is read once, here (thread-safe static initialisation).
struct Store {
    std::atomic<long> v[kCount];
    Store() {
        for (int i = 0; i < kCount; ++i) {
            long x = kDefs[i].dflt;
            if (const char* e = std::getenv(kDefs[i].name); e && *e) {
                // Presence-style knobs (BLBRS_EC_PERSISTENT=yes) count as 1.
                char* end = nullptr;
                const long p = std::strtol(e, &end, 10);
                x = end != e ? p : 1;
            }
            v[i].store(x, std::memory_order_relaxed);
        }
    }
};
Store& store() {
    static Store s;
    return s;
}
int index_of(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < kCount; ++i)
        if (std::strcmp(name, kDefs[i].name) == 0) return i;
    return -1;
}

}  // namespace

long get(Knob k) { return store().v[k].load(std::memory_order_relaxed); }

bool set(const char* name, long value) {
    const int i = index_of(name);
    if (i < 0) return false;
    store().v[i].store(value, std::memory_order_relaxed);
    return true;
}

bool get(const char* name, long* value) {
    const int i = index_of(name);
    if (i < 0 || !value) return false;
    *value = store().v[i].load(std::memory_order_relaxed);
    return true;
}

}  // namespace tune
}  // namespace blbrs

extern "C" int blbrs_set_tuning(const char* name, long value) {
    return blbrs::tune::set(name, value) ? BLBRS_OK : BLBRS_ERR_INVALID_ARG;
}

extern "C" int blbrs_get_tuning(const char* name, long* value) {
    return blbrs::tune::get(name, value) ? BLBRS_OK : BLBRS_ERR_INVALID_ARG;
}
