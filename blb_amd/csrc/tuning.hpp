// tuning.hpp -- the library's A/B knobs, read once.
//
// Each knob starts from its BLBRS_* environment variable, read once when the library first
// asks for a knob, and changes only through blbrs_set_tuning (include/blb_rs.h).  Hot paths
// read an atomic, never getenv: an A/B driver that flips a knob between launches calls the
// setter instead of changing the environment under live worker threads (setenv racing
// getenv is undefined behaviour).
#pragma once

namespace blbrs {
namespace tune {

// Only knobs that choose between policies the library ships; the variants measured and rejected
// in rounds 1-4 (CSE temporaries, waves-per-EU requests, occupancy caps, segment-kernel flags,
// PackTracts variants, run-time encode networks) are no longer built.
enum Knob : int {
    kBitslice = 0,   // BLBRS_BITSLICE: compiled encode network 0 = never, 1 = where faster (default), 2 = always
    kEcPersistent,   // BLBRS_EC_PERSISTENT: fused encode+CRC on the persistent segment kernel, the fallback
                     // for shapes the tile-grid kernel does not take (0; 1 forces it where it applies)
    kRtc,            // BLBRS_RTC: run-time decode networks 0 = off, 1 = compiled in the
                     // background (default since round 6), 2 = compiled by the caller (rtc.hpp)
    kRtcWide,        // BLBRS_RTC_WIDE: a decode pass takes a network when k + rows > this (13: RS(12,5)-wide
                     // passes, where the tables are VALU-bound; narrower ones measured +-1-3 %)
    kDoneWord,       // BLBRS_DONE_WORD: small single-launch host calls end on their kernel's completion
                     // word (1, default since round 6) or on a stream wait (0); runtime.hpp kDoneMaxBytes
    kCount
};

long get(Knob k);
// By BLBRS_* name; false when the name is unknown.
bool set(const char* name, long value);
bool get(const char* name, long* value);

}  // namespace tune
}  // namespace blbrs
