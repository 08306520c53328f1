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

enum Knob : int {
    kBitslice = 0,   // BLBRS_BITSLICE: compiled encode network 0 = never, 1 = where faster (default), 2 = always
    kOccLds,         // BLBRS_OCC_LDS: dynamic LDS bytes per workgroup of rs_code_kernel network launches (0)
    kOccLdsEct,      // BLBRS_OCC_LDS_ECT: the same for the fused encode+CRC tile kernel (0)
    kPackVariant,    // BLBRS_PACK_VARIANT: PackTracts kernel variant (-1 = default)
    kPeCmWide,       // BLBRS_PE_CM_WIDE: PackTracts+Encode network at U = 2 for wide k (1)
    kHostZc,         // BLBRS_HOST_ZC: host calls zero copy 1 / by DMA 0 / policy -1 (default)
    kEcPersistent,   // BLBRS_EC_PERSISTENT: fused encode+CRC on the persistent segment kernel (0)
    kEcFlags,        // BLBRS_EC_FLAGS: segment-kernel A/B flags (0)
    kRtc,            // BLBRS_RTC: run-time decode networks 0 = off, 1 = compiled in the background (default), 2 = compiled by the caller
    kRtcCse,         // BLBRS_RTC_CSE: explicit shared XOR temporaries in generated networks (0: LLVM already
                     // shares terms; the temporaries raise VGPRs 156 -> 252-280 at RS(12,5))
    kRtcWide,        // BLBRS_RTC_WIDE: a decode pass takes a network when k + rows > this (13: RS(12,5)-wide
                     // passes, where the tables are VALU-bound; narrower ones measured +-1-3 %)
    kRtcEncode,      // BLBRS_RTC_ENCODE: encode passes too take run-time networks instead of the compiled ones (0; A/B)
    kRtcWpe,         // BLBRS_RTC_WPE: waves per SIMD run-time networks of k + rows <= 14 ask for (0 = the compiler's choice)
    kRtcRowStores,   // BLBRS_RTC_ROW_STORES: run-time networks store each row as it is formed (1) or all rows at the end (0)
    kCount
};

long get(Knob k);
// Bumped by every set(): lookups cached under the knobs (run-time network per pass) compare it
// to notice a change.
unsigned generation();
// By BLBRS_* name; false when the name is unknown.
bool set(const char* name, long value);
bool get(const char* name, long* value);

}  // namespace tune
}  // namespace blbrs
