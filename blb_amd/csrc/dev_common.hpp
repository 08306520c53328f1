// dev_common.hpp -- small gfx950 device helpers shared by the coding and CRC kernels.
//
// Also compiled by hipRTC (rtc.hip: decode networks built per erasure pattern at run time), where
// no standard headers exist: the fixed-width types come from hipRTC's own runtime header.
#pragma once
#ifdef __HIPCC_RTC__
using uint8_t = __hip_internal::uint8_t;
using uint32_t = __hip_internal::uint32_t;
using uint64_t = __hip_internal::uint64_t;
using int32_t = __hip_internal::int32_t;
using uintptr_t = unsigned long;
#else
#include <hip/hip_runtime.h>
#include <cstdint>
#endif

namespace blbrs {
namespace dev {

// Read-only metadata (tables, shard indices, pointer tables, CRC matrices) is read through
// the constant address space so the compiler may use scalar (s_load) loads for it.
using cu32 = const uint32_t __attribute__((address_space(4)))*;
using ci32 = const int32_t __attribute__((address_space(4)))*;
using cu64 = const uint64_t __attribute__((address_space(4)))*;
__device__ __forceinline__ cu32 as_const(const uint32_t* p) { return (cu32)(uintptr_t)p; }
__device__ __forceinline__ ci32 as_const(const int32_t* p) { return (ci32)(uintptr_t)p; }
__device__ __forceinline__ cu64 as_const(const uint64_t* p) { return (cu64)(uintptr_t)p; }

// 3-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96 = a ^ b ^ c); hipcc
// does not form it from a ^ b ^ c by itself.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

using u32x4 = uint32_t __attribute__((ext_vector_type(4)));

}  // namespace dev
}  // namespace blbrs
