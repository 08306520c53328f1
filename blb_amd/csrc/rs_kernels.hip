// rs_kernels.hip -- launch policy and ahead-of-time instantiations of rs_code_kernel
// (rs_code.hpp): the v_perm table path for every shape and the compiled encode networks; and
// rs_small_kernel (rs_small.hpp), the latency kernel of small host calls.
#include "rs_kernels.hpp"

#include <algorithm>

#include "rs_code.hpp"
#include "rs_small.hpp"
#include "rtc.hpp"
#include "tuning.hpp"

namespace blbrs {
namespace {

using code::rs_code_kernel;

using KernelFn = void (*)(CodeArgs);

// Compile-time input counts: blb's classes RS(6,3), RS(8,3), RS(10,3), RS(12,5)
// (internal/core/StorageClass.go:7-13), the bench's RS(10,4), the reference tests' RS(3,2)
// (store_test.go:750,818) and RS(4,2); rows 1..5 cover every encode and decode of those.
#define BLBRS_K_LIST(X) X(3) X(4) X(6) X(8) X(10) X(12)
constexpr int kMaxTemplRows = 5;

// Launch policy, measured on MI355X (tools/tune_kernels.hip, profiles/r01/tune*.txt):
//  * nontemporal loads and stores (every byte is touched once): +2-5 %;
//  * store mode: U = 4 chunks per lane (16 KiB tiles) when K + MR <= 9, else U = 2 -- wider
//    shapes at U = 4 drop to one wave per SIMD (RS(10,4) 4.6 vs 6.2 TB/s);
//  * verify mode (check shards prefetched with the inputs): U = 2 -- 6.8 TB/s, faster than
//    a plain 9-shard read stream; U = 4 needs too many VGPRs; U = 1 when K + MR > 13:
//    RS(12,5) at U = 2 holds 256 VGPRs (one wave per SIMD) and verified in 20.0 ms, at U = 1
//    147 VGPRs and 13.4 ms; RS(10,4) 10.45 -> 9.9-10.3 ms (tools/code_ab.py, r02);
//  * one tile per block in dispatch order (no persistent grid-stride), with each XCD given
//    a contiguous eighth of the tiles: +10-16 % over a resident persistent grid.
constexpr int kNT = 3;
#ifndef BLBRS_U_WIDE
#define BLBRS_U_WIDE 2         // store mode, K + MR > 9
#endif
#ifndef BLBRS_U_VERIFY_WIDE
#define BLBRS_U_VERIFY_WIDE 1  // verify mode, K + MR > 13
#endif
constexpr int pick_u(int K, int MR, int MODE) {
    return MODE == 0 ? ((K > 0 && K + MR <= 9) ? 4 : BLBRS_U_WIDE) : (K + MR > 13 ? BLBRS_U_VERIFY_WIDE : 2);  // MODE 1, 2
}


template <int K, int MR, int MODE, int ADDR>
constexpr KernelFn fn_of() { return rs_code_kernel<K, MR, MODE, ADDR, pick_u(K, MR, MODE), kNT>; }

struct Choice {
    KernelFn fn = nullptr;
    int u = 0;
    bool fixed = false;
    bool cm = false;  // the compiled encode network
};

// Encode / Verify passes of parity rows: the compiled network where the shape has one.
template <int K, int MR, int MODE, int ADDR>
Choice choice_of(bool cm) {
    constexpr int UC = network_u(K, MR, MODE);
    if constexpr (K > 0 && MODE != 2) {
        if (cm) return {rs_code_kernel<K, MR, MODE, ADDR, UC, kNT, bs::EncodeNet<K>>, UC, true, true};
    }
    return {fn_of<K, MR, MODE, ADDR>(), pick_u(K, MR, MODE), K > 0, false};
}

template <int K, int MODE, int ADDR>
Choice pick_rows(int rows, bool cm = false) {
    switch (rows) {
        case 1: return choice_of<K, 1, MODE, ADDR>(cm);
        case 2: return choice_of<K, 2, MODE, ADDR>(cm);
        case 3: return choice_of<K, 3, MODE, ADDR>(cm);
        case 4: return choice_of<K, 4, MODE, ADDR>(cm);
        case 5: return choice_of<K, 5, MODE, ADDR>(cm);
        case 6: return {fn_of<0, 6, MODE, ADDR>(), pick_u(0, 6, MODE), false};
        case 7: return {fn_of<0, 7, MODE, ADDR>(), pick_u(0, 7, MODE), false};
        case 8: return {fn_of<0, 8, MODE, ADDR>(), pick_u(0, 8, MODE), false};
        default: return {};
    }
}

template <int MODE, int ADDR>
Choice pick_k(int k, int rows, bool cm) {
    if (rows <= kMaxTemplRows) {
        switch (k) {
#define BLBRS_CASE(KK) case KK: return pick_rows<KK, MODE, ADDR>(rows, cm);
            BLBRS_K_LIST(BLBRS_CASE)
#undef BLBRS_CASE
            default: break;
        }
    }
    return pick_rows<0, MODE, ADDR>(rows);
}

Choice pick(int k, int rows, Mode mode, bool strided, bool cm = false) {
    if (mode == Mode::kStore) return strided ? pick_k<0, 0>(k, rows, cm) : pick_k<0, 1>(k, rows, cm);
    if (mode == Mode::kVerify) return strided ? pick_k<1, 0>(k, rows, cm) : pick_k<1, 1>(k, rows, cm);
    return strided ? pick_k<2, 0>(k, rows, false) : pick_k<2, 1>(k, rows, false);
}

}  // namespace

hipError_t launch_code(const CodeArgs& args, Mode mode, hipStream_t stream, rtc::NetKernel* net) {
    if (args.rows < 1 || args.rows > kMaxRows || args.k < 1) return hipErrorInvalidValue;
    if (mode != Mode::kStore && !args.mismatch) return hipErrorInvalidValue;
    if (mode == Mode::kStoreVerify && (args.nstore < 0 || args.nstore > args.rows)) return hipErrorInvalidValue;
    if (args.B == 0 || args.S == 0) return hipSuccess;
    Choice ch = pick(args.k, args.rows, mode, args.base != nullptr, bs::use(args.parity, args.k, args.rows, bs::kWideCode));
    // A run-time network replaces the table kernel once loaded (the caller asks for one only where
    // no compiled encode network applies).
    hipFunction_t rfn = rtc::ready(net);
    if (rfn) {
        ch.u = net->u;
        ch.cm = true;
    }
    if (!ch.fn && !rfn) return hipErrorInvalidValue;
    const uint64_t tile = static_cast<uint64_t>(kTileBytes) * ch.u;
    const uint64_t tps = (args.S + tile - 1) / tile;
    // Tiles are numbered with 32-bit ints: split huge batches.
    const uint64_t max_b = std::max<uint64_t>(1, 0x7FFFFFFFull / tps);
    if (!args.base && !args.ptrs && static_cast<uint64_t>(args.B) * args.nshards > kInlinePtrs) return hipErrorInvalidValue;
    for (uint64_t b0 = 0; b0 < args.B; b0 += max_b) {
        CodeArgs a = args;
        a.B = static_cast<uint32_t>(std::min<uint64_t>(max_b, args.B - b0));
        if (a.base) a.base += b0 * a.stripe_stride;
        else if (a.ptrs) a.ptrs += b0 * a.nshards;  // an inline table never splits (B * nshards <= kInlinePtrs)
        if (a.mismatch) a.mismatch += b0;
        a.tiles_per_stripe = static_cast<uint32_t>(tps);
        const uint64_t total = static_cast<uint64_t>(a.B) * tps;
        uint64_t grid = total;
        a.xcd_remap = 0;
        if (total >= 64) {  // one tile per block; a multiple of 8 blocks for the XCD remap
            grid = total & ~uint64_t{7};
            a.xcd_remap = 1;
        }
        hipError_t e;
        if (rfn) {
            void* params[] = {&a};
            e = hipModuleLaunchKernel(rfn, static_cast<unsigned>(grid), 1, 1, kThreads, 1, 1, 0, stream, params, nullptr);
        } else {
            hipLaunchKernelGGL(ch.fn, dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, stream, a);
            e = hipGetLastError();
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

namespace {

using SmallFn = void (*)(code::SmallArgs);

template <int K>
SmallFn small_rows(int rows) {
    switch (rows) {
        case 1: return code::rs_small_kernel<K, 1>;
        case 2: return code::rs_small_kernel<K, 2>;
        case 3: return code::rs_small_kernel<K, 3>;
        case 4: return code::rs_small_kernel<K, 4>;
        case 5: return code::rs_small_kernel<K, 5>;
        default: break;
    }
    if constexpr (K == 0) {
        switch (rows) {
            case 6: return code::rs_small_kernel<0, 6>;
            case 7: return code::rs_small_kernel<0, 7>;
            case 8: return code::rs_small_kernel<0, 8>;
            default: break;
        }
    }
    return nullptr;
}

SmallFn pick_small(int k, int rows) {
    if (rows <= kMaxTemplRows) {
        switch (k) {
#define BLBRS_CASE(KK) case KK: return small_rows<KK>(rows);
            BLBRS_K_LIST(BLBRS_CASE)
#undef BLBRS_CASE
            default: break;
        }
    }
    return small_rows<0>(rows);
}

}  // namespace

hipError_t launch_small(const CodeArgs& args, uint32_t* done_word, uint32_t* done_count, uint32_t seq,
                        hipStream_t stream) {
    if (args.rows < 1 || args.rows > kMaxRows || args.k < 1 || args.base) return hipErrorInvalidValue;
    if (done_word && (!done_count || seq == 0)) return hipErrorInvalidValue;
    if (!args.ptrs && static_cast<uint64_t>(args.B) * args.nshards > kInlinePtrs) return hipErrorInvalidValue;
    const uint64_t chunks = (args.S + kTileBytes - 1) / kTileBytes;
    const uint64_t total = static_cast<uint64_t>(args.B) * chunks;
    if (args.B == 0 || args.S == 0 || total > 0x7FFFFFFFull) return hipErrorInvalidValue;  // callers: small calls
    const SmallFn fn = pick_small(args.k, args.rows);
    if (!fn) return hipErrorInvalidValue;
    code::SmallArgs s{};
    s.c = args;
    s.c.tiles_per_stripe = static_cast<uint32_t>(chunks);
    s.c.xcd_remap = 0;
    s.done_word = done_word;
    s.done_count = done_count;
    s.done_seq = seq;
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(total, 4096));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, s);
    return hipGetLastError();
}

namespace {

using Small1Fn = void (*)(code::Small1Args);

template <int K>
Small1Fn small1_rows(int rows) {
    switch (rows) {
        case 1: return code::rs_small1_kernel<K, 1>;
        case 2: return code::rs_small1_kernel<K, 2>;
        case 3: return code::rs_small1_kernel<K, 3>;
        case 4: return code::rs_small1_kernel<K, 4>;
        case 5: return code::rs_small1_kernel<K, 5>;
        default: return nullptr;
    }
}

Small1Fn pick_small1(int k, int rows) {
    switch (k) {
#define BLBRS_CASE(KK) case KK: return small1_rows<KK>(rows);
        BLBRS_K_LIST(BLBRS_CASE)
#undef BLBRS_CASE
        default: return nullptr;
    }
}

}  // namespace

hipError_t launch_small1(const CodeArgs& args, const int32_t* in_idx, const int32_t* out_idx, uint32_t* done_word,
                         uint32_t* done_count, uint32_t seq, hipStream_t stream) {
    if (args.B != 1 || args.base || args.ptrs || !in_idx || !out_idx) return hipErrorNotSupported;
    if (args.k > code::kSmall1MaxIn || args.rows < 1 || args.rows > kMaxRows) return hipErrorNotSupported;
    const Small1Fn fn = pick_small1(args.k, args.rows);
    if (!fn) return hipErrorNotSupported;
    if (done_word && (!done_count || seq == 0)) return hipErrorInvalidValue;
    if (args.S == 0) return hipErrorInvalidValue;
    code::Small1Args s{};
    s.tables = args.tables;
    s.S = args.S;
    s.fault = args.fault;
    s.done_word = done_word;
    s.done_count = done_count;
    s.done_seq = seq;
    s.ptr_tag = args.ptr_tag;
    const uint64_t chunks = (args.S + kTileBytes - 1) / kTileBytes;
    if (chunks > 0x7FFFFFFFull) return hipErrorInvalidValue;
    s.chunks = static_cast<uint32_t>(chunks);
    s.rows = args.rows;
    s.aligned = args.aligned;
    for (int j = 0; j < args.k; ++j) {
        if (in_idx[j] < 0 || static_cast<uint32_t>(in_idx[j]) >= args.nshards || in_idx[j] >= kInlinePtrs)
            return hipErrorInvalidValue;
        s.in_e[j] = args.inl[in_idx[j]];
        s.in_slot[j] = static_cast<uint8_t>(in_idx[j]);
    }
    for (int r = 0; r < args.rows; ++r) {
        if (out_idx[r] < 0 || static_cast<uint32_t>(out_idx[r]) >= args.nshards || out_idx[r] >= kInlinePtrs)
            return hipErrorInvalidValue;
        s.out_e[r] = args.inl[out_idx[r]];
        s.out_slot[r] = static_cast<uint8_t>(out_idx[r]);
    }
    const unsigned grid = static_cast<unsigned>(std::min<uint64_t>(chunks, 4096));
    hipLaunchKernelGGL(fn, dim3(grid), dim3(kThreads), 0, stream, s);
    return hipGetLastError();
}

const char* kernel_name(int k, int rows, Mode mode, bool parity) {
    const Choice ch = pick(k, rows, mode, true, bs::use(parity, k, rows, bs::kWideCode));
    return ch.cm      ? "rs_code_kernel<K,MR,MODE,ADDR,U,NT,true>"
           : ch.fixed ? "rs_code_kernel<K,MR,MODE,ADDR,U,NT>"
                      : "rs_code_kernel<0,MR,MODE,ADDR,U,NT>";
}

}  // namespace blbrs
