// kernel_hooks.h -- the places where the diagnostic build's timing-only
// variants (diag_variants.h) differ from the product, as one policy type.
//
// The product kernels (k_rs_bs in rs_bitsliced.hip, k_rs_jitw in rs_jit.hip)
// and the generated-code words (rs_jit.h Wide) read `Hooks`.  In the product
// build Hooks = ProductHooks: every hook is the identity or a compile-time
// constant, and the kernels compile to exactly what they compute.  Only the
// diagnostic library (make diag DIAG_VARIANT=n -> tools/diag/, never
// rsgpu/librsgpu.so) defines RSGPU_DIAG_VARIANT and swaps in
// diag::Variant<n>, whose outputs are WRONG by design.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RH_HD __host__ __device__
#else
#define RH_HD
#endif

namespace rsgpu {

struct ProductHooks {
    static constexpr int kVariant = 0;
    // row data: the block whose rows a workgroup reads and writes, and the
    // byte offset within them of its lane (o: the product's offset; wg: the
    // workgroup's tile index)
    RH_HD static constexpr long long data_block(long long b) { return b; }
    RH_HD static constexpr long long data_offset(long long o, long long /*wg*/, int /*lane*/) { return o; }
    // k_rs_jitw: the block and chunk whose generated code a wave runs
    RH_HD static constexpr long long code_block(long long b) { return b; }
    RH_HD static constexpr int code_chunk(int ch, bool /*full_chunk*/) { return ch; }
    // source transposes done / their planes kept
    static constexpr bool kTransposes = true;
    static constexpr bool kZeroPlanes = false;
    // k_rs_bs: the planes fed to the multiply-accumulates come from LDS
    static constexpr bool kZeroValuPlanes = false;
    // k_rs_jitw: per-phase clock stamps
    static constexpr bool kPhaseStamps = false;
    // generated code words (rs_jit.h Wide): extra preamble bytes per source,
    // a replaced preamble word, the composite operands of a multiply-accumulate
    static constexpr int kPreExtra = 0;
    RH_HD static constexpr bool pre_word(int /*t*/, int /*i*/, int /*pl*/, int /*cl*/, int /*addr*/,
                                         uint32_t* /*w*/)
    {
        return false;
    }
    RH_HD static constexpr int pre_index(int i) { return i; }
    RH_HD static constexpr int mac_lo(int lo) { return lo; }
    RH_HD static constexpr int mac_hi(int hi) { return hi; }
};

#if defined(__HIP__)
// a source's planes after its transpose: kept (product), or zeros the
// compiler cannot see through (variant 2: the transpose done, its result quiet)
template <class H>
__device__ inline __attribute__((always_inline)) void hook_planes(uint32_t (&W)[8])
{
    if constexpr (H::kZeroPlanes) {
        asm volatile("" ::"v"(W[0]), "v"(W[1]), "v"(W[2]), "v"(W[3]), "v"(W[4]), "v"(W[5]), "v"(W[6]), "v"(W[7]));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            W[i] = 0;
    }
}
#endif

}  // namespace rsgpu

#if defined(RSGPU_DIAG_VARIANT)
#if !defined(RSGPU_DIAG_CLOCK)
#error "RSGPU_DIAG_VARIANT builds wrong outputs by design: only the diagnostic library (make diag) may set it"
#endif
#include "diag_variants.h"
namespace rsgpu {
using Hooks = diag::Variant<RSGPU_DIAG_VARIANT>;
}
#else
namespace rsgpu {
using Hooks = ProductHooks;
}
#endif
