// diag_variants.h -- the timing-only energy variants of the DIAGNOSTIC build
// (round 5; make -C storage-benchmarks_amd diag DIAG_VARIANT=n ->
// tools/diag/librsgpu_diag_vn.so, tools/energy_run.sh).  Each is the product
// instruction stream with one component's data made quiet or one phase
// removed; their outputs are WRONG by construction.  Only kernel_hooks.h
// includes this file, and only when RSGPU_DIAG_VARIANT is set together with
// RSGPU_DIAG_CLOCK (the diagnostic library's own flag).
//   1 hbmq    sources read from, rows written to, a window of two blocks x
//             16 KB per row that stays in the XCD's L2 (HBM I/O quiet)
//   2 zplane  the transposes write zero planes (LDS plane writes and reads,
//             the VALU of the multiply-accumulates and the row stores quiet)
//   3 valuq   the planes are read from LDS as usual but land in dead
//             registers, the VALU works on zero planes (VALU quiet)
//   4 nowait  the generated decode's per-source LDS wait removed
//   5 notr    the source transposes skipped (raw bytes used as planes)
//   6 phases  the product stream plus s_memtime stamps between the phases of
//             k_rs_jitw (per-wave cycle sums of one workgroup in kEvery)
//   7 code0   k_rs_jitw runs block 0's code in every block (L2-resident code)
//   8 chunk0  k_rs_jitw runs each wave's chunk-0 code for every full chunk
//             (instruction-cache-resident code)
//   9, 10     marginal LDS / VALU prices of the generated decode: two more
//             LDS reads / eight more VALU per source
//   11 lfix   every multiply-accumulate of the generated code reads the same
//             low-nibble composite (one operand's data constant between
//             consecutive instructions; same instruction count)
//   12 lhfix  both composite operands fixed the same way
#pragma once
#include "jit_enc.h"

namespace rsgpu {
namespace diag {

template <int V>
struct Variant : ProductHooks {
    static_assert(V >= 1 && V <= 12, "diagnostic variants are 1..12");
    static constexpr int kVariant = V;
    RH_HD static constexpr long long data_block(long long b) { return V == 1 ? (b & 1) : b; }
    RH_HD static constexpr long long data_offset(long long o, long long wg, int lane)
    {
        return V == 1 ? (wg & 7) * 2048 + lane * 32 : o;
    }
    RH_HD static constexpr long long code_block(long long b) { return V == 7 ? 0 : b; }
    RH_HD static constexpr int code_chunk(int ch, bool full_chunk) { return V == 8 && full_chunk ? 0 : ch; }
    static constexpr bool kTransposes = V != 5;
    static constexpr bool kZeroPlanes = V == 2;
    static constexpr bool kZeroValuPlanes = V == 3;
    static constexpr bool kPhaseStamps = V == 6;
    static constexpr int kPreExtra = V == 9 ? 16 : V == 10 ? 32 : 0;
    // preamble word i of source t (rs_jit.h Wide::pre_u32; pl / cl: the plane
    // and composite registers, addr: the LDS address register)
    RH_HD static constexpr bool pre_word(int t, int i, int pl, int cl, int addr, uint32_t* w)
    {
        using namespace jit;
        if (V == 3 && i < 4) {  // the planes land in the composite registers
            const uint64_t d = enc_ds_read_b128(i < 2 ? cl : cl + 4, addr, t * LDS_SRC + (i < 2 ? 0 : LDS_HALF));
            *w = (i & 1) ? (uint32_t)(d >> 32) : (uint32_t)d;
            return true;
        }
        if (V == 4 && i == 4) {  // no wait for them
            *w = S_NOP0;
            return true;
        }
        if (V == 9 && i >= 4 && i < 8) {  // the planes read a second time, into v18..v25
            const uint64_t d = enc_ds_read_b128(i < 6 ? cl : cl + 4, addr, t * LDS_SRC + (i < 6 ? 0 : LDS_HALF));
            *w = (i & 1) ? (uint32_t)(d >> 32) : (uint32_t)d;
            return true;
        }
        if (V == 10 && i >= 27) {  // after the composites: v18..v21 ^= v10 twice
            *w = i < 35 ? enc_xor_e32(cl + ((i - 27) >> 1), pl, cl + ((i - 27) >> 1)) : S_NOP0;
            return true;
        }
        return false;
    }
    RH_HD static constexpr int pre_index(int i) { return V == 9 && i >= 8 ? i - 4 : i; }
    RH_HD static constexpr int mac_lo(int lo) { return (V == 11 || V == 12) && lo ? 1 : lo; }
    RH_HD static constexpr int mac_hi(int hi) { return V == 12 && hi ? 1 : hi; }
};

}  // namespace diag
}  // namespace rsgpu
