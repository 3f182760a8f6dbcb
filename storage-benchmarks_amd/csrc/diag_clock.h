// diag_clock.h -- in-kernel clock stamps for the DIAGNOSTIC build only
// (make -C storage-benchmarks_amd diag -> tools/diag/librsgpu_diag.so; read
// by tools/bound_probe.py).  The product library is built without
// RSGPU_DIAG_CLOCK and the macros below expand to nothing, so no stamp
// executes in the shipped kernels.
//
// Method: MI355X_MICROARCH.md "DVFS give-back" item 6 -- the in-kernel clock
// is delta s_memtime / delta s_memrealtime x 100 MHz, stamped once around a
// workgroup's whole life (wave 0, lane 0) after seconds of back-to-back
// launches.  The stamps go to a buffer of their own (g_clk below) that no
// other code reads; no output is computed from them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Timing-only energy variants of the diagnostic build (round 5,
// tools/energy_run.sh; make diag DIAG_VARIANT=n): the same instruction
// stream with one component's data made quiet, or one phase removed.  Their
// outputs are WRONG by construction; the product build always has 0.
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
//   9, 10     marginal LDS / VALU prices of the generated decode (rs_jit.h)
//   11 lfix   every multiply-accumulate of the generated code reads the same
//             low-nibble composite (one operand's data constant between
//             consecutive instructions; same instruction count)
//   12 lhfix  both composite operands fixed the same way
#if defined(RSGPU_DIAG_CLOCK) && defined(RSGPU_DIAG_VARIANT)
#define RSGPU_DIAG_VAR RSGPU_DIAG_VARIANT
#else
#define RSGPU_DIAG_VAR 0
#endif

#ifdef RSGPU_DIAG_CLOCK
namespace rsgpu {
namespace diag {

constexpr int kSlots = 16384;  // one workgroup in kEvery is stamped
constexpr int kEvery = 32;

__device__ __forceinline__ unsigned long long memtime()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long memrealtime()
{
    unsigned long long t;
    asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

}  // namespace diag
}  // namespace rsgpu

// one stamp table per translation unit (no relocatable device code)
#define RSGPU_DIAG_TABLE static __device__ unsigned long long g_rsgpu_clk[::rsgpu::diag::kSlots][4];
#define RSGPU_DIAG_BEGIN()                                                                          \
    const unsigned long long dg_t0_ = ::rsgpu::diag::memtime();                                     \
    const unsigned long long dg_r0_ = ::rsgpu::diag::memrealtime();
#define RSGPU_DIAG_END()                                                                            \
    do {                                                                                            \
        const unsigned lin_ = blockIdx.x + gridDim.x * blockIdx.y;                                  \
        if (threadIdx.x == 0 && lin_ % ::rsgpu::diag::kEvery == 0) {                                \
            const unsigned long long t1_ = ::rsgpu::diag::memtime();                                \
            const unsigned long long r1_ = ::rsgpu::diag::memrealtime();                            \
            unsigned long long* s_ = g_rsgpu_clk[(lin_ / ::rsgpu::diag::kEvery) % ::rsgpu::diag::kSlots]; \
            s_[0] = dg_t0_;                                                                         \
            s_[1] = dg_r0_;                                                                         \
            s_[2] = t1_;                                                                            \
            s_[3] = r1_;                                                                            \
        }                                                                                           \
    } while (0)
// variant 6: per-wave cycle sums per phase of the stamped workgroups
#define RSGPU_DIAG_PHASE_TABLE \
    static __device__ unsigned long long g_rsgpu_phase[::rsgpu::diag::kSlots][::rsgpu::diag::kPhaseWaves][::rsgpu::diag::kPhases];
namespace rsgpu {
namespace diag {
constexpr int kPhases = 8;
constexpr int kPhaseWaves = 4;
struct PhaseTimer {
    unsigned long long sum[kPhases] = {}, t, start;
    __device__ PhaseTimer() : t(memtime()), start(t) {}
    __device__ void mark(int p)
    {
        const unsigned long long n = memtime();
        sum[p] += n - t;
        t = n;
    }
    template <class Table>
    __device__ void end(Table& tab, int wave)
    {
        sum[kPhases - 1] = memtime() - start;
        const unsigned lin = blockIdx.x + gridDim.x * blockIdx.y;
        if ((threadIdx.x & 63) == 0 && lin % kEvery == 0 && wave < kPhaseWaves)
            for (int i = 0; i < kPhases; ++i)
                tab[(lin / kEvery) % kSlots][wave][i] = sum[i];
    }
};
}  // namespace diag
}  // namespace rsgpu
#define RSGPU_DIAG_PHASE_READER(NAME)                                                               \
    hipError_t NAME(void* host, size_t bytes)                                                       \
    {                                                                                               \
        return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rsgpu_phase),                                 \
                                   bytes < sizeof(g_rsgpu_phase) ? bytes : sizeof(g_rsgpu_phase), 0, \
                                   hipMemcpyDeviceToHost);                                          \
    }

// host side, in the same translation unit as the table
#define RSGPU_DIAG_READER(NAME)                                                                     \
    hipError_t NAME(void* host, size_t bytes)                                                       \
    {                                                                                               \
        return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_rsgpu_clk),                                   \
                                   bytes < sizeof(g_rsgpu_clk) ? bytes : sizeof(g_rsgpu_clk), 0,    \
                                   hipMemcpyDeviceToHost);                                          \
    }                                                                                               \
    hipError_t NAME##_clear()                                                                       \
    {                                                                                               \
        void* p = nullptr;                                                                          \
        hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(g_rsgpu_clk));                            \
        return e != hipSuccess ? e : hipMemset(p, 0, sizeof(g_rsgpu_clk));                         \
    }
#else
#define RSGPU_DIAG_TABLE
#define RSGPU_DIAG_PHASE_TABLE
#define RSGPU_DIAG_PHASE_READER(NAME)
#define RSGPU_DIAG_BEGIN()
#define RSGPU_DIAG_END() \
    do {                 \
    } while (0)
#define RSGPU_DIAG_READER(NAME)
#endif
