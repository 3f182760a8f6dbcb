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

// The timing-only energy variants (DIAG_VARIANT=n) are policies of their own:
// kernel_hooks.h / diag_variants.h.

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
// variant 6: per-wave cycle sums per phase of the stamped workgroups (one
// table per translation unit, as the clock table)
namespace rsgpu {
namespace diag {
constexpr int kPhases = 8;
constexpr int kPhaseWaves = 4;
}  // namespace diag
}  // namespace rsgpu
static __device__ unsigned long long g_rsgpu_phase[::rsgpu::diag::kSlots][::rsgpu::diag::kPhaseWaves]
                                                  [::rsgpu::diag::kPhases];
namespace rsgpu {
namespace diag {
struct PhaseTimer {
    unsigned long long sum[kPhases] = {}, t, start;
    __device__ PhaseTimer() : t(memtime()), start(t) {}
    __device__ void mark(int p)
    {
        const unsigned long long n = memtime();
        sum[p] += n - t;
        t = n;
    }
    __device__ void end(int wave)
    {
        sum[kPhases - 1] = memtime() - start;
        const unsigned lin = blockIdx.x + gridDim.x * blockIdx.y;
        if ((threadIdx.x & 63) == 0 && lin % kEvery == 0 && wave < kPhaseWaves)
            for (int i = 0; i < kPhases; ++i)
                g_rsgpu_phase[(lin / kEvery) % kSlots][wave][i] = sum[i];
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
#define RSGPU_DIAG_PHASE_READER(NAME)
#define RSGPU_DIAG_BEGIN()
#define RSGPU_DIAG_END() \
    do {                 \
    } while (0)
#define RSGPU_DIAG_READER(NAME)
#endif

namespace rsgpu {
namespace diag {
// phase stamps of k_rs_jitw: the diagnostic PhaseTimer when the hooks ask
// for them (variant 6), nothing otherwise
struct NoPhases {
    __device__ void mark(int) {}
    __device__ void end(int) {}
};
}  // namespace diag
}  // namespace rsgpu
