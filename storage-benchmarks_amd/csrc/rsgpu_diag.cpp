// rsgpu_diag.cpp -- exports of the DIAGNOSTIC build only (make diag ->
// tools/diag/librsgpu_diag.so, compiled with RSGPU_DIAG_CLOCK): the in-kernel
// clock stamps of k_rs_bs and k_rs_jitw (diag_clock.h).  Not part of
// include/rsgpu.h; the product library does not contain this file.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "diag_clock.h"

#ifndef RSGPU_DIAG_CLOCK
#error "rsgpu_diag.cpp belongs to the diagnostic build (-DRSGPU_DIAG_CLOCK)"
#endif

namespace rsgpu {
namespace bs {
hipError_t diag_read_bs(void* host, size_t bytes);
hipError_t diag_read_bs_clear();
}  // namespace bs
namespace jitk {
hipError_t diag_read_jitw(void* host, size_t bytes);
hipError_t diag_read_jitw_clear();
hipError_t diag_read_jitw_phase(void* host, size_t bytes);
}  // namespace jitk
}  // namespace rsgpu

extern "C" {

// which 0: k_rs_bs (compiled encode), 1: k_rs_jitw (generated two-wave
// layouts); out receives [kSlots][4] = (s_memtime, s_memrealtime) at the
// start and end of one workgroup in kEvery (zeros where none was stamped)
int rsgpu_diag_clock_read(int which, unsigned long long* out, size_t bytes)
{
    const hipError_t e = which == 0 ? rsgpu::bs::diag_read_bs(out, bytes) : rsgpu::jitk::diag_read_jitw(out, bytes);
    return e == hipSuccess ? 0 : -2;
}

int rsgpu_diag_clock_clear(void)
{
    return rsgpu::bs::diag_read_bs_clear() == hipSuccess && rsgpu::jitk::diag_read_jitw_clear() == hipSuccess ? 0
                                                                                                              : -2;
}

int rsgpu_diag_clock_slots(void) { return rsgpu::diag::kSlots; }

// variant 6 only: k_rs_jitw's per-wave phase cycle sums,
// [kSlots][kPhaseWaves][kPhases] (diag_clock.h); zeros in other builds
int rsgpu_diag_phase_read(unsigned long long* out, size_t bytes)
{
    return rsgpu::jitk::diag_read_jitw_phase(out, bytes) == hipSuccess ? 0 : -2;
}

}  // extern "C"
