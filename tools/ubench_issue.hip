// ubench_issue.hip -- the VALU issue ceiling of gfx950 for the engine's
// instruction, measured the way the kernels are (tool, not product).
//
// Every lane runs 16 independent chains acc_i = v_bitop3(acc_i, X_i, Y_i,
// 0x96) on random data (the accumulators toggle about half their bits per
// instruction, as the real MACs do), ITER times, fixed in inline asm so the
// compiler cannot fold the XORs.  WPS waves per SIMD are resident (WPS
// 256-thread workgroups per CU: a grid of 256 x WPS), long enough (~30 ms at
// 4 waves per SIMD) for the clock to settle under load.
//
// Read it with one rocprofv3 pass that holds both counters:
//   rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES -- tools/ubench_issue WPS
// SIMD-cycles per wave64 VALU = (GRBM_GUI_ACTIVE / 8 XCDs) * 1024 SIMDs /
// SQ_INSTS_VALU -- no wall clock involved (tools/valu_ceiling.py).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define B3(i) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[i]) : "v"(x[i]), "v"(y[i]))

__global__ __launch_bounds__(256) void k_issue(unsigned* out, int iters)
{
    unsigned a[16], x[16], y[16];
    unsigned s = (blockIdx.x * 256u + threadIdx.x) * 2654435761u + 12345u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        s = s * 1664525u + 1013904223u;
        a[i] = s;
        s = s * 1664525u + 1013904223u;
        x[i] = s;
        s = s * 1664525u + 1013904223u;
        y[i] = s ^ (s >> 7);
    }
    for (int it = 0; it < iters; ++it) {
        B3(0); B3(1); B3(2); B3(3); B3(4); B3(5); B3(6); B3(7);
        B3(8); B3(9); B3(10); B3(11); B3(12); B3(13); B3(14); B3(15);
    }
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main(int argc, char** argv)
{
    const int wps = argc > 1 ? atoi(argv[1]) : 4;       // waves per SIMD
    const int iters = argc > 2 ? atoi(argv[2]) : 400000;
    const int grid = 256 * wps;                          // 256-thread WGs: one per SIMD-wave set
    unsigned* out;
    if (hipMalloc(&out, (size_t)grid * 256 * 4) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(k_issue, dim3(grid), dim3(256), 0, 0, out, iters / 20);  // warm-up
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_issue, dim3(grid), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess)
        return 1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double insts = (double)grid * 4 * iters * 16;  // wave-instructions of the loop
    std::printf("waves_per_simd=%d iters=%d ms=%.3f loop_valu=%.4g  (at 2.4 GHz: %.2f SIMD-cycles per VALU)\n",
                wps, iters, ms, insts, ms * 1e-3 * 2.4e9 * 1024 / insts);
    return 0;
}
