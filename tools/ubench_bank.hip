// ubench_bank.hip -- does the VGPR bank of v_bitop3 operands matter on gfx950?
// (tool, not product).  16 independent accumulator chains per lane,
// acc_i ^= X_i ^ Y_i, with the operand registers fixed in asm so their banks
// (register number mod 4) are known:
//   mode 0: acc, X, Y all in bank 0
//   mode 1: acc bank 0, X bank 1, Y bank 2
//   mode 2: acc bank 0, X and Y both bank 1
//   mode 3: acc bank 0, X bank 0, Y bank 1
//   mode 4: acc bank i % 4 (the JIT's accumulator layout), X bank 1, Y bank 2
// Reports SIMD cycles per wave-instruction at 1, 2 and 4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_bank tools/ubench_bank.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define N_IT 4096
#define S(x) #x
#define XS(x) S(x)

// acc registers v64 + 4 i (bank 0) or v64 + i
#define B1(A, X, Y) "v_bitop3_b32 v" XS(A) ", v" XS(A) ", v" XS(X) ", v" XS(Y) " bitop3:0x96\n"

#define BODY_M0                                                                                  \
    B1(64, 32, 36) B1(68, 32, 36) B1(72, 32, 36) B1(76, 32, 36) B1(80, 32, 36) B1(84, 32, 36)    \
    B1(88, 32, 36) B1(92, 32, 36) B1(96, 32, 36) B1(100, 32, 36) B1(104, 32, 36) B1(108, 32, 36) \
    B1(112, 32, 36) B1(116, 32, 36) B1(120, 32, 36) B1(124, 32, 36)
#define BODY_M1                                                                                  \
    B1(64, 33, 34) B1(68, 33, 34) B1(72, 33, 34) B1(76, 33, 34) B1(80, 33, 34) B1(84, 33, 34)    \
    B1(88, 33, 34) B1(92, 33, 34) B1(96, 33, 34) B1(100, 33, 34) B1(104, 33, 34) B1(108, 33, 34) \
    B1(112, 33, 34) B1(116, 33, 34) B1(120, 33, 34) B1(124, 33, 34)
#define BODY_M2                                                                                  \
    B1(64, 33, 37) B1(68, 33, 37) B1(72, 33, 37) B1(76, 33, 37) B1(80, 33, 37) B1(84, 33, 37)    \
    B1(88, 33, 37) B1(92, 33, 37) B1(96, 33, 37) B1(100, 33, 37) B1(104, 33, 37) B1(108, 33, 37) \
    B1(112, 33, 37) B1(116, 33, 37) B1(120, 33, 37) B1(124, 33, 37)
#define BODY_M3                                                                                  \
    B1(64, 32, 33) B1(68, 32, 33) B1(72, 32, 33) B1(76, 32, 33) B1(80, 32, 33) B1(84, 32, 33)    \
    B1(88, 32, 33) B1(92, 32, 33) B1(96, 32, 33) B1(100, 32, 33) B1(104, 32, 33) B1(108, 32, 33) \
    B1(112, 32, 33) B1(116, 32, 33) B1(120, 32, 33) B1(124, 32, 33)
#define BODY_M4                                                                                  \
    B1(64, 33, 34) B1(65, 33, 34) B1(66, 33, 34) B1(67, 33, 34) B1(68, 33, 34) B1(69, 33, 34)    \
    B1(70, 33, 34) B1(71, 33, 34) B1(72, 33, 34) B1(73, 33, 34) B1(74, 33, 34) B1(75, 33, 34)    \
    B1(76, 33, 34) B1(77, 33, 34) B1(78, 33, 34) B1(79, 33, 34)

#define BODY_M5                                                                                  \
    B1(40, 33, 34) B1(41, 33, 34) B1(42, 33, 34) B1(43, 33, 34) B1(44, 33, 34) B1(45, 33, 34)    \
    B1(46, 33, 34) B1(47, 33, 34) B1(48, 33, 34) B1(49, 33, 34) B1(50, 33, 34) B1(51, 33, 34)    \
    B1(52, 33, 34) B1(53, 33, 34) B1(54, 33, 34) B1(55, 33, 34)
#define CLOB5 "v32", "v33", "v34", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", \
              "v50", "v51", "v52", "v53", "v54", "v55"

#define CLOB                                                                                      \
    "v32", "v33", "v34", "v35", "v36", "v37", "v64", "v65", "v66", "v67", "v68", "v69", "v70",     \
        "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v84", "v88", "v92", \
        "v96", "v100", "v104", "v108", "v112", "v116", "v120", "v124"

__global__ __launch_bounds__(256, 8) __attribute__((amdgpu_num_vgpr(64))) void kern5(unsigned* out,
                                                                                    unsigned long long* clk)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    unsigned v;
    asm volatile(
        "v_mov_b32 v32, %1\n v_mov_b32 v33, %1\n v_mov_b32 v34, %1\n"
        "v_mov_b32 v40, 0\n v_mov_b32 v41, 0\n v_mov_b32 v42, 0\n v_mov_b32 v43, 0\n"
        "v_mov_b32 v44, 0\n v_mov_b32 v45, 0\n v_mov_b32 v46, 0\n v_mov_b32 v47, 0\n"
        "v_mov_b32 v48, 0\n v_mov_b32 v49, 0\n v_mov_b32 v50, 0\n v_mov_b32 v51, 0\n"
        "v_mov_b32 v52, 0\n v_mov_b32 v53, 0\n v_mov_b32 v54, 0\n v_mov_b32 v55, 0\n"
        "s_mov_b32 s40, %2\n"
        "1:\n" BODY_M5
        "s_sub_u32 s40, s40, 1\n"
        "s_cmp_lg_u32 s40, 0\n"
        "s_cbranch_scc1 1b\n"
        "v_xor_b32 %0, v40, v48\n v_xor_b32 %0, %0, v55\n"
        : "=v"(v)
        : "v"(threadIdx.x * 0x9E3779B9u), "i"(N_IT)
        : CLOB5, "s40", "scc");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int M>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32))) void kern(unsigned* out,
                                                                                  unsigned long long* clk)
{
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    unsigned v;
#define RUN(BODY)                                                                               \
    asm volatile(                                                                               \
        "v_mov_b32 v32, %1\n v_mov_b32 v33, %1\n v_mov_b32 v34, %1\n v_mov_b32 v35, %1\n"        \
        "v_mov_b32 v36, %1\n v_mov_b32 v37, %1\n"                                               \
        "v_mov_b32 v64, 0\n v_mov_b32 v65, 0\n v_mov_b32 v66, 0\n v_mov_b32 v67, 0\n"            \
        "v_mov_b32 v68, 0\n v_mov_b32 v69, 0\n v_mov_b32 v70, 0\n v_mov_b32 v71, 0\n"            \
        "v_mov_b32 v72, 0\n v_mov_b32 v73, 0\n v_mov_b32 v74, 0\n v_mov_b32 v75, 0\n"            \
        "v_mov_b32 v76, 0\n v_mov_b32 v77, 0\n v_mov_b32 v78, 0\n v_mov_b32 v79, 0\n"            \
        "v_mov_b32 v80, 0\n v_mov_b32 v84, 0\n v_mov_b32 v88, 0\n v_mov_b32 v92, 0\n"            \
        "v_mov_b32 v96, 0\n v_mov_b32 v100, 0\n v_mov_b32 v104, 0\n v_mov_b32 v108, 0\n"         \
        "v_mov_b32 v112, 0\n v_mov_b32 v116, 0\n v_mov_b32 v120, 0\n v_mov_b32 v124, 0\n"        \
        "s_mov_b32 s40, %2\n"                                                                    \
        "1:\n" BODY                                                                             \
        "s_sub_u32 s40, s40, 1\n"                                                                \
        "s_cmp_lg_u32 s40, 0\n"                                                                  \
        "s_cbranch_scc1 1b\n"                                                                    \
        "v_xor_b32 %0, v64, v68\n v_xor_b32 %0, %0, v72\n v_xor_b32 %0, %0, v79\n"                \
        : "=v"(v)                                                                               \
        : "v"(threadIdx.x * 0x9E3779B9u), "i"(N_IT)                                             \
        : CLOB, "s40", "scc")
    if constexpr (M == 0) RUN(BODY_M0);
    if constexpr (M == 1) RUN(BODY_M1);
    if constexpr (M == 2) RUN(BODY_M2);
    if constexpr (M == 3) RUN(BODY_M3);
    if constexpr (M == 4) RUN(BODY_M4);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    unsigned* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, (size_t)cus * 16 * 256 * 4);
    (void)hipMalloc(&clk, 16);
    const char* names[6] = {"acc,X,Y all bank 0", "acc 0, X 1, Y 2", "acc 0, X 1, Y 1", "acc 0, X 0, Y 1",
                            "acc i%4, X 1, Y 2", "<=64 VGPRs"};
    for (int m = 0; m < 6; ++m)
        for (int wps = 1; wps <= (m == 5 ? 8 : 4); wps = m == 5 ? wps + 1 : wps * 2) {
            // wps waves per SIMD: wps * 4 waves per CU -> one WG of 64 * 4 * wps threads... use
            // 256-thread WGs, wps WGs per CU
            const int grid = cus * wps;
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                switch (m) {
                case 0: hipLaunchKernelGGL(kern<0>, dim3(grid), dim3(256), 0, 0, out, clk); break;
                case 1: hipLaunchKernelGGL(kern<1>, dim3(grid), dim3(256), 0, 0, out, clk); break;
                case 2: hipLaunchKernelGGL(kern<2>, dim3(grid), dim3(256), 0, 0, out, clk); break;
                case 3: hipLaunchKernelGGL(kern<3>, dim3(grid), dim3(256), 0, 0, out, clk); break;
                case 4: hipLaunchKernelGGL(kern<4>, dim3(grid), dim3(256), 0, 0, out, clk); break;
                default: hipLaunchKernelGGL(kern5, dim3(grid), dim3(256), 0, 0, out, clk); break;
                }
                (void)hipEventRecord(e1);
                (void)hipDeviceSynchronize();
            }
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            unsigned long long c[2];
            (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
            const double ghz = c[1] ? (double)c[0] / (double)c[1] * 0.1 : 0;
            const double instr = (double)N_IT * 16 * wps;  // per SIMD: wps waves x N_IT x 16
            printf("  %-20s waves/SIMD=%d  clk=%.2f GHz  in-kernel cycles/instr/SIMD=%.2f  (event %.3f ms)\n",
                   names[m], wps, ghz, (double)c[0] / ((double)N_IT * 16) / wps, ms);
            (void)instr;
        }
    return 0;
}
