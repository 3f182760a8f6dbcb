// ubench_idx.hip -- is GPR-index mode itself costly on gfx950? (tool, not
// product)  No jumps: 8 "coefficients" of 8 v_bitop3 each per iteration,
// 4 waves per SIMD, cycles per coefficient per SIMD (s_memtime).
//   V0  8 accumulator slots addressed directly (v64..v127)
//   V1  the same VALU with slot 0's registers relocated by s_set_gpr_idx_idx
//       8*slot inside one s_set_gpr_idx_on/off (the threaded-code pattern)
//   V2  V0 plus one dummy s_mov_b32 per coefficient (SALU count of V1)
//   V3  V1 with the index set once (idx 0 for all slots: mode on, no changes)
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_idx tools/ubench_idx.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define N_IT 4096
#define B8(A)                                                                 \
    "v_bitop3_b32 v" #A "0, v" #A "0, v20, v36 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "1, v" #A "1, v21, v37 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "2, v" #A "2, v22, v38 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "3, v" #A "3, v23, v39 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "4, v" #A "4, v24, v40 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "5, v" #A "5, v25, v41 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "6, v" #A "6, v26, v42 bitop3:0x96\n"                 \
    "v_bitop3_b32 v" #A "7, v" #A "7, v27, v43 bitop3:0x96\n"
// slot s of V0: v[64+8s ..] -- written out with decimal register names
#define S0 B8(6) /* v60..v67: slot base 60 */
#define ACC_CLOB                                                                                 \
    "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72",   \
        "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84",      \
        "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96",      \
        "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",     \
        "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",  \
        "v119", "v120", "v121", "v122", "v123"
#define TAB_CLOB "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "s88"

#define OPS8(base)                                                                               \
    "v_bitop3_b32 v" base "0, v" base "0, v20, v36 bitop3:0x96\n"
// explicit slot bodies (acc base 60 + 8 s)
#define SLOT(a0, a1, a2, a3, a4, a5, a6, a7)                          \
    "v_bitop3_b32 v" #a0 ", v" #a0 ", v20, v36 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a1 ", v" #a1 ", v21, v37 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a2 ", v" #a2 ", v22, v38 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a3 ", v" #a3 ", v23, v39 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a4 ", v" #a4 ", v24, v40 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a5 ", v" #a5 ", v25, v41 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a6 ", v" #a6 ", v26, v42 bitop3:0x96\n"         \
    "v_bitop3_b32 v" #a7 ", v" #a7 ", v27, v43 bitop3:0x96\n"
#define SL0 SLOT(60, 61, 62, 63, 64, 65, 66, 67)
#define SL1 SLOT(68, 69, 70, 71, 72, 73, 74, 75)
#define SL2 SLOT(76, 77, 78, 79, 80, 81, 82, 83)
#define SL3 SLOT(84, 85, 86, 87, 88, 89, 90, 91)
#define SL4 SLOT(92, 93, 94, 95, 96, 97, 98, 99)
#define SL5 SLOT(100, 101, 102, 103, 104, 105, 106, 107)
#define SL6 SLOT(108, 109, 110, 111, 112, 113, 114, 115)
#define SL7 SLOT(116, 117, 118, 119, 120, 121, 122, 123)
#define DUM "s_mov_b32 s88, 7\n"
#define XX(a, l, h) "v_xor_b32_e32 v" #a ", v" #a ", v" #l "\n" "v_xor_b32_e32 v" #a ", v" #a ", v" #h "\n"
#define X2 XX(60, 20, 36) XX(61, 21, 37) XX(62, 22, 38) XX(63, 23, 39) XX(64, 24, 40) XX(65, 25, 41) XX(66, 26, 42) XX(67, 27, 43)

template <int V>
__global__ __launch_bounds__(256) void kern(unsigned* out, unsigned long long* clk, unsigned seed)
{
    unsigned r = threadIdx.x ^ seed;
    asm volatile("v_mov_b32 v20, %0\n v_mov_b32 v21, 2\n v_mov_b32 v22, 3\n v_mov_b32 v23, 4\n"
                 "v_mov_b32 v24, 5\n v_mov_b32 v25, 6\n v_mov_b32 v26, 7\n v_mov_b32 v27, 8\n"
                 "v_mov_b32 v36, 9\n v_mov_b32 v37, 10\n v_mov_b32 v38, 11\n v_mov_b32 v39, 12\n"
                 "v_mov_b32 v40, 13\n v_mov_b32 v41, 14\n v_mov_b32 v42, 15\n v_mov_b32 v43, 16\n"
                 :: "v"(r) : TAB_CLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
        if constexpr (V == 0)
            asm volatile(SL0 SL1 SL2 SL3 SL4 SL5 SL6 SL7 ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 2)
            asm volatile(DUM SL0 DUM SL1 DUM SL2 DUM SL3 DUM SL4 DUM SL5 DUM SL6 DUM SL7 ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 1)
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n" SL0
                         "s_set_gpr_idx_idx 8\n" SL0 "s_set_gpr_idx_idx 16\n" SL0
                         "s_set_gpr_idx_idx 24\n" SL0 "s_set_gpr_idx_idx 32\n" SL0
                         "s_set_gpr_idx_idx 40\n" SL0 "s_set_gpr_idx_idx 48\n" SL0
                         "s_set_gpr_idx_idx 56\n" SL0 "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 4)
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(DST)\n" SL0 SL0 SL0 SL0 SL0 SL0 SL0 SL0
                         "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 5)
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC0)\n" SL0 SL0 SL0 SL0 SL0 SL0 SL0 SL0
                         "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 6)
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC2)\n" SL0 SL0 SL0 SL0 SL0 SL0 SL0 SL0
                         "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 7)  // 2-source VOP2 xors under SRC0|DST: 16 per coefficient
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n" X2 X2 X2 X2 X2 X2 X2 X2
                         "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 8)  // the same VOP2 xors without index mode
            asm volatile(X2 X2 X2 X2 X2 X2 X2 X2 ::: ACC_CLOB, TAB_CLOB);
        if constexpr (V == 3)
            asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n" SL0 SL0 SL0 SL0 SL0 SL0 SL0 SL0
                         "s_set_gpr_idx_off\n" ::: ACC_CLOB, TAB_CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned v;
    asm volatile("v_xor_b32 %0, v60, v123" : "=v"(v) :: ACC_CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0)
        atomicAdd(clk, t1 - t0);
}

template <int V>
void run(const char* name, unsigned* out, unsigned long long* clk)
{
    const int blocks = 256 * 4;  // 4 waves per SIMD
    (void)hipMemset(clk, 0, 8);
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    (void)hipDeviceSynchronize();
    (void)hipMemset(clk, 0, 8);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern<V>, dim3(blocks), dim3(256), 0, 0, out, clk, 1u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long c;
    (void)hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
    const double wave_cycles = (double)c / blocks;  // one sampled wave per block
    const double coefs = (double)N_IT * 8;
    printf("  %-44s %.2f cycles per coef per SIMD (4 waves)   kernel %.3f ms  %s\n", name,
           wave_cycles / coefs / 4, ms, hipGetErrorString(hipGetLastError()));
}

int main()
{
    unsigned* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, 256 * 1024 * 4 * sizeof(unsigned));
    (void)hipMalloc(&clk, 8);
    run<0>("V0 direct slots", out, clk);
    run<2>("V2 direct slots + 1 dummy SALU per coef", out, clk);
    run<3>("V3 gpr_idx mode on, index never changed", out, clk);
    run<1>("V1 gpr_idx mode, s_set_gpr_idx_idx per coef", out, clk);
    run<4>("V4 gpr_idx(DST) only", out, clk);
    run<5>("V5 gpr_idx(SRC0) only", out, clk);
    run<6>("V6 gpr_idx(SRC2) only", out, clk);
    run<7>("V7 gpr_idx(SRC0,DST), 16 v_xor_e32 per coef", out, clk);
    run<8>("V8 16 v_xor_e32 per coef, no index mode", out, clk);
    run<0>("V0 direct slots (again)", out, clk);
    return 0;
}
