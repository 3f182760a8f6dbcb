// ubench_jump.hip -- cost of threaded-code dispatch on gfx950 (tool, not
// product): each "coefficient" is an s_swappc_b64 into one of 256 handler
// blocks of 8 v_bitop3 (the bit-sliced multiply-accumulate of one GF(2^8)
// coefficient) that returns with s_setpc_b64.  Variants:
//   0: the 8 v_bitop3 inline, no jump (VALU floor)
//   1: jump to handler chosen per coefficient (targets preloaded in SGPRs)
//   2: as 1, plus s_set_gpr_idx_on/off so the handler's accumulator operand
//      is relative to a runtime slot index (one handler set for all slots)
//   3: as 1, but the 8 targets per group come from s_load_dwordx16 of a
//      device table (what a real kernel would do)
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_jump tools/ubench_jump.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <string>

#define N_IT 2048

#define CLOB                                                                                     \
    "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v20", "v21", "v22", "v23", "v24",   \
        "v25", "v26", "v27", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "s90", "s91", \
        "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "scc"

// one handler block = 8 bitop3 + (optional gpr_idx_off) + return, padded to 64 B
#define HANDLER_ABS                                                                               \
    ".p2align 6\n"                                                                                \
    "v_bitop3_b32 v10, v10, v20, v36 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v11, v11, v21, v37 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v12, v12, v22, v38 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v13, v13, v23, v39 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v14, v14, v24, v40 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v15, v15, v25, v41 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v16, v16, v26, v42 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v17, v17, v27, v43 bitop3:0x96\n"                                               \
    "s_setpc_b64 s[90:91]\n"
#define HANDLER_REL                                                                               \
    ".p2align 6\n"                                                                                \
    "v_bitop3_b32 v10, v10, v20, v36 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v11, v11, v21, v37 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v12, v12, v22, v38 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v13, v13, v23, v39 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v14, v14, v24, v40 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v15, v15, v25, v41 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v16, v16, v26, v42 bitop3:0x96\n"                                               \
    "v_bitop3_b32 v17, v17, v27, v43 bitop3:0x96\n"                                               \
    "s_set_gpr_idx_off\n"                                                                         \
    "s_setpc_b64 s[90:91]\n"
#define X4(H) H H H H
#define X16(H) X4(H) X4(H) X4(H) X4(H)
#define X256(H) X16(X16(H))

#define HSET0 ".p2align 6\n" "v_bitop3_b32 v10, v10, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v11, v11, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v12, v12, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v13, v13, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v14, v14, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v15, v15, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v16, v16, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v17, v17, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET1 ".p2align 6\n" "v_bitop3_b32 v44, v44, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v45, v45, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v46, v46, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v47, v47, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v48, v48, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v49, v49, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v50, v50, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v51, v51, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET2 ".p2align 6\n" "v_bitop3_b32 v52, v52, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v53, v53, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v54, v54, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v55, v55, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v56, v56, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v57, v57, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v58, v58, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v59, v59, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET3 ".p2align 6\n" "v_bitop3_b32 v60, v60, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v61, v61, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v62, v62, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v63, v63, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v64, v64, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v65, v65, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v66, v66, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v67, v67, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET4 ".p2align 6\n" "v_bitop3_b32 v68, v68, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v69, v69, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v70, v70, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v71, v71, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v72, v72, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v73, v73, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v74, v74, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v75, v75, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET5 ".p2align 6\n" "v_bitop3_b32 v76, v76, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v77, v77, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v78, v78, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v79, v79, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v80, v80, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v81, v81, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v82, v82, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v83, v83, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET6 ".p2align 6\n" "v_bitop3_b32 v84, v84, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v85, v85, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v86, v86, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v87, v87, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v88, v88, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v89, v89, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v90, v90, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v91, v91, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HSET7 ".p2align 6\n" "v_bitop3_b32 v92, v92, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v93, v93, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v94, v94, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v95, v95, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v96, v96, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v97, v97, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v98, v98, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v99, v99, v27, v43 bitop3:0x96\n" "s_setpc_b64 s[90:91]\n"
#define HREL ".p2align 6\n" "v_bitop3_b32 v10, v10, v20, v36 bitop3:0x96\n" "v_bitop3_b32 v11, v11, v21, v37 bitop3:0x96\n" "v_bitop3_b32 v12, v12, v22, v38 bitop3:0x96\n" "v_bitop3_b32 v13, v13, v23, v39 bitop3:0x96\n" "v_bitop3_b32 v14, v14, v24, v40 bitop3:0x96\n" "v_bitop3_b32 v15, v15, v25, v41 bitop3:0x96\n" "v_bitop3_b32 v16, v16, v26, v42 bitop3:0x96\n" "v_bitop3_b32 v17, v17, v27, v43 bitop3:0x96\n" "s_set_gpr_idx_off\n" "s_setpc_b64 s[90:91]\n"
#define CLOB8 CLOB, "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107"

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, unsigned long long* clk,
                                            const uint64_t* offs, uint32_t seed)
{
    uint32_t r = threadIdx.x ^ seed;
    // base address of the handler table, and 8 handler targets in s[80:89]
    // (s[80:81].. are rewritten per group from `offs` for OP 3)
    asm volatile(
        "v_mov_b32 v10, %0\n v_mov_b32 v11, %0\n v_mov_b32 v12, %0\n v_mov_b32 v13, %0\n"
        "v_mov_b32 v14, %0\n v_mov_b32 v15, %0\n v_mov_b32 v16, %0\n v_mov_b32 v17, %0\n"
        "v_mov_b32 v20, 1\n v_mov_b32 v21, 2\n v_mov_b32 v22, 3\n v_mov_b32 v23, 4\n"
        "v_mov_b32 v24, 5\n v_mov_b32 v25, 6\n v_mov_b32 v26, 7\n v_mov_b32 v27, 8\n"
        "v_mov_b32 v36, 9\n v_mov_b32 v37, 10\n v_mov_b32 v38, 11\n v_mov_b32 v39, 12\n"
        "v_mov_b32 v40, 13\n v_mov_b32 v41, 14\n v_mov_b32 v42, 15\n v_mov_b32 v43, 16\n"
        :
        : "v"(r)
        : CLOB);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
        if constexpr (OP == 0) {
            asm volatile(X4(
                             "v_bitop3_b32 v10, v10, v20, v36 bitop3:0x96\n"
                             "v_bitop3_b32 v11, v11, v21, v37 bitop3:0x96\n"
                             "v_bitop3_b32 v12, v12, v22, v38 bitop3:0x96\n"
                             "v_bitop3_b32 v13, v13, v23, v39 bitop3:0x96\n"
                             "v_bitop3_b32 v14, v14, v24, v40 bitop3:0x96\n"
                             "v_bitop3_b32 v15, v15, v25, v41 bitop3:0x96\n"
                             "v_bitop3_b32 v16, v16, v26, v42 bitop3:0x96\n"
                             "v_bitop3_b32 v17, v17, v27, v43 bitop3:0x96\n")::
                             : CLOB);
        } else {
            // 4 coefficients per iteration: targets = base + ((it*4+j)*off-hash & 255)*64
            const uint32_t sidx = __builtin_amdgcn_readfirstlane((uint32_t)it * 2654435761u ^ seed);
            if constexpr (OP == 4) {
                const uint64_t* p = offs + ((it & 63) * 4);
                asm volatile(
                    "s_load_dwordx8 s[80:87], %0, 0\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    "s_swappc_b64 s[90:91], s[80:81]\n"
                    "s_swappc_b64 s[90:91], s[82:83]\n"
                    "s_swappc_b64 s[90:91], s[84:85]\n"
                    "s_swappc_b64 s[90:91], s[86:87]\n"
                    :
                    : "s"(p)
                    : CLOB8, "memory");
            } else if constexpr (OP == 5) {
                const uint64_t* p = offs + ((it & 63) * 4);
                asm volatile(
                    "s_load_dwordx8 s[80:87], %0, 0\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    "s_mov_b32 s88, 0\n"
                    "s_set_gpr_idx_on s88, gpr_idx(SRC0,DST)\n"
                    "s_swappc_b64 s[90:91], s[80:81]\n"
                    "s_mov_b32 s88, 34\n"
                    "s_set_gpr_idx_on s88, gpr_idx(SRC0,DST)\n"
                    "s_swappc_b64 s[90:91], s[82:83]\n"
                    "s_mov_b32 s88, 42\n"
                    "s_set_gpr_idx_on s88, gpr_idx(SRC0,DST)\n"
                    "s_swappc_b64 s[90:91], s[84:85]\n"
                    "s_mov_b32 s88, 50\n"
                    "s_set_gpr_idx_on s88, gpr_idx(SRC0,DST)\n"
                    "s_swappc_b64 s[90:91], s[86:87]\n"
                    :
                    : "s"(p)
                    : CLOB8, "memory");
            } else if constexpr (OP == 3) {
                const uint64_t* p = offs + ((it & 63) * 4);
                asm volatile(
                    "s_load_dwordx8 s[80:87], %0, 0\n"
                    "s_waitcnt lgkmcnt(0)\n"
                    "s_swappc_b64 s[90:91], s[80:81]\n"
                    "s_swappc_b64 s[90:91], s[82:83]\n"
                    "s_swappc_b64 s[90:91], s[84:85]\n"
                    "s_swappc_b64 s[90:91], s[86:87]\n"
                    :
                    : "s"(p)
                    : CLOB, "memory");
            } else {
                // compute 4 targets from the handler base with cheap SALU (not timed
                // separately; OP 3 is the realistic variant)
                asm volatile(
                    "s_getpc_b64 s[88:89]\n"
                    "GP_%=:\n"
                    "s_add_u32 s88, s88, HB_%=-GP_%=\n"
                    "s_addc_u32 s89, s89, 0\n"
                    "s_and_b32 s80, %0, 0x3fc0\n"
                    "s_add_u32 s80, s80, s88\n s_addc_u32 s81, s89, 0\n"
                    "s_lshr_b32 s82, %0, 8\n s_and_b32 s82, s82, 0x3fc0\n"
                    "s_add_u32 s82, s82, s88\n s_addc_u32 s83, s89, 0\n"
                    "s_lshr_b32 s84, %0, 16\n s_and_b32 s84, s84, 0x3fc0\n"
                    "s_add_u32 s84, s84, s88\n s_addc_u32 s85, s89, 0\n"
                    "s_lshr_b32 s86, %0, 20\n s_and_b32 s86, s86, 0x3fc0\n"
                    "s_add_u32 s86, s86, s88\n s_addc_u32 s87, s89, 0\n"
                    "s_branch GO_%=\n"
                    ".p2align 6\n"
                    "HB_%=:\n" X256(HANDLER_ABS)
                    "GO_%=:\n"
                    "s_swappc_b64 s[90:91], s[80:81]\n"
                    "s_swappc_b64 s[90:91], s[82:83]\n"
                    "s_swappc_b64 s[90:91], s[84:85]\n"
                    "s_swappc_b64 s[90:91], s[86:87]\n"
                    :
                    : "s"(sidx)
                    : CLOB);
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t v;
    asm volatile("v_xor_b32 %0, v10, v17" : "=v"(v) : : CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        clk[0] = t1 - t0;
}

// Handler block for OP 3 lives in its own kernel-less asm function so its
// address can be taken: a __device__ function whose body is the handler set.
extern "C" __global__ void handler_anchor(uint64_t* base)
{
    uint64_t b;
    asm volatile(
        "s_getpc_b64 s[88:89]\n"
        "GPA:\n"
        "s_add_u32 s88, s88, HA-GPA\n"
        "s_addc_u32 s89, s89, 0\n"
        "s_mov_b64 %0, s[88:89]\n"
        "s_branch HAEND\n"
        ".p2align 6\n"
        "HA:\n" X256(HANDLER_ABS) "HAEND:\n"
        : "=s"(b)
        :
        : "s88", "s89", "scc");
    if (threadIdx.x == 0)
        *base = b;
}

extern "C" __global__ void handler_anchor8(uint64_t* base)
{
    uint64_t b;
    asm volatile(
        "s_getpc_b64 s[88:89]\n"
        "GPA8:\n"
        "s_add_u32 s88, s88, HA8-GPA8\n"
        "s_addc_u32 s89, s89, 0\n"
        "s_mov_b64 %0, s[88:89]\n"
        "s_getpc_b64 s[86:87]\n"
        "GPB8:\n"
        "s_add_u32 s86, s86, HAEND8-GPB8\n"
        "s_addc_u32 s87, s87, 0\n"
        "s_setpc_b64 s[86:87]\n"
        ".p2align 6\n"
        "HA8:\n" X256(HSET0) X256(HSET1) X256(HSET2) X256(HSET3) X256(HSET4) X256(HSET5)
        X256(HSET6) X256(HSET7) "HAEND8:\n"
        : "=s"(b)
        :
        : "s88", "s89", "scc");
    if (threadIdx.x == 0)
        *base = b;
}

extern "C" __global__ void handler_anchor_rel(uint64_t* base)
{
    uint64_t b;
    asm volatile(
        "s_getpc_b64 s[88:89]\n"
        "GPAR:\n"
        "s_add_u32 s88, s88, HAR-GPAR\n"
        "s_addc_u32 s89, s89, 0\n"
        "s_mov_b64 %0, s[88:89]\n"
        "s_branch HAENDR\n"
        ".p2align 6\n"
        "HAR:\n" X256(HREL) "HAENDR:\n"
        : "=s"(b)
        :
        : "s88", "s89", "scc");
    if (threadIdx.x == 0)
        *base = b;
}

template <int OP>
void run(const char* name, int wg_per_cu, uint32_t* d, unsigned long long* c, const uint64_t* offs,
         double units)
{
    dim3 grid(256 * wg_per_cu), block(256);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, c, offs, 3u);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, c, offs, 5u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long h;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    const double cyc = ms * 1e6 * 2.2;
    printf("  %-34s waves/SIMD=%d  cycles per coef per SIMD=%.2f  (one wave: %.2f)  err=%s\n", name,
           wg_per_cu, cyc / (wg_per_cu * N_IT * units), (double)h / (N_IT * units),
           hipGetErrorString(hipGetLastError()));
}

int main(int argc, char** argv)
{
    const int op = argc > 1 ? atoi(argv[1]) : 0;
    uint32_t* d;
    unsigned long long* c;
    uint64_t *offs, *dbase;
    (void)hipMalloc(&d, 256 * 256 * 8 * 4);
    (void)hipMalloc(&c, 16);
    (void)hipMalloc(&offs, 256 * 8);
    (void)hipMalloc(&dbase, 8);
    if (op == 4)
        hipLaunchKernelGGL(handler_anchor8, dim3(1), dim3(64), 0, 0, dbase);
    else if (op == 5)
        hipLaunchKernelGGL(handler_anchor_rel, dim3(1), dim3(64), 0, 0, dbase);
    else
        hipLaunchKernelGGL(handler_anchor, dim3(1), dim3(64), 0, 0, dbase);
    uint64_t base = 0;
    (void)hipMemcpy(&base, dbase, 8, hipMemcpyDeviceToHost);
    std::vector<uint64_t> h(256);
    uint32_t x = 12345;
    const uint32_t nh = op == 4 ? 2048 : 256;
    for (auto& t : h) {
        x = x * 1664525u + 1013904223u;
        t = base + (uint64_t)((x >> 11) % nh) * 64;
    }
    (void)hipMemcpy(offs, h.data(), 256 * 8, hipMemcpyHostToDevice);
    printf("handler base %#llx\n", (unsigned long long)base);
    for (int w : {1, 4, 8}) {
        if (op == 0) run<0>("inline 8 bitop3 (unit=coef)", w, d, c, offs, 4);
        if (op == 1) run<1>("jump, SALU-computed targets", w, d, c, offs, 4);
        if (op == 3) run<3>("jump, s_load targets", w, d, c, offs, 4);
        if (op == 4) run<4>("jump, 8 handler sets (128 KB)", w, d, c, offs, 4);
        if (op == 5) run<5>("jump, gpr_idx relative acc", w, d, c, offs, 4);
        fflush(stdout);
    }
    return 0;
}
