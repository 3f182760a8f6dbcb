// ubench_salu.hip -- scalar-unit issue rate and computed-jump cost on gfx950
// (tool, not product).  Reports cycles per instruction per CU/SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_salu tools/ubench_salu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define N_IT 4096

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, unsigned long long* clk, uint32_t seed)
{
    uint32_t s0 = __builtin_amdgcn_readfirstlane(seed), s1 = s0 ^ 7, s2 = s0 + 3, s3 = s0 * 5;
    uint32_t v0 = threadIdx.x, v1 = v0 ^ seed, v2 = v0 + 1, v3 = v0 + 9;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
        if constexpr (OP == 0) {  // 16 independent-ish SALU ops
#pragma unroll
            for (int i = 0; i < 4; ++i)
                asm volatile("s_add_u32 %0, %0, 1\n s_xor_b32 %1, %1, %0\n s_add_u32 %2, %2, %1\n s_xor_b32 %3, %3, %2"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) : : "scc");
        } else if constexpr (OP == 1) {  // 16 SALU interleaved with 16 VALU
#pragma unroll
            for (int i = 0; i < 4; ++i)
                asm volatile("s_add_u32 %0, %0, 1\n v_xor_b32 %4, %4, %5\n s_xor_b32 %1, %1, %0\n v_xor_b32 %5, %5, %6\n"
                             " s_add_u32 %2, %2, %1\n v_xor_b32 %6, %6, %7\n s_xor_b32 %3, %3, %2\n v_xor_b32 %7, %7, %4"
                             : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : : "scc");
        } else if constexpr (OP == 2) {  // computed jump over one of 2 equal blocks, 8 VALU each
            asm volatile(
                "s_and_b32 s40, %4, 1\n"
                "s_mul_i32 s40, s40, 32\n"
                "s_getpc_b64 s[42:43]\n"
                "GPC_%=:\n"
                "s_add_u32 s42, s42, s40\n"
                "s_addc_u32 s43, s43, 0\n"
                "s_add_u32 s42, s42, BLK0_%=-GPC_%=\n"
                "s_addc_u32 s43, s43, 0\n"
                "s_setpc_b64 s[42:43]\n"
                "BLK0_%=:\n"
                "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_xor_b32 %2, %2, %3\n v_xor_b32 %3, %3, %0\n"
                "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_xor_b32 %2, %2, %3\n s_branch END_%=\n"
                "BLK1_%=:\n"
                "v_xor_b32 %3, %3, %0\n v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_xor_b32 %2, %2, %3\n"
                "v_xor_b32 %3, %3, %0\n v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n s_branch END_%=\n"
                "END_%=:\n"
                : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3)
                : "s"(s0 + it)
                : "s40", "s42", "s43", "scc");
        } else if constexpr (OP == 3) {  // same VALU work, no jump
            asm volatile(
                "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_xor_b32 %2, %2, %3\n v_xor_b32 %3, %3, %0\n"
                "v_xor_b32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_xor_b32 %2, %2, %3\n"
                : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        } else if constexpr (OP == 4) {  // uniform compare+branch tree depth 4 around 8 VALU
            int c = __builtin_amdgcn_readfirstlane((int)((s0 + it) & 15));
            if (c < 8) {
                if (c < 4) { v0 ^= v1; v1 ^= v2; } else { v1 ^= v3; v2 ^= v0; }
            } else {
                if (c < 12) { v2 ^= v1; v3 ^= v2; } else { v3 ^= v0; v0 ^= v2; }
            }
            v0 ^= v3; v1 ^= v0; v2 ^= v1; v3 ^= v2; v0 ^= v1; v1 ^= v3;
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = s0 ^ s1 ^ s2 ^ s3 ^ v0 ^ v1 ^ v2 ^ v3;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        clk[0] = t1 - t0;
}

template <int OP>
void run(const char* name, int wg_per_cu, uint32_t* d, unsigned long long* c, double units)
{
    dim3 grid(256 * wg_per_cu), block(256);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, c, 3u);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, c, 5u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long h;
    (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    // per SIMD: wg_per_cu waves; total units per SIMD = wg_per_cu * N_IT * units
    const double cyc = ms * 1e6 * 2.2;  // assume 2.2 GHz
    printf("  %-28s waves/SIMD=%d  wall-cycles per unit per SIMD=%.2f  (one wave: %.2f)\n", name,
           wg_per_cu, cyc / (wg_per_cu * N_IT * units), (double)h / (N_IT * units));
}

int main(int argc, char** argv)
{
    const int op = argc > 1 ? atoi(argv[1]) : 0;
    uint32_t* d;
    unsigned long long* c;
    (void)hipMalloc(&d, 256 * 256 * 8 * 4);
    (void)hipMalloc(&c, 16);
    for (int w : {1, 4, 8}) {
        if (op == 0) run<0>("salu x16 (unit=salu)", w, d, c, 16);
        if (op == 1) run<1>("salu16+valu16 (unit=pair)", w, d, c, 16);
        if (op == 2) run<2>("jump+7valu (unit=iter)", w, d, c, 1);
        if (op == 3) run<3>("7valu (unit=iter)", w, d, c, 1);
        if (op == 4) run<4>("branchtree+8valu (unit=iter)", w, d, c, 1);
        fflush(stdout);
    }
    return 0;
}
