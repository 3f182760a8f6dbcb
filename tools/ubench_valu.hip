// ubench_valu.hip -- VALU issue-rate microbenchmark for the instruction mix of
// the GF(2^8) kernels (tool, not product).  Each thread runs 16 independent
// chains of one instruction (inline asm, so the count is exact); the kernel
// measures its own shader clock (s_memtime vs s_memrealtime @100 MHz) and
// reports cycles per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_IT 2048

#define BODY(ASM)                                                                         \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) { ASM; }

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, unsigned long long* clk, uint32_t seed)
{
    uint32_t r[16], t[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        r[i] = seed * (threadIdx.x + 1) * (i + 3);
        t[i] = seed ^ (i * 0x01010101u) ^ threadIdx.x;
    }
    const uint32_t s = __builtin_amdgcn_readfirstlane(seed ^ 0x5a5a5a5au);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < N_IT; ++it) {
        if constexpr (OP == 0) BODY(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 1) BODY(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(t[i]), "v"(t[(i + 1) & 15])))
        if constexpr (OP == 2) BODY(asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(r[i]) : "v"(t[i]), "v"(t[(i + 1) & 15])))
        if constexpr (OP == 3) BODY(asm volatile("v_perm_b32 %0, %1, %1, %0" : "+v"(r[i]) : "s"(s)))
        if constexpr (OP == 4) BODY(asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(r[i])))
        if constexpr (OP == 5) BODY(asm volatile("v_and_b32 %0, %0, %1" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 6) BODY(asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 7) BODY(asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 8) BODY(asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(t[i]), "v"(t[(i + 1) & 15])))
        if constexpr (OP == 9) BODY(asm volatile("v_alignbit_b32 %0, %0, %1, 3" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 10) BODY(asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r[i]) : "s"(s)))
        if constexpr (OP == 11) BODY(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(t[i]), "s"(s)))
        if constexpr (OP == 12) BODY(asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(r[i])))
        if constexpr (OP == 13) BODY(asm volatile("v_mov_b32 %0, %1" : "=v"(r[i]) : "v"(r[(i + 1) & 15])))
        if constexpr (OP == 14) BODY(asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 15) BODY(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[i]) : "v"(t[i])))
        if constexpr (OP == 16) {
            // 64-bit shifts on register pairs (8 pairs = the 16 chains)
            _Pragma("unroll") for (int i = 0; i < 16; i += 2) {
                unsigned long long x = ((unsigned long long)r[i + 1] << 32) | r[i];
                asm volatile("v_lshlrev_b64 %0, 4, %0" : "+v"(x));
                asm volatile("v_lshrrev_b64 %0, 2, %0" : "+v"(x));
                r[i] = (uint32_t)x;
                r[i + 1] = (uint32_t)(x >> 32);
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        acc ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
void run(const char* name, int wg_per_cu, uint32_t* d, unsigned long long* dclk)
{
    const int cus = 256;
    dim3 grid(cus * wg_per_cu), block(256);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, dclk, 12345u);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(kern<OP>, grid, block, 0, 0, d, dclk, 777u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    unsigned long long h[2];
    (void)hipMemcpy(h, dclk, sizeof(h), hipMemcpyDeviceToHost);
    const double ghz = (double)h[0] / ((double)h[1] * 10.0);  // realtime = 100 MHz
    // per SIMD: wg_per_cu waves (256-thread WG = 4 waves = 1 per SIMD)
    const double instr_per_simd = (double)wg_per_cu * N_IT * 16.0;
    const double cycles = ms * 1e6 * ghz;  // kernel cycles (approx., includes launch)
    printf("  %-18s waves/SIMD=%d  clk=%.2f GHz  cycles/instr/SIMD=%.2f  (in-kernel %.2f)\n", name,
           wg_per_cu, ghz, cycles / instr_per_simd, (double)h[0] / (N_IT * 16.0) / wg_per_cu);
}

int main()
{
    uint32_t* d;
    unsigned long long* c;
    (void)hipMalloc(&d, 256 * 256 * 8 * sizeof(uint32_t));
    (void)hipMalloc(&c, 16);
    for (int w : {1, 2, 4, 8}) {
        run<0>("v_xor", w, d, c);
        run<10>("v_xor(sgpr)", w, d, c);
        run<1>("v_bitop3", w, d, c);
        run<11>("v_bitop3(sgpr)", w, d, c);
        run<2>("v_perm", w, d, c);
        run<3>("v_perm(sgpr,sgpr)", w, d, c);
        run<4>("v_lshlrev", w, d, c);
        run<12>("v_lshrrev", w, d, c);
        run<5>("v_and", w, d, c);
        run<6>("v_pk_mul_lo_u16", w, d, c);
        run<14>("v_pk_add_u16", w, d, c);
        run<7>("v_lshl_or", w, d, c);
        run<8>("v_bfi", w, d, c);
        run<9>("v_alignbit", w, d, c);
        run<13>("v_mov", w, d, c);
        run<15>("v_cndmask", w, d, c);
        run<16>("v_lshl/rrev_b64", w, d, c);
    }
    return 0;
}
