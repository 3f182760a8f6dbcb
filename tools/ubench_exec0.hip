// ubench_exec0.hip -- round 6 probe (a tool, not the product): how many
// cycles a wave64 spends issuing a straight run of v_bitop3_b32 with EXEC = 0
// against EXEC = all lanes, one wave per SIMD and 3 waves per SIMD, measured
// with s_memtime around the run.  Question: can a wave walk the generated
// code with EXEC = 0 (to pull its lines into the instruction cache ahead of
// the working waves) for much less than running it?
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_exec0 tools/ubench_exec0.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define OPS16 \
    "v_bitop3_b32 v10, v10, v11, v12 bitop3:0x96\n v_bitop3_b32 v13, v13, v14, v15 bitop3:0x96\n" \
    "v_bitop3_b32 v16, v16, v17, v18 bitop3:0x96\n v_bitop3_b32 v19, v19, v20, v21 bitop3:0x96\n" \
    "v_bitop3_b32 v10, v10, v11, v12 bitop3:0x96\n v_bitop3_b32 v13, v13, v14, v15 bitop3:0x96\n" \
    "v_bitop3_b32 v16, v16, v17, v18 bitop3:0x96\n v_bitop3_b32 v19, v19, v20, v21 bitop3:0x96\n" \
    "v_bitop3_b32 v10, v10, v11, v12 bitop3:0x96\n v_bitop3_b32 v13, v13, v14, v15 bitop3:0x96\n" \
    "v_bitop3_b32 v16, v16, v17, v18 bitop3:0x96\n v_bitop3_b32 v19, v19, v20, v21 bitop3:0x96\n" \
    "v_bitop3_b32 v10, v10, v11, v12 bitop3:0x96\n v_bitop3_b32 v13, v13, v14, v15 bitop3:0x96\n" \
    "v_bitop3_b32 v16, v16, v17, v18 bitop3:0x96\n v_bitop3_b32 v19, v19, v20, v21 bitop3:0x96\n"
#define OPS64 OPS16 OPS16 OPS16 OPS16
#define OPS256 OPS64 OPS64 OPS64 OPS64

__global__ void k_run(unsigned long long* out, int exec0, int reps)
{
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int r = 0; r < reps; ++r) {
        if (exec0)
            asm volatile("s_mov_b64 s[20:21], exec\n s_mov_b64 exec, 0\n" OPS256 "s_mov_b64 exec, s[20:21]"
                         ::: "s20", "s21", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19",
                           "v20", "v21", "memory");
        else
            asm volatile(OPS256 ::: "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20",
                         "v21", "memory");
    }
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x % 64 == 0)
        out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main()
{
    const int reps = 200;  // 51200 instructions per wave
    unsigned long long* d;
    hipMalloc(&d, 1 << 20);
    std::vector<unsigned long long> h(1 << 17);
    for (int wps : {1, 3}) {  // waves per SIMD: 256 CUs x 4 SIMDs
        for (int e0 : {0, 1}) {
            const int blocks = 256 * wps, threads = 256;  // 4 waves per workgroup, one per SIMD
            hipLaunchKernelGGL(k_run, dim3(blocks), dim3(threads), 0, 0, d, e0, reps);
            hipLaunchKernelGGL(k_run, dim3(blocks), dim3(threads), 0, 0, d, e0, reps);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < blocks * 4; ++i)
                s += (double)h[i];
            const double per = s / (blocks * 4) / (reps * 256.0);
            std::printf("waves/SIMD %d exec0 %d: %.3f s_memtime ticks per instruction per wave\n", wps, e0, per);
        }
    }
    return 0;
}
