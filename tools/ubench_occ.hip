// ubench_occ.hip -- how many 256-thread workgroups of a given static LDS size
// and 96 VGPRs are resident per CU at once (tool, not product).  Every wave
// sleeps a fixed time; a grid of 256 x W workgroups takes one sleep when W
// fit per CU, two when they do not.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_occ tools/ubench_occ.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int LDS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32))) void k_occ(int* sink)
{
    __shared__ uint32_t buf[LDS / 4];
    buf[threadIdx.x] = threadIdx.x;
    // 96 VGPRs in the descriptor, as k_rs_jit
    asm volatile("v_mov_b32 v95, 0" ::: "v95");
    for (int i = 0; i < 400; ++i)
        __builtin_amdgcn_s_sleep(127);
    __syncthreads();
    if (buf[(threadIdx.x + 1) & 255] == 12345)
        sink[0] = 1;
}

template <int LDS>
void run(int* sink)
{
    for (int w = 3; w <= 6; ++w) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        hipLaunchKernelGGL(k_occ<LDS>, dim3(256 * w), dim3(256), 0, 0, sink);  // warm
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_occ<LDS>, dim3(256 * w), dim3(256), 0, 0, sink);
        (void)hipEventRecord(b);
        (void)hipDeviceSynchronize();
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        printf("LDS %6d B, %d workgroups per CU asked: %.3f ms\n", LDS, w, ms);
    }
}

int main()
{
    int* sink;
    (void)hipMalloc(&sink, 4);
    run<32768>(sink);
    run<32256>(sink);
    run<32000>(sink);
    run<31744>(sink);
    run<24576>(sink);
    return 0;
}
