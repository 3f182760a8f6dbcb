// hbm_bw.hip -- achievable HBM bandwidth on the box for the access mixes of
// the RS kernels (tool, not product): read-only, write-only, copy (1 read :
// 1 write) and 2:1 read:write (the encode's 64 source rows : 32 parity rows),
// each with 16-byte per-lane accesses over large buffers, several grid
// shapes.  Reports GB/s (1e9) of algorithmic bytes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_bw tools/hbm_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// each thread handles UNROLL consecutive 16-byte chunks per grid stride
template <int R, int W, int UNROLL>
__global__ __launch_bounds__(256) void kern(const v4u* __restrict__ in, v4u* __restrict__ out,
                                            size_t n16, unsigned sink)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x * UNROLL;
    v4u acc = {0, 0, 0, 0};
    for (size_t base = ((size_t)blockIdx.x * blockDim.x) * UNROLL + threadIdx.x; base < n16;
         base += stride) {
        v4u v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t i = base + (size_t)u * blockDim.x;
            v[u] = (v4u){0, 0, 0, 0};
            if (R && i < n16) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    v[u] ^= in[i + (size_t)r * n16];
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t i = base + (size_t)u * blockDim.x;
            if (W && i < n16) {
#pragma unroll
                for (int w = 0; w < W; ++w)
                    out[i + (size_t)w * n16] = v[u] ^ (v4u){(unsigned)w, 0, 0, sink};
            } else {
                acc ^= v[u];
            }
        }
    }
    if (acc.x == sink && acc.y == 0x12345 && W == 0)
        out[0] = acc;  // keeps read-only loads alive
}

template <int R, int W, int UNROLL>
void run(const char* name, v4u* in, v4u* out, size_t n16, int blocks_per_cu)
{
    dim3 grid(256 * blocks_per_cu), block(256);
    hipLaunchKernelGGL((kern<R, W, UNROLL>), grid, block, 0, 0, in, out, n16, 7u);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int reps = 5;
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((kern<R, W, UNROLL>), grid, block, 0, 0, in, out, n16, 7u);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)n16 * 16.0 * (R + W) * reps;
    printf("  %-22s blocks/CU=%-3d unroll=%d  %8.1f GB/s\n", name, blocks_per_cu, UNROLL,
           bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
}

int main()
{
    // 2 GiB per "row set": read sets R x 2 GiB, write sets W x 2 GiB
    const size_t n16 = (size_t)2 << 30 >> 4;
    v4u *in, *out;
    if (hipMalloc(&in, n16 * 16 * 2) != hipSuccess || hipMalloc(&out, n16 * 16 * 2) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(in, 1, n16 * 16 * 2);
    (void)hipMemset(out, 0, n16 * 16 * 2);
    for (int bpc : {4, 8, 16}) {
        run<1, 0, 4>("read 1:0", in, out, n16, bpc);
        run<0, 1, 4>("write 0:1", in, out, n16, bpc);
        run<1, 1, 4>("copy 1:1", in, out, n16, bpc);
        run<2, 1, 4>("read2 write1 (2:1)", in, out, n16, bpc);
    }
    run<1, 1, 8>("copy 1:1", in, out, n16, 8);
    run<2, 1, 2>("read2 write1 (2:1)", in, out, n16, 8);
    return 0;
}
