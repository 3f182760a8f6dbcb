// hwid_probe.hip -- which CU a workgroup lands on (tool, not the product;
// round 5): every workgroup of a large grid records XCC_ID and HW_ID, so
// the field layout (CU / SH / SE ids) and the dispatch order can be read.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hwid_probe tools/hwid_probe.hip
//   tools/hwid_probe > out.txt
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ void k_id(unsigned* out)
{
    if (threadIdx.x != 0)
        return;
    unsigned x, h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\n s_getreg_b32 %1, hwreg(HW_REG_HW_ID)" : "=s"(x), "=s"(h));
    out[2 * blockIdx.x] = x;
    out[2 * blockIdx.x + 1] = h;
    // keep the workgroup resident a little so the dispatcher spreads them
    for (int i = 0; i < 2000; ++i)
        asm volatile("s_nop 7");
}

int main()
{
    const int n = 8192;
    unsigned* d;
    if (hipMalloc(&d, 2 * n * 4) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(k_id, dim3(n), dim3(256), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess)
        return 1;
    std::vector<unsigned> h(2 * n);
    (void)hipMemcpy(h.data(), d, 2 * n * 4, hipMemcpyDeviceToHost);
    std::map<unsigned, int> cu;  // (xcc, se, sh, cu) -> count
    for (int i = 0; i < n; ++i) {
        const unsigned x = h[2 * i] & 0xf, w = h[2 * i + 1];
        const unsigned cuid = (w >> 8) & 0xf, sh = (w >> 12) & 1, se = (w >> 13) & 0x7;
        cu[(x << 12) | (se << 8) | (sh << 4) | cuid]++;
        if (i < 48)
            printf("wg %d xcc %u hw_id 0x%08x se %u sh %u cu %u simd %u wave %u\n", i, x, w, se, sh, cuid,
                   (w >> 4) & 3, w & 0xf);
    }
    printf("# distinct (xcc, se, sh, cu): %zu\n", cu.size());
    for (auto& [k, c] : cu)
        printf("xcc %u se %u sh %u cu %u : %d\n", k >> 12, (k >> 8) & 0xf, (k >> 4) & 1, k & 0xf, c);
    return 0;
}
