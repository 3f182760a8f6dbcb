// numa_probe.hip -- does an XCD see some HBM addresses closer than others?
// (tool, not the product; round 5, after the energy split showed the HBM
// path -- DRAM, PHY, the IOD fabric -- at ~5 ms of the C3 kernels' 22 ms.)
//
// One wave per workgroup, 8 workgroups per XCD (workgroups are dealt
// round-robin over the XCDs; each records its XCC_ID to prove it).  Lane 0
// issues dependent loads, each to an address never touched before by any
// workgroup, and times each with s_memtime.  The address of sample s of
// class c for workgroup w is ((w * S + s) * NC + c) << G, so the class is
// address bits [G, G + log2 NC).  Per (XCD, class): the mean latency.  An
// XCD whose latency depends on the class reveals which addresses are local
// to its IOD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/numa_probe tools/numa_probe.hip
//   tools/numa_probe G NC S   (defaults 12 64 48)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_probe(const unsigned* buf, int G, int NC, int S, unsigned long long* out, unsigned* xcc)
{
    if (threadIdx.x != 0)
        return;
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    const int w = blockIdx.x;
    xcc[w] = x;
    for (int c = 0; c < NC; ++c) {
        unsigned long long sum = 0;
        for (int s = 0; s < S; ++s) {
            const size_t byte = (((size_t)w * S + s) * NC + c) << G;
            const unsigned* p = buf + byte / 4;
            unsigned long long t0, t1;
            unsigned v;
            asm volatile(
                "s_memtime %[t0]\n"
                "s_waitcnt lgkmcnt(0)\n"
                "global_load_dword %[v], %[p], off\n"
                "s_waitcnt vmcnt(0)\n"
                "s_memtime %[t1]\n"
                "s_waitcnt lgkmcnt(0)\n"
                : [t0] "=&s"(t0), [t1] "=&s"(t1), [v] "=&v"(v)
                : [p] "v"(p)
                : "memory");
            (void)v;
            sum += t1 - t0;
        }
        out[(size_t)w * NC + c] = sum;
    }
}

int main(int argc, char** argv)
{
    const int G = argc > 1 ? atoi(argv[1]) : 12;
    const int NC = argc > 2 ? atoi(argv[2]) : 64;
    const int S = argc > 3 ? atoi(argv[3]) : 48;
    const int W = 64;
    const size_t need = ((size_t)W * S * NC) << G;
    const size_t bytes = std::max(need + ((size_t)1 << 30), (size_t)2 << 30);  // + 1 GB that evicts the MALL
    unsigned* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    unsigned long long* d_out;
    unsigned* d_x;
    CK(hipMalloc(&d_out, (size_t)W * NC * 8));
    CK(hipMalloc(&d_x, W * 4));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_probe, dim3(W), dim3(64), 0, 0, buf, G, NC, S, d_out, d_x);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> out((size_t)W * NC);
    std::vector<unsigned> x(W);
    CK(hipMemcpy(out.data(), d_out, out.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(x.data(), d_x, W * 4, hipMemcpyDeviceToHost));
    // per (xcc, class) mean cycles
    std::vector<double> lat(8 * NC, 0.0);
    std::vector<int> cnt(8 * NC, 0);
    for (int w = 0; w < W; ++w)
        for (int c = 0; c < NC; ++c) {
            lat[(x[w] & 7) * NC + c] += (double)out[(size_t)w * NC + c] / S;
            cnt[(x[w] & 7) * NC + c] += 1;
        }
    printf("# G=%d NC=%d S=%d; workgroup -> XCC:", G, NC, S);
    for (int w = 0; w < 16; ++w)
        printf(" %u", x[w]);
    printf(" ...\n# class: mean cycles per XCC 0..7 (s_memtime ticks)\n");
    for (int c = 0; c < NC; ++c) {
        printf("%4d", c);
        for (int q = 0; q < 8; ++q)
            printf(" %7.0f", cnt[q * NC + c] ? lat[q * NC + c] / cnt[q * NC + c] : -1.0);
        printf("\n");
    }
    CK(hipFree(buf));
    return 0;
}
