// numa_map.hip -- which HBM addresses are near which XCDs (tool, not the
// product; round 5).  tools/numa_probe showed two groups of XCDs, {0,3,4,7}
// and {1,2,5,6}, each ~20 % closer to half of the addresses.  Here one wave
// on XCC 0 (workgroup 0) and one on XCC 1 (workgroup 1) each time one load
// per listed offset, XCC 1 at offset + 128 (a fresh line of the same 256 B),
// so every load misses every cache.  Prints "offset lat0 lat1" per offset;
// tools/numa_fit.py fits the group as a function of the address bits.
//   hipcc --offload-arch=gfx950 -O3 -o tools/numa_map tools/numa_map.hip
//   tools/numa_map MODE > out.txt   (MODE 0: every 256 B of 32 MB; 1: bits
//   8..33 one at a time over 256 random bases; 2: 16 lines per 4 KB page of
//   the first 16 MB and of 2048 random pages)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_map(const unsigned char* buf, const unsigned long long* offs, int n, unsigned* lat,
                      unsigned* xcc)
{
    if (threadIdx.x != 0 || blockIdx.x > 1)
        return;
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    xcc[blockIdx.x] = x;
    for (int i = 0; i < n; ++i) {
        const unsigned* p = (const unsigned*)(buf + offs[i] + 128 * blockIdx.x);
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
        lat[(size_t)blockIdx.x * n + i] = (unsigned)(t1 - t0);
    }
}

int main(int argc, char** argv)
{
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t bytes = (size_t)20 << 30;  // 20 GB: bits up to 34
    std::vector<unsigned long long> offs;
    if (mode == 0) {
        for (unsigned long long o = 0; o < (32ull << 20); o += 256)
            offs.push_back(o);
    } else if (mode == 2) {
        // 16 fresh 256-byte lines of each 4 KB page (XCC 1 takes the +128
        // line of each): the first 4096 pages (16 MB), then 2048 random pages
        std::mt19937_64 rng(11);
        std::vector<unsigned long long> pages;
        for (unsigned long long p = 0; p < 4096; ++p)
            pages.push_back(p << 12);
        for (int i = 0; i < 2048; ++i)
            pages.push_back((rng() % ((bytes >> 1) >> 12)) << 12);
        for (unsigned long long pg : pages)
            for (int l = 0; l < 16; ++l)
                offs.push_back(pg + 256ull * l);
    } else {
        std::mt19937_64 rng(7);
        for (int b = 0; b < 256; ++b) {
            const unsigned long long base = (rng() % ((bytes >> 1) >> 8)) << 8;
            offs.push_back(base);
            for (int bit = 8; bit < 34; ++bit)
                offs.push_back(base ^ (1ull << bit));
        }
    }
    unsigned char* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    unsigned long long* d_offs;
    unsigned *d_lat, *d_x;
    const int n = (int)offs.size();
    CK(hipMalloc(&d_offs, n * 8));
    CK(hipMalloc(&d_lat, 2 * (size_t)n * 4));
    CK(hipMalloc(&d_x, 8));
    CK(hipMemcpy(d_offs, offs.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_map, dim3(8), dim3(64), 0, 0, buf, d_offs, n, d_lat, d_x);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<unsigned> lat(2 * (size_t)n);
    unsigned x[2];
    CK(hipMemcpy(lat.data(), d_lat, lat.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(x, d_x, 8, hipMemcpyDeviceToHost));
    printf("# mode %d, workgroup 0 on XCC %u, workgroup 1 on XCC %u; buffer at %p\n", mode, x[0], x[1], (void*)buf);
    for (int i = 0; i < n; ++i)
        printf("%llu %u %u\n", offs[i], lat[i], lat[(size_t)n + i]);
    CK(hipFree(buf));
    return 0;
}
