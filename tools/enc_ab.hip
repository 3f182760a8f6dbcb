// enc_ab.hip -- A/B timing of the compile-time encode k_rs_bs<64,32> (tool,
// not product): the kernel source compiled with different -D switches into
// different binaries; random rows; median of R launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -fconstexpr-steps=50000000 \
//     -Istorage-benchmarks_amd/csrc [-DRSGPU_BS_PREFETCH] -o tools/enc_ab_X tools/enc_ab.hip
#include "../storage-benchmarks_amd/csrc/rs_bitsliced.hip"

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 1024;
    const int R = argc > 2 ? atoi(argv[2]) : 7;
    const int k = 64, e = 32;
    const long long L = 1000000, pitch = 1000192;
    uint8_t *src, *out;
    if (hipMalloc(&src, (size_t)B * k * pitch) != hipSuccess ||
        hipMalloc(&out, (size_t)B * e * pitch) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    std::mt19937 rng(7);
    {
        const size_t chunk = 64u << 20;
        std::vector<uint32_t> h(chunk / 4);
        for (auto& x : h)
            x = rng();
        uint8_t* d;
        (void)hipMalloc(&d, chunk);
        (void)hipMemcpy(d, h.data(), chunk, hipMemcpyHostToDevice);
        const size_t n = (size_t)B * k * pitch;
        for (size_t o = 0; o < n; o += chunk)
            (void)hipMemcpy(src + o, d + (o / chunk % 7) * 4096, std::min(chunk - 7 * 4096, n - o),
                            hipMemcpyDeviceToDevice);
        (void)hipFree(d);
    }
    auto run = [&] { return launch_rs_bitsliced(k, e, src, out, pitch, L, B, 0); };
    (void)run();
    (void)run();
    if (hipDeviceSynchronize() != hipSuccess) {
        printf("launch failed\n");
        return 1;
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> ms(R);
    for (int i = 0; i < R; ++i) {
        (void)hipEventRecord(e0);
        (void)run();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms[i], e0, e1);
    }
    std::sort(ms.begin(), ms.end());
    printf("%s k_rs_bs<64,32> B=%d: median %.3f ms  min %.3f  max %.3f  (%.1f GB/s alg)\n",
           argc > 3 ? argv[3] : "", B, ms[R / 2], ms[0], ms[R - 1],
           (double)(k + e) * L * B / (ms[R / 2] * 1e-3) / 1e9);
    return 0;
}
