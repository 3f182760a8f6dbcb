// fused_profile.hip -- where the waves of k_rs_decode_fused spend their time
// (tool, not product): the kernel compiled with -DRSGPU_FUSED_PROF, run on
// synthetic rows with random erasures and random solve coefficients.
//   make -C storage-benchmarks_amd build/tc_handlers.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -DRSGPU_FUSED_PROF \
//     -Istorage-benchmarks_amd/csrc -Istorage-benchmarks_amd/build \
//     -o tools/fused_profile tools/fused_profile.hip
#include "../storage-benchmarks_amd/csrc/rs_tc.hip"
#include "../storage-benchmarks_amd/csrc/rs_decode_fused.hip"

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 256;
    const int k = 64, e = 32;
    const long long L = 1000000, pitch = 1000192;
    uint8_t *src, *par, *out;
    if (hipMalloc(&src, (size_t)B * k * pitch) != hipSuccess ||
        hipMalloc(&par, (size_t)B * e * pitch) != hipSuccess ||
        hipMalloc(&out, (size_t)B * e * pitch) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(src, 0x5A, (size_t)B * k * pitch);
    (void)hipMemset(par, 0x3C, (size_t)B * e * pitch);
    std::mt19937 rng(7);
    std::vector<unsigned long long> em(2 * B, 0);
    for (int b = 0; b < B; ++b) {
        std::vector<int> idx(k);
        std::iota(idx.begin(), idx.end(), 0);
        std::shuffle(idx.begin(), idx.end(), rng);
        for (int i = 0; i < e; ++i)
            em[2 * b] |= 1ull << idx[i];
    }
    unsigned long long *d_em, *d_q, *d_addr;
    int* d_status;
    (void)hipMalloc(&d_em, em.size() * 8);
    (void)hipMemcpy(d_em, em.data(), em.size() * 8, hipMemcpyHostToDevice);
    (void)hipMalloc(&d_q, 16);
    (void)tc_query_handlers(d_q, 0);
    unsigned long long q[2];
    (void)hipMemcpy(q, d_q, 16, hipMemcpyDeviceToHost);
    if (q[1] - q[0] != (unsigned long long)tc_handler_count() * tc_handler_stride()) {
        printf("bad handler table\n");
        return 1;
    }
    std::vector<unsigned long long> addr((size_t)B * e * 32);
    // every slot uses the handler copy that serves it (chained dispatch)
    auto odd = [](size_t i) { return 256ull * tc_slot_copy((int)(i % 8)); };  // the slot's handler copy
    for (size_t i = 0; i < addr.size(); ++i)
        addr[i] = q[0] + (odd(i) + (rng() & 255)) * tc_handler_stride();
    (void)hipMalloc(&d_addr, addr.size() * 8);
    (void)hipMemcpy(d_addr, addr.data(), addr.size() * 8, hipMemcpyHostToDevice);
    std::vector<unsigned long long> sa((size_t)B * (k - e) * 32);
    for (size_t i = 0; i < sa.size(); ++i)
        sa[i] = q[0] + (odd(i) + (rng() & 255)) * tc_handler_stride();
    unsigned long long* d_sa;
    (void)hipMalloc(&d_sa, sa.size() * 8);
    (void)hipMemcpy(d_sa, sa.data(), sa.size() * 8, hipMemcpyHostToDevice);
    (void)hipMalloc(&d_status, B * sizeof(int));
    (void)hipMemset(d_status, 0, B * sizeof(int));

    auto run = [&] {
        return launch_rs_decode_fused(k, e, src, par, out, pitch, L, B, (const uint64_t*)d_em,
                                      d_addr, d_sa, d_status, 0);
    };
    (void)run();
    (void)run();
    unsigned long long zero[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(fused::rsgpu_fused_prof), zero, sizeof zero);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    (void)run();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long prof[16];
    (void)hipMemcpyFromSymbol(prof, HIP_SYMBOL(fused::rsgpu_fused_prof), sizeof prof);
    const double waves = (double)(((L + 2047) / 2048 + 63) / 64) * B * 4;  // sampled WGs
    const char* names[16] = {"p1 issue DMA", "p1 wait vmcnt", "p1 transpose in", "p1 barrier 1",
                             "p1 syndrome MAC", "p1 barrier 2+loop", "parity+syn store",
                             "p2 issue+wait", "p2 barrier 1", "p2 chunk asm", "p2 barrier 2+loop",
                             "output store", "prologue (parity)", "", "", "wave lifetime"};
    printf("k_rs_decode_fused<64,32>: B=%d L=%lld  %.3f ms  (%.1f GB/s alg)\n", B, L, ms,
           (double)(k + e) * L * B / (ms * 1e-3) / 1e9);
    for (int i = 0; i < 16; ++i)
        if (names[i][0])
            printf("  %-20s %10.0f cycles/wave  %5.1f %%\n", names[i], prof[i] / waves,
                   100.0 * prof[i] / prof[15]);
    return 0;
}
