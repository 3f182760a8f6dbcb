// tc_profile.hip -- where the waves of k_rs_tc spend their time (tool, not
// product).  Compiles the kernel source with -DRSGPU_TC_PROF (per-wave
// s_memtime sums per phase), runs it on synthetic rows with random
// coefficients, and prints the average cycles per wave in each phase.
//   make -C storage-benchmarks_amd build/tc_handlers.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -DRSGPU_TC_PROF \
//     -Istorage-benchmarks_amd/csrc -Istorage-benchmarks_amd/build \
//     -o tools/tc_profile tools/tc_profile.hip
#include "../storage-benchmarks_amd/csrc/rs_tc.hip"

#include <cstdio>
#include <vector>

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 256;
    const int k = argc > 2 ? atoi(argv[2]) : 32;
    const int nrows = argc > 3 ? atoi(argv[3]) : k;  // output rows (the C3 decode: k 64, rows 32)
    const long long L = 1000000, pitch = 1000192;
    uint8_t* rows;
    if (hipMalloc(&rows, (size_t)B * k * pitch) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(rows, 0x5A, (size_t)B * k * pitch);
    std::vector<const uint8_t*> ptr((size_t)B * k);
    for (size_t i = 0; i < ptr.size(); ++i)
        ptr[i] = rows + i * pitch;
    const uint8_t** d_ptr;
    (void)hipMalloc(&d_ptr, ptr.size() * sizeof(void*));
    (void)hipMemcpy(d_ptr, ptr.data(), ptr.size() * sizeof(void*), hipMemcpyHostToDevice);

    unsigned long long* d_q;
    (void)hipMalloc(&d_q, 16);
    (void)tc_query_handlers(d_q, 0);
    unsigned long long q[2];
    (void)hipMemcpy(q, d_q, 16, hipMemcpyDeviceToHost);
    if (q[1] - q[0] != (unsigned long long)tc_handler_count() * tc_handler_stride()) {
        printf("bad handler table\n");
        return 1;
    }
    const int slots = tc_rows_per_pass(nrows);
    std::vector<unsigned long long> addr((size_t)B * k * slots);
    uint32_t x = 12345;
    for (size_t i = 0; i < addr.size(); ++i) {  // the handler copy serving the slot
        x = x * 1664525u + 1013904223u;
        const unsigned long long h = 256ull * tc_slot_copy((int)(i % 8)) + ((x >> 13) & 255);
        addr[i] = q[0] + h * tc_handler_stride();
    }
    unsigned long long* d_addr;
    (void)hipMalloc(&d_addr, addr.size() * 8);
    (void)hipMemcpy(d_addr, addr.data(), addr.size() * 8, hipMemcpyHostToDevice);

    TcArgs a{};
    a.srcs = d_ptr;
    a.dsts = (uint8_t* const*)d_ptr;
    a.addr = d_addr;
    a.k = k;
    a.rows = nrows;
    a.addr_stride = (long long)k * slots;
    a.len = L;
    a.status = nullptr;
    for (int i = 0; i < 2; ++i)
        (void)launch_rs_tc(a, B, 0);
    unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(tc::rsgpu_tc_prof), zero, sizeof zero);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    (void)launch_rs_tc(a, B, 0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long prof[8];
    (void)hipMemcpyFromSymbol(prof, HIP_SYMBOL(tc::rsgpu_tc_prof), sizeof prof);
    const double waves = (double)(((L + 2047) / 2048 + 63) / 64) * B * (slots / 8);  // sampled WGs
    // one barrier per step: phase 0 is the wait, phase 1 empty, phase 3 the barrier plus the next issue
    const char* names[8] = {"wait vmcnt", "-", "transpose in", "barrier + issue DMA",
                            "chunk asm", "store out", "loop", "wave lifetime"};
    printf("k_rs_tc<%d>: B=%d k=%d rows=%d L=%lld  %.3f ms  (%.1f GB/s alg)\n", slots / 8, B, k, nrows,
           L, ms, (double)(k + nrows) * L * B / (ms * 1e-3) / 1e9);
    for (int i = 0; i < 8; ++i)
        printf("  %-18s %10.0f cycles/wave  %5.1f %%\n", names[i], prof[i] / waves,
               100.0 * prof[i] / prof[7]);
    return 0;
}
