// tc_profile.hip -- where the waves of k_rs_tc spend their time (tool, not
// product).  Instantiates the product kernel with a hooks policy whose Timer
// sums s_memtime per phase, runs it on synthetic rows with random
// coefficients, and prints the average cycles per wave in each phase.
// `tc_profile fused B k e` does the same for the one-launch small decode
// k_rs_tc_fused (C2: fused 1 16 4).
//   make -C storage-benchmarks_amd build/tc_handlers.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 \
//     -Istorage-benchmarks_amd/csrc -Istorage-benchmarks_amd/build \
//     -o tools/tc_profile tools/tc_profile.hip
#include "../storage-benchmarks_amd/csrc/rs_tc.hip"

namespace tcprof {
__device__ unsigned long long rsgpu_tc_prof[8];
struct ProfHooks {
    struct Timer {
        unsigned long long sum[8] = {}, t, start;
        __device__ Timer() : t(__builtin_amdgcn_s_memtime()), start(t) {}
        __device__ void mark(int p)
        {
            const unsigned long long n = __builtin_amdgcn_s_memtime();
            sum[p] += n - t;
            t = n;
        }
        __device__ void end(int lane)
        {
            sum[7] = __builtin_amdgcn_s_memtime() - start;
            if (lane == 0 && (blockIdx.x & 63) == 0)  // sampled: same-address atomics serialise
                for (int i = 0; i < 8; ++i)
                    atomicAdd(&rsgpu_tc_prof[i], sum[i]);
        }
    };
};
void launch(const rsgpu::TcArgs& a, int B)
{
    const int nw = rsgpu::tc_rows_per_pass(a.rows) / 8;
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)B);
    switch (nw) {
    case 1: hipLaunchKernelGGL((rsgpu::tc::k_rs_tc<1, ProfHooks>), grid, dim3(64), 0, 0, a, 1); break;
    case 2: hipLaunchKernelGGL((rsgpu::tc::k_rs_tc<2, ProfHooks>), grid, dim3(128), 0, 0, a, 1); break;
    case 3: hipLaunchKernelGGL((rsgpu::tc::k_rs_tc<3, ProfHooks>), grid, dim3(192), 0, 0, a, 1); break;
    default: hipLaunchKernelGGL((rsgpu::tc::k_rs_tc<4, ProfHooks>), grid, dim3(256), 0, 0, a, 1); break;
    }
}
void launch_fused(const rsgpu::TcFusedArgs& f)
{
    dim3 grid((unsigned)((f.len + 2047) / 2048), (unsigned)f.blocks);
    hipLaunchKernelGGL((rsgpu::tc::k_rs_tc_fused<4, ProfHooks>), grid, dim3(256), 0, 0, f);
}
}  // namespace tcprof

#include <cstdio>
#include <string>
#include <vector>

static int fused_main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 2 ? atoi(argv[2]) : 1;
    const int k = argc > 3 ? atoi(argv[3]) : 16;
    const int e = argc > 4 ? atoi(argv[4]) : 4;
    const long long L = 1000000, pitch = 1000192;
    uint8_t *src, *par, *out, *err;
    int* status;
    if (hipMalloc(&src, (size_t)B * k * pitch) != hipSuccess || hipMalloc(&par, (size_t)B * e * pitch) ||
        hipMalloc(&out, (size_t)B * e * pitch) || hipMalloc(&err, (size_t)B * e) || hipMalloc(&status, 4 * B)) {
        printf("alloc failed\n");
        return 1;
    }
    (void)hipMemset(src, 0x5A, (size_t)B * k * pitch);
    (void)hipMemset(par, 0x3C, (size_t)B * e * pitch);
    std::vector<uint8_t> er((size_t)B * e);
    for (int b = 0; b < B; ++b)
        for (int i = 0; i < e; ++i)
            er[(size_t)b * e + i] = (uint8_t)(i * k / e);  // spread, strictly ascending
    (void)hipMemcpy(err, er.data(), er.size(), hipMemcpyHostToDevice);
    unsigned long long* d_q;
    (void)hipMalloc(&d_q, 16);
    (void)tc_query_handlers(d_q, 0);
    unsigned long long q[2];
    (void)hipMemcpy(q, d_q, 16, hipMemcpyDeviceToHost);
    TcFusedArgs f{};
    f.k = k;
    f.e = e;
    f.len = L;
    f.pitch = pitch;
    f.blocks = B;
    f.err = err;
    f.src = src;
    f.par = par;
    f.out = out;
    f.status = status;
    f.map_base = q[0];
    f.map_stride = tc_handler_stride();
    for (int sl = 0; sl < 8; ++sl)
        f.map_copy[sl] = tc_slot_copy(sl);
    for (int i = 0; i < 3; ++i)
        tcprof::launch_fused(f);
    unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(tcprof::rsgpu_tc_prof), zero, sizeof zero);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    tcprof::launch_fused(f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long prof[8];
    (void)hipMemcpyFromSymbol(prof, HIP_SYMBOL(tcprof::rsgpu_tc_prof), sizeof prof);
    const double waves = (double)(((L + 2047) / 2048 + 63) / 64) * B * 4;  // sampled WGs x 4 waves
    const char* names[8] = {"erasures arrive", "survivors + issue", "closed form", "wait + transpose",
                            "chunk asm", "partials + bar", "reduce + store", "wave lifetime"};
    printf("k_rs_tc_fused<4>: B=%d k=%d e=%d L=%lld  %.3f ms  (%.1f GB/s alg)\n", B, k, e, L, ms,
           (double)(k + e) * L * B / (ms * 1e-3) / 1e9);
    for (int i = 0; i < 8; ++i)
        printf("  %-18s %10.0f cycles/wave  %5.1f %%\n", names[i], prof[i] / waves, 100.0 * prof[i] / prof[7]);
    return 0;
}

int main(int argc, char** argv)
{
    using namespace rsgpu;
    if (argc > 1 && std::string(argv[1]) == "fused")
        return fused_main(argc, argv);
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
    a.dst_stride = k;  // block b writes its own rows (dsts == srcs)
    a.addr_stride = (long long)k * slots;
    a.len = L;
    a.status = nullptr;
    for (int i = 0; i < 2; ++i)
        tcprof::launch(a, B);
    unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(tcprof::rsgpu_tc_prof), zero, sizeof zero);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    tcprof::launch(a, B);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long prof[8];
    (void)hipMemcpyFromSymbol(prof, HIP_SYMBOL(tcprof::rsgpu_tc_prof), sizeof prof);
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
