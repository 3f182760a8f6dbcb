// jit_profile.hip -- where the waves of k_rs_jit spend their time (tool, not
// product).  Instantiates the product kernel with its own hooks policy
// (ProfHooks below: per-wave s_memtime sums per phase, and timing-only
// variants that run other code than the block's own), writes
// random-coefficient code for every block with the host emitters of rs_jit.h,
// copies it into executable device memory, runs the decode kernel on
// synthetic rows and prints the average cycles per wave in each phase.
//   make -C storage-benchmarks_amd build/tc_handlers.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 \
//     -Istorage-benchmarks_amd/csrc -Istorage-benchmarks_amd/build \
//     -o tools/jit_profile tools/jit_profile.hip -lhsa-runtime64
//   tools/jit_profile [blocks=512] [k=64] [rows=32] [extra_lds] [mac_order] [xcd]
//                     [share=0|1|2] [inv=1|0]
//   share 1: every wave runs wave 0's code, 2: block 0's too; inv 0: no
//   s_icache_inv (both timing only: wrong results)
#include "../storage-benchmarks_amd/csrc/rs_jit.hip"

namespace jitprof {
__device__ unsigned long long rsgpu_jit_prof[8];

template <int SHARE, bool INV>
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
            if (lane == 0 && (blockIdx.x & 63) == 0)
                for (int i = 0; i < 8; ++i)
                    atomicAdd(&rsgpu_jit_prof[i], sum[i]);
        }
    };
    static constexpr bool kInvalidate = INV;
    __device__ static const uint8_t* code(const rsgpu::JitArgs& a, bool shared, int b, int wave, int nch)
    {
        if (SHARE == 0)
            return rsgpu::jitk::JitHooks::code(a, shared, b, wave, nch);
        return a.code + (size_t)(SHARE == 2 ? 0 : b) * a.block_stride;
    }
};

template <int NW, int SHARE, bool INV>
void launch(const rsgpu::JitArgs& a, int B, int extra_lds)
{
    hipLaunchKernelGGL((rsgpu::jitk::k_rs_jit<NW, false, ProfHooks<SHARE, INV>>),
                       dim3((unsigned)((a.len + 2047) / 2048), (unsigned)B), dim3(64 * NW), extra_lds, 0, a);
}

template <int NW>
void launch_mode(const rsgpu::JitArgs& a, int B, int extra_lds, int share, bool inv)
{
    if (share == 1)
        inv ? launch<NW, 1, true>(a, B, extra_lds) : launch<NW, 1, false>(a, B, extra_lds);
    else if (share == 2)
        inv ? launch<NW, 2, true>(a, B, extra_lds) : launch<NW, 2, false>(a, B, extra_lds);
    else
        inv ? launch<NW, 0, true>(a, B, extra_lds) : launch<NW, 0, false>(a, B, extra_lds);
}
}  // namespace jitprof

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>
#include <vector>

static hsa_status_t pick(hsa_amd_memory_pool_t p, void* d)
{
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc) {
        *(hsa_amd_memory_pool_t*)d = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

__global__ void k_fill_random(uint64_t* p, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

__global__ void k_copy(uint64_t* dst, const uint64_t* src, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 512;
    const int k = argc > 2 ? atoi(argv[2]) : 64;
    const int e = argc > 3 ? atoi(argv[3]) : 32;
    // extra dynamic LDS per workgroup: caps workgroups per CU (occupancy A/B)
    const int extra_lds = argc > 4 ? atoi(argv[4]) : 0;
    // order of the independent multiply-accumulate words of a source (A/B of
    // operand locality): 0 = as emitted (slot, plane), 1 = by (L, H) operand
    // registers, 2 = by (H, L)
    const int mac_order = argc > 5 ? atoi(argv[5]) : 0;
    const int xcd = argc > 6 ? atoi(argv[6]) : 0;  // XCD-contiguous (block, tile) order
    const int share = argc > 7 ? atoi(argv[7]) : 0;
    const bool inv = argc > 8 ? atoi(argv[8]) != 0 : true;
    const long long L = 1000000, pitch = 1000192;
    uint8_t* rows;
    if (hipMalloc(&rows, (size_t)B * (k + e) * pitch) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    // random rows (constant data runs the decode ~10 % faster: power)
    hipLaunchKernelGGL(k_fill_random, dim3(8192), dim3(256), 0, 0, (uint64_t*)rows,
                       (long long)((size_t)B * (k + e) * pitch / 8));
    std::vector<const uint8_t*> sp((size_t)B * k), dp((size_t)B * e);
    for (int b = 0; b < B; ++b) {
        for (int j = 0; j < k; ++j)
            sp[(size_t)b * k + j] = rows + ((size_t)b * (k + e) + j) * pitch;
        for (int i = 0; i < e; ++i)
            dp[(size_t)b * e + i] = rows + ((size_t)b * (k + e) + k + i) * pitch;
    }
    const uint8_t** d_sp;
    uint8_t** d_dp;
    (void)hipMalloc(&d_sp, sp.size() * 8);
    (void)hipMalloc(&d_dp, dp.size() * 8);
    (void)hipMemcpy(d_sp, sp.data(), sp.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_dp, dp.data(), dp.size() * 8, hipMemcpyHostToDevice);
    int* d_st;
    (void)hipMalloc(&d_st, B * sizeof(int));
    (void)hipMemset(d_st, 0, B * sizeof(int));

    // random-coefficient code of every block, host-emitted
    const size_t per = jit_code_bytes(k, e, 1);
    std::vector<uint64_t> code(per / 8 * B);
    const int NW = (e + 7) / 8, nch = (k + 7) / 8;
    const size_t stride = (size_t)jit::chunk_stride(8);
    uint32_t x = 12345;
    for (int b = 0; b < B; ++b) {
        uint8_t* cb = (uint8_t*)code.data() + (size_t)b * per;
        for (size_t i = 0; i < per / 8; ++i)
            ((uint64_t*)cb)[i] = (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
        std::vector<uint8_t> rows((size_t)e * k);
        for (auto& c : rows) {
            x = x * 1664525u + 1013904223u;
            c = (uint8_t)(x >> 13);
        }
        const int stride_w = (int)(stride / 8);
        for (int w = 0; w < NW; ++w)
            for (int ch = 0; ch < nch; ++ch)
            {
                for (int o = 0; o < stride_w; ++o) {
                    uint64_t word;
                    if (jit::code_word(rows.data() + (size_t)8 * w * k, k, std::min(8, e - 8 * w), ch, o, &word))
                        ((uint64_t*)cb)[((size_t)w * nch + ch) * stride_w + o] = word;
                }
                    if (mac_order) {
                        const int nt = std::min(8, k - 8 * ch), nslot = std::min(8, e - 8 * w);
                        for (int t = 0; t < nt; ++t) {
                            uint64_t* m = (uint64_t*)(cb + ((size_t)w * nch + ch) * stride + jit::PRO_BYTES +
                                                      (size_t)t * jit::src_bytes(nslot) + jit::PRE_BYTES);
                            auto key = [&](uint64_t wd) {
                                const uint32_t w1 = (uint32_t)(wd >> 32);
                                const uint32_t L = (w1 >> 9) & 511, H = (w1 >> 18) & 511;
                                return mac_order == 1 ? (L << 9 | H) : (H << 9 | L);
                            };
                            std::stable_sort(m, m + 8 * nslot, [&](uint64_t x, uint64_t y) { return key(x) < key(y); });
                        }
                    }
                }
    }
    uint64_t* d_stage;
    (void)hipMalloc(&d_stage, code.size() * 8);
    (void)hipMemcpy(d_stage, code.data(), code.size() * 8, hipMemcpyHostToDevice);
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    hsa_amd_pointer_info(d_stage, &info, nullptr, nullptr, nullptr);
    hsa_amd_memory_pool_t pool{};
    hsa_amd_agent_iterate_memory_pools(info.agentOwner, pick, &pool);
    void* exec = nullptr;
    if (hsa_amd_memory_pool_allocate(pool, code.size() * 8, HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, &exec) !=
        HSA_STATUS_SUCCESS) {
        printf("exec alloc failed\n");
        return 1;
    }
    hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (uint64_t*)exec, d_stage, (long long)code.size());

    JitArgs a{};
    a.srcs = d_sp;
    a.dsts = d_dp;
    a.code = (const uint8_t*)exec;
    a.chunk_stride = (long long)stride;
    a.block_stride = (long long)NW * nch * stride;
    a.dst_stride = e;
    a.k = k;
    a.rows = e;
    a.len = L;
    a.status = d_st;
    a.xcd_order = xcd;
    for (int rep = 0; rep < 4; ++rep) {  // warm, then measured
        unsigned long long z[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(jitprof::rsgpu_jit_prof), z, sizeof z);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        switch (NW) {
        case 1: jitprof::launch_mode<1>(a, B, extra_lds, share, inv); break;
        case 2: jitprof::launch_mode<2>(a, B, extra_lds, share, inv); break;
        case 3: jitprof::launch_mode<3>(a, B, extra_lds, share, inv); break;
        default: jitprof::launch_mode<4>(a, B, extra_lds, share, inv); break;
        }
        (void)hipEventRecord(e1);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 1;
        }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long p[8];
        (void)hipMemcpyFromSymbol(p, HIP_SYMBOL(jitprof::rsgpu_jit_prof), sizeof p);
        const double waves = (double)p[7] > 0 ? 1 : 1;
        (void)waves;
        const char* names[8] = {"wait vmcnt (LDS-DMA)", "transpose in", "barrier",
                                "issue DMA", "generated code", "store out", "-", "wave lifetime"};
        const long long wg = ((L + 2047) / 2048 + 63) / 64 * (long long)B;  // sampled WGs ~ x & 63 == 0
        printf("rep %d: %.3f ms for %d blocks (%.2f TB/s alg)\n", rep, ms, B,
               (double)B * (k + e) * L / (ms * 1e-3) / 1e12);
        for (int i = 0; i < 8; ++i)
            printf("  %-22s %12.0f cycles per wave (%.1f %%)\n", names[i],
                   (double)p[i] / (wg * NW), 100.0 * p[i] / p[7]);
    }
    return 0;
}
