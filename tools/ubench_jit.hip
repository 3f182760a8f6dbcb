// ubench_jit.hip -- probe for runtime-generated device code (the decode
// kernel's per-block code):
//   1. executable device memory from the GPU's coarse-grained pool
//      (hsa_amd_memory_pool_allocate with HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG)
//      is writable by a kernel's vector stores and callable by s_swappc;
//   2. code rewritten at the same address between two launches is seen by
//      the next launch when it runs s_icache_inv first (without it a run
//      mixed old and new lines and hit an illegal instruction: the dispatch
//      does not invalidate the instruction cache);
//   3. the cost of STREAMING straight-line code through the instruction
//      cache: the same number of VALU instructions run (a) from a 4 KB block
//      called repeatedly (cache resident), (b) from one 256 KB straight-line
//      block shared by every workgroup, (c) from a distinct 256 KB block per
//      group of workgroups (per-block code in the decode).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_jit.hip \
//          -o tools/ubench_jit -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

struct PoolFind {
    hsa_amd_memory_pool_t pool;
    bool found;
};

static hsa_status_t pick_pool(hsa_amd_memory_pool_t p, void* d)
{
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc) {
        ((PoolFind*)d)->pool = p;
        ((PoolFind*)d)->found = true;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

static void* exec_alloc(size_t bytes)
{
    void* probe = nullptr;
    CHECK(hipMalloc(&probe, 4096));
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    if (hsa_amd_pointer_info(probe, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) {
        std::printf("hsa_amd_pointer_info failed\n");
        std::exit(1);
    }
    PoolFind f{};
    hsa_amd_agent_iterate_memory_pools(info.agentOwner, pick_pool, &f);
    CHECK(hipFree(probe));
    if (!f.found) {
        std::printf("no coarse-grained pool\n");
        std::exit(1);
    }
    void* p = nullptr;
    hsa_status_t st = hsa_amd_memory_pool_allocate(f.pool, bytes, HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, &p);
    if (st != HSA_STATUS_SUCCESS || !p) {
        std::printf("executable allocation failed (%d)\n", (int)st);
        std::exit(1);
    }
    return p;
}

// gfx950 encodings (llvm-mc -mcpu=gfx950 -show-encoding)
__host__ __device__ inline uint64_t enc_bitop3_96(int d, int a, int b, int c)
{
    const uint32_t w0 = 0xd2340200u | (uint32_t)d;
    const uint32_t w1 = 0xd0000000u | ((uint32_t)(256 + c) << 18) | ((uint32_t)(256 + b) << 9) |
                        (uint32_t)(256 + a);
    return (uint64_t)w1 << 32 | w0;
}
__host__ __device__ inline uint64_t enc_xor_e64(int d, int a, int b)
{
    const uint32_t w0 = 0xd1150000u | (uint32_t)d;
    const uint32_t w1 = ((uint32_t)(256 + b) << 9) | (uint32_t)(256 + a);
    return (uint64_t)w1 << 32 | w0;
}
constexpr uint32_t SETPC_82 = 0xbe801d52u;  // s_setpc_b64 s[82:83]
constexpr uint32_t SNOP0 = 0xbf800000u;

// every 8-byte slot "s_setpc_b64 s[82:83]; s_nop 0": a return wherever a
// wave lands
__global__ void k_fill_ret(uint64_t* code, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        code[i] = (uint64_t)SNOP0 << 32 | SETPC_82;
}

// code[i] for i < n: variant 0 -> v_bitop3 v10 ^= v11 ^ v12; variant 1 ->
// v_xor v10 ^= v11; then the return
__global__ void k_gen_small(uint64_t* code, int n, int variant)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        code[i] = variant == 0 ? enc_bitop3_96(10, 10, 11, 12) : enc_xor_e64(10, 10, 11);
    if (i == n)
        code[i] = (uint64_t)SNOP0 << 32 | SETPC_82;
}

__global__ void k_run_small(const void* code, uint32_t* out, int inv)
{
    uint32_t v = threadIdx.x;
    if (inv)  // drop instruction-cache lines left by an earlier launch
        asm volatile("s_icache_inv\n s_nop 15\n s_nop 15" ::: "memory");
    asm volatile(
        "v_mov_b32 v10, %0\n"
        "v_mov_b32 v11, 0x1111\n"
        "v_mov_b32 v12, 0x2222\n"
        "s_swappc_b64 s[82:83], %1\n"
        "v_mov_b32 %0, v10\n"
        : "+v"(v)
        : "s"(code)
        : "v10", "v11", "v12", "s82", "s83", "memory");
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// n bitop3 over 64 accumulators v64..v127 with operands v24..v53, return
__global__ void k_gen_big(uint64_t* code, long long n, int nblk, long long stride)
{
    const long long tot = (long long)nblk * stride;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i % stride;
        if (r < n) {
            const int acc = 64 + (int)(r % 64);
            code[i] = enc_bitop3_96(acc, acc, 24 + (int)((r / 64) % 8), 32 + (int)((r * 7) % 22));
        } else if (r == n) {
            code[i] = (uint64_t)SNOP0 << 32 | SETPC_82;
        } else {
            code[i] = (uint64_t)SNOP0 << 32 | SNOP0;
        }
    }
}

// each workgroup calls code block (blockIdx.x / group) `calls` times
__global__ __launch_bounds__(256) void k_run_big(const uint64_t* code, long long stride, int group,
                                                 int calls, uint32_t* out, int inv)
{
    const uint64_t* c = code + (long long)(blockIdx.x / group) * stride;
    if (inv)
        asm volatile("s_icache_inv\n s_nop 15\n s_nop 15" ::: "memory");
    uint32_t seed = threadIdx.x * 2654435761u;
    asm volatile(
        "v_mov_b32 v24, %0\n v_mov_b32 v25, %0\n v_mov_b32 v26, %0\n v_mov_b32 v27, %0\n"
        "v_mov_b32 v28, %0\n v_mov_b32 v29, %0\n v_mov_b32 v30, %0\n v_mov_b32 v31, %0\n"
        :
        : "v"(seed)
        : "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31");
    for (int k = 0; k < calls; ++k)
        asm volatile("s_swappc_b64 s[82:83], %0\n" ::"s"(c)
                     : "s82", "s83", "memory", "v24", "v25", "v26", "v27", "v28", "v29", "v30",
                       "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41",
                       "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52",
                       "v53", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73",
                       "v74", "v75", "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84",
                       "v85", "v86", "v87", "v88", "v89", "v90", "v91", "v92", "v93", "v94", "v95",
                       "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105",
                       "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114",
                       "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123",
                       "v124", "v125", "v126", "v127");
    uint32_t r;
    asm volatile("v_mov_b32 %0, v64" : "=v"(r));
    if (r == 0x12345678u)
        out[0] = r;  // keeps the work alive
}

int main()
{
    // 1 + 2: correctness and coherence
    void* code = exec_alloc(64 << 20);
    hipLaunchKernelGGL(k_fill_ret, dim3(4096), dim3(256), 0, 0, (uint64_t*)code, (64ll << 20) / 8);
    std::printf("executable allocation at %p\n", code);
    uint32_t* d_out;
    CHECK(hipMalloc(&d_out, 4096 * sizeof(uint32_t)));
    std::vector<uint32_t> h(256);
    int bad = 0, bad_noinv = 0;
    for (int it = 0; it < 40; ++it) {
        const int variant = it & 1, n = 3 + (it % 6);  // odd / even counts
        const int inv = 1;
        hipLaunchKernelGGL(k_gen_small, dim3(1), dim3(64), 0, 0, (uint64_t*)code, n, variant);
        hipLaunchKernelGGL(k_run_small, dim3(1), dim3(256), 0, 0, code, d_out, inv);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(h.data(), d_out, 256 * 4, hipMemcpyDeviceToHost));
        for (int t = 0; t < 256; ++t) {
            const uint32_t x = variant == 0 ? 0x3333u : 0x1111u;
            const uint32_t want = (n & 1) ? (t ^ x) : (uint32_t)t;
            if (h[t] != want) {
                if (inv && bad < 4)
                    std::printf("it %d lane %d: got %#x want %#x\n", it, t, h[t], want);
                (inv ? bad : bad_noinv)++;
            }
        }
    }
    std::printf("coherence with s_icache_inv: %d stale lanes of %d\n", bad, 40 * 256);
    (void)bad_noinv;
    if (bad)
        return 1;

    // 3: streaming straight-line code
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const long long NBIG = 32768;  // 256 KB of bitop3 per call
    const long long SMALL = 512;   // 4 KB
    const int wgs = 8192;          // 32768 waves
    struct Case {
        const char* name;
        long long n;
        int nblk, group, calls, inv;
    } cases[] = {
        // every case invalidates the instruction cache first: code rewritten
        // at an address an earlier launch executed is otherwise stale (a run
        // without it mixed old and new lines and hit an illegal instruction)
        {"resident 4 KB x 64 calls, inv", SMALL, 1, wgs, 64, 1},
        {"shared 256 KB x 1 call, inv", NBIG, 1, wgs, 1, 1},
        {"per 64 WGs 256 KB (128 blocks), inv", NBIG, wgs / 64, 64, 1, 1},
        {"per 8 WGs 256 KB (1024 blocks), inv", NBIG, wgs / 8, 8, 1, 1},
    };
    for (auto& c : cases) {
        const long long stride = c.n + 8;
        if ((long long)c.nblk * stride * 8 > (64ll << 20))
            continue;
        hipLaunchKernelGGL(k_gen_big, dim3(4096), dim3(256), 0, 0, (uint64_t*)code, c.n, c.nblk, stride);
        CHECK(hipDeviceSynchronize());
        for (int rep = 0; rep < 3; ++rep) {
            CHECK(hipEventRecord(a));
            hipLaunchKernelGGL(k_run_big, dim3(wgs), dim3(256), 0, 0, (const uint64_t*)code, stride,
                               c.group, c.calls, d_out, c.inv);
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, a, b));
            const double winst = (double)wgs * 4 * c.n * c.calls;  // wave-instructions
            std::printf("%-34s %8.3f ms  %.3f ns per wave-instr per SIMD (1024 SIMDs)\n", c.name, ms,
                        ms * 1e6 * 1024 / winst);
        }
    }
    return 0;
}
