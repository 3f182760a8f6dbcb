// jit16_ab.hip -- A/B of the generated decode with 16 output rows per wave
// (tool, not product).  The product kernel k_rs_jit gives each of 4 waves 8
// rows (64 accumulators, 128 VGPRs, 4 waves per SIMD) and every wave builds
// the 22 four-Russians composites of every source; here 2 waves own 16 rows
// each (128 accumulators in v40..v167, 168 VGPRs, 3 waves per SIMD), so the
// composites are built once per 16 rows (6765 -> ~5950 VALU per 8 rows), at
// the price of one wave per SIMD less.  Sources in LDS chunks of CS = 6
// (2 x 12 KiB: 6 workgroups of 2 waves per CU).  Both kernels run on the same
// random rows with random per-block coefficients, code emitted on the host.
//   python3 tools/gen_jit16_inc.py > build_ab/jit16.inc
//   make -C storage-benchmarks_amd build/tc_handlers.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -Ibuild_ab \
//     -Istorage-benchmarks_amd/csrc -Istorage-benchmarks_amd/build \
//     -o tools/jit16_ab tools/jit16_ab.hip -lhsa-runtime64
//   tools/jit16_ab [blocks=1024] [reps=5] [check=1] [late=0] [variants=2]
// variants: 0 base (k_rs_jit), 1 the tool's 16-row kernel, 2 rs_jit.hip's
// k_rs_jitw<16>, 3 the same in XCD-contiguous (block, tile) order
#include "../storage-benchmarks_amd/csrc/rs_jit.hip"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "jit16.inc"

namespace j16 {
using namespace rsgpu;
constexpr int CS = 6;          // sources per LDS chunk
constexpr int ADDR = 9;        // v9: LDS address of the chunk's first source + 16 lane
constexpr int PL = 10;         // v10..v17 planes L1 L2 L4 L8 H1 H2 H4 H8
constexpr int CL = 18;         // v18..v28 composites L[n], v29..v39 H[n]
constexpr int ACC = 40;        // v40..v167
constexpr int SRC_BYTES = 16 + 4 + 22 * 4 + 4 + 16 * 64;   // per source, 16 slots
constexpr int CHUNK_STRIDE = (CS * SRC_BYTES + 8 + 63) / 64 * 64;

inline int treg(int hi, int n)
{
    if ((n & (n - 1)) == 0) {
        const int a = n == 1 ? 0 : n == 2 ? 1 : n == 4 ? 2 : 3;
        return PL + 4 * hi + a;
    }
    const int below = 1 + (n > 2) + (n > 4) + (n > 8);
    return CL + 11 * hi + (n - below - 1);
}

// code of one chunk (nt sources) for one wave's 16 rows: coef[s][t].
// late = 1: the multiply-accumulates that read a plane register run first,
// then the next source's planes are loaded into those registers while the
// rest (composites only) run -- the LDS latency hides behind them.
int g_late = 0;
size_t emit_chunk(uint8_t* dst, int nt, const uint8_t (*coef)[CS])
{
    size_t o = 0;
    auto p32 = [&](uint32_t w) {
        for (int i = 0; i < 4; ++i)
            dst[o++] = (uint8_t)(w >> (8 * i));
    };
    auto p64 = [&](uint64_t w) {
        for (int i = 0; i < 8; ++i)
            dst[o++] = (uint8_t)(w >> (8 * i));
    };
    for (int t = 0; t < nt; ++t) {
        if (!g_late || t == 0) {
            p64(jit::enc_ds_read_b128(PL, ADDR, t * 2048));
            p64(jit::enc_ds_read_b128(PL + 4, ADDR, t * 2048 + 1024));
        }
        p32(jit::enc_waitcnt_lgkm(0));
        for (int hi = 0; hi < 2; ++hi)
            for (int n = 3; n < 16; ++n) {
                const int low = n & -n;
                if (n == low)
                    continue;
                p32(jit::enc_xor_e32(treg(hi, n), treg(hi, n ^ low), treg(hi, low)));
            }
        p32(jit::S_NOP0);
        auto single = [](int n) { return n && (n & (n - 1)) == 0; };
        for (int pass = 0; pass < (g_late ? 2 : 1); ++pass) {
            if (pass == 1 && t + 1 < nt) {  // planes dead: the next source's planes
                p64(jit::enc_ds_read_b128(PL, ADDR, (t + 1) * 2048));
                p64(jit::enc_ds_read_b128(PL + 4, ADDR, (t + 1) * 2048 + 1024));
            }
            for (int s = 0; s < 16; ++s)
                for (int b = 0; b < 8; ++b) {
                    const uint8_t m = jit::mat_row(coef[s][t], b);
                    const int acc = ACC + 8 * s + b, lo = m & 15, hi = m >> 4;
                    const bool plane = single(lo) || single(hi);
                    if (g_late && plane != (pass == 0))
                        continue;
                    p64(lo && hi ? jit::enc_bitop3_96(acc, acc, treg(0, lo), treg(1, hi))
                        : lo     ? jit::enc_xor_e64(acc, acc, treg(0, lo))
                        : hi     ? jit::enc_xor_e64(acc, acc, treg(1, hi))
                                 : (uint64_t)jit::S_NOP0 << 32 | jit::S_NOP0);
                }
        }
    }
    p64((uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82);
    return o;
}

template <int S>
__device__ __forceinline__ void read_slot(uint32_t (&W)[8])
{
    uint64_t P[4];
#define J16_RD(TEXT) asm volatile(TEXT : "=v"(P[0]), "=v"(P[1]), "=v"(P[2]), "=v"(P[3]))
    if constexpr (S == 0) J16_RD(J16_READ_SLOT_0);
    if constexpr (S == 1) J16_RD(J16_READ_SLOT_1);
    if constexpr (S == 2) J16_RD(J16_READ_SLOT_2);
    if constexpr (S == 3) J16_RD(J16_READ_SLOT_3);
    if constexpr (S == 4) J16_RD(J16_READ_SLOT_4);
    if constexpr (S == 5) J16_RD(J16_READ_SLOT_5);
    if constexpr (S == 6) J16_RD(J16_READ_SLOT_6);
    if constexpr (S == 7) J16_RD(J16_READ_SLOT_7);
    if constexpr (S == 8) J16_RD(J16_READ_SLOT_8);
    if constexpr (S == 9) J16_RD(J16_READ_SLOT_9);
    if constexpr (S == 10) J16_RD(J16_READ_SLOT_10);
    if constexpr (S == 11) J16_RD(J16_READ_SLOT_11);
    if constexpr (S == 12) J16_RD(J16_READ_SLOT_12);
    if constexpr (S == 13) J16_RD(J16_READ_SLOT_13);
    if constexpr (S == 14) J16_RD(J16_READ_SLOT_14);
    if constexpr (S == 15) J16_RD(J16_READ_SLOT_15);
#undef J16_RD
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        W[2 * q] = (uint32_t)P[q];
        W[2 * q + 1] = (uint32_t)(P[q] >> 32);
    }
}

// 2 waves x 16 rows; compiler-allocated VGPRs v0..v39, of which the call
// clobbers v9..v39 (so what lives across it fits v0..v8)
__global__ __launch_bounds__(128) __attribute__((amdgpu_num_vgpr(40))) void k_jit16(JitArgs a)
{
    __shared__ uint4 lds[2][CS * 2 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    const long long tile = blockIdx.x;
    const int k = a.k;
    const int nch = (k + CS - 1) / CS;
    const uint8_t* const* srcs = a.srcs + (size_t)b * k;
    uint8_t* const* dsts = a.dsts + (size_t)b * a.dst_stride;
    const uint8_t* code = a.code + (size_t)b * a.block_stride + (size_t)wave * nch * a.chunk_stride;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];
    const long long off = tile * 2048 + lane * 32;
    const uint32_t loff = off + 32 <= a.len ? (uint32_t)off : 0u;
    if (wave == 0)
        asm volatile("s_icache_inv\n s_nop 15\n s_nop 15" ::: "memory");
    auto issue = [&](int ch) {
        const int c0 = ch * CS, nt = min(CS, k - c0);
        const uint32_t base = lds0 + (uint32_t)((ch & 1) * CS * 2 * 64 * 16);
        for (int t = wave; t < nt; t += 2)
            bs::glds32(bs::sload_ptr(srcs + c0 + t), loff, base + (uint32_t)(t * 2 * 64 * 16));
    };
    asm volatile(J16_ZERO ::: J16_ACC_CLOBBERS);
    issue(0);
    for (int ch = 0; ch < nch; ++ch) {
        const int nt = min(CS, k - ch * CS);
        uint4* buf = lds[ch & 1];
        bs::wait_vm(0);
        {
            const uint32_t m4 = bs::vconst(0x0F0F0F0Fu), m2 = bs::vconst(0x33333333u), m1 = bs::vconst(0x55555555u);
            for (int t = wave; t < nt; t += 2) {
                uint4 u = buf[(t * 2 + 0) * 64 + lane], v = buf[(t * 2 + 1) * 64 + lane];
                uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                bs::tr8(W, m4, m2, m1);
                buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
                buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
            }
        }
        bs::barrier_lds();
        if (ch + 1 < nch)
            issue(ch + 1);
        const uint32_t la = lds0 + (uint32_t)((ch & 1) * CS * 2 * 64 * 16) + lane * 16;
        const uint8_t* fn = code + (size_t)ch * a.chunk_stride;
        asm volatile("s_swappc_b64 s[82:83], %[fn]"
                     :
                     : [fn] "s"(fn), "{v9}"(la)
                     : "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                       "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33",
                       "v34", "v35", "v36", "v37", "v38", "v39", "s82", "s83", "scc", "memory",
                       J16_ACC_CLOBBERS);
    }
    if (off + 32 <= a.len) {
        const uint32_t m4 = bs::vconst(0x0F0F0F0Fu), m2 = bs::vconst(0x33333333u), m1 = bs::vconst(0x55555555u);
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            (
                [&] {
                    const int r = wave * 16 + Ss;
                    if (r < a.rows) {
                        uint32_t W[8];
                        read_slot<Ss>(W);
                        bs::tr8(W, m4, m2, m1);
                        bs::store32((uint8_t*)bs::sload_ptr((const uint8_t* const*)(dsts + r)), off, W);
                    }
                }(),
                ...);
        }(std::make_integer_sequence<int, 16>{});
    }
}
}  // namespace j16

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

__global__ void k_copy64(uint64_t* dst, const uint64_t* src, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static void* to_exec(const std::vector<uint8_t>& code)
{
    uint64_t* stage;
    (void)hipMalloc(&stage, code.size());
    (void)hipMemcpy(stage, code.data(), code.size(), hipMemcpyHostToDevice);
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    hsa_amd_pointer_info(stage, &info, nullptr, nullptr, nullptr);
    hsa_amd_memory_pool_t pool{};
    hsa_amd_agent_iterate_memory_pools(info.agentOwner, pick, &pool);
    void* exec = nullptr;
    if (hsa_amd_memory_pool_allocate(pool, code.size(), HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, &exec) !=
        HSA_STATUS_SUCCESS)
        return nullptr;
    hipLaunchKernelGGL(k_copy64, dim3(4096), dim3(256), 0, 0, (uint64_t*)exec, stage, (long long)(code.size() / 8));
    (void)hipDeviceSynchronize();
    (void)hipFree(stage);
    return exec;
}

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 1024;
    const int R = argc > 2 ? atoi(argv[2]) : 5;
    const bool check = argc > 3 ? atoi(argv[3]) != 0 : true;
    j16::g_late = argc > 4 ? atoi(argv[4]) : 0;
    const int k = 64, e = 32;
    const long long L = 1000000, pitch = 1000192;
    uint8_t *rows, *out2;
    if (hipMalloc(&rows, (size_t)B * (k + e) * pitch) != hipSuccess ||
        hipMalloc(&out2, (size_t)B * e * pitch) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipLaunchKernelGGL(k_fill_random, dim3(8192), dim3(256), 0, 0, (uint64_t*)rows,
                       (long long)((size_t)B * (k + e) * pitch / 8));
    std::vector<const uint8_t*> sp((size_t)B * k);
    std::vector<uint8_t*> dp((size_t)B * e), dp2((size_t)B * e);
    for (int b = 0; b < B; ++b) {
        for (int j = 0; j < k; ++j)
            sp[(size_t)b * k + j] = rows + ((size_t)b * (k + e) + j) * pitch;
        for (int i = 0; i < e; ++i) {
            dp[(size_t)b * e + i] = rows + ((size_t)b * (k + e) + k + i) * pitch;
            dp2[(size_t)b * e + i] = out2 + ((size_t)b * e + i) * pitch;
        }
    }
    const uint8_t** d_sp;
    uint8_t **d_dp, **d_dp2;
    (void)hipMalloc(&d_sp, sp.size() * 8);
    (void)hipMalloc(&d_dp, dp.size() * 8);
    (void)hipMalloc(&d_dp2, dp2.size() * 8);
    (void)hipMemcpy(d_sp, sp.data(), sp.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_dp, dp.data(), dp.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_dp2, dp2.data(), dp2.size() * 8, hipMemcpyHostToDevice);
    int* d_st;
    (void)hipMalloc(&d_st, B * sizeof(int));
    (void)hipMemset(d_st, 0, B * sizeof(int));

    // the same random e x k matrix per block for both kernels
    std::vector<uint8_t> coef((size_t)B * e * k);
    uint32_t x = 12345;
    for (auto& c : coef) {
        x = x * 1664525u + 1013904223u;
        c = (uint8_t)(x >> 13);
    }
    // product layout (rs_jit.h): 4 waves x 8 rows, chunks of 8
    const size_t per = jit_code_bytes(k, e, 1);
    std::vector<uint8_t> code1(per * B);
    const int nch8 = (k + 7) / 8, stride_w = jit::chunk_stride(8) / 8;
    for (int b = 0; b < B; ++b) {
        uint64_t* cb = (uint64_t*)(code1.data() + (size_t)b * per);
        for (size_t i = 0; i < per / 8; ++i)
            cb[i] = (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
        for (int w = 0; w < 4; ++w)
            for (int ch = 0; ch < nch8; ++ch)
                for (int o = 0; o < stride_w; ++o) {
                    uint64_t word;
                    if (jit::code_word(coef.data() + ((size_t)b * e + 8 * w) * k, k, 8, ch, o, &word))
                        cb[((size_t)w * nch8 + ch) * stride_w + o] = word;
                }
    }
    // 16-row layout: 2 waves x 16 rows, chunks of CS
    const int nch6 = (k + j16::CS - 1) / j16::CS;
    const size_t per2 = (size_t)2 * nch6 * j16::CHUNK_STRIDE;
    std::vector<uint8_t> code2(per2 * B);
    for (int b = 0; b < B; ++b)
        for (int w = 0; w < 2; ++w)
            for (int ch = 0; ch < nch6; ++ch) {
                const int nt = std::min(j16::CS, k - ch * j16::CS);
                uint8_t cf[16][j16::CS];
                for (int s = 0; s < 16; ++s)
                    for (int t = 0; t < nt; ++t)
                        cf[s][t] = coef[((size_t)b * e + 16 * w + s) * k + ch * j16::CS + t];
                j16::emit_chunk(code2.data() + (size_t)b * per2 + ((size_t)w * nch6 + ch) * j16::CHUNK_STRIDE, nt,
                                cf);
            }
    void* x1 = to_exec(code1);
    void* x2 = to_exec(code2);
    if (!x1 || !x2) {
        printf("exec alloc failed\n");
        return 1;
    }
    JitArgs a{};
    a.srcs = d_sp;
    a.dsts = d_dp;
    a.code = (const uint8_t*)x1;
    a.chunk_stride = jit::chunk_stride(8);
    a.block_stride = (long long)per;
    a.dst_stride = e;
    a.k = k;
    a.rows = e;
    a.len = L;
    a.status = d_st;
    JitArgs a2 = a;
    a2.dsts = d_dp2;
    a2.code = (const uint8_t*)x2;
    a2.chunk_stride = j16::CHUNK_STRIDE;
    a2.block_stride = (long long)per2;
    const dim3 grid((unsigned)((L + 2047) / 2048), (unsigned)B);
    JitArgs a3 = a2;  // the product kernel (rs_jit.hip k_rs_jit16) in XCD-contiguous order
    a3.xcd_order = 1;
    auto run = [&](int which) {
        if (which == 0)
            return launch_rs_jit(a, B, 0);
        if (which == 2)
            return launch_rs_jitw(a2, B, 0);
        if (which == 3)
            return launch_rs_jitw(a3, B, 0);
        hipLaunchKernelGGL(j16::k_jit16, grid, dim3(128), 0, 0, a2);
        return hipGetLastError();
    };
    const int nvar = argc > 5 ? atoi(argv[5]) : 2;  // variants timed: base, tool rows16, product, product xcd
    if (check) {  // both write the same bytes (the product kernel into the parity rows)
        (void)run(0);
        (void)run(1);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("kernel failed\n");
            return 1;
        }
        std::vector<uint8_t> h1(L), h2(L);
        long long bad = 0;
        for (int b = 0; b < B; b += std::max(1, B / 16))
            for (int i = 0; i < e; ++i) {
                (void)hipMemcpy(h1.data(), dp[(size_t)b * e + i], L, hipMemcpyDeviceToHost);
                (void)hipMemcpy(h2.data(), dp2[(size_t)b * e + i], L, hipMemcpyDeviceToHost);
                for (long long j = 0; j < L; ++j)
                    bad += h1[j] != h2[j];
            }
        printf("check: %lld differing bytes (sampled blocks)\n", bad);
    }
    for (int rep = 0; rep < R; ++rep)
        for (int which = 0; which < nvar; ++which) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            (void)run(which);
            (void)hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) {
                printf("kernel failed\n");
                return 1;
            }
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            static const char* nm[4] = {"base  ", "rows16", "prod16", "prodx "};
            printf("%s rep %d: %.3f ms (%.2f TB/s alg)\n", nm[which], rep, ms,
                   (double)B * (k + e) * L / (ms * 1e-3) / 1e12);
        }
    return 0;
}
