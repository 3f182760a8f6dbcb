// fused_ab.hip -- A/B timing of k_rs_decode_fused<64,32> (tool, not product):
// the same driver compiled against different generated asm (gen_tc_handlers.py
// variants in different include dirs), random rows, random erasures and random
// handler tables; prints the median of R launches.
//   RSGPU_TC_LAYOUT=late python3 storage-benchmarks_amd/csrc/gen_tc_handlers.py \
//     D/tc_handlers.inc D/syn_blocks.inc
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -Istorage-benchmarks_amd/csrc -ID \
//     -o tools/fused_ab_X tools/fused_ab.hip
#include "../storage-benchmarks_amd/csrc/rs_tc.hip"
#include "../storage-benchmarks_amd/csrc/rs_decode_fused.hip"

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <random>
#include <string>
#include <vector>

int main(int argc, char** argv)
{
    using namespace rsgpu;
    const int B = argc > 1 ? atoi(argv[1]) : 1024;
    const int R = argc > 2 ? atoi(argv[2]) : 7;
    const int k = 64, e = 32;
    // RSGPU_AB_NC=n: coefficients drawn from 1..n only (instruction-cache
    // working set experiment; products wrong, timing only)
    const unsigned nc = std::getenv("RSGPU_AB_NC") ? (unsigned)atoi(std::getenv("RSGPU_AB_NC")) : 255u;

    const long long L = 1000000, pitch = 1000192;
    uint8_t *src, *par, *out;
    if (hipMalloc(&src, (size_t)B * k * pitch) != hipSuccess ||
        hipMalloc(&par, (size_t)B * e * pitch) != hipSuccess ||
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
        for (auto [p, n] : {std::pair<uint8_t*, size_t>{src, (size_t)B * k * pitch},
                            std::pair<uint8_t*, size_t>{par, (size_t)B * e * pitch}})
            for (size_t o = 0; o < n; o += chunk)
                (void)hipMemcpy(p + o, d + (o / chunk % 7) * 4096, std::min(chunk - 7 * 4096, n - o),
                                hipMemcpyDeviceToDevice);
        (void)hipFree(d);
    }
    std::vector<unsigned long long> em(2 * B, 0);
    for (int b = 0; b < B; ++b) {
        std::vector<int> idx(k);
        std::iota(idx.begin(), idx.end(), 0);
        std::shuffle(idx.begin(), idx.end(), rng);
        for (int i = 0; i < e; ++i)
            em[2 * b] |= 1ull << idx[i];
    }
    unsigned long long *d_em, *d_q, *d_addr, *d_sa;
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
    auto table = [&](size_t n) {
        std::vector<unsigned long long> v(n);
        for (size_t i = 0; i < n; ++i) {  // the handler copy of slot / source parity
            v[i] = q[0] + (unsigned long long)(tc_slot_copy((int)(i % 8)) * 256 + 1 + rng() % nc) *
                              tc_handler_stride();
        }
        unsigned long long* d;
        (void)hipMalloc(&d, n * 8);
        (void)hipMemcpy(d, v.data(), n * 8, hipMemcpyHostToDevice);
        return d;
    };
    d_addr = table((size_t)B * e * 32);
    d_sa = table((size_t)B * (k - e) * 32);
    (void)hipMalloc(&d_status, B * sizeof(int));
    (void)hipMemset(d_status, 0, B * sizeof(int));
    // mode "tc": the one-matrix decode through k_rs_tc instead (64 sources =
    // 32 survivors + 32 parity rows, 32 output rows, random coefficients)
    const bool tc_mode = argc > 4 && std::string(argv[4]) == "tc";
    TcArgs ta{};
    if (tc_mode) {
        std::vector<const uint8_t*> sp((size_t)B * k);
        std::vector<uint8_t*> dp((size_t)B * e);
        for (int b = 0; b < B; ++b) {
            int n = 0;
            for (int j = 0; j < k; ++j)
                if (!((em[2 * b] >> j) & 1))
                    sp[(size_t)b * k + n++] = src + ((size_t)b * k + j) * pitch;
            for (int r = 0; r < e; ++r)
                sp[(size_t)b * k + n++] = par + ((size_t)b * e + r) * pitch;
            for (int r = 0; r < e; ++r)
                dp[(size_t)b * e + r] = out + ((size_t)b * e + r) * pitch;
        }
        const uint8_t** d_sp;
        uint8_t** d_dp;
        (void)hipMalloc(&d_sp, sp.size() * 8);
        (void)hipMalloc(&d_dp, dp.size() * 8);
        (void)hipMemcpy(d_sp, sp.data(), sp.size() * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_dp, dp.data(), dp.size() * 8, hipMemcpyHostToDevice);
        ta.srcs = d_sp;
        ta.dsts = d_dp;
        ta.addr = table((size_t)B * k * 32);
        ta.addr_stride = (long long)k * 32;
        ta.k = k;
        ta.rows = e;
        ta.len = L;
        ta.status = d_status;
    }
    auto run = [&] {
        if (tc_mode)
            return launch_rs_tc(ta, B, 0);
        return launch_rs_decode_fused(k, e, src, par, out, pitch, L, B, (const uint64_t*)d_em,
                                      d_addr, d_sa, d_status, 0);
    };
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
    std::vector<float> s = ms;
    std::sort(s.begin(), s.end());
    printf("%s %s<64,32> B=%d: median %.3f ms  min %.3f  max %.3f  (%.1f GB/s alg)\n",
           argc > 3 ? argv[3] : "", tc_mode ? "k_rs_tc" : "k_rs_decode_fused", B, s[R / 2], s[0], s[R - 1],
           (double)(k + e) * L * B / (s[R / 2] * 1e-3) / 1e9);
    return 0;
}
