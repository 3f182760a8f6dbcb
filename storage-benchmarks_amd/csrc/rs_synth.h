// rs_synth.h -- seeded synthetic symbols and erasure patterns (host + device).
//
// The reference fills source symbols with libc rand() after srand(time(0))
// (benchmark/isa_throughput/isa.cpp:56-58, :324) and draws `erased` distinct
// original indices with rand() % k into a std::set (isa.cpp:137-153).  The
// engine replaces rand() by a counter-based mix so that any device, any rank
// and the CPU oracle produce identical bytes for (seed, row, word).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RS_SYN_HD __host__ __device__
#else
#define RS_SYN_HD
#endif

namespace rsgpu {

RS_SYN_HD inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// 8 bytes (little endian) at byte offset 8*word of synthetic row `row`.
RS_SYN_HD inline uint64_t synth_word(uint64_t seed, uint64_t row, uint64_t word)
{
    return mix64(seed * 0x9E3779B97F4A7C15ull + row * 0xD1B54A32D192ED03ull + word);
}

// Erasure list of block `blk`: e distinct originals in [0, k), ascending.
inline void erasure_pattern(uint64_t seed, uint64_t blk, int k, int e, uint8_t* err_list)
{
    uint8_t in[256] = {0};
    if (e > k || k > 256 || e < 0)
        return;
    int have = 0;
    uint64_t ctr = 0;
    while (have < e) {
        const uint64_t r = mix64(seed ^ 0xA5A5A5A55A5A5A5Aull) ^ mix64(blk * 0x2545F4914F6CDD1Dull + ctr++);
        const int s = (int)(mix64(r) % (uint64_t)k);
        if (in[s])
            continue;
        in[s] = 1;
        ++have;
    }
    for (int i = 0, n = 0; i < k; ++i)
        if (in[i])
            err_list[n++] = (uint8_t)i;
}

}  // namespace rsgpu
