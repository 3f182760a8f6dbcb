// jit_enc.h -- gfx950 instruction words of the generated code (rs_jit.h,
// jit_prog.cpp) and the LDS layout they address; shared with the diagnostic
// build's code-word variants (diag_variants.h).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RJ_HD __host__ __device__
#else
#define RJ_HD
#endif

namespace rsgpu {
namespace jit {

constexpr int LDS_SRC = 2048;    // LDS bytes per source: [2 halves][64 lanes] x 16 B
constexpr int LDS_HALF = 1024;

// ---- gfx950 encodings (llvm-mc -mcpu=gfx950 -show-encoding) -------------

RJ_HD constexpr uint64_t enc_bitop3_96(int d, int a, int b, int c)  // d = a ^ b ^ c
{
    const uint32_t w0 = 0xd2340200u | (uint32_t)d;
    const uint32_t w1 = 0xd0000000u | ((uint32_t)(256 + c) << 18) | ((uint32_t)(256 + b) << 9) |
                        (uint32_t)(256 + a);
    return (uint64_t)w1 << 32 | w0;
}
RJ_HD constexpr uint64_t enc_xor_e64(int d, int a, int b)  // VOP3 form, 8 bytes
{
    const uint32_t w0 = 0xd1150000u | (uint32_t)d;
    const uint32_t w1 = ((uint32_t)(256 + b) << 9) | (uint32_t)(256 + a);
    return (uint64_t)w1 << 32 | w0;
}
RJ_HD constexpr uint32_t enc_xor_e32(int d, int a, int b)  // VOP2, 4 bytes
{
    return 0x2a000000u | ((uint32_t)d << 17) | ((uint32_t)b << 9) | (uint32_t)(256 + a);
}
RJ_HD constexpr uint64_t enc_ds_read_b128(int vd, int vaddr, int offset)
{
    return (uint64_t)(((uint32_t)vd << 24) | (uint32_t)vaddr) << 32 | (0xd9fe0000u | (uint32_t)offset);
}
constexpr uint32_t S_NOP0 = 0xbf800000u;
constexpr uint64_t NOP2 = (uint64_t)S_NOP0 << 32 | S_NOP0;  // two s_nop 0: a zero-mask word
constexpr uint32_t S_SETPC_82 = 0xbe801d52u;  // s_setpc_b64 s[82:83]
RJ_HD constexpr uint32_t enc_waitcnt_lgkm(int n) { return 0xbf8cc07fu | ((uint32_t)n << 8); }

}  // namespace jit
}  // namespace rsgpu
