// gf256.h -- GF(2^8) arithmetic for the MI355X RS engine (host + device, constexpr).
//
// Field: GF(2^8) with primitive polynomial x^8+x^4+x^3+x^2+1 (0x11D) and
// generator 2, the field of ISA-L 2.13 (isa/ec_base.h:35 gff_base,
// isa/ec_base.c:159-161 0x1d reduction).  Everything here is computed, not
// tabulated from the reference.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RS_HD __host__ __device__
#else
#define RS_HD
#endif

namespace rsgpu {

// Carry-less multiply with reduction by 0x11D (shift-and-add form).
RS_HD constexpr uint8_t gf_mul_slow(uint8_t a, uint8_t b)
{
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1)
            p ^= a;
        const bool hi = (a & 0x80) != 0;
        a = (uint8_t)(a << 1);
        if (hi)
            a ^= 0x1D;
        b >>= 1;
    }
    return p;
}

RS_HD constexpr uint8_t gf_pow(uint8_t a, int e)
{
    uint8_t r = 1;
    for (int i = 0; i < e; ++i)
        r = gf_mul_slow(r, a);
    return r;
}

// 2^e with e taken mod 255 (2 is primitive).
RS_HD constexpr uint8_t gf_exp2(int e)
{
    e %= 255;
    if (e < 0)
        e += 255;
    uint8_t r = 1;
    for (int i = 0; i < e; ++i)
        r = gf_mul_slow(r, 2);
    return r;
}

// Coefficient of the parity row p, column j of gf_gen_rs_matrix
// (isa/ec_base.c:62-79): row k+p is gen^j with gen = 2^p, i.e. 2^(p*j).
RS_HD constexpr uint8_t rs_vand_coef(int p, int j) { return gf_exp2((p * j) % 255); }

// Runtime field with log/antilog tables (host side and device LDS copies).
struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
};

RS_HD inline void gf_build_tables(GfTables& t)
{
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = (uint8_t)v;
        t.exp[i + 255] = (uint8_t)v;
        t.log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    t.log[0] = 0;
}

// The same tables as a constant expression (device code copies them into
// LDS with one load per thread instead of building them serially).
RS_HD constexpr GfTables make_gf_tables()
{
    GfTables t{};
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = (uint8_t)v;
        t.exp[i + 255] = (uint8_t)v;
        t.log[v] = (uint8_t)i;
        v <<= 1;
        if (v & 0x100)
            v ^= 0x11D;
    }
    t.exp[510] = t.exp[0];
    t.exp[511] = t.exp[1];
    t.log[0] = 0;
    return t;
}

// The v_perm lookup tables of one coefficient c for the runtime-coefficient
// kernel (see rs_kernels.hip, "generic dot product"):
//   t[0] = c*{0,1,2,3}        t[1] = c*{4,5,6,7}          (bits 0-2)
//   t[2] = c*{0,8,16,24}      t[3] = c*{32,40,48,56}      (bits 3-5)
//   t[4] = c*{0,64,128,192}                                (bits 6-7)
// Byte n of t[0..1] is c*n, etc.  Little-endian packing.
RS_HD inline void perm_tables(uint8_t c, uint32_t t[5])
{
    uint8_t v[20];
    for (int n = 0; n < 8; ++n) {
        v[n] = gf_mul_slow(c, (uint8_t)n);
        v[8 + n] = gf_mul_slow(c, (uint8_t)(n << 3));
    }
    for (int n = 0; n < 4; ++n)
        v[16 + n] = gf_mul_slow(c, (uint8_t)(n << 6));
    for (int w = 0; w < 5; ++w)
        t[w] = (uint32_t)v[4 * w] | ((uint32_t)v[4 * w + 1] << 8) | ((uint32_t)v[4 * w + 2] << 16) |
               ((uint32_t)v[4 * w + 3] << 24);
}

}  // namespace rsgpu
