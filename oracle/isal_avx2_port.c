/*
 * isal_avx2_port.c -- CPU BASELINE ONLY (test infrastructure; the engine never
 * links it).  ISA-L 2.13's AVX2 dot-product path restated in C intrinsics,
 * because the reference's yasm sources cannot be assembled in this image
 * (no yasm/nasm).  Linked into oracle/_ref/libisal_ref.so next
 * to the reference's own ec_base.c / ec_highlevel_func.c, so matrices, tables
 * and inversion stay the reference's code and only the data kernel is ported.
 *
 *   ec_encode_data_avx2    isa/ec_highlevel_func.c:106-135: len < 32 -> base;
 *                          rows in passes of 4, then a 3/2/1 tail; every pass
 *                          re-streams all k sources
 *   gf_4vect_dot_prod_avx2 isa/gf_4vect_dot_prod_avx2.asm:303-451 (and the
 *                          3/2/1-output twins): per 32-byte position and
 *                          source, split the bytes into nibbles (vpand,
 *                          vpsraw 4), per output two vpshufb on the source's
 *                          broadcast 16-byte lo/hi tables (ec_init_tables
 *                          layout: table of (row r, source j) at
 *                          g + (r*k + j)*32), vpxor into the accumulator
 *
 * The asm handles len % 32 with an overlapped final chunk
 * (gf_vect_dot_prod_avx2.asm:255-261); here the last 32 bytes are recomputed
 * at len - 32, which writes the same bytes.
 */
#include <immintrin.h>
#include <stdint.h>

void ec_encode_data_base(int len, int srcs, int dests, unsigned char *v,
                         unsigned char **src, unsigned char **dest);

#define PORT_AVX2 __attribute__((target("avx2"), always_inline)) static inline

PORT_AVX2 void dot_chunk(int off, int k, int nout, const unsigned char *g,
                         unsigned char **src, unsigned char **dest)
{
    const __m256i mask = _mm256_set1_epi8(0x0f);
    __m256i acc0 = _mm256_setzero_si256(), acc1 = acc0, acc2 = acc0, acc3 = acc0;
    const size_t row = (size_t)k * 32;
    for (int j = 0; j < k; ++j) {
        const __m256i x = _mm256_loadu_si256((const __m256i *)(src[j] + off));
        const __m256i lo = _mm256_and_si256(x, mask);
        const __m256i hi = _mm256_and_si256(_mm256_srli_epi16(x, 4), mask);
        const unsigned char *t = g + (size_t)j * 32;
#define PORT_MAC(ACC, R)                                                                         \
    do {                                                                                         \
        const __m256i tl = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t + (R) * row)));      \
        const __m256i th = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)(t + (R) * row + 16))); \
        ACC = _mm256_xor_si256(ACC, _mm256_xor_si256(_mm256_shuffle_epi8(tl, lo),                \
                                                     _mm256_shuffle_epi8(th, hi)));              \
    } while (0)
        PORT_MAC(acc0, 0);
        if (nout > 1)
            PORT_MAC(acc1, 1);
        if (nout > 2)
            PORT_MAC(acc2, 2);
        if (nout > 3)
            PORT_MAC(acc3, 3);
#undef PORT_MAC
    }
    _mm256_storeu_si256((__m256i *)(dest[0] + off), acc0);
    if (nout > 1)
        _mm256_storeu_si256((__m256i *)(dest[1] + off), acc1);
    if (nout > 2)
        _mm256_storeu_si256((__m256i *)(dest[2] + off), acc2);
    if (nout > 3)
        _mm256_storeu_si256((__m256i *)(dest[3] + off), acc3);
}

/* gf_{1,2,3,4}vect_dot_prod_avx2: nout outputs, compile-time after inlining */
PORT_AVX2 void dot_prod_n(int len, int k, int nout, const unsigned char *g,
                          unsigned char **src, unsigned char **dest)
{
    int off = 0;
    for (; off + 32 <= len; off += 32)
        dot_chunk(off, k, nout, g, src, dest);
    if (off < len)
        dot_chunk(len - 32, k, nout, g, src, dest);
}

__attribute__((target("avx2"))) static void dot4(int len, int k, const unsigned char *g,
                                                 unsigned char **s, unsigned char **d)
{
    dot_prod_n(len, k, 4, g, s, d);
}
__attribute__((target("avx2"))) static void dot3(int len, int k, const unsigned char *g,
                                                 unsigned char **s, unsigned char **d)
{
    dot_prod_n(len, k, 3, g, s, d);
}
__attribute__((target("avx2"))) static void dot2(int len, int k, const unsigned char *g,
                                                 unsigned char **s, unsigned char **d)
{
    dot_prod_n(len, k, 2, g, s, d);
}
__attribute__((target("avx2"))) static void dot1(int len, int k, const unsigned char *g,
                                                 unsigned char **s, unsigned char **d)
{
    dot_prod_n(len, k, 1, g, s, d);
}

int port_have_avx2(void)
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") ? 1 : 0;
}

/* ec_encode_data_avx2 (isa/ec_highlevel_func.c:106-135) */
void port_ec_encode_data_avx2(int len, int k, int rows, unsigned char *g, unsigned char **data,
                              unsigned char **coding)
{
    if (len < 32 || !port_have_avx2()) {
        ec_encode_data_base(len, k, rows, g, data, coding);
        return;
    }
    while (rows >= 4) {
        dot4(len, k, g, data, coding);
        g += 4 * k * 32;
        coding += 4;
        rows -= 4;
    }
    switch (rows) {
    case 3: dot3(len, k, g, data, coding); break;
    case 2: dot2(len, k, g, data, coding); break;
    case 1: dot1(len, k, g, data, coding); break;
    default: break;
    }
}
