// rs_jit.h -- generated decode / encode code (k_rs_jit, rs_jit.hip).
//
// The one-matrix decode applies an e x k coefficient matrix that differs per
// block (random erasures).  k_rs_tc dispatches each coefficient through a
// handler (a jump, SALU work and GPR-index mode per coefficient); here
// k_jit_emit instead WRITES the straight-line code of every (block, wave,
// chunk of 8 sources) into executable device memory, with the coefficients
// baked into the register operands, and the decode kernel makes one call per
// chunk.  The encode of a matrix shared by every block gets the same kind of
// code, built once on the host (jit_prog.h).  Only vector-ALU, LDS-read,
// s_waitcnt, s_nop and s_setpc instructions are ever generated.
//
// Register contract (the decode kernel's asm statement clobbers all of it):
//   v20            LDS byte address of the chunk's first source + 16 lane
//   v24..v31       planes of the current source, bank A: L1 L2 L4 L8 H1 H2
//                  H4 H8 (plane a of the 32 bytes of a lane, bit-sliced as in
//                  rs_bitsliced.hip / bitslice.h tr8)
//   v54..v61       the same, bank B (odd sources: the next source's planes
//                  land in the other bank while this one is consumed)
//   v32..v42       composite four-Russians entries L[n], n = 3 5 6 7 9 ... 15
//   v43..v53       composite entries H[n]
//   v64..v127      accumulators: slot s (output row 8 w + s) planes v[64+8s ..]
//   s[82:83]       return address (s_swappc_b64 s[82:83], code)
//
// Code of one chunk (nt <= 8 sources, nslot <= 8 output rows of the wave):
//   prologue   ds_read_b128 x2: source 0's planes into bank A      16 B
//   source t   [ds_read_b128 x2 of source t+1 into bank (t+1)&1, or 2 x
//              (s_nop; s_nop)], s_waitcnt lgkmcnt(2 or 0), 22 v_xor_b32
//              composites from bank t&1, s_nop, then per slot 8
//              multiply-accumulates of 8 bytes each (v_bitop3_b32 0x96 /
//              v_xor_b32_e64 / s_nop pair for a zero row)       112 + 64 nslot B
//   epilogue   s_setpc_b64 s[82:83]; s_nop                           8 B
// The layout depends on (nt, nslot) only, never on the coefficients (the
// host-built shared programs of jit_prog.h size each preamble to its cover).
#pragma once
#include <stdint.h>

#include "jit_enc.h"
#include "kernel_hooks.h"

namespace rsgpu {
namespace jit {

constexpr int ACC = 64;          // accumulator base register
constexpr int PRO_BYTES = 16;
constexpr int PRE_BYTES = 112;   // per source before the multiply-accumulates
constexpr int EPI_BYTES = 8;

RJ_HD constexpr int src_bytes(int nslot) { return PRE_BYTES + 64 * nslot; }
RJ_HD constexpr int chunk_bytes(int nt, int nslot) { return PRO_BYTES + nt * src_bytes(nslot) + EPI_BYTES; }
// stride between chunks: the largest chunk, rounded to 64-byte lines
RJ_HD constexpr int chunk_stride(int nslot) { return (chunk_bytes(8, nslot) + 63) / 64 * 64; }

// plane registers of bank `bank`: entry 0..3 = L1 L2 L4 L8, 4..7 = H1 H2 H4 H8
RJ_HD constexpr int plane_reg(int bank, int a) { return (bank ? 54 : 24) + a; }

// four-Russians table register of L[n] (hi = 0) or H[n] (hi = 1), n = 1..15
RJ_HD constexpr int table_reg(int bank, int hi, int n)
{
    if ((n & (n - 1)) == 0) {  // single plane
        const int a = n == 1 ? 0 : n == 2 ? 1 : n == 4 ? 2 : 3;
        return plane_reg(bank, 4 * hi + a);
    }
    // composites n = 3 5 6 7 9 10 11 12 13 14 15 -> 0..10: n minus the
    // single-plane values below it (1, 2, 4, 8) minus 1
    const int below = 1 + (n > 2) + (n > 4) + (n > 8);
    return 32 + 11 * hi + (n - below - 1);
}

// Row b of the 8 x 8 GF(2) matrix of x -> c x: bit a set iff bit b of c 2^a.
RJ_HD constexpr uint8_t mat_row(uint8_t c, int b)
{
    uint8_t x = c, r = 0;
    for (int a = 0; a < 8; ++a) {
        r |= (uint8_t)(((x >> b) & 1) << a);
        x = (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1D : 0));
    }
    return r;
}

// The eight words of coefficient c on slot s at once (one matrix per call)
RJ_HD inline void mac_words(uint8_t c, int s, int bank, uint64_t (&wd)[8])
{
    uint8_t x = c, row[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int a = 0; a < 8; ++a) {  // row b bit a = bit b of c 2^a
        for (int b = 0; b < 8; ++b)
            row[b] |= (uint8_t)(((x >> b) & 1) << a);
        x = (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1D : 0));
    }
    for (int b = 0; b < 8; ++b) {
        const int acc = ACC + 8 * s + b, lo = row[b] & 15, hi = row[b] >> 4;
        wd[b] = lo && hi ? enc_bitop3_96(acc, acc, table_reg(bank, 0, lo), table_reg(bank, 1, hi))
                : lo     ? enc_xor_e64(acc, acc, table_reg(bank, 0, lo))
                : hi     ? enc_xor_e64(acc, acc, table_reg(bank, 1, hi))
                         : (uint64_t)S_NOP0 << 32 | S_NOP0;
    }
}

// 32-bit word i (< PRE_BYTES / 4 = 28) of source t's preamble: the next
// source's two plane loads (or no-ops for the chunk's last source), the wait
// for this source's planes, the 22 four-Russians composites, one s_nop
RJ_HD inline uint32_t pre_u32(int t, int nt, int i)
{
    const int bank = t & 1, nb = (t + 1) & 1;
    if (i < 4) {
        if (t + 1 >= nt)
            return S_NOP0;
        const uint64_t d = enc_ds_read_b128(plane_reg(nb, i < 2 ? 0 : 4), 20,
                                            (t + 1) * LDS_SRC + (i < 2 ? 0 : LDS_HALF));
        return (i & 1) ? (uint32_t)(d >> 32) : (uint32_t)d;
    }
    if (i == 4)
        return enc_waitcnt_lgkm(t + 1 < nt ? 2 : 0);
    const int j = i - 5;
    if (j >= 22)
        return S_NOP0;
    // composites n = 3 5 6 7 9 10 11 12 13 14 15 of L, then of H
    const int hi = j / 11, c = j - 11 * hi;
    const int n = c < 1 ? 3 : c < 4 ? 4 + c : 5 + c;
    const int low = n & -n;
    return enc_xor_e32(table_reg(bank, hi, n), table_reg(bank, hi, n ^ low), table_reg(bank, hi, low));
}

// Word o (8 bytes) of chunk ch of a wave's code, for the wave's nslot rows
// rows[s * k + q] (coefficient of row s, source q).  Returns false for words
// past the chunk's return (never executed, not written).  k_jit_emit runs it
// one word per thread; rsgpu_internal_jit_emit, for the CPU suite, too.
RJ_HD inline bool code_word(const uint8_t* rows, int k, int nslot, int ch, int o, uint64_t* word)
{
    const int nt = k - 8 * ch < 8 ? k - 8 * ch : 8;
    const int per_src = PRE_BYTES / 8 + 8 * nslot;
    if (o < 2) {  // prologue: source 0's planes into bank A
        *word = enc_ds_read_b128(plane_reg(0, 4 * o), 20, o * LDS_HALF);
    } else if (o < 2 + nt * per_src) {
        const int t = (o - 2) / per_src, r = o - 2 - t * per_src;
        if (r < PRE_BYTES / 8) {
            *word = (uint64_t)pre_u32(t, nt, 2 * r + 1) << 32 | pre_u32(t, nt, 2 * r);
        } else {
            const int m = r - PRE_BYTES / 8, s = m >> 3, pl = m & 7;
            uint64_t wd[8];
            mac_words(rows[s * k + 8 * ch + t], s, t & 1, wd);
            *word = wd[pl];
        }
    } else if (o == 2 + nt * per_src) {
        *word = (uint64_t)S_NOP0 << 32 | S_SETPC_82;
    } else {
        return false;
    }
    return true;
}

// ---- R rows per wave (k_rs_jitw<R>) ---------------------------------------
//
// Two waves per column tile, R output rows each, so the composites of a
// source are built once per R rows instead of once per 8:
//   R = 16 (k_rs_jit16, 24 < e <= 32): 128 accumulators, 168 VGPRs, 3 waves
//          per SIMD, chunks of 6 sources (6 workgroups per CU); 10 % fewer
//          VALU instructions, 40 % fewer instruction-cache misses than 4 x 8
//   R = 12 (k_rs_jit12, 20 < e <= 24): 96 accumulators, 136 VGPRs, 3 waves
//          per SIMD, chunks of 6 sources; composites twice per source and
//          tile instead of three times (8 + 8 + 8 rows)
//   R = 10 (k_rs_jit10, 16 < e <= 20): 80 accumulators, 120 VGPRs, 4 waves
//          per SIMD, chunks of 5 sources (8 workgroups per CU); composites
//          twice per source and tile instead of three times (8 + 8 + 4 rows)
// Four waves per column tile for 32 < e <= 64 (R = 10 / 12 / 16 for e up to
// 40 / 48 / 64), so a tile's sources are loaded and transposed once for all
// e rows (the 8-row layout runs passes of 32 rows, each reading every source).
// Wave w of NV = wide_waves(e) holds rows wide_row0(e, w) .. wide_row0(e, w + 1)
// - 1 (balanced: at most one row apart).
// Register contract (all):
//   v9             LDS byte address of the chunk's first source + 16 lane
//   v10..v17       planes of the current source: L1 L2 L4 L8 H1 H2 H4 H8
//   v18..v28       composites L[n], n = 3 5 6 7 9 ... 15; v29..v39 H[n]
//   v40..v40+8R-1  accumulators: slot s (row wide_row0(e, w) + s) plane b at v40+8s+b
//   s[82:83]       return address
// Code of one chunk (nt <= CS sources, nslot <= R rows of the wave):
//   source t   ds_read_b128 x2 of its own planes, s_waitcnt lgkmcnt(0), the
//              22 composites (v_xor_b32), s_nop, then per slot 8
//              multiply-accumulates (as mac_words)          112 + 64 nslot B
//   epilogue   s_setpc_b64 s[82:83]; s_nop                           8 B
// No next-source prefetch (no register bank for it): the other waves of the
// SIMD cover the LDS latency.
RJ_HD constexpr int wide_waves(int e) { return e > 32 ? 4 : 2; }
RJ_HD constexpr int wide_row0(int e, int w) { return w * e / wide_waves(e); }
// e > 64 (k + e <= 250 allows e up to 125): passes of at most 64 rows, split
// evenly (e = 100 as 50 + 50, e = 65 as 32 + 33), each pass one launch in the
// layout of its own row count; pass p holds rows wide_pass_row0(e, p) ..
// wide_pass_row0(e, p + 1) - 1.  A block's code is its passes' code in order.
RJ_HD constexpr int wide_passes(int e) { return e > 64 ? (e + 63) / 64 : 1; }
RJ_HD constexpr int wide_pass_row0(int e, int p) { return p * e / wide_passes(e); }
RJ_HD constexpr int wide_pass_rows(int e, int p) { return wide_pass_row0(e, p + 1) - wide_pass_row0(e, p); }

template <int R_, int CS_>
struct Wide {
    static constexpr int R = R_, CS = CS_;
    static constexpr int ADDR = 9, PL = 10, CL = 18, ACC = 40;
    // bytes per source before the multiply-accumulates (kernel_hooks.h: 112
    // in the product)
    static constexpr int PRE = 112 + Hooks::kPreExtra;
    RJ_HD static constexpr int src_bytes(int nslot) { return PRE + 64 * nslot; }
    RJ_HD static constexpr int chunk_stride() { return (CS * src_bytes(R) + 8 + 63) / 64 * 64; }

    RJ_HD static constexpr int treg(int hi, int n)
    {
        if ((n & (n - 1)) == 0) {
            const int a = n == 1 ? 0 : n == 2 ? 1 : n == 4 ? 2 : 3;
            return PL + 4 * hi + a;
        }
        const int below = 1 + (n > 2) + (n > 4) + (n > 8);
        return CL + 11 * hi + (n - below - 1);
    }

    // the multiply-accumulate word for mask m with the accumulator fields
    // zero: acc ^= L[m & 15] ^ H[m >> 4] (v_bitop3_b32 0x96, or v_xor_b32 in
    // the VOP3 form when one nibble is 0; an s_nop pair for m = 0).  The
    // accumulator is both the destination (low byte of the first dword) and
    // src0 (256 + acc, low 9 bits of the second), so for acc < 256 the word of
    // accumulator acc is this base OR (acc << 32 | acc).
    RJ_HD static constexpr uint64_t mac_base(uint8_t m)
    {
        const int lo = m & 15, hi = m >> 4, l = Hooks::mac_lo(lo), h = Hooks::mac_hi(hi);
        return lo && hi ? enc_bitop3_96(0, 0, treg(0, l), treg(1, h))
               : lo     ? enc_xor_e64(0, 0, treg(0, l))
               : hi     ? enc_xor_e64(0, 0, treg(1, h))
                        : NOP2;
    }
    RJ_HD static constexpr uint64_t with_acc(uint64_t base, int acc)
    {
        return base == NOP2 ? NOP2 : base | ((uint64_t)acc << 32 | (uint64_t)acc);
    }

    // the multiply-accumulate word of output plane b of slot s, for row b
    // (mask m = mat_row(c, b)) of the coefficient's matrix
    RJ_HD static constexpr uint64_t mac_word(uint8_t m, int s, int b) { return with_acc(mac_base(m), ACC + 8 * s + b); }

    RJ_HD static void mac_words(uint8_t c, int s, uint64_t (&wd)[8])
    {
        for (int b = 0; b < 8; ++b)
            wd[b] = mac_word(mat_row(c, b), s, b);
    }

    // 32-bit word i (< PRE / 4 = 28) of source t's preamble
    RJ_HD static constexpr uint32_t pre_u32(int t, int i)
    {
        if (uint32_t w = 0; Hooks::pre_word(t, i, PL, CL, ADDR, &w))
            return w;
        i = Hooks::pre_index(i);
        if (i < 4) {
            const uint64_t d = enc_ds_read_b128(i < 2 ? PL : PL + 4, ADDR, t * LDS_SRC + (i < 2 ? 0 : LDS_HALF));
            return (i & 1) ? (uint32_t)(d >> 32) : (uint32_t)d;
        }
        if (i == 4)
            return enc_waitcnt_lgkm(0);
        const int j = i - 5;
        if (j >= 22)
            return S_NOP0;
        const int hi = j / 11, c = j - 11 * hi;
        const int n = c < 1 ? 3 : c < 4 ? 4 + c : 5 + c;
        const int low = n & -n;
        return enc_xor_e32(treg(hi, n), treg(hi, n ^ low), treg(hi, low));
    }

    // Word o (8 bytes) of chunk ch of a wave's code, rows[s * k + q] as in
    // jit::code_word; false past the chunk's return.
    RJ_HD static bool code_word(const uint8_t* rows, int k, int nslot, int ch, int o, uint64_t* word)
    {
        const int nt = k - CS * ch < CS ? k - CS * ch : CS;
        const int per_src = PRE / 8 + 8 * nslot;
        if (o < nt * per_src) {
            const int t = o / per_src, r = o - t * per_src;
            if (r < PRE / 8) {
                *word = (uint64_t)pre_u32(t, 2 * r + 1) << 32 | pre_u32(t, 2 * r);
            } else {
                const int m = r - PRE / 8, s = m >> 3;
                uint64_t wd[8];
                mac_words(rows[s * k + CS * ch + t], s, wd);
                *word = wd[m & 7];
            }
        } else if (o == nt * per_src) {
            *word = (uint64_t)S_NOP0 << 32 | S_SETPC_82;
        } else {
            return false;
        }
        return true;
    }
};
using J16 = Wide<16, 6>;
using J12 = Wide<12, 6>;
using J10 = Wide<10, 5>;

// Word tables of the device emitter k_jitw_emit (the register contract, and
// so every table, is the same for all R): the base word (mac_base) of
// coefficient c for output plane b at [8 c + b], and the 14 preamble words
// of chunk position t at [14 t + i / 2] (i = 0 .. 27 as pre_u32).
struct WideTables {
    static constexpr int PW = Wide<16, 6>::PRE / 8;  // preamble words per source (14)
    uint64_t mac[256 * 8];
    uint64_t pre[6 * PW];
};
RJ_HD constexpr WideTables wide_tables()
{
    WideTables w{};
    for (int c = 0; c < 256; ++c)
        for (int b = 0; b < 8; ++b)
            w.mac[8 * c + b] = J16::mac_base(mat_row((uint8_t)c, b));
    for (int t = 0; t < 6; ++t)
        for (int r = 0; r < WideTables::PW; ++r)
            w.pre[WideTables::PW * t + r] = (uint64_t)J16::pre_u32(t, 2 * r + 1) << 32 | J16::pre_u32(t, 2 * r);
    return w;
}

}  // namespace jit
}  // namespace rsgpu
