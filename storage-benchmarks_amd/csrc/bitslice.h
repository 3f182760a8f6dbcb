// bitslice.h -- device helpers shared by the bit-sliced kernels
// (rs_bitsliced.hip: compile-time coefficients; rs_tc.hip: runtime
// coefficients through threaded-code handlers).  A lane holds 32 consecutive
// bytes of a row; tr8 turns its 8 dwords into 8 bit-planes and back.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsgpu {
namespace bs {

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Opaque VGPR copy of a constant: keeps masks out of SGPR operands (an SGPR
// operand makes v_bitop3 a 4-cycle issue, profiles/r1_ubench_valu.log).
__device__ __forceinline__ uint32_t vconst(uint32_t c)
{
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "i"(c));
    return v;
}

// Two (lo, hi) block swaps of the SWAR 8x8 bit transpose at once, per byte
// lane:  lo' = (lo & m) | ((hi << s) & ~m),  hi' = ((lo >> s) & m) | (hi & ~m)
// for (lo0, hi0) and (lo1, hi1).  The two lo are shifted as ONE 64-bit value
// (lo1:lo0) >> s, the two hi as (hi1:hi0) << s: the s bits that cross the
// dword boundary land at the top of lo0 >> s / the bottom of hi1 << s, where
// m (0x0F0F0F0F, 0x33333333, 0x55555555 for s = 4, 2, 1) selects the other
// operand, so they never reach a result.  12 shifts per tr8 instead of 24
// (hipcc splits a C++ 64-bit shift whose halves are used separately into
// v_alignbit + v_lshrrev, hence the asm; it pairs the operands in aligned
// VGPR pairs without a move, tools/tr8_codegen: 24 v_bitop3 + 12 64-bit shifts).
// bitop3 truth table (src0=0xF0, src1=0xCC, src2=0xAA):
//   f(a, b, m) = (a & m) | (b & ~m)  -> (0xF0 & 0xAA) | (0xCC & 0x55) = 0xE4
template <int S>
__device__ __forceinline__ void swap_blk2(uint32_t& lo0, uint32_t& lo1, uint32_t& hi0, uint32_t& hi1, uint32_t m)
{
    uint64_t l, h;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(l) : "i"(S), "v"((uint64_t)lo1 << 32 | lo0));
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(h) : "i"(S), "v"((uint64_t)hi1 << 32 | hi0));
    const uint32_t nl0 = __builtin_amdgcn_bitop3_b32(lo0, (uint32_t)h, m, 0xE4);
    const uint32_t nl1 = __builtin_amdgcn_bitop3_b32(lo1, (uint32_t)(h >> 32), m, 0xE4);
    const uint32_t nh0 = __builtin_amdgcn_bitop3_b32((uint32_t)l, hi0, m, 0xE4);
    const uint32_t nh1 = __builtin_amdgcn_bitop3_b32((uint32_t)(l >> 32), hi1, m, 0xE4);
    lo0 = nl0;
    lo1 = nl1;
    hi0 = nh0;
    hi1 = nh1;
}

// In place: W[w] byte q = byte (4w+q) of a 32-byte segment  <->  plane
// layout W[a] byte q bit w = bit a of that byte.  Self-inverse.  Block swaps
// (0,4)(1,5)(2,6)(3,7) by 4 bits, (0,2)(1,3)(4,6)(5,7) by 2, (0,1)(2,3)(4,5)(6,7)
// by 1, grouped in pairs whose lo (and hi) halves are shifted together.
__device__ __forceinline__ void tr8(uint32_t (&W)[8], uint32_t m4, uint32_t m2, uint32_t m1)
{
    swap_blk2<4>(W[0], W[1], W[4], W[5], m4);
    swap_blk2<4>(W[2], W[3], W[6], W[7], m4);
    swap_blk2<2>(W[0], W[1], W[2], W[3], m2);
    swap_blk2<2>(W[4], W[5], W[6], W[7], m2);
    swap_blk2<1>(W[0], W[2], W[1], W[3], m1);
    swap_blk2<1>(W[4], W[6], W[5], W[7], m1);
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4u gcv4u;
typedef __attribute__((address_space(1))) v4u gv4u;

__device__ __forceinline__ void load32(const uint8_t* row, long long off, bool ok, uint32_t (&W)[8])
{
    if (ok) {
        const v4u a = *(gcv4u*)(row + off);
        const v4u b = *(gcv4u*)(row + off + 16);
        W[0] = a.x; W[1] = a.y; W[2] = a.z; W[3] = a.w;
        W[4] = b.x; W[5] = b.y; W[6] = b.z; W[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            W[i] = 0;
    }
}

__device__ __forceinline__ void store32(uint8_t* row, long long off, const uint32_t (&W)[8])
{
    v4u a, b;
    a.x = W[0]; a.y = W[1]; a.z = W[2]; a.w = W[3];
    b.x = W[4]; b.y = W[5]; b.z = W[6]; b.w = W[7];
    // non-temporal (`nt`): the rows are written once and not read back by
    // this launch.  Same box, three interleaved passes (profiles/r04_nt/):
    // C4 1262-1264 vs 1242-1246 GiB/s (generated decode 3.26 vs 3.35 ms per
    // 4096 blocks), C5 740-741 vs 734-736, C3 1323-1326 vs 1315-1325; nt on
    // the LDS-DMA source loads as well: C3 -1.6 % (the encode 22.7 vs 22.3 ms)
    __builtin_nontemporal_store(a, (gv4u*)(row + off));
    __builtin_nontemporal_store(b, (gv4u*)(row + off + 16));
}

// 16 bytes per lane global -> LDS (LDS-DMA, no VGPR destination): lane i's
// bytes land at lds_byte + 16 i.  M0 holds the LDS base and is restored.
__device__ __forceinline__ void glds16(const void* g, uint32_t lds_byte)
{
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n"
        "s_mov_b32 m0, %2\n"
        "s_nop 0\n"
        "global_load_lds_dwordx4 %1, off\n"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_byte))
        : "memory");
}

// 32 bytes per lane of the wave-uniform row `row` at per-lane byte offset
// `voff` -> LDS (two LDS-DMA pieces: bytes 0-15 of every lane at lds_lo +
// 16 lane, bytes 16-31 at lds_lo + 1024 + 16 lane).  SGPR base + VGPR
// offset addressing: no per-lane 64-bit address arithmetic per piece, one
// M0 save/restore for both pieces.  (The instruction offset field would be
// added to the LDS address as well, so the second piece gets its own base.)
__device__ __forceinline__ void glds32(const uint8_t* row, uint32_t voff, uint32_t lds_lo)
{
    const uint64_t r = (uint64_t)row;
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(r >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r);
    const uint64_t base16 = base + 16;
    const uint32_t lo = __builtin_amdgcn_readfirstlane(lds_lo);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n"
        "s_mov_b32 m0, %4\n"
        "s_nop 0\n"
        "global_load_lds_dwordx4 %1, %2\n"
        "s_add_u32 m0, %4, 0x400\n"
        "s_nop 0\n"
        "global_load_lds_dwordx4 %1, %3\n"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(base), "s"(base16), "s"(lo)
        : "memory", "scc");
}

// glds32 with the non-temporal policy: streamed sources that should not
// displace other lines (the generated decode's code) from the XCD's L2
__device__ __forceinline__ void glds32_nt(const uint8_t* row, uint32_t voff, uint32_t lds_lo)
{
    const uint64_t r = (uint64_t)row;
    const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(r >> 32)) << 32) |
                          (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r);
    const uint64_t base16 = base + 16;
    const uint32_t lo = __builtin_amdgcn_readfirstlane(lds_lo);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n"
        "s_mov_b32 m0, %4\n"
        "s_nop 0\n"
        "global_load_lds_dwordx4 %1, %2 nt\n"
        "s_add_u32 m0, %4, 0x400\n"
        "s_nop 0\n"
        "global_load_lds_dwordx4 %1, %3 nt\n"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(base), "s"(base16), "s"(lo)
        : "memory", "scc");
}

// Wave-uniform pointer from a table through the scalar cache.  (hipcc would
// use a vector load for it -- it cannot prove the table is not written -- and
// its vmcnt(0) would drain the LDS-DMA in flight.)
__device__ __forceinline__ const uint8_t* sload_ptr(const uint8_t* const* p)
{
    const uint8_t* r;
    asm volatile("s_load_dwordx2 %0, %1, 0\n s_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
    return r;
}

// wait until at most N of this wave's vector-memory operations are pending
__device__ __forceinline__ void wait_vm(int n)
{
    switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

// workgroup barrier that does not drain the LDS-DMA in flight
__device__ __forceinline__ void barrier_lds()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n s_barrier" ::: "memory");
}

}  // namespace bs
}  // namespace rsgpu
