// rs_decode_fused.hip -- one-pass syndrome decode for the gf_gen_rs_matrix
// codes: recovered data rows from the surviving data rows and the parity rows
// of each block, with HBM traffic (k + e) * L per block (read k, write e)
// plus the parked syndromes of the waves beyond the LDS hand-off.
//
// Status: the default decode is the one-matrix k_rs_tc (rsgpu_capi.cpp
// decode_mode); this kernel is the default for (k 100, e 20), where it
// measured 3 % faster, and RSGPU_DECODE=fused selects it elsewhere.  Its
// phase 1 runs on threaded code by default (TC1 below); the compile-time
// Horner form described next is kept behind RSGPU_FUSED_SYN=horner.
//
// The two-kernel decode (k_rs_bs<SYN> writes the e syndrome rows to HBM,
// k_rs_tc reads them back and overwrites them with the data) moves 2 e L
// more bytes.  Here one workgroup does both for its 2 KB column tile:
//
//   phase 1  s = P ^ V_kept d_kept        compile-time coefficients 2^(r j)
//            (the k_rs_bs syndrome: sources streamed by LDS-DMA, bit-
//            transposed in LDS, Horner over chunks of C sources).  The
//            parity rows are loaded into the accumulators first, scaled by
//            2^(-C r (NCH-1)) so the Horner twiddles return them to P_r: their
//            load overlaps the first LDS-DMA part instead of ending the phase.
//            The e syndrome rows are stored to this tile of the output rows in
//            bit-plane form (they stay L2/MALL resident)
//   phase 2  x = V_E^-1 s                 runtime coefficients, threaded code
//            (k_rs_tc's chunk asm over the e syndrome rows read back by
//            LDS-DMA -- already planes, so no input transposes), then the
//            rows are transposed to bytes and overwrite the syndromes.
//
// Both phases keep the accumulators in asm-owned v64..v127 (the compiler is
// capped at v0..v63, amdgpu_num_vgpr(64)): phase 1's compile-time MAC blocks
// are generated asm too (gen_tc_handlers.py -> build/syn_blocks.inc).
// Wave w owns rows 8w..8w+7; NW = ceil(e / 8) waves per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <cstring>
#include <utility>

#include "bitslice.h"
#include "rs_kernels.h"
#include "tc_handlers.inc"

namespace rsgpu {
namespace fused {

template <int K, int E, int G, int T>
struct SynBlock;
template <int K, int E, int C, int G>
struct SynTwiddle;
template <int K, int E, int C, int G>
struct SynPreScale;
template <int S>
struct XorSlot;
#include "syn_blocks.inc"

using bs::barrier_lds;
using bs::glds32;
using bs::store32;
using bs::tr8;
using bs::vconst;
using bs::wait_vm;

constexpr int S = 8;  // sources per LDS part (two parts double-buffer the stream)

// Phase accounting for tools/fused_profile.hip (-DRSGPU_FUSED_PROF only):
// per-wave s_memtime sums per phase, sampled WGs, added into
// rsgpu_fused_prof[phase] at the end of the wave.
#ifdef RSGPU_FUSED_PROF
__device__ unsigned long long rsgpu_fused_prof[16];
#define FP_DECL unsigned long long fp_sum[16] = {}, fp_t = __builtin_amdgcn_s_memtime(), fp_start = fp_t;
#define FP_MARK(P)                                                      \
    do {                                                                \
        const unsigned long long fp_n = __builtin_amdgcn_s_memtime();   \
        fp_sum[P] += fp_n - fp_t;                                       \
        fp_t = fp_n;                                                    \
    } while (0)
#define FP_END                                                                  \
    do {                                                                        \
        fp_sum[15] = __builtin_amdgcn_s_memtime() - fp_start;                   \
        if (lane == 0 && (blockIdx.x & 63) == 0)                                \
            for (int i = 0; i < 16; ++i)                                        \
                atomicAdd(&rsgpu_fused_prof[i], fp_sum[i]);                     \
    } while (0)
#else
#define FP_DECL
#define FP_MARK(P) \
    do {           \
    } while (0)
#define FP_END \
    do {       \
    } while (0)
#endif
static_assert(S == RSGPU_TC_C, "phase 2 chunk asm reads parts of RSGPU_TC_C sources");

struct Args {
    const uint8_t* src;                // [B][K] rows
    const uint8_t* par;                // [B][E] rows
    uint8_t* out;                      // [B][E] rows (syndromes, then the data)
    long long pitch, len;
    const uint64_t* emask;             // [B][2] erased originals
    const unsigned long long* addr;    // [B][E][8 NW] handler addresses of V_E^-1
    const unsigned long long* syn_addr;  // [B][K-E][8 NW] handlers of 2^(r j), survivors j
    const int* status;                 // [B]
};

__device__ __forceinline__ uint64_t uniform64(uint64_t x)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Read accumulator slot SL (asm-owned v[64+8SL .. 64+8SL+7]) into W.
template <int SL>
__device__ __forceinline__ void read_slot(uint32_t (&W)[8])
{
#define RSGPU_RD(TEXT)                                                                          \
    asm volatile(TEXT : "=v"(W[0]), "=v"(W[1]), "=v"(W[2]), "=v"(W[3]), "=v"(W[4]), "=v"(W[5]), \
                        "=v"(W[6]), "=v"(W[7]))
    if constexpr (SL == 0) RSGPU_RD(RSGPU_TC_READ_SLOT0);
    if constexpr (SL == 1) RSGPU_RD(RSGPU_TC_READ_SLOT1);
    if constexpr (SL == 2) RSGPU_RD(RSGPU_TC_READ_SLOT2);
    if constexpr (SL == 3) RSGPU_RD(RSGPU_TC_READ_SLOT3);
    if constexpr (SL == 4) RSGPU_RD(RSGPU_TC_READ_SLOT4);
    if constexpr (SL == 5) RSGPU_RD(RSGPU_TC_READ_SLOT5);
    if constexpr (SL == 6) RSGPU_RD(RSGPU_TC_READ_SLOT6);
    if constexpr (SL == 7) RSGPU_RD(RSGPU_TC_READ_SLOT7);
#undef RSGPU_RD
}

// Write W into accumulator slot SL.
template <int SL>
__device__ __forceinline__ void write_slot(const uint32_t (&W)[8])
{
#define RSGPU_WR(TEXT)                                                                          \
    asm volatile(TEXT ::"v"(W[0]), "v"(W[1]), "v"(W[2]), "v"(W[3]), "v"(W[4]), "v"(W[5]), \
                 "v"(W[6]), "v"(W[7]))
    if constexpr (SL == 0) RSGPU_WR(RSGPU_TC_WRITE_SLOT0);
    if constexpr (SL == 1) RSGPU_WR(RSGPU_TC_WRITE_SLOT1);
    if constexpr (SL == 2) RSGPU_WR(RSGPU_TC_WRITE_SLOT2);
    if constexpr (SL == 3) RSGPU_WR(RSGPU_TC_WRITE_SLOT3);
    if constexpr (SL == 4) RSGPU_WR(RSGPU_TC_WRITE_SLOT4);
    if constexpr (SL == 5) RSGPU_WR(RSGPU_TC_WRITE_SLOT5);
    if constexpr (SL == 6) RSGPU_WR(RSGPU_TC_WRITE_SLOT6);
    if constexpr (SL == 7) RSGPU_WR(RSGPU_TC_WRITE_SLOT7);
#undef RSGPU_WR
}

// Start loading 32 bytes per lane of `row` into accumulator slot SL (two
// global_load_dwordx4, counted in vmcnt; the caller waits before reading it).
template <int SL>
__device__ __forceinline__ void load_slot(const uint8_t* row)
{
#define RSGPU_LD(TEXT) asm volatile(TEXT ::"v"(row) : "memory")
    if constexpr (SL == 0) RSGPU_LD(RSGPU_TC_LOAD_SLOT0);
    if constexpr (SL == 1) RSGPU_LD(RSGPU_TC_LOAD_SLOT1);
    if constexpr (SL == 2) RSGPU_LD(RSGPU_TC_LOAD_SLOT2);
    if constexpr (SL == 3) RSGPU_LD(RSGPU_TC_LOAD_SLOT3);
    if constexpr (SL == 4) RSGPU_LD(RSGPU_TC_LOAD_SLOT4);
    if constexpr (SL == 5) RSGPU_LD(RSGPU_TC_LOAD_SLOT5);
    if constexpr (SL == 6) RSGPU_LD(RSGPU_TC_LOAD_SLOT6);
    if constexpr (SL == 7) RSGPU_LD(RSGPU_TC_LOAD_SLOT7);
#undef RSGPU_LD
}

// SynBlock<K, E, g, T> for the runtime (wave-uniform) wave group g
template <int K, int E, int T, int NW>
__device__ __forceinline__ void syn_block(int g, const uint32_t (&P)[8])
{
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((g == Gs ? SynBlock<K, E, Gs, T>::run(P) : void()), ...);
    }(std::make_integer_sequence<int, NW>{});
}

template <int K, int E, int C, int NW>
__device__ __forceinline__ void syn_twiddle(int g)
{
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((g == Gs ? SynTwiddle<K, E, C, Gs>::run() : void()), ...);
    }(std::make_integer_sequence<int, NW>{});
}

template <int K, int E, int C, int NW>
__device__ __forceinline__ void syn_prescale(int g)
{
    [&]<int... Gs>(std::integer_sequence<int, Gs...>) {
        ((g == Gs ? SynPreScale<K, E, C, Gs>::run() : void()), ...);
    }(std::make_integer_sequence<int, NW>{});
}

template <int K, int C, int E, int NW, int PART>
__device__ __forceinline__ void syn_part(int G, const uint4* buf, int lane, int j0, uint64_t em0,
                                         uint64_t em1)
{
    [&]<int... Ts>(std::integer_sequence<int, Ts...>) {
        (
            [&] {
                constexpr int T = PART * S + Ts;
                if constexpr (T < C) {
                    const int j = j0 + Ts;
                    const bool live = j < K && !(((j < 64 ? em0 >> j : em1 >> (j - 64)) & 1));
                    if (live) {
                        const uint4 u = buf[(Ts * 2 + 0) * 64 + lane];
                        const uint4 v = buf[(Ts * 2 + 1) * 64 + lane];
                        const uint32_t P[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                        syn_block<K, E, T, NW>(G, P);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, S>{});
}

// One LDS part of nt sources through the threaded-code chunk asm
// (gen_tc_handlers.py): la = part base + 16 lane, pa = this wave's handler
// addresses of the part's first source (NW * 8 per source).
template <int NW>
__device__ __forceinline__ void tc_chunk(uint32_t la, const unsigned long long* pa, int nt)
{
#define RSGPU_TC_RUN(N)                                                                          \
    asm volatile(RSGPU_TC_CHUNK##N                                                               \
                 :                                                                               \
                 : [la] "v"(la), [pa] "s"(pa), [o1] "i"(1 * NW * 64), [o2] "i"(2 * NW * 64),      \
                   [o3] "i"(3 * NW * 64), [o4] "i"(4 * NW * 64), [o5] "i"(5 * NW * 64),           \
                   [o6] "i"(6 * NW * 64), [o7] "i"(7 * NW * 64)                                  \
                 : RSGPU_TC_CLOBBERS, RSGPU_TC_ACC_CLOBBERS, "memory")
    switch (nt) {
    case 1: RSGPU_TC_RUN(1); break;
    case 2: RSGPU_TC_RUN(2); break;
    case 3: RSGPU_TC_RUN(3); break;
    case 4: RSGPU_TC_RUN(4); break;
    case 5: RSGPU_TC_RUN(5); break;
    case 6: RSGPU_TC_RUN(6); break;
    case 7: RSGPU_TC_RUN(7); break;
    default: RSGPU_TC_RUN(8); break;
    }
#undef RSGPU_TC_RUN
}

// The scaffolding is shared by every wave group (G runtime, wave-uniform):
// only the generated MAC / twiddle blocks differ per group, which keeps the
// executed code of all groups plus the 256 handlers inside the I-cache.
template <int K, int E, int C, int NW, bool TC1>
__device__ __forceinline__ void run_group(const Args& a, uint4 (*lds)[S * 2 * 64], uint8_t* items,
                                          int G)
{
    constexpr int NCH = (K + C - 1) / C;
    constexpr int NP = (C + S - 1) / S;
    constexpr int NSTEP = NCH * NP;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const bool inb = off + 32 <= a.len;
    const long long loff = inb ? off : 0;  // out-of-range lanes re-read the row head
    const uint8_t* sb = a.src + (size_t)b * K * a.pitch;
    uint8_t* ob = a.out + (size_t)b * E * a.pitch;
    const uint64_t em0 = uniform64(a.emask[2 * b]), em1 = uniform64(a.emask[2 * b + 1]);
    auto live = [&](int j) { return j < K && !(((j < 64 ? em0 >> j : em1 >> (j - 64)) & 1)); };
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];

    // ---------------- phase 1: syndromes ----------------
    FP_DECL
    if constexpr (TC1) {
        // Threaded code (the phase-2 machinery): the K-E survivors in
        // ascending order, S per LDS part, each wave moving and transposing
        // slots t = G, G+NW, ...; coefficient 2^(r j) of survivor j for
        // syndrome row r comes as a handler address from the prepare
        // kernel's table.  No Horner chunks, so no twiddles and the parity
        // rows enter the accumulators unscaled.
        constexpr int NL = K - E;
        constexpr int NSTEP = (NL + S - 1) / S;
        static_assert(K <= 128, "survivor list: one byte per survivor, two lanes' words");
        uint32_t vi0 = 0, vi1 = 0;  // lane q: survivor q (q < 64) / 64 + q
        {
            auto range = [](int lo, int hi) -> uint64_t {  // bits [lo, hi) of one word
                lo = max(lo, 0);
                hi = min(hi, 64);
                if (hi <= lo)
                    return 0;
                const uint64_t below_hi = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
                return below_hi & ~((1ull << lo) - 1);
            };
            const uint64_t lv0 = ~em0 & range(0, K), lv1 = ~em1 & range(0, K - 64);
            for (int j = lane; j < K; j += 64)
                if (live(j))
                    items[__popcll(lv0 & range(0, j)) + __popcll(lv1 & range(-64, j - 64))] = (uint8_t)j;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own lanes' writes, in order
            vi0 = lane < NL ? items[lane] : 0;
            if constexpr (NL > 64)
                vi1 = 64 + lane < NL ? items[64 + lane] : 0;
        }
        auto survivor = [&](int q) -> int {
            if constexpr (NL > 64)
                return __builtin_amdgcn_readlane((int)(q < 64 ? vi0 : vi1), q & 63);
            return __builtin_amdgcn_readlane((int)vi0, q);
        };
        auto part_n = [&](int n) { return min(S, NL - n * S); };
        auto issue1 = [&](int n) {
            const uint32_t base = lds0 + (uint32_t)((n & 1) * S * 2 * 64 * 16);
            for (int t = G; t < part_n(n); t += NW)
                glds32(sb + (size_t)survivor(n * S + t) * a.pitch, (uint32_t)loff,
                       base + (uint32_t)(t * 2 * 64 * 16));
        };
        auto own1 = [&](int n) {
            const int nt = part_n(n);
            return nt > G ? 2 * ((nt - G + NW - 1) / NW) : 0;
        };
        asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
        // parity rows straight into this wave's accumulators (unscaled)
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            ((G * 8 + Ss < E ? load_slot<Ss>(a.par + ((size_t)b * E + G * 8 + Ss) * a.pitch + loff)
                             : void()),
             ...);
        }(std::make_integer_sequence<int, 8>{});
        issue1(0);
        if (NSTEP > 1)
            issue1(1);
        wait_vm(own1(0) + (NSTEP > 1 ? own1(1) : 0));  // the (older) parity loads have landed
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            (
                [&] {
                    if (G * 8 + Ss < E) {
                        uint32_t W[8];
                        read_slot<Ss>(W);
                        tr8(W, m4, m2, m1);
                        write_slot<Ss>(W);
                    }
                }(),
                ...);
        }(std::make_integer_sequence<int, 8>{});
        FP_MARK(12);
        const unsigned long long* sp = a.syn_addr + (size_t)b * NL * (NW * 8) + G * 8;
        for (int n = 0; n < NSTEP; ++n) {
            const int nt = part_n(n);
            FP_MARK(5);
            if (n == 0) {
                FP_MARK(0);
                wait_vm(NSTEP > 1 ? own1(1) : 0);
            } else if (n + 1 < NSTEP) {
                issue1(n + 1);
                FP_MARK(0);
                wait_vm(own1(n + 1));
            } else {
                wait_vm(0);
            }
            FP_MARK(1);
            uint4* buf = lds[n & 1];
            for (int t = G; t < nt; t += NW) {
                uint4 u = buf[(t * 2 + 0) * 64 + lane];
                uint4 v = buf[(t * 2 + 1) * 64 + lane];
                uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                tr8(W, m4, m2, m1);
                buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
                buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
            }
            FP_MARK(2);
            barrier_lds();
            FP_MARK(3);
            tc_chunk<NW>(lds0 + (uint32_t)((n & 1) * S * 2 * 64 * 16) + lane * 16,
                         sp + (size_t)(n * S) * (NW * 8), nt);
            FP_MARK(4);
            barrier_lds();  // buffer n & 1 is refilled by part n + 2
        }
        FP_MARK(5);
    } else {
    auto first_src = [&](int n) { return (NCH - 1 - n / NP) * C + (n % NP) * S; };
    auto part_len = [&](int n) { return min(S, C - (n % NP) * S); };
    // The live sources of step n are dealt round-robin over the waves by
    // rank (starting at wave n % NW), so every wave moves and transposes
    // the same number of rows, +-1, whatever the erasure pattern.
    auto live_bits = [&](int n) -> uint32_t {  // bit t: slot t of step n is a live source
        const int j0 = first_src(n);
        const int nt = min(part_len(n), K - j0);  // slots past K hold nothing
        const uint64_t er = j0 == 0 ? em0 : j0 < 64 ? (em0 >> j0) | (em1 << (64 - j0)) : em1 >> (j0 - 64);
        return ~(uint32_t)er & ((1u << nt) - 1);  // nt <= S = 8
    };
    auto dealt = [&](int n, uint32_t m) -> uint32_t {  // this wave's slots of step n
        uint32_t mine = 0;
        for (int rk = n % NW; m; m &= m - 1, rk = rk + 1 == NW ? 0 : rk + 1)
            mine |= rk == G ? m & (0u - m) : 0u;
        return mine;
    };
    auto issue1 = [&](int n, uint32_t mine) {
        const int j0 = first_src(n);
        const uint32_t base = lds0 + (uint32_t)((n & 1) * S * 2 * 64 * 16);
        for (; mine; mine &= mine - 1) {
            const int t = __builtin_ctz(mine);
            glds32(sb + (size_t)(j0 + t) * a.pitch, (uint32_t)loff, base + (uint32_t)(t * 2 * 64 * 16));
        }
    };
    auto issued1 = [&](uint32_t mine) { return 2 * __builtin_popcount(mine); };

    // Parity rows straight into this wave's accumulators; their latency
    // overlaps the first two LDS-DMA parts.  (Streaming one parity row per
    // step instead, scaled for the twiddles still to come, removed this
    // prologue but measured 1-2 % slower overall.)
    asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        ((G * 8 + Ss < E ? load_slot<Ss>(a.par + ((size_t)b * E + G * 8 + Ss) * a.pitch + loff)
                         : void()),
         ...);
    }(std::make_integer_sequence<int, 8>{});
    uint32_t mine_next = dealt(0, live_bits(0));
    issue1(0, mine_next);
    // buffer 1 is free from the start: part 1 flies during the parity work
    const uint32_t mine1 = NSTEP > 1 ? dealt(1, live_bits(1)) : 0u;
    if (NSTEP > 1)
        issue1(1, mine1);
    wait_vm(issued1(mine_next) + issued1(mine1));  // the (older) parity loads have landed
    // bytes -> planes, scaled by 2^(-C r (NCH-1)): the NCH-1 Horner twiddles
    // of the chunk loop bring them back to P_r
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        (
            [&] {
                if (G * 8 + Ss < E) {
                    uint32_t W[8];
                    read_slot<Ss>(W);
                    tr8(W, m4, m2, m1);
                    write_slot<Ss>(W);
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, 8>{});
    syn_prescale<K, E, C, NW>(G);
    FP_MARK(12);
    for (int n = 0; n < NSTEP; ++n) {
        uint4* buf = lds[n & 1];
        const int j0 = first_src(n);
        const uint32_t mine = mine_next;
        FP_MARK(5);
        if (n == 0 && NSTEP > 1) {  // part 1 already issued in the prologue
            mine_next = mine1;
            FP_MARK(0);
            wait_vm(issued1(mine_next));
        } else if (n + 1 < NSTEP) {
            mine_next = dealt(n + 1, live_bits(n + 1));
            issue1(n + 1, mine_next);
            FP_MARK(0);
            wait_vm(issued1(mine_next));
        } else {
            wait_vm(0);
        }
        FP_MARK(1);
        for (uint32_t mm = mine; mm; mm &= mm - 1) {
            const int t = __builtin_ctz(mm);
            uint4 u = buf[(t * 2 + 0) * 64 + lane];
            uint4 v = buf[(t * 2 + 1) * 64 + lane];
            uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            tr8(W, m4, m2, m1);
            buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        FP_MARK(2);
        barrier_lds();
        FP_MARK(3);
        const int part = n % NP;
        if (part == 0 && n != 0)
            syn_twiddle<K, E, C, NW>(G);
        [&]<int... Ps>(std::integer_sequence<int, Ps...>) {
            ((part == Ps ? syn_part<K, C, E, NW, Ps>(G, buf, lane, j0, em0, em1) : void()), ...);
        }(std::make_integer_sequence<int, NP>{});
        FP_MARK(4);
        barrier_lds();
    }
    FP_MARK(5);

    }

    // The syndromes (parity included), in plane form, are phase 2's sources:
    // wave G's rows are its chunk G.  Waves 0 and 1 write theirs straight
    // into the two LDS part buffers (both free after the last barrier);
    // later waves park theirs in this tile of the output rows (L2 / MALL)
    // and phase 2 fetches them back by LDS-DMA one chunk ahead.
    constexpr int NLDS = 2;  // chunks handed over through LDS
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        (
            [&] {
                const int r = G * 8 + Ss;
                if (r < E) {
                    uint32_t W[8];
                    read_slot<Ss>(W);
                    if (G < NLDS) {
                        uint4* dst = lds[G];
                        dst[(Ss * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
                        dst[(Ss * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
                    } else if (inb) {
                        store32(ob + (size_t)r * a.pitch, off, W);
                    }
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, 8>{});
    barrier_lds();  // the LDS-held chunks are complete
    FP_MARK(6);

    // ---------------- phase 2: x = V_E^-1 s (threaded code) ----------------
    constexpr int NCH2 = (E + S - 1) / S;
    const unsigned long long* ap = a.addr + (size_t)b * E * (NW * 8) + G * 8;
    auto issue2 = [&](int ch) {
        const int c0 = ch * S, nt = min(S, E - c0);
        const uint32_t base = lds0 + (uint32_t)((ch & 1) * S * 2 * 64 * 16);
        for (int t = G; t < nt; t += NW) {
            glds32(ob + (size_t)(c0 + t) * a.pitch, (uint32_t)loff, base + (uint32_t)(t * 2 * 64 * 16));
        }
    };
    auto own2 = [&](int ch) {
        const int nt = min(S, E - ch * S);
        return nt > G ? 2 * ((nt - G + NW - 1) / NW) : 0;
    };
    asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
    for (int ch = 0; ch < NCH2; ++ch) {
        const int nt = min(S, E - ch * S);
        FP_MARK(10);
        // chunk ch + 1 >= NLDS comes by LDS-DMA into buffer (ch + 1) & 1,
        // free since the last barrier; chunk ch >= NLDS was issued one step
        // ago and must have landed (own pieces; the barrier covers the rest)
        if (ch + 1 < NCH2 && ch + 1 >= NLDS) {
            issue2(ch + 1);
            if (ch >= NLDS)
                wait_vm(own2(ch + 1));
        } else if (ch >= NLDS) {
            wait_vm(0);
        }
        FP_MARK(7);
        barrier_lds();  // every wave's part of this chunk has landed
        FP_MARK(8);
        const uint32_t la = lds0 + (uint32_t)((ch & 1) * S * 2 * 64 * 16) + lane * 16;
        const unsigned long long* pa = ap + (size_t)(ch * S) * (NW * 8);
tc_chunk<NW>(la, pa, nt);
        FP_MARK(9);
        if (ch == 0 && G >= NLDS)  // parked syndromes written before chunk NLDS is fetched
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier_lds();  // buffer ch & 1 is refilled by chunk ch + 2
    }
    FP_MARK(10);

    if (!inb) {
        FP_END;
        return;
    }
    // all syndrome rows of this tile were read before the last barrier: the
    // data may overwrite them
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        (
            [&] {
                const int r = G * 8 + Ss;
                if (r < E) {
                    uint32_t W[8];
                    read_slot<Ss>(W);
                    tr8(W, m4, m2, m1);
                    store32(ob + (size_t)r * a.pitch, off, W);
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, 8>{});
    FP_MARK(11);
    FP_END;
}

template <int K, int E, int C, bool TC1>
__global__ __launch_bounds__(64 * ((E + 7) / 8)) __attribute__((amdgpu_num_vgpr(64))) void
k_rs_decode_fused(Args a)
{
    constexpr int NW = (E + 7) / 8;
    __shared__ uint4 lds[2][S * 2 * 64];
    __shared__ uint8_t items[NW][128];  // per-wave survivor list (TC1)
    if (a.status[blockIdx.y] != 0)
        return;  // singular or malformed: the whole block is skipped
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    run_group<K, E, C, NW, TC1>(a, lds, items[wave], wave);
}

// Syndrome phase: threaded code (default) or the compile-time Horner blocks
// (RSGPU_FUSED_SYN=horner, kept for comparison).
bool fused_syn_tc()
{
    static const bool tc = [] {
        const char* v = std::getenv("RSGPU_FUSED_SYN");
        return !(v && std::strcmp(v, "horner") == 0);
    }();
    return tc;
}

template <int K, int E, int C>
hipError_t launch(const Args& a, long long blocks, hipStream_t st)
{
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)blocks);
    if (fused_syn_tc() && a.syn_addr)
        hipLaunchKernelGGL((k_rs_decode_fused<K, E, C, true>), grid, dim3(64 * ((E + 7) / 8)), 0,
                           st, a);
    else
        hipLaunchKernelGGL((k_rs_decode_fused<K, E, C, false>), grid, dim3(64 * ((E + 7) / 8)), 0,
                           st, a);
    return hipGetLastError();
}

}  // namespace fused

bool rs_decode_fused_available(int k, int e)
{
    return (k == 16 && e == 4) || (k == 16 && e == 8) || (k == 64 && e == 32) ||
           (k == 64 && e == 16) || (k == 100 && e == 20) || (k == 5 && e == 4) ||
           (k == 20 && e == 7);
}

hipError_t launch_rs_decode_fused(int k, int e, const uint8_t* src, const uint8_t* par,
                                  uint8_t* out, long long pitch, long long len, long long blocks,
                                  const uint64_t* emask, const unsigned long long* addr,
                                  const unsigned long long* syn_addr, const int* status,
                                  hipStream_t st)
{
    fused::Args a{src, par, out, pitch, len, emask, addr, syn_addr, status};
    if (k == 16 && e == 4) return fused::launch<16, 4, 8>(a, blocks, st);
    if (k == 16 && e == 8) return fused::launch<16, 8, 8>(a, blocks, st);
    if (k == 64 && e == 32) return fused::launch<64, 32, 8>(a, blocks, st);
    if (k == 64 && e == 16) return fused::launch<64, 16, 8>(a, blocks, st);
    if (k == 100 && e == 20) return fused::launch<100, 20, 8>(a, blocks, st);
    if (k == 5 && e == 4) return fused::launch<5, 4, 5>(a, blocks, st);
    if (k == 20 && e == 7) return fused::launch<20, 7, 8>(a, blocks, st);
    return hipErrorInvalidValue;
}

}  // namespace rsgpu
