// rs_decode_fused.hip -- one-pass syndrome decode for the gf_gen_rs_matrix
// codes: recovered data rows from the surviving data rows and the parity rows
// of each block, with HBM traffic (k + e) * L per block (read k, write e)
// plus the parked syndromes of the waves beyond the LDS hand-off.
//
// Status: the default decode is the one-matrix k_rs_tc (rsgpu_capi.cpp
// decode_kernel); this kernel is the default for (k 100, e 20), where it
// measured 3 % faster, and RSGPU_DECODE_FUSED (rsgpu_set_decode_kernel)
// selects it for any k <= 128, e <= 32.
//
// The two-kernel decode (syndrome rows to HBM, then the solve reading them
// back) moves 2 e L more bytes.  Here one workgroup does both for its 2 KB
// column tile, both phases on threaded code (rs_tc.hip's chunk asm):
//
//   phase 1  s = P ^ V_kept d_kept        coefficients 2^(r j) of the k - e
//            surviving originals j (handler addresses from the prepare
//            kernel), sources streamed by LDS-DMA and bit-transposed in LDS;
//            the parity rows enter the accumulators first.  Wave G's e/NW
//            syndrome rows are phase 2's chunk G: waves 0 and 1 hand theirs
//            over in LDS, later waves park theirs in this tile of the output
//            rows (L2 / MALL resident) in bit-plane form
//   phase 2  x = V_E^-1 s                 runtime e x e coefficients over the
//            syndrome rows (already planes: no input transposes), then the
//            rows are transposed to bytes and overwrite the syndromes.
//
// Both phases keep the accumulators in asm-owned v64..v127 (the compiler is
// capped at v0..v63, amdgpu_num_vgpr(64)).  Wave w owns rows 8w..8w+7; NW =
// ceil(e / 8) waves per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "bitslice.h"
#include "rs_kernels.h"
#include "tc_handlers.inc"

namespace rsgpu {
namespace fused {

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
    int K, E;
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

// One wave group G (runtime, wave-uniform) of NW: rows 8G..8G+7.
template <int NW>
__device__ __forceinline__ void run_group(const Args& a, uint4 (*lds)[S * 2 * 64], uint8_t* items,
                                          int G)
{
    const int K = a.K, E = a.E;
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
    // The K-E survivors in ascending order, S per LDS part, each wave moving
    // and transposing slots t = G, G+NW, ...; coefficient 2^(r j) of
    // survivor j for syndrome row r comes as a handler address from the
    // prepare kernel's table.  The parity rows enter the accumulators
    // unscaled.
    FP_DECL
    const int NL = K - E;
    const int NSTEP = (NL + S - 1) / S;
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
        vi1 = 64 + lane < NL ? items[64 + lane] : 0;
    }
    auto survivor = [&](int q) -> int {
        return __builtin_amdgcn_readlane((int)(q < 64 ? vi0 : vi1), q & 63);
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
    issue1(0);  // NL >= 1 (rs_decode_fused_available)
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
    const int NCH2 = (E + S - 1) / S;
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

template <int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_num_vgpr(64))) void
k_rs_decode_fused(Args a)
{
    __shared__ uint4 lds[2][S * 2 * 64];
    __shared__ uint8_t items[NW][128];  // per-wave survivor list
    if (a.status[blockIdx.y] != 0)
        return;  // singular or malformed: the whole block is skipped
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    run_group<NW>(a, lds, items[wave], wave);
}

}  // namespace fused

// any gf_gen_rs_matrix code with 1 <= e <= 32 parity rows, k <= 128 (the
// survivor list is two lanes' words) and at least one surviving original
bool rs_decode_fused_available(int k, int e)
{
    return e >= 1 && e <= 32 && k <= 128 && k > e;
}

hipError_t launch_rs_decode_fused(int k, int e, const uint8_t* src, const uint8_t* par,
                                  uint8_t* out, long long pitch, long long len, long long blocks,
                                  const uint64_t* emask, const unsigned long long* addr,
                                  const unsigned long long* syn_addr, const int* status,
                                  hipStream_t st)
{
    if (!rs_decode_fused_available(k, e) || !syn_addr)
        return hipErrorInvalidValue;
    fused::Args a{src, par, out, k, e, pitch, len, emask, addr, syn_addr, status};
    dim3 grid((unsigned)((len + 2047) / 2048), (unsigned)blocks);
    switch ((e + 7) / 8) {
    case 1: hipLaunchKernelGGL(fused::k_rs_decode_fused<1>, grid, dim3(64), 0, st, a); break;
    case 2: hipLaunchKernelGGL(fused::k_rs_decode_fused<2>, grid, dim3(128), 0, st, a); break;
    case 3: hipLaunchKernelGGL(fused::k_rs_decode_fused<3>, grid, dim3(192), 0, st, a); break;
    default: hipLaunchKernelGGL(fused::k_rs_decode_fused<4>, grid, dim3(256), 0, st, a); break;
    }
    return hipGetLastError();
}

}  // namespace rsgpu
