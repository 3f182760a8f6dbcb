// rs_tc.hip -- bit-sliced GF(2^8) dot product with RUNTIME coefficients via
// threaded code: out_i = sum_p c[i][p] * src_p for per-block matrices c.
// Uses: the decode (the e x k rows of inv(b) over the k - e survivors and the
// e parity rows, rsgpu_capi.cpp / k_decode_prepare_syn; or the rows of the
// k x k inversion for codes without compile-time kernels), the split
// decode's solve, and every runtime-coefficient encode (ec_encode_data with
// any tables, Cauchy).
//
// The bit-sliced multiply-accumulate of one coefficient is 8 full-rate
// v_bitop3 whose REGISTER operands depend on the coefficient value
// (rs_bitsliced.hip, gen_tc_handlers.py).  Register numbers cannot be chosen
// at run time without indexing overhead, so all 256 variants exist as code:
// handler c (RSGPU_TC_STRIDE = 72 bytes, generated) applies coefficient c to
// an accumulator slot from the four-Russians tables of the current source.
// Slot s is reached by GPR indexing (s_set_gpr_idx_on / _idx, one index per
// slot group), and the handlers chain in groups of three (slots 0-2, 3-5,
// 6-7; RSGPU_TC_CHAIN): the kernel s_swappc's to the group's first handler,
// which jumps to the next slot's handler (another copy of the 256 working on
// the next 8 accumulators), and the group's last handler returns.  Group 0
// runs before index mode is switched on.  The 8 handler addresses of a
// source are one s_load_dwordx16 of the table the prepare kernel writes
// ([source][slot], address of the slot's handler copy for coefficient c).  GPR index mode costs every VALU it covers about one
// issue cycle (tools/ubench_idx.hip), the price of reusing one table build
// for 8 rows without per-slot handler copies.
//
// Register contract (gen_tc_handlers.py): accumulators v[64:127] (8 slots x 8
// planes); the source planes v[24:31] (read from LDS straight into the
// single-plane table entries after the previous source's dispatch) and the
// 22 composite L/H entries v[32:53]; handler addresses in the other of two
// banks s[64:79] / s[84:99] while the current source dispatches (one asm
// statement per LDS part, so every load it starts is also waited for inside
// it); return address s[82:83], chain continuation s[80:81], M0 saved in s63.
// The kernel uses exactly 128 VGPRs: 4 waves per SIMD.
//
// Work split: as k_rs_bs -- a workgroup of NW waves covers 64 lanes x 32 bytes
// of every row of one block; wave w owns output rows [8w, 8w+8); the waves
// share the loading + bit transposing of each part of C sources through LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "bitslice.h"
#include "gf256.h"
#include "rs_kernels.h"
#include "tc_handlers.inc"

namespace rsgpu {
namespace tc {

using bs::barrier_lds;
using bs::glds16;
using bs::glds32;
using bs::sload_ptr;
using bs::store32;
using bs::wait_vm;
using bs::tr8;
using bs::vconst;

constexpr int C = RSGPU_TC_C;  // sources per LDS chunk (double-buffered)

// Holds the handler table; launched once per context to report where the
// table sits (out[0] = first handler, out[1] = end of the table).  The
// handlers are reached only through s_swappc from k_rs_tc.
__global__ void k_tc_handlers(unsigned long long* out)
{
    unsigned long long base, end;
    asm volatile(
        "s_getpc_b64 s[84:85]\n"
        "TCQ0:\n"
        "s_add_u32 s84, s84, TC_HANDLERS-TCQ0\n"
        "s_addc_u32 s85, s85, 0\n"
        "s_getpc_b64 s[86:87]\n"
        "TCQ1:\n"
        "s_add_u32 s86, s86, TC_HANDLERS_END-TCQ1\n"
        "s_addc_u32 s87, s87, 0\n"
        "s_mov_b64 %0, s[84:85]\n"
        "s_mov_b64 %1, s[86:87]\n"
        "s_branch TC_SKIP\n"
        ".p2align 6\n"
        "TC_HANDLERS:\n" RSGPU_TC_HANDLERS
        "TC_HANDLERS_END:\n"
        "TC_SKIP:\n"
        : "=s"(base), "=s"(end)
        :
        : "s84", "s85", "s86", "s87", "scc");
    if (threadIdx.x == 0) {
        out[0] = base;
        out[1] = end;
    }
}

// Instrumentation point of k_rs_tc: the product's TcHooks time nothing;
// tools/tc_profile.hip instantiates the kernel with a policy whose Timer sums
// s_memtime per phase.
struct TcHooks {
    struct Timer {
        __device__ void mark(int) {}
        __device__ void end(int) {}
    };
};

// Read accumulator slot S (asm-owned v[64+8S : 64+8S+7]) into W, two planes
// per v_mov_b64.
template <int S>
__device__ __forceinline__ void read_slot(uint32_t (&W)[8])
{
    uint64_t P[4];
#define RSGPU_TC_RD(TEXT) asm volatile(TEXT : "=v"(P[0]), "=v"(P[1]), "=v"(P[2]), "=v"(P[3]))
    if constexpr (S == 0) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_0);
    if constexpr (S == 1) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_1);
    if constexpr (S == 2) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_2);
    if constexpr (S == 3) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_3);
    if constexpr (S == 4) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_4);
    if constexpr (S == 5) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_5);
    if constexpr (S == 6) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_6);
    if constexpr (S == 7) RSGPU_TC_RD(RSGPU_TC_READ_SLOT64_7);
#undef RSGPU_TC_RD
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        W[2 * q] = (uint32_t)P[q];
        W[2 * q + 1] = (uint32_t)(P[q] >> 32);
    }
}

// amdgpu_num_vgpr(64): the compiler allocates v0..v63 only; the accumulators
// v64..v127 are touched by asm alone, so they stay put across the loops (the
// kernel descriptor still reserves 128 VGPRs because the asm names v127).
template <int NW, class H = TcHooks>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_num_vgpr(64))) void k_rs_tc(TcArgs a, int tiles_per_wg)
{
    // two chunk buffers [C][2 halves][64 lanes] of 16 bytes: 2 x 16 KiB
    __shared__ uint4 lds[2][C * 2 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    if (a.status && a.status[b] != 0)
        return;  // uniform per workgroup: the whole block is skipped
    // this workgroup's consecutive 2 KB column tiles of block b
    const long long ntile = (a.len + 2047) / 2048;
    const long long tile0 = (long long)blockIdx.x * tiles_per_wg;
    const int my_tiles = (int)min((long long)tiles_per_wg, ntile - tile0);
    const int k = a.k;
    const int nch = (k + C - 1) / C;
    const int total = my_tiles * nch;  // (tile, chunk) steps, pipelined across tiles
    const uint8_t* const* srcs = a.srcs + (size_t)b * k;
    uint8_t* const* dsts = a.dsts + (size_t)b * a.dst_stride;
    // addresses [B][k][NW*8]: this wave's 8 slots of source j at ap + j*NW*8
    const unsigned long long* ap = a.addr + (size_t)b * a.addr_stride + wave * 8;
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];

    auto issue = [&](int n) {
        const int ch = n % nch;
        const long long off = (tile0 + n / nch) * 2048 + lane * 32;
        const long long loff = off + 32 <= a.len ? off : 0;  // out-of-range lanes re-read the row head
        const int c0 = ch * C, nt = min(C, k - c0);
        const uint32_t base = lds0 + (uint32_t)((n & 1) * C * 2 * 64 * 16);
        // this wave's row pointers of the chunk, two scalar loads under one
        // wait when it owns two sources (load and wait in ONE asm statement:
        // the compiler must not see an output before it has landed)
        int t = wave;
        for (; t + NW < nt; t += 2 * NW) {
            const uint8_t *r0, *r1;
            asm volatile("s_load_dwordx2 %0, %2, 0\n s_load_dwordx2 %1, %3, 0\n s_waitcnt lgkmcnt(0)"
                         : "=&s"(r0), "=&s"(r1)
                         : "s"(srcs + c0 + t), "s"(srcs + c0 + t + NW)
                         : "memory");
            glds32(r0, (uint32_t)loff, base + (uint32_t)(t * 2 * 64 * 16));
            glds32(r1, (uint32_t)loff, base + (uint32_t)((t + NW) * 2 * 64 * 16));
        }
        if (t < nt)
            glds32(sload_ptr(srcs + c0 + t), (uint32_t)loff, base + (uint32_t)(t * 2 * 64 * 16));
    };

    typename H::Timer tp;
    issue(0);
    for (int n = 0; n < total; ++n) {
        const int ch = n % nch;
        const int nt = min(C, k - ch * C);
        uint4* buf = lds[n & 1];
        tp.mark(6);
        wait_vm(0);  // this step's own sources, issued behind the previous step's barrier
        tp.mark(0);
        tp.mark(1);
        // own share of this chunk: bytes -> bit-planes, in place
        for (int t = wave; t < nt; t += NW) {
            uint4 u = buf[(t * 2 + 0) * 64 + lane];
            uint4 v = buf[(t * 2 + 1) * 64 + lane];
            uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            tr8(W, m4, m2, m1);
            buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        tp.mark(2);
        barrier_lds();
        // one barrier per step: every wave is past its dispatch of step
        // n - 1, which read buffer (n + 1) & 1, so the next step's sources
        // may land there now and arrive during this step's dispatch
        if (n + 1 < total)
            issue(n + 1);
        tp.mark(3);
        if (ch == 0)
            asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
        // the chunk's nt sources: one asm statement (gen_tc_handlers.py)
        {
            const uint32_t la = lds0 + (uint32_t)((n & 1) * C * 2 * 64 * 16) + lane * 16;
            const unsigned long long* pa = ap + (size_t)(ch * C) * (NW * 8);
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
        tp.mark(4);
        if (ch == nch - 1) {
            // tile done: outputs back to bytes and out (all of this tile's
            // sources were read before the previous barrier: in-place safe)
            const long long off = (tile0 + n / nch) * 2048 + lane * 32;
            if (off + 32 <= a.len) {
                [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
                    (
                        [&] {
                            const int r = wave * 8 + Ss;
                            if (r < a.rows) {
                                uint32_t W[8];
                                read_slot<Ss>(W);
                                tr8(W, m4, m2, m1);
                                store32((uint8_t*)sload_ptr((const uint8_t* const*)(dsts + r)), off, W);
                            }
                        }(),
                        ...);
                }(std::make_integer_sequence<int, 8>{});
            }
        }
        tp.mark(5);
    }
    tp.mark(6);
    tp.end(lane);
}

// Small batches, rows <= 8 (C2: one block of (16, 4, 1e6), 489 tiles): one
// wave per tile would leave most SIMDs idle and walk all k sources in series
// (13 us at C2).  Here SPL waves split a tile's sources: wave w takes the
// contiguous range [w k / SPL, (w+1) k / SPL), loads it by LDS-DMA into its
// own LDS part, transposes it and runs the same threaded code over it into
// all rows (the address table [B][k][8] of tc_rows_per_pass(rows) = 8); then
// the partial accumulators meet in LDS and wave w finishes rows w, w + SPL,
// ...  No barrier until the reduction: each wave reads only its own part.
template <int SPL>
__global__ __launch_bounds__(64 * SPL) __attribute__((amdgpu_num_vgpr(64))) void k_rs_tc_split(TcArgs a)
{
    // per wave: C sources x [2 halves][64 lanes] x 16 B = 16 KiB, reused for
    // the wave's partial accumulators (8 slots x 8 planes x 64 lanes x 4 B)
    __shared__ uint4 lds[SPL][C * 2 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    if (a.status && a.status[b] != 0)
        return;
    const int k = a.k;
    const int j0 = wave * k / SPL, j1 = (wave + 1) * k / SPL;
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const uint32_t loff = off + 32 <= a.len ? (uint32_t)off : 0u;  // out-of-range lanes re-read the row head
    const uint8_t* const* srcs = a.srcs + (size_t)b * k;
    const unsigned long long* ap = a.addr + (size_t)b * a.addr_stride;
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    uint4* mine = lds[wave];
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)mine;
    asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
    for (int c0 = j0; c0 < j1; c0 += C) {
        const int nt = min(C, j1 - c0);
        for (int t = 0; t < nt; ++t)
            glds32(sload_ptr(srcs + c0 + t), loff, base + (uint32_t)(t * 2 * 64 * 16));
        wait_vm(0);
        for (int t = 0; t < nt; ++t) {
            uint4 u = mine[(t * 2 + 0) * 64 + lane];
            uint4 v = mine[(t * 2 + 1) * 64 + lane];
            uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            tr8(W, m4, m2, m1);
            mine[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            mine[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const uint32_t la = base + lane * 16;
        const unsigned long long* pa = ap + (size_t)c0 * 8;
#define RSGPU_TC_RUN(N)                                                                          \
    asm volatile(RSGPU_TC_CHUNK##N                                                               \
                 :                                                                               \
                 : [la] "v"(la), [pa] "s"(pa), [o1] "i"(64), [o2] "i"(128), [o3] "i"(192),        \
                   [o4] "i"(256), [o5] "i"(320), [o6] "i"(384), [o7] "i"(448)                     \
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
    // partial accumulators -> this wave's part: [slot][plane][lane]
    uint32_t* part = reinterpret_cast<uint32_t*>(mine);
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        (
            [&] {
                if (Ss < a.rows) {
                    uint32_t W[8];
                    read_slot<Ss>(W);
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        part[(Ss * 8 + q) * 64 + lane] = W[q];
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, 8>{});
    __syncthreads();
    if (off + 32 > a.len)
        return;
    uint8_t* const* dsts = a.dsts + (size_t)b * a.dst_stride;
    for (int r = wave; r < a.rows; r += SPL) {
        uint32_t W[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < SPL; ++w) {
            const uint32_t* pw = reinterpret_cast<const uint32_t*>(lds[w]);
#pragma unroll
            for (int q = 0; q < 8; ++q)
                W[q] ^= pw[(r * 8 + q) * 64 + lane];
        }
        tr8(W, m4, m2, m1);
        store32((uint8_t*)sload_ptr((const uint8_t* const*)(dsts + r)), off, W);
    }
}

// The whole decode of a small batch in ONE launch (rsgpu_decode_blocks, C2:
// one block of (16, 4, 1e6), e <= 8, k <= 64): every wave first builds the
// coefficients of its own sources from the e x k decode rows V_E^-1 [V_kept | I]
// in closed form (the rows of k_decode_prepare_syn, rs_kernels.hip, as
// Lagrange bases: logs for the survivors, Q_i = prod_{l != i} (z + a_l) built
// lane-parallel in registers for the parity sources) while its source loads
// fly, with no barrier, then runs k_rs_tc_split's work with
// the handler addresses computed from the rows (handler of slot s for
// coefficient c at map.base + (map.copy[s] 256 + c) map.stride) and handed
// to the threaded code in a VGPR (RSGPU_TC_CHUNKV, v_readlane) instead of a
// table in memory.  Saves the prepare launch and its table round trip.
alignas(16) __device__ const GfTables kGfTc = make_gf_tables();

template <int SPL, class H = TcHooks>
__global__ __launch_bounds__(64 * SPL) __attribute__((amdgpu_num_vgpr(64))) void k_rs_tc_fused(TcFusedArgs a)
{
    typename H::Timer tp;
    __shared__ uint4 lds[SPL][C * 2 * 64];  // per wave: its sources, then its partial rows
    __shared__ uint32_t gtw[SPL][192];         // per wave: its copy of exp[512] | log[256]
    __shared__ uint8_t coef[8 * 64], lvw[SPL][64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y, k = a.k, e = a.e, nl = k - e;
    // every wave: the GF tables and its block's erasure list (one round trip),
    // the list validated, and the survivors (ascending) -- all it needs to
    // start its own source loads at once, before the decode rows exist
    const uint32_t* tsrc = reinterpret_cast<const uint32_t*>(&kGfTc);
    const uint32_t t0 = tsrc[lane], t1 = tsrc[64 + lane], t2 = tsrc[128 + lane];
    const int j = lane < e ? a.err[(size_t)b * e + lane] : 255;  // lane i: erased original j_i
    const int jp = __shfl_up(j, 1);
    if (__ballot(lane < e && (j >= k || (lane > 0 && j <= jp))) != 0) {  // strictly ascending, < k
        if (blockIdx.x == 0 && threadIdx.x == 0)
            a.status[b] = -2;
        return;  // uniform per workgroup
    }
    tp.mark(0);
    uint32_t* gw = gtw[wave];
    gw[lane] = t0;
    gw[64 + lane] = t1;
    gw[128 + lane] = t2;
    const uint8_t* gexp = reinterpret_cast<const uint8_t*>(gw);
    const uint8_t* glog = gexp + 512;
    bool er = false;
    for (int i = 0; i < e; ++i)
        er |= __builtin_amdgcn_readlane(j, i) == lane;
    const unsigned long long surv = __ballot(lane < k && !er);
    const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(surv >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)surv, 0u));
    uint8_t* lv = lvw[wave];
    if (lane < k && !er)
        lv[rank] = (uint8_t)lane;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int j0 = wave * k / SPL, j1 = (wave + 1) * k / SPL;
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const uint32_t loff = off + 32 <= a.len ? (uint32_t)off : 0u;
    uint4* mine = lds[wave];
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)mine;
    auto issue = [&](int g0) {
        for (int t = 0; t < min(4, j1 - g0); ++t) {
            const int q = g0 + t;
            const uint8_t* row = q < nl ? a.src + ((size_t)b * k + lv[q]) * a.pitch
                                        : a.par + ((size_t)b * e + (q - nl)) * a.pitch;
            glds32(row, loff, base + (uint32_t)(t * 2 * 64 * 16));
        }
    };
    if (j0 < j1)
        issue(j0);
    tp.mark(1);
    // While the loads fly, each wave builds the coefficients of its own
    // sources (closed form, the rows k_decode_prepare_syn builds): row i of
    // V_E^-1 [V_kept | I] is the Lagrange basis L_i(z) = Q_i(z) / w_i with
    // Q_i = prod_{l != i} (z + a_l), a_l = 2^(j_l), w_i = Q_i(a_i); survivor q
    // gets L_i(b_q) through logs, parity source nl + m the coefficient of z^m.
    const int al = lane < e ? gexp[j] : 0;  // lane l: a_l
    // a_l in SGPRs, unused l < 8 marked (readlane outside any ?:, which clang
    // lowers to branches around a convergent call)
    int A[8];
    bool use[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        A[l] = __builtin_amdgcn_readlane(al, l);
        use[l] = l < e;
    }
    auto pick = [&](int idx) {  // a_idx, idx per lane
        int r = 0;
#pragma unroll
        for (int l = 0; l < 8; ++l)
            r = idx == l ? A[l] : r;
        return r;
    };
    auto log_w = [&](int i) {  // log w_i = sum_{l != i} log (a_i + a_l)
        const int ai = pick(i);
        int sw = 0;
#pragma unroll
        for (int l = 0; l < 8; ++l)
            sw += glog[(use[l] && l != i) ? ai ^ A[l] : 1];  // log 1 = 0
        return sw % 255;
    };
    const int s1 = min(j1, nl);
    for (int p = j0 * 8; p < s1 * 8; p += 64) {  // (survivor q, row i) on lane 8 q + i
        const int q = (p + lane) >> 3, i = lane & 7;
        if (q < s1 && i < e) {
            const int bq = gexp[lv[q]];
            int lb = 0;  // log Lambda(b_q)
#pragma unroll
            for (int l = 0; l < 8; ++l)
                lb += glog[use[l] ? bq ^ A[l] : 1];
            coef[i * k + q] = gexp[(lb + 2 * 255 - glog[bq ^ pick(i)] - log_w(i)) % 255];
        }
    }
    if (j1 > nl) {  // parity sources: Q_i's coefficients, z^m on lane 8 i + m
        const int i = lane >> 3, m = lane & 7;
        int J[8];
#pragma unroll
        for (int l = 0; l < 8; ++l)
            J[l] = __builtin_amdgcn_readlane(j, l);
        int ji = 0;
#pragma unroll
        for (int l = 0; l < 8; ++l)
            ji = i == l ? J[l] : ji;
        const int tv = gexp[ji + m];  // lane 8 l + c: a_l x^c = 2^(j_l + c)
        int qv = m == 0;
        for (int l = 0; l < e; ++l) {
            int pr = 0;  // a_l q_m: the x^c multiples of a_l where q_m has bit c
#pragma unroll
            for (int c = 0; c < 8; ++c)
                pr ^= __builtin_amdgcn_readlane(tv, l * 8 + c) & -((qv >> c) & 1);
            int sh = __builtin_amdgcn_update_dpp(0, qv, 0x111, 0xF, 0xF, true);  // row_shr:1, q_{m-1}
            sh = m ? sh : 0;
            qv = l == i ? qv : (sh ^ pr);
        }
        if (i < e && m < e && nl + m >= j0 && nl + m < j1)
            coef[i * k + nl + m] = qv ? gexp[(glog[qv] + 255 - log_w(i)) % 255] : 0;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own coefficients, read back below
    tp.mark(2);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        a.status[b] = 0;
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
    for (int g0 = j0; g0 < j1; g0 += 4) {
        const int nt = min(4, j1 - g0);
        if (g0 != j0)
            issue(g0);  // the part is free: the previous group's dispatch is done
        // lane 16 t + w: dword w of source g0 + t's 8 handler addresses
        uint32_t av = 0;
        {
            const int t = lane >> 4, s = (lane & 15) >> 1;
            if (t < nt) {
                const int c = s < e ? coef[s * k + g0 + t] : 0;
                const unsigned long long ad =
                    a.map_base + (unsigned long long)(a.map_copy[s] * 256 + c) * (unsigned long long)a.map_stride;
                av = (lane & 1) ? (uint32_t)(ad >> 32) : (uint32_t)ad;
            }
        }
        wait_vm(0);
        for (int t = 0; t < nt; ++t) {
            uint4 u = mine[(t * 2 + 0) * 64 + lane];
            uint4 v = mine[(t * 2 + 1) * 64 + lane];
            uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            tr8(W, m4, m2, m1);
            mine[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            mine[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        tp.mark(3);
        const uint32_t la = base + lane * 16;
#define RSGPU_TC_RUNV(N)                                                                          \
    asm volatile(RSGPU_TC_CHUNKV##N                                                               \
                 :                                                                                \
                 : [la] "v"(la), [av] "v"(av)                                                     \
                 : RSGPU_TC_CLOBBERS, RSGPU_TC_ACC_CLOBBERS, "memory")
        switch (nt) {
        case 1: RSGPU_TC_RUNV(1); break;
        case 2: RSGPU_TC_RUNV(2); break;
        case 3: RSGPU_TC_RUNV(3); break;
        default: RSGPU_TC_RUNV(4); break;
        }
#undef RSGPU_TC_RUNV
        // the next group reuses this wave's part and av
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        tp.mark(4);
    }
    uint32_t* part = reinterpret_cast<uint32_t*>(mine);
    [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
        (
            [&] {
                if (Ss < e) {
                    uint32_t W[8];
                    read_slot<Ss>(W);
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        part[(Ss * 8 + q) * 64 + lane] = W[q];
                }
            }(),
            ...);
    }(std::make_integer_sequence<int, 8>{});
    __syncthreads();
    tp.mark(5);
    if (off + 32 > a.len)
        return;
    for (int r = wave; r < e; r += SPL) {
        uint32_t W[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < SPL; ++w) {
            const uint32_t* pw = reinterpret_cast<const uint32_t*>(lds[w]);
#pragma unroll
            for (int q = 0; q < 8; ++q)
                W[q] ^= pw[(r * 8 + q) * 64 + lane];
        }
        tr8(W, m4, m2, m1);
        store32(a.out + ((size_t)b * e + r) * a.pitch, off, W);
    }
    tp.mark(6);
    tp.end(lane);
}

}  // namespace tc

hipError_t tc_query_handlers(unsigned long long* d_out, hipStream_t st)
{
    hipLaunchKernelGGL(tc::k_tc_handlers, dim3(1), dim3(64), 0, st, d_out);
    return hipGetLastError();
}

int tc_handler_stride() { return RSGPU_TC_STRIDE; }

int tc_handler_count() { return RSGPU_TC_NHANDLERS; }

int tc_slot_copy(int slot)
{
    static constexpr int copy[8] = RSGPU_TC_SLOT_COPY;
    return copy[slot & 7];
}

hipError_t launch_rs_tc_split(const TcArgs& a, long long blocks, hipStream_t st)
{
    if (a.rows <= 0 || a.rows > 8 || a.k < 4)
        return hipErrorInvalidValue;
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)blocks);
    hipLaunchKernelGGL(tc::k_rs_tc_split<4>, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_rs_tc_fused(const TcFusedArgs& a, hipStream_t st)
{
    if (a.e <= 0 || a.e > 8 || a.k <= 0 || a.k > 64 || a.k < a.e || a.len % 32 || a.blocks <= 0 ||
        a.blocks > 65535)
        return hipErrorInvalidValue;
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)a.blocks);
    hipLaunchKernelGGL(tc::k_rs_tc_fused<4>, grid, dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_rs_tc(const TcArgs& a, long long blocks, hipStream_t st)
{
    const int nw = tc_rows_per_pass(a.rows) / 8;
    if (a.rows <= 0 || a.rows > 32 || a.k <= 0)
        return hipErrorInvalidValue;
    const long long ntile = (a.len + 2047) / 2048;
    // one 2 KB column tile per workgroup (several consecutive tiles per
    // workgroup, the LDS-DMA pipeline running across them, measured equal)
    const int tpw = 1;
    const unsigned pad = 0;
    dim3 grid((unsigned)ntile, (unsigned)blocks);
    switch (nw) {
    case 1: hipLaunchKernelGGL(tc::k_rs_tc<1>, grid, dim3(64), pad, st, a, tpw); break;
    case 2: hipLaunchKernelGGL(tc::k_rs_tc<2>, grid, dim3(128), pad, st, a, tpw); break;
    case 3: hipLaunchKernelGGL(tc::k_rs_tc<3>, grid, dim3(192), pad, st, a, tpw); break;
    case 4: hipLaunchKernelGGL(tc::k_rs_tc<4>, grid, dim3(256), pad, st, a, tpw); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rsgpu
