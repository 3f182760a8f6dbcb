// rs_jit.hip -- the one-matrix decode through per-block generated code
// (rs_jit.h): dsts[b][i] = sum_p c_b[i][p] * srcs[b][p] with the e x k matrix
// of block b baked into code that k_jit_emit wrote into executable
// device memory (rsgpu_capi.cpp allocates it from the GPU's coarse-grained
// pool with HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG).
//
// Work split as k_rs_tc (rs_tc.hip): a workgroup of NW waves covers one 2 KB
// column tile (64 lanes x 32 bytes) of every row of one block; wave w owns
// output rows [8w, 8w+8); the waves share the loading (LDS-DMA) and bit
// transposing of each chunk of 8 sources through LDS.  Per chunk a wave makes
// ONE call into its generated code, which reads the planes from LDS, builds
// the four-Russians tables and applies its 8 x 8 coefficients: no
// per-coefficient jumps, no scalar loads of handler addresses, no GPR index
// mode.
//
// The instruction cache is not invalidated between kernel launches
// (tools/ubench_jit.hip: code rewritten between two launches runs stale
// without it), and the code of a block is rewritten by every prepare, so
// wave 0 of every workgroup executes s_icache_inv before the workgroup's
// first call.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <utility>

#include "bitslice.h"
#include "diag_clock.h"
#include "rs_jit.h"
#include "rs_kernels.h"
#include "tc_handlers.inc"

namespace rsgpu {
namespace jitk {

using bs::barrier_lds;
using bs::glds32;
using bs::glds32_nt;
using bs::sload_ptr;
using bs::store32;
using bs::tr8;
using bs::vconst;
using bs::wait_vm;

constexpr int C = 8;  // sources per LDS chunk (double-buffered)

RSGPU_DIAG_TABLE

// k_rs_jitw's phase stamps (the diagnostic build's variant 6, kernel_hooks.h)
#ifdef RSGPU_DIAG_CLOCK
using JitwPhases = std::conditional_t<Hooks::kPhaseStamps, diag::PhaseTimer, diag::NoPhases>;
#else
using JitwPhases = diag::NoPhases;
#endif

// Instrumentation points of k_rs_jit.  The product instantiates JitHooks:
// no timers, every wave runs its own block's code, wave 0 invalidates the
// instruction cache.  tools/jit_profile.hip supplies its own policy (per-phase
// s_memtime sums, timing-only code substitution) without touching this file.
struct JitHooks {
    struct Timer {
        __device__ void mark(int) {}
        __device__ void end(int) {}
    };
    static constexpr bool kInvalidate = true;
    // this wave's generated code: chunk ch at code + ch * chunk_stride
    __device__ static const uint8_t* code(const JitArgs& a, bool shared, int b, int wave, int nch)
    {
        return a.code + (shared ? 0 : (size_t)b * a.block_stride) + (size_t)wave * nch * a.chunk_stride;
    }
};

template <int S>
__device__ __forceinline__ void read_slot(uint32_t (&W)[8])
{
    uint64_t P[4];
#define RSGPU_JIT_RD(TEXT) asm volatile(TEXT : "=v"(P[0]), "=v"(P[1]), "=v"(P[2]), "=v"(P[3]))
    if constexpr (S == 0) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_0);
    if constexpr (S == 1) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_1);
    if constexpr (S == 2) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_2);
    if constexpr (S == 3) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_3);
    if constexpr (S == 4) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_4);
    if constexpr (S == 5) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_5);
    if constexpr (S == 6) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_6);
    if constexpr (S == 7) RSGPU_JIT_RD(RSGPU_TC_READ_SLOT64_7);
#undef RSGPU_JIT_RD
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        W[2 * q] = (uint32_t)P[q];
        W[2 * q + 1] = (uint32_t)(P[q] >> 32);
    }
}

// amdgpu_num_vgpr(64): the compiler allocates v0..v63 only (minus the
// registers the call clobbers); the accumulators v64..v127 are touched by asm
// and generated code alone.  (Holding the block's row pointers in VGPRs and
// reading them with v_readlane instead of scalar loads measured slower:
// 26.3 vs 25.1 ms at C3, tools/jit_profile.)
// SH: one program shared by every block (the GENERATED encode; a distinct
// symbol, so profiles tell it from the per-block decode)
template <int NW, bool SH, class H = JitHooks>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_num_vgpr(64))) void k_rs_jit(JitArgs a)
{
    __shared__ uint4 lds[2][C * 2 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    int b = blockIdx.y;
    long long tile = blockIdx.x;
    if (a.xcd_order) {
        // workgroups are dealt round-robin over the 8 XCDs: give each XCD a
        // contiguous range of (block, tile), so all tiles of a block (and its
        // code) stay in one XCD's L2 -- it matters when a block has few tiles
        const unsigned g = blockIdx.x + gridDim.x * blockIdx.y, tot = gridDim.x * gridDim.y;
        const unsigned xcd = g & 7, q8 = tot >> 3, r8 = tot & 7;
        const unsigned lin = xcd * q8 + min(xcd, r8) + (g >> 3);
        b = (int)(lin / gridDim.x);
        tile = lin - (unsigned)b * gridDim.x;
    }
    if (a.status && a.status[b] != 0)
        return;  // uniform per workgroup: the whole block is skipped
    const int k = a.k;
    const int nch = (k + C - 1) / C;
    const uint8_t* const* srcs = a.srcs + (size_t)b * k;
    uint8_t* const* dsts = a.dsts + (size_t)b * a.dst_stride;
    const uint8_t* code = H::code(a, SH, b, wave, nch);
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][0];
    const long long off = tile * 2048 + lane * 32;
    const long long loff = off + 32 <= a.len ? off : 0;  // out-of-range lanes re-read the row head

    // The instruction cache is shared by the waves of a CU pair and keeps
    // lines across launches: wave 0 invalidates it before any wave of this
    // workgroup calls code (the calls follow the first chunk barrier).  Every
    // wave invalidating measured 1.3 % slower (it wipes the other workgroups'
    // lines too; profiles/r02_ab/jit_icache_inv.log).
    if (H::kInvalidate && wave == 0)
        asm volatile("s_icache_inv\n s_nop 15\n s_nop 15" ::: "memory");

    // chunk ch's sources this wave moves: t = wave, wave + NW, ... (two row
    // pointers per scalar wait)
    auto issue = [&](int ch) {
        const int c0 = ch * C, nt = min(C, k - c0);
        const uint32_t base = lds0 + (uint32_t)((ch & 1) * C * 2 * 64 * 16);
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

    asm volatile(RSGPU_TC_ZERO ::: RSGPU_TC_ACC_CLOBBERS);
    typename H::Timer jp;
    issue(0);
    jp.mark(3);
    for (int ch = 0; ch < nch; ++ch) {
        const int nt = min(C, k - ch * C);
        uint4* buf = lds[ch & 1];
        wait_vm(0);  // this chunk's own sources, issued behind the previous barrier
        jp.mark(0);
        if (a.prio)  // the transposes up to the barrier over other waves' code (as k_rs_jitw)
            asm volatile("s_setprio 2" ::: "memory");
        // own share of this chunk: bytes -> bit-planes, in place, two
        // sources at a time (both sets of LDS reads in flight together)
        int t = wave;
        for (; t + NW < nt; t += 2 * NW) {
            const int t1 = t + NW;
            uint4 u0 = buf[(t * 2 + 0) * 64 + lane], v0 = buf[(t * 2 + 1) * 64 + lane];
            uint4 u1 = buf[(t1 * 2 + 0) * 64 + lane], v1 = buf[(t1 * 2 + 1) * 64 + lane];
            uint32_t W0[8] = {u0.x, u0.y, u0.z, u0.w, v0.x, v0.y, v0.z, v0.w};
            uint32_t W1[8] = {u1.x, u1.y, u1.z, u1.w, v1.x, v1.y, v1.z, v1.w};
            tr8(W0, m4, m2, m1);
            tr8(W1, m4, m2, m1);
            buf[(t * 2 + 0) * 64 + lane] = make_uint4(W0[0], W0[1], W0[2], W0[3]);
            buf[(t * 2 + 1) * 64 + lane] = make_uint4(W0[4], W0[5], W0[6], W0[7]);
            buf[(t1 * 2 + 0) * 64 + lane] = make_uint4(W1[0], W1[1], W1[2], W1[3]);
            buf[(t1 * 2 + 1) * 64 + lane] = make_uint4(W1[4], W1[5], W1[6], W1[7]);
        }
        if (t < nt) {
            uint4 u = buf[(t * 2 + 0) * 64 + lane];
            uint4 v = buf[(t * 2 + 1) * 64 + lane];
            uint32_t W[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            tr8(W, m4, m2, m1);
            buf[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            buf[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        jp.mark(1);
        barrier_lds();
        if (a.prio)
            asm volatile("s_setprio 0" ::: "memory");
        jp.mark(2);
        // one barrier per chunk: every wave is past its call of chunk ch - 1,
        // which read buffer (ch + 1) & 1, so chunk ch + 1 may land there now
        if (ch + 1 < nch)
            issue(ch + 1);
        jp.mark(3);
        const uint32_t la = lds0 + (uint32_t)((ch & 1) * C * 2 * 64 * 16) + lane * 16;
        const uint8_t* fn = code + (size_t)ch * a.chunk_stride;
        asm volatile("s_swappc_b64 s[82:83], %[fn]"
                     :
                     : [fn] "s"(fn), "{v20}"(la)
                     : "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34",
                       "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
                       "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56",
                       "v57", "v58", "v59", "v60", "v61", "s82", "s83", "scc", "memory",
                       RSGPU_TC_ACC_CLOBBERS);
        jp.mark(4);
    }
    // outputs back to bytes and out (every source of this tile was read
    // before the last barrier)
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
    jp.mark(5);
    jp.end(lane);
}

template <int S>
__device__ __forceinline__ void read_slotw(uint32_t (&W)[8])
{
    uint64_t P[4];
#define RSGPU_JW_RD(TEXT) asm volatile(TEXT : "=v"(P[0]), "=v"(P[1]), "=v"(P[2]), "=v"(P[3]))
    if constexpr (S == 0) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_0);
    if constexpr (S == 1) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_1);
    if constexpr (S == 2) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_2);
    if constexpr (S == 3) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_3);
    if constexpr (S == 4) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_4);
    if constexpr (S == 5) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_5);
    if constexpr (S == 6) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_6);
    if constexpr (S == 7) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_7);
    if constexpr (S == 8) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_8);
    if constexpr (S == 9) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_9);
    if constexpr (S == 10) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_10);
    if constexpr (S == 11) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_11);
    if constexpr (S == 12) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_12);
    if constexpr (S == 13) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_13);
    if constexpr (S == 14) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_14);
    if constexpr (S == 15) RSGPU_JW_RD(RSGPU_JW_READ_SLOT64_15);
#undef RSGPU_JW_RD
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        W[2 * q] = (uint32_t)P[q];
        W[2 * q + 1] = (uint32_t)(P[q] >> 32);
    }
}

// The same decode with R rows per wave (rs_jit.h Wide): 2 waves per column
// tile; R = 16: 168 VGPRs (3 waves per SIMD), chunks of 6 sources (6
// workgroups per CU); R = 10: 120 VGPRs (4 waves per SIMD), chunks of 5 (8
// workgroups per CU).  The compiler gets v0..v39; the call clobbers
// v10..v39 and the accumulators, so what lives across it sits in v0..v8.
// hipcc warns that v129..v167 in the clobber lists are "reserved": it does
// not allocate them itself, and the kernel descriptor still gives the wave
// 168 VGPRs (.amdhsa_next_free_vgpr 168, no AGPRs), which only the asm and
// the generated code touch.
// NV = 4 (e > 32): four waves per tile, the same chunk of sources in LDS for
// all of them (rs_jit.h wide_waves / wide_row0), one tile per workgroup.
// TPW > 1 (NV = 2): one workgroup covers TPW consecutive column tiles of a block (2
// TPW waves; wave w: tile w / 2, rows of wave w % 2), so the TPW waves with
// the same rows run the same code between the same chunk barriers and share
// its instruction-cache lines.
template <class W, int TPW, int NV>
__global__ __launch_bounds__(64 * NV * TPW) __attribute__((amdgpu_num_vgpr(40))) void k_rs_jitw(JitArgs a)
{
    constexpr int CS = W::CS, R = W::R;
    __shared__ uint4 lds[2][TPW][CS * 2 * 64];
    RSGPU_DIAG_BEGIN()
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wave = wv % NV, tw = wv / NV;  // rows of the wave, its tile in the workgroup
    const int lane = threadIdx.x & 63;
    int b = blockIdx.y;
    long long tile = blockIdx.x;
    if (a.xcd_order) {  // as k_rs_jit
        const unsigned g = blockIdx.x + gridDim.x * blockIdx.y, tot = gridDim.x * gridDim.y;
        const unsigned xcd = g & 7, q8 = tot >> 3, r8 = tot & 7;
        const unsigned lin = xcd * q8 + min(xcd, r8) + (g >> 3);
        b = (int)(lin / gridDim.x);
        tile = lin - (unsigned)b * gridDim.x;
    }
    const long long wg = tile;  // this workgroup's index within its block
    tile = tile * TPW + tw;
    if (a.status && a.status[b] != 0)
        return;
    const int k = a.k;
    const int nch = (k + CS - 1) / CS;
    const int bw = (int)Hooks::data_block(b);
    const uint8_t* const* srcs = a.srcs + (size_t)bw * k;
    uint8_t* const* dsts = a.dsts + (size_t)bw * a.dst_stride;
    const uint8_t* code = a.code + (size_t)Hooks::code_block(b) * a.block_stride + (size_t)wave * nch * a.chunk_stride;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)&lds[0][tw][0];
    constexpr uint32_t kBuf = TPW * CS * 2 * 64 * 16;  // bytes between the two chunk buffers
    const long long off = Hooks::data_offset(tile * 2048 + lane * 32, tile, lane);
    // lanes past the row end re-read its head (results never stored; at C4
    // 24 of 64 lanes of every row's last tile).  Loading nothing there cut
    // the C4 decode's HBM bytes but not its time (3.26-3.28 vs 3.26-3.27 ms
    // per slice, same box x3, round 5): the head is in L2.
    const uint32_t loff = off + 32 <= a.len ? (uint32_t)off : 0u;
    if (wv == 0)
        asm volatile("s_icache_inv\n s_nop 15\n s_nop 15" ::: "memory");
    // the row pointers through the constant address space: scalar loads the
    // compiler issues together and waits for once, a chunk ahead of their
    // use (one s_load + wait per source measured 5-7 % of the wave's time)
    typedef const uint8_t* const __attribute__((address_space(4)))* CPtrs;
    const CPtrs csrcs = (CPtrs)srcs;
    constexpr int PW = (CS + NV - 1) / NV;  // this wave's sources per chunk: t = wave, wave + NV, ...
    auto ptrs = [&](int ch, const uint8_t* (&p)[PW]) {
        const int c0 = ch * CS, nt = min(CS, k - c0);
#pragma unroll
        for (int i = 0; i < PW; ++i)
            p[i] = csrcs[c0 + min(wave + NV * i, nt - 1)];  // in bounds, unconditional
    };
    // NOTE: the first word of chunk buffer 1 carries the chunk rotation
    // (below) until every wave has read it, before the first chunk barrier:
    // no LDS-DMA may target buffer 1 (par 1) before that barrier.
    auto issue = [&](int ch, int par, const uint8_t* const (&p)[PW]) {
        const int c0 = ch * CS, nt = min(CS, k - c0);
        const uint32_t base = lds0 + (uint32_t)(par * kBuf);
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            const int t = wave + NV * i;
            if (t < nt) {
                if (a.code_prefetch)  // short rows: keep the block's code in L2
                    glds32_nt(p[i], loff, base + (uint32_t)(t * 2 * 64 * 16));
                else
                    glds32(p[i], loff, base + (uint32_t)(t * 2 * 64 * 16));
            }
        }
    };
    if constexpr (R == 16)
        asm volatile(RSGPU_J16_ZERO ::: RSGPU_J16_ACC_CLOBBERS);
    else if constexpr (R == 12)
        asm volatile(RSGPU_J12_ZERO ::: RSGPU_J12_ACC_CLOBBERS);
    else
        asm volatile(RSGPU_J10_ZERO ::: RSGPU_J10_ACC_CLOBBERS);
    JitwPhases ph;
    // Wave priority: a wave's transposes up to the chunk barrier run at level
    // 2 (a.prio != 0, the default) over the other waves' generated code, so
    // the workgroup's last wave reaches the barrier sooner (same process ABBA,
    // round 6, profiles/r06_prio/: C3 decode -2.5 %, C4 slices -2 %, C5 -2.4 %)
    // The chunks' order is free (each chunk's code only adds into the
    // accumulators).  A rotation by the time the workgroup starts, chunk
    // (t / kRot) % nch first, keeps the workgroups that share a CU pair's
    // instruction cache at about the same chunk of their block's code
    // (workgroups that start later begin where the others are).
    // Rounded to the nearest period, so a workgroup starts with the chunk the
    // others are about to be in (same box x3, profiles/r05_rot/: C3 decode
    // 22.53-22.58 ms at 600 ticks, 23.04-23.08 in order; 450-800 all gain;
    // one process ABBA x10: the step -0.39 ms).  Re-picking the chunk before
    // every barrier by the clock measured 0.8 ms slower than this
    // (ab_knob_rot_mode2.json).
    int rot = 0;
    if (a.chunk_rot_ticks > 0) {
        // broadcast through the first word of chunk buffer 1, which no
        // LDS-DMA writes before the first chunk barrier: a separate
        // __shared__ int made the 10-row two-tile kernel 40964 bytes, four
        // bytes too many for four workgroups per CU
        volatile int& s_rot = *(volatile int*)&lds[1][0][0];
        if (threadIdx.x == 0) {
            unsigned long long t;
            asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            const unsigned long long p = (unsigned long long)a.chunk_rot_ticks;
            s_rot = (int)(((t + p / 2) / p) % (unsigned long long)nch);
        }
        __syncthreads();
        rot = __builtin_amdgcn_readfirstlane(s_rot);
    }
    auto chunk_of = [&](int i) { return i + rot >= nch ? i + rot - nch : i + rot; };
    const uint8_t* pc[PW];
    const uint8_t* pn[PW];
    ptrs(chunk_of(0), pc);
    issue(chunk_of(0), 0, pc);
    ptrs(chunk_of(min(1, nch - 1)), pn);
    if (a.code_prefetch) {
        // the block's workgroups split its code (both row halves) and pull
        // it into L2 with vector loads, every line in flight at once, so the
        // instruction fetch, which misses line by line, finds it there; the
        // wait also covers the sources just issued, needed next anyway
        const uint8_t* cb = a.code + (size_t)b * a.block_stride;
        const long long lines = ((long long)NV * nch * a.chunk_stride) >> 7;
        const long long lo = wg * lines / gridDim.x, hi = (wg + 1) * lines / gridDim.x;
        for (long long i = lo + threadIdx.x; i < hi; i += 64 * NV * TPW) {
            uint32_t d;
            asm volatile("global_load_dword %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(d) : "v"(cb + (i << 7)) : "memory");
        }
    }
    for (int i = 0; i < nch; ++i) {
        const int ch = chunk_of(i), par = i & 1;  // the chunk, its LDS buffer
        const int nt = min(CS, k - ch * CS);
        uint4* buf = lds[par][tw];
        ph.mark(0);  // phase 0: the previous call's return .. here (loop overhead, start)
        wait_vm(0);
        ph.mark(1);  // phase 1: this chunk's LDS-DMA
        if (a.prio)
            asm volatile("s_setprio 2" ::: "memory");
        {
            // (Tried, round 5: the wave's three sources' LDS reads batched in
            // hand-allocated asm, one exposed LDS latency per chunk instead of
            // three -- the step unchanged in a same-process ABBA x10,
            // profiles/r05_energy/ab_knob_asm_transposes.json; not kept.)
            const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
            for (int t = wave; t < nt && Hooks::kTransposes; t += NV) {
                uint4 u = buf[(t * 2 + 0) * 64 + lane], v = buf[(t * 2 + 1) * 64 + lane];
                uint32_t Wd[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
                tr8(Wd, m4, m2, m1);
                hook_planes<Hooks>(Wd);
                buf[(t * 2 + 0) * 64 + lane] = make_uint4(Wd[0], Wd[1], Wd[2], Wd[3]);
                buf[(t * 2 + 1) * 64 + lane] = make_uint4(Wd[4], Wd[5], Wd[6], Wd[7]);
            }
        }
        ph.mark(2);  // phase 2: transposes
        barrier_lds();
        ph.mark(3);  // phase 3: the chunk barrier
        if (a.prio)
            asm volatile("s_setprio 0" ::: "memory");
        if (i + 1 < nch)
            issue(chunk_of(i + 1), par ^ 1, pn);
        ptrs(chunk_of(min(i + 2, nch - 1)), pn);  // in flight during this chunk's code
        ph.mark(4);  // phase 4: next chunk's LDS-DMA issue, row pointers
        const uint32_t la = lds0 + (uint32_t)(par * kBuf) + lane * 16;
        const uint8_t* fn = code + (size_t)Hooks::code_chunk(ch, nt == CS) * a.chunk_stride;
        if constexpr (Hooks::kZeroValuPlanes)  // the diagnostic build's variant 3 (kernel_hooks.h)
            asm volatile("v_mov_b32 v10, 0\n v_mov_b32 v11, 0\n v_mov_b32 v12, 0\n v_mov_b32 v13, 0\n"
                         " v_mov_b32 v14, 0\n v_mov_b32 v15, 0\n v_mov_b32 v16, 0\n v_mov_b32 v17, 0"
                         ::: "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17");
        if constexpr (R == 16)
            asm volatile("s_swappc_b64 s[82:83], %[fn]"
                         :
                         : [fn] "s"(fn), "{v9}"(la)
                         : RSGPU_JW_CALL_CLOBBERS, "s82", "s83", "scc", "memory", RSGPU_J16_ACC_CLOBBERS);
        else if constexpr (R == 12)
            asm volatile("s_swappc_b64 s[82:83], %[fn]"
                         :
                         : [fn] "s"(fn), "{v9}"(la)
                         : RSGPU_JW_CALL_CLOBBERS, "s82", "s83", "scc", "memory", RSGPU_J12_ACC_CLOBBERS);
        else
            asm volatile("s_swappc_b64 s[82:83], %[fn]"
                         :
                         : [fn] "s"(fn), "{v9}"(la)
                         : RSGPU_JW_CALL_CLOBBERS, "s82", "s83", "scc", "memory", RSGPU_J10_ACC_CLOBBERS);
        ph.mark(5);  // phase 5: the generated code
    }
    // the output pointers likewise: all R loads under one wait
    typedef uint8_t* const __attribute__((address_space(4)))* CDsts;
    const int r0 = jit::wide_row0(a.rows, wave), nrow = jit::wide_row0(a.rows, wave + 1) - r0;
    uint8_t* dp[R];
#pragma unroll
    for (int i = 0; i < R; ++i)
        dp[i] = ((CDsts)dsts)[min(r0 + i, a.rows - 1)];
    if (off + 32 <= a.len) {
        const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
        [&]<int... Ss>(std::integer_sequence<int, Ss...>) {
            (
                [&] {
                    if (Ss < nrow) {
                        uint32_t Wd[8];
                        read_slotw<Ss>(Wd);
                        tr8(Wd, m4, m2, m1);
                        store32(dp[Ss], off, Wd);
                    }
                }(),
                ...);
        }(std::make_integer_sequence<int, R>{});
    }
    ph.mark(6);  // phase 6: output transposes and stores
    ph.end(wv);
    RSGPU_DIAG_END();
}

// every 8-byte slot a return: a call that lands in code never written
// comes straight back
__global__ void k_jit_fill(uint64_t* code, long long n)
{
    const uint64_t ret = (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        code[i] = ret;
}

RSGPU_DIAG_READER(diag_read_jitw)
RSGPU_DIAG_PHASE_READER(diag_read_jitw_phase)

}  // namespace jitk

// One workgroup per (block, wave), the wave's rows of the block's matrix
// staged in LDS first: a thread per (source, slot) writes that coefficient's
// eight multiply-accumulate words (one 64-byte run, consecutive threads
// consecutive runs), a thread per preamble word, then the chunks' ends.
// Layout as rs_jit.h describes; the words are those of jit::code_word (the
// host emitter the CPU suite interprets).  (Earlier forms: emission inside
// the prepare kernel, 0.41 ms at C3; one workgroup per (block, wave, chunk),
// dispatch-bound at 0.49 ms; one thread per word with the index arithmetic
// and the coefficient's matrix recomputed per word, 0.19 ms.)
__global__ __launch_bounds__(256) void k_jit_emit(int k, int e, const uint8_t* coef, const int* status,
                                                  uint8_t* code)
{
    __shared__ uint8_t cw[8 * 256];  // rows 8 w .. 8 w + 7 (k <= 250)
    const int b = blockIdx.y, w = blockIdx.x;
    if (status[b] != 0)
        return;
    const int nw = (e + 7) / 8, nch = (k + 7) / 8;
    const int nslot = min(8, e - 8 * w);
    const size_t stride = (size_t)jit::chunk_stride(8);
    uint8_t* cbase = code + ((size_t)b * nw + w) * nch * stride;
    const int sb = jit::src_bytes(nslot);
    for (int i = threadIdx.x; i < nslot * k; i += blockDim.x)
        cw[i] = coef[((size_t)b * e + 8 * w) * k + i];
    __syncthreads();
    for (int i = threadIdx.x; i < 8 * k; i += blockDim.x) {
        const int q = i >> 3, s = i & 7;
        if (s >= nslot)
            continue;
        const int ch = q >> 3, t = q & 7;
        uint64_t wd[8];
        jit::mac_words(cw[s * k + q], s, t & 1, wd);
        uint4* dst = reinterpret_cast<uint4*>(cbase + (size_t)ch * stride + jit::PRO_BYTES + (size_t)t * sb +
                                              jit::PRE_BYTES + 64 * s);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            dst[j] = make_uint4((uint32_t)wd[2 * j], (uint32_t)(wd[2 * j] >> 32), (uint32_t)wd[2 * j + 1],
                                (uint32_t)(wd[2 * j + 1] >> 32));
    }
    constexpr int PW = jit::PRE_BYTES / 8;  // preamble words per source
    for (int i = threadIdx.x; i < PW * k; i += blockDim.x) {
        const int q = i / PW, r = i - q * PW;
        const int ch = q >> 3, t = q & 7, nt = min(8, k - 8 * ch);
        reinterpret_cast<uint64_t*>(cbase + (size_t)ch * stride + jit::PRO_BYTES + (size_t)t * sb)[r] =
            (uint64_t)jit::pre_u32(t, nt, 2 * r + 1) << 32 | jit::pre_u32(t, nt, 2 * r);
    }
    for (int i = threadIdx.x; i < 3 * nch; i += blockDim.x) {  // prologue words, return
        const int ch = i / 3, o = i - 3 * ch, nt = min(8, k - 8 * ch);
        uint64_t word;
        (void)jit::code_word(cw, k, nslot, ch, o < 2 ? o : 2 + nt * (PW + 8 * nslot), &word);
        reinterpret_cast<uint64_t*>(cbase + (size_t)ch * stride)[o < 2 ? o : 2 + nt * (PW + 8 * nslot)] = word;
    }
}

// The word tables of k_jitw_emit (rs_jit.h wide_tables), built at compile time.
__constant__ jit::WideTables kWideTab = jit::wide_tables();

// k_rs_jitw<R>'s code (rs_jit.h Wide), one workgroup per (block, wave) as
// k_jit_emit: rows wide_row0(e, w) .. wide_row0(e, w + 1) - 1 of the block's decode rows.  Each word
// is a table entry (the coefficient's matrix row and register operands are
// fixed per (c, plane)) with the accumulator ORed in: per 16 bytes of code
// one 16-byte table load, two selects and ORs.  (Computing every word from
// the coefficient's 8 x 8 matrix took ~3500 VALU + 2400 SALU per wave; the
// emission of a C4 batch, 2.5 GB of code, 0.85-0.9 ms.)
// e > 64: one launch per pass of the rows (rs_jit.h wide_passes), rows
// row_base .. row_base + rows - 1 of the block's e decode rows, the pass's code
// at pass_off in each block's block_stride bytes.
template <class W>
__global__ __launch_bounds__(256) void k_jitw_emit(int k, int e, int row_base, int rows, long long block_stride,
                                                   long long pass_off, const uint8_t* coef, const int* status,
                                                   uint8_t* code)
{
    constexpr int R = W::R, CS = W::CS, PW = W::PRE / 8;
    static_assert(PW == jit::WideTables::PW && CS <= 6, "preamble table: PW words per source, chunk positions < 6");
    __shared__ uint8_t cw[R * 256];
    const int b = blockIdx.y, w = blockIdx.x;
    if (status[b] != 0)
        return;
    const int nch = (k + CS - 1) / CS;
    const int r0 = row_base + jit::wide_row0(rows, w), nslot = jit::wide_row0(rows, w + 1) - jit::wide_row0(rows, w);
    const size_t stride = (size_t)W::chunk_stride();
    uint8_t* cbase = code + (size_t)b * block_stride + pass_off + (size_t)w * nch * stride;
    const int sb = W::src_bytes(nslot);
    // every load of a phase in flight before its first use: the loops below
    // would otherwise wait a full memory latency per iteration
    {
        const uint8_t* cr = coef + ((size_t)b * e + r0) * k;
        constexpr int NB = R * 256 / 256;  // bytes per thread, nslot * k <= R * 250
        uint8_t v[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            const int i = threadIdx.x + 256 * j;
            v[j] = i < nslot * k ? cr[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j)
            cw[threadIdx.x + 256 * j] = v[j];
    }
    __syncthreads();
    // (source, slot) runs of 64 bytes, one 16-byte quarter (planes 2j, 2j+1)
    // per thread, so a wave's store covers 1 KB of consecutive code; U table
    // loads issued together
    constexpr int U = 8;
    for (int i0 = threadIdx.x; i0 < R * k * 4; i0 += 256 * U) {
        uint4 bw[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + 256 * u, run = i >> 2, q = run / R, s = run - q * R;
            const int c = i < R * k * 4 && s < nslot ? cw[s * k + q] : 0;
            bw[u] = *reinterpret_cast<const uint4*>(&kWideTab.mac[8 * c + 2 * (i & 3)]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + 256 * u, run = i >> 2, j = i & 3, q = run / R, s = run - q * R;
            if (i >= R * k * 4 || s >= nslot)
                continue;
            const int ch = q / CS, t = q - ch * CS;
            const int acc = W::ACC + 8 * s + 2 * j;
            const uint64_t w0 = W::with_acc((uint64_t)bw[u].y << 32 | bw[u].x, acc);
            const uint64_t w1 = W::with_acc((uint64_t)bw[u].w << 32 | bw[u].z, acc + 1);
            reinterpret_cast<uint4*>(cbase + (size_t)ch * stride + (size_t)t * sb + W::PRE + 64 * s)[j] =
                make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
        }
    }
    // preambles: this thread's words of the table are fixed by its index mod 14
    for (int i0 = threadIdx.x; i0 < PW * k; i0 += 256 * 4) {
        uint64_t pw[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + 256 * u, q = i / PW, r = i - q * PW, t = q % CS;
            pw[u] = kWideTab.pre[i < PW * k ? PW * t + r : 0];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + 256 * u, q = i / PW, r = i - q * PW;
            if (i >= PW * k)
                continue;
            const int ch = q / CS, t = q - ch * CS;
            reinterpret_cast<uint64_t*>(cbase + (size_t)ch * stride + (size_t)t * sb)[r] = pw[u];
        }
    }
    for (int ch = threadIdx.x; ch < nch; ch += blockDim.x) {  // returns
        const int nt = min(CS, k - CS * ch);
        reinterpret_cast<uint64_t*>(cbase + (size_t)ch * stride)[nt * (PW + 8 * nslot)] =
            (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
    }
}

// rows per wave of the 2-wave layout for e rows, 0 = the 8-row layout
// (e > 64: the layout of each pass, jitw_pass_rows)
int jitw_rows(int e)
{
    if (e > 32)  // four waves
        return e > 48 && e <= 64 ? 16 : e > 40 && e <= 64 ? 12 : e > 32 && e <= 64 ? 10 : 0;
    return e > 24 ? 16 : e > 20 ? 12 : e > 16 ? 10 : 0;
}

int jitw_rot_ticks(int rows)
{
    // one chunk's work per wave, CS (8 R + 24) VALU, times the waves sharing
    // a SIMD (4 for the 10-row kernels, 3 otherwise), scaled from C3's
    // measured optimum (R 16, CS 6, 3 waves: 600 ticks).  C5 (R 10): 456;
    // 500 measured 0.6 % faster than 342 and 200 1.1 % slower
    // (profiles/r05_rot/c5_period.json); 456 against 342 same process ABBA
    // x6: -0.14 ms per C5 step (c5_period_456_vs_342.json)
    const int r = jitw_rows(rows), cs = jitw_cs(rows), waves = r == 10 ? 4 : 3;
    return r ? 600 * cs * (8 * r + 24) * waves / (6 * (8 * 16 + 24) * 3) : 0;
}

int jitw_cs(int e) { return jitw_rows(e) == 16 ? jit::J16::CS : jitw_rows(e) == 12 ? jit::J12::CS : jit::J10::CS; }

size_t jitw_chunk_stride(int e)
{
    const int r = jitw_rows(e);
    return r == 16 ? jit::J16::chunk_stride() : r == 12 ? jit::J12::chunk_stride() : jit::J10::chunk_stride();
}

// the layout covers e: 16 < e <= 64 in one launch, 64 < e <= 125 in passes
bool jitw_layout(int e)
{
    return e > 16 && (e <= 64 || (e <= 128 && jitw_rows(jit::wide_pass_rows(e, 0)) &&
                                                        jitw_rows(jit::wide_pass_rows(e, jit::wide_passes(e) - 1))));
}

// one block's code of a pass of `rows` (<= 64) rows
size_t jitw_pass_bytes(int k, int rows)
{
    const int cs = jitw_cs(rows);
    return (size_t)jit::wide_waves(rows) * ((k + cs - 1) / cs) * jitw_chunk_stride(rows);
}

size_t jitw_pass_offset(int k, int e, int p)
{
    size_t o = 0;
    for (int q = 0; q < p; ++q)
        o += jitw_pass_bytes(k, jit::wide_pass_rows(e, q));
    return o;
}

size_t jitw_code_bytes(int k, int e, long long blocks)
{
    return (size_t)blocks * jitw_pass_offset(k, e, jit::wide_passes(e));
}

hipError_t launch_jitw_emit(int k, int e, long long blocks, const uint8_t* coef, const int* status,
                            uint8_t* code, hipStream_t st)
{
    if (k <= 0 || k > 250 || !jitw_layout(e) || k + e > 250 || blocks <= 0 || !coef || !status || !code)
        return hipErrorInvalidValue;
    const long long bs = (long long)jitw_code_bytes(k, e, 1);
    for (int p = 0; p < jit::wide_passes(e); ++p) {
        const int r0 = jit::wide_pass_row0(e, p), rows = jit::wide_pass_rows(e, p);
        const long long off = (long long)jitw_pass_offset(k, e, p);
        const dim3 grid(jit::wide_waves(rows), (unsigned)blocks);
        if (jitw_rows(rows) == 16)
            hipLaunchKernelGGL(k_jitw_emit<jit::J16>, grid, dim3(256), 0, st, k, e, r0, rows, bs, off, coef, status, code);
        else if (jitw_rows(rows) == 12)
            hipLaunchKernelGGL(k_jitw_emit<jit::J12>, grid, dim3(256), 0, st, k, e, r0, rows, bs, off, coef, status, code);
        else
            hipLaunchKernelGGL(k_jitw_emit<jit::J10>, grid, dim3(256), 0, st, k, e, r0, rows, bs, off, coef, status, code);
    }
    return hipGetLastError();
}

hipError_t launch_rs_jitw(const JitArgs& a, long long blocks, hipStream_t st)
{
    if (!jitw_rows(a.rows) || a.dst_stride < a.rows || a.k <= 0 || !a.code || a.chunk_stride <= 0)
        return hipErrorInvalidValue;
    // four waves per tile (e > 32): one tile per workgroup, three 4-wave
    // workgroups fill a CU's 12 wave slots
    const int nv = jit::wide_waves(a.rows);
    const int tpw = nv == 4 ? 1 : a.tiles_per_wg >= 3 ? 3 : a.tiles_per_wg == 2 ? 2 : 1;
    const long long ntile = (a.len + 2047) / 2048;
    dim3 grid((unsigned)((ntile + tpw - 1) / tpw), (unsigned)blocks);
    dim3 blk(64 * nv * tpw);
#define RSGPU_JW_LAUNCH(WT)                                                                          \
    if (nv == 4)                                                                                     \
        hipLaunchKernelGGL((jitk::k_rs_jitw<WT, 1, 4>), grid, blk, 0, st, a);                        \
    else                                                                                             \
        switch (tpw) {                                                                               \
        case 3: hipLaunchKernelGGL((jitk::k_rs_jitw<WT, 3, 2>), grid, blk, 0, st, a); break;        \
        case 2: hipLaunchKernelGGL((jitk::k_rs_jitw<WT, 2, 2>), grid, blk, 0, st, a); break;        \
        default: hipLaunchKernelGGL((jitk::k_rs_jitw<WT, 1, 2>), grid, blk, 0, st, a); break;       \
        }
    if (jitw_rows(a.rows) == 16) {
        RSGPU_JW_LAUNCH(jit::J16)
    } else if (jitw_rows(a.rows) == 12) {
        RSGPU_JW_LAUNCH(jit::J12)
    } else {
        RSGPU_JW_LAUNCH(jit::J10)
    }
#undef RSGPU_JW_LAUNCH
    return hipGetLastError();
}

size_t jit_code_bytes(int k, int e, long long blocks)
{
    const int nw = (e + 7) / 8, nch = (k + 7) / 8;
    return (size_t)blocks * nw * nch * jit::chunk_stride(8);
}

hipError_t launch_jit_fill(void* code, size_t bytes, hipStream_t st)
{
    hipLaunchKernelGGL(jitk::k_jit_fill, dim3(4096), dim3(256), 0, st, (uint64_t*)code,
                       (long long)(bytes / 8));
    return hipGetLastError();
}

hipError_t launch_jit_emit(int k, int e, long long blocks, const uint8_t* coef, const int* status,
                           uint8_t* code, hipStream_t st)
{
    if (k <= 0 || k > 250 || e <= 0 || k + e > 250 || blocks <= 0 || !coef || !status || !code)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_jit_emit, dim3((unsigned)((e + 7) / 8), (unsigned)blocks), dim3(256), 0, st, k, e,
                       coef, status, code);
    return hipGetLastError();
}

__global__ void k_jit_copy(uint64_t* dst, const uint64_t* src, long long n)
{
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// up to PutArgs::kWords 8-byte words from the kernel arguments to device
// memory: a small upload (a call's row pointers) without a host staging
// buffer, its copy and the host's wait for the previous one
__global__ void k_put_words(PutArgs a)
{
    if ((int)threadIdx.x < a.n)
        a.dst[threadIdx.x] = a.w[threadIdx.x];
}

hipError_t launch_put_words(void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (bytes % 8 || bytes > sizeof(PutArgs::w) || !dst)
        return hipErrorInvalidValue;
    PutArgs a{};
    a.dst = (uint64_t*)dst;
    a.n = (int)(bytes / 8);
    std::memcpy(a.w, src, bytes);
    hipLaunchKernelGGL(k_put_words, dim3(1), dim3(PutArgs::kWords), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_jit_copy(void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (bytes % 8)
        return hipErrorInvalidValue;
    const long long n = (long long)(bytes / 8);
    const unsigned grid = (unsigned)std::min<long long>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_jit_copy, dim3(grid), dim3(256), 0, st, (uint64_t*)dst, (const uint64_t*)src, n);
    return hipGetLastError();
}

hipError_t launch_rs_jit(const JitArgs& a, long long blocks, hipStream_t st)
{
    if (a.rows <= 0 || a.rows > 32 || a.dst_stride < a.rows || a.k <= 0 || !a.code || a.chunk_stride <= 0)
        return hipErrorInvalidValue;
    const int nw = (a.rows + 7) / 8;
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)blocks);
    const bool sh = a.block_stride == 0;
    switch (nw * 2 + (sh ? 1 : 0)) {
    case 2: hipLaunchKernelGGL((jitk::k_rs_jit<1, false>), grid, dim3(64), 0, st, a); break;
    case 3: hipLaunchKernelGGL((jitk::k_rs_jit<1, true>), grid, dim3(64), 0, st, a); break;
    case 4: hipLaunchKernelGGL((jitk::k_rs_jit<2, false>), grid, dim3(128), 0, st, a); break;
    case 5: hipLaunchKernelGGL((jitk::k_rs_jit<2, true>), grid, dim3(128), 0, st, a); break;
    case 6: hipLaunchKernelGGL((jitk::k_rs_jit<3, false>), grid, dim3(192), 0, st, a); break;
    case 7: hipLaunchKernelGGL((jitk::k_rs_jit<3, true>), grid, dim3(192), 0, st, a); break;
    case 8: hipLaunchKernelGGL((jitk::k_rs_jit<4, false>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((jitk::k_rs_jit<4, true>), grid, dim3(256), 0, st, a); break;
    }
    return hipGetLastError();
}

}  // namespace rsgpu
