// rs_tc.hip -- bit-sliced GF(2^8) dot product with RUNTIME coefficients via
// threaded code: out_i = sum_p c[i][p] * src_p for per-block matrices c
// (the decode solve x = V_E^-1 s of the syndrome decoder, rsgpu_capi.cpp).
//
// The bit-sliced multiply-accumulate of one coefficient is 8 full-rate
// v_bitop3 whose REGISTER operands depend on the coefficient value
// (rs_bitsliced.hip, gen_tc_handlers.py).  Register numbers cannot be chosen
// at run time without indexing overhead, so all 256 variants exist as code:
// handler c (72 bytes, generated) applies coefficient c to accumulator slot 0
// from the four-Russians tables of the current source, and returns with
// s_setpc_b64.  The kernel dispatches one coefficient with
//     s_set_gpr_idx_on 8*slot, gpr_idx(SRC0,DST)   (accumulator slot)
//     s_swappc_b64 ret, addr[slot]                 (handler of the coefficient)
// where the 8 handler addresses of a source are one s_load_dwordx16 of a
// table the prepare kernel writes (address = base + c * 72).  Measured on
// gfx950: ~25-35 SIMD cycles per coefficient and 32 bytes, against ~120 for
// the v_perm table lookups of k_dot_generic (profiles/r1_ubench_jump.log).
//
// Register contract (gen_tc_handlers.py): accumulators v[64:127] (8 slots x 8
// planes), L/H tables v[32:61] with the source planes pinned at their
// single-bit entries, handler addresses s[64:79], return address s[82:83].
// The kernel therefore uses exactly 128 VGPRs: 4 waves per SIMD.
//
// Work split: as k_rs_bs -- a workgroup of NW waves covers 64 lanes x 32 bytes
// of every row of one block; wave w owns output rows [8w, 8w+8); the waves
// share the loading + bit transposing of each chunk of C sources through LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bitslice.h"
#include "rs_kernels.h"
#include "tc_handlers.inc"

namespace rsgpu {
namespace tc {

using bs::load32;
using bs::store32;
using bs::tr8;
using bs::vconst;

constexpr int C = 16;  // sources per LDS chunk

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

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_rs_tc(TcArgs a)
{
    __shared__ uint4 lds[C * 2 * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y;
    if (a.status && a.status[b] != 0)
        return;  // uniform per workgroup: the whole block is skipped
    const long long off = (long long)blockIdx.x * 2048 + lane * 32;
    const bool inb = off + 32 <= a.len;
    const int k = a.k;
    const uint8_t* const* srcs = a.srcs + (size_t)b * k;
    // addresses [B][k][NW*8]: this wave's 8 slots of source j at ap + j*NW*8
    const unsigned long long* ap = a.addr + (size_t)b * k * (NW * 8) + wave * 8;
    const uint32_t m4 = vconst(0x0F0F0F0Fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);

    uint32_t acc[64];
#pragma unroll
    for (int i = 0; i < 64; ++i)
        acc[i] = 0;

    for (int c0 = 0; c0 < k; c0 += C) {
        const int nt = min(C, k - c0);
        for (int t = wave; t < nt; t += NW) {
            uint32_t W[8];
            load32(srcs[c0 + t], off, inb, W);
            tr8(W, m4, m2, m1);
            lds[(t * 2 + 0) * 64 + lane] = make_uint4(W[0], W[1], W[2], W[3]);
            lds[(t * 2 + 1) * 64 + lane] = make_uint4(W[4], W[5], W[6], W[7]);
        }
        __syncthreads();
        for (int t = 0; t < nt; ++t) {
            const uint4 u = lds[(t * 2 + 0) * 64 + lane];
            const uint4 v = lds[(t * 2 + 1) * 64 + lane];
            const uint32_t P[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
            const unsigned long long* pa = ap + (size_t)(c0 + t) * (NW * 8);
            asm volatile(RSGPU_TC_CONSUME
                         : RSGPU_TC_ACC_OPS(acc)
                         : RSGPU_TC_PLANE_OPS(P), [pa] "s"(pa)
                         : RSGPU_TC_CLOBBERS);
        }
        __syncthreads();
    }

    if (!inb)
        return;
    uint8_t* const* dsts = a.dsts + (size_t)b * a.rows;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int r = wave * 8 + s;
        if (r < a.rows) {
            uint32_t W[8];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                W[q] = acc[s * 8 + q];
            tr8(W, m4, m2, m1);
            store32(dsts[r], off, W);
        }
    }
}

}  // namespace tc

hipError_t tc_query_handlers(unsigned long long* d_out, hipStream_t st)
{
    hipLaunchKernelGGL(tc::k_tc_handlers, dim3(1), dim3(64), 0, st, d_out);
    return hipGetLastError();
}

int tc_handler_stride() { return RSGPU_TC_STRIDE; }

int tc_rows_per_pass(int rows) { return rows <= 0 ? 8 : (rows + 7) / 8 * 8; }

hipError_t launch_rs_tc(const TcArgs& a, long long blocks, hipStream_t st)
{
    const int nw = tc_rows_per_pass(a.rows) / 8;
    dim3 grid((unsigned)((a.len + 2047) / 2048), (unsigned)blocks);
    switch (nw) {
    case 1: hipLaunchKernelGGL(tc::k_rs_tc<1>, grid, dim3(64), 0, st, a); break;
    case 2: hipLaunchKernelGGL(tc::k_rs_tc<2>, grid, dim3(128), 0, st, a); break;
    case 3: hipLaunchKernelGGL(tc::k_rs_tc<3>, grid, dim3(192), 0, st, a); break;
    case 4: hipLaunchKernelGGL(tc::k_rs_tc<4>, grid, dim3(256), 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rsgpu
