// rsgpu_testhooks.cpp -- test and A/B hooks, built into their OWN library
// (rsgpu/librsgpu_testhooks.so), never into librsgpu.so, whose exports are
// exactly include/rsgpu.h (rsgpu.map).  The CPU suite interprets the code
// the host emitters write (tests/test_jit.py), the GPU suite compares the
// device emitter with them and drives the generated decode's layout knobs,
// and tools/ab_lib.py uses the knobs for same-box A/Bs.  The context hooks
// write fields of an rsgpu_ctx created by librsgpu.so (the struct is
// rsgpu_ctx.h, compiled into both); the emitters link their own copies of
// jit_prog.o and rs_jit.o.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/rsgpu.h"
#include "jit_prog.h"
#include "rs_jit.h"
#include "rs_kernels.h"
#include "rsgpu_ctx.h"

using namespace rsgpu;

namespace {

constexpr size_t kMaxGridBlocks = 65535;

// One pass's code in the two- / four-wave layout (rs_jit.h Wide<R, CS>):
// rows row_base .. row_base + rows - 1 of the e x k matrix coef, from
// Wide::code_word: wave w, chunk ch at (w nch + ch) chunk_stride from o64;
// unused words are returns.
template <class W>
void jitw_emit_host(int k, int row_base, int rows, const unsigned char* coef, uint64_t* o64)
{
    const int nch = (k + W::CS - 1) / W::CS, stride_w = W::chunk_stride() / 8;
    for (int w = 0; w < jit::wide_waves(rows); ++w) {
        const int r0 = row_base + jit::wide_row0(rows, w);
        const int nslot = jit::wide_row0(rows, w + 1) - jit::wide_row0(rows, w);
        const unsigned char* cr = coef + (size_t)r0 * k;
        for (int ch = 0; ch < nch; ++ch)
            for (int o = 0; o < stride_w; ++o) {
                uint64_t word;
                if (W::code_word(cr, k, nslot, ch, o, &word))
                    o64[((size_t)w * nch + ch) * stride_w + o] = word;
            }
    }
}

}  // namespace

extern "C" {

// Test / A-B hook (not part of include/rsgpu.h): column tiles per workgroup
// of the two-wave generated decode (1, 2, 3; 0 = the library's choice).
int rsgpu_internal_set_jitw_tiles(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < 0 || n > 3)
        return RSGPU_ERR_ARG;
    ctx->jitw_tpw = n;
    return RSGPU_OK;
}

// A-B hook (not part of include/rsgpu.h): k_rs_jitw's code prefetch into L2
// (0 off, 1 on, -1 the library's choice).
int rsgpu_internal_set_jitw_prefetch(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < -1 || n > 1)
        return RSGPU_ERR_ARG;
    ctx->jitw_prefetch = n;
    return RSGPU_OK;
}

// A-B hook (not part of include/rsgpu.h): k_rs_jitw's chunk rotation period
// in 100 MHz ticks (0 chunks in order, -1 the library's choice).
int rsgpu_internal_set_jitw_rot(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < -1 || n > 1000000)
        return RSGPU_ERR_ARG;
    ctx->jitw_rot = n;
    return RSGPU_OK;
}

// A-B hook (not part of include/rsgpu.h): the generated-code kernels
// (k_rs_jitw, k_rs_jit) raise their waves' priority (to level 2) from the
// transposes to the chunk barrier (n != 0, the default 2) or not (0).
int rsgpu_internal_set_jitw_prio(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < 0 || n > 3)
        return RSGPU_ERR_ARG;
    ctx->jitw_prio = n;
    return RSGPU_OK;
}

// A-B hook (not part of include/rsgpu.h): k_rs_bs raises its waves'
// priority (to level 2) from the transposes to the part barrier (n != 0, the
// default 2; its own instantiation) or not (0).
int rsgpu_internal_set_bs_prio(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < 0 || n > 3)
        return RSGPU_ERR_ARG;
    ctx->bs_prio = n;
    return RSGPU_OK;
}

// Test / A-B hook (not part of include/rsgpu.h): slices of the short-row
// generated decode whose prepare and emission run beside the decode
// (rsgpu_decode_blocks; 0 or 1 off, -1 the library's choice).
int rsgpu_internal_set_decode_pipeline(rsgpu_ctx* ctx, int n)
{
    if (!ctx || n < -1 || n > 64)
        return RSGPU_ERR_ARG;
    ctx->decode_pipe = n;
    return RSGPU_OK;
}

// Test hook (not in include/rsgpu.h): the host-built code of an e x k matrix
// shared by every block (jit_prog.h, the GENERATED encode), for the CPU
// suite to disassemble and interpret.  Returns the bytes needed, or -1;
// writes only when out_bytes is large enough; *chunk_stride gets the stride.
long long rsgpu_internal_jit_matrix_code(int k, int e, const unsigned char* coef, unsigned char* out,
                                         size_t out_bytes, int* chunk_stride, int max_ops)
{
    if (k <= 0 || k > 250 || e <= 0 || e > 255 || !coef || !chunk_stride)
        return -1;
    const std::vector<uint8_t> code = jit::build_matrix_code(coef, k, e, chunk_stride, max_ops);
    if (out && out_bytes >= code.size())
        std::memcpy(out, code.data(), code.size());
    return (long long)code.size();
}

// Test hook (not part of include/rsgpu.h): the generated decode code of ONE
// block for coefficient matrix coef[e][k], written on the host by the same
// emitters the prepare kernel runs (rs_jit.h), so the CPU suite can
// disassemble and interpret it.  Returns the bytes needed (jit_code_bytes)
// or -1 for bad arguments; writes only when out_bytes is large enough.
long long rsgpu_internal_jit_emit(int k, int e, const unsigned char* coef, unsigned char* out,
                                  size_t out_bytes)
{
    if (k <= 0 || e <= 0 || k + e > 250 || !coef)
        return -1;
    const size_t need = jit_code_bytes(k, e, 1);
    if (!out || out_bytes < need)
        return (long long)need;
    const int nw = (e + 7) / 8, nch = (k + 7) / 8, stride_w = jit::chunk_stride(8) / 8;
    uint64_t* o64 = reinterpret_cast<uint64_t*>(out);
    for (size_t i = 0; i < need / 8; ++i)
        o64[i] = (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
    // the words k_jit_emit writes, from the same function
    for (int w = 0; w < nw; ++w) {
        const int nslot = std::min(8, e - 8 * w);
        const unsigned char* rows = coef + (size_t)8 * w * k;
        for (int ch = 0; ch < nch; ++ch)
            for (int o = 0; o < stride_w; ++o) {
                uint64_t word;
                if (jit::code_word(rows, k, nslot, ch, o, &word))
                    o64[((size_t)w * nch + ch) * stride_w + o] = word;
            }
    }
    return (long long)need;
}

// Test hook (not part of include/rsgpu.h): the same for the two- and
// four-wave layouts of k_rs_jitw (rs_jit.h Wide, jitw_rows, wide_waves; e >
// 64 as passes of <= 64 rows, wide_passes), from Wide::code_word (the words
// k_jitw_emit writes).
long long rsgpu_internal_jitw_emit(int k, int e, const unsigned char* coef, unsigned char* out,
                                   size_t out_bytes)
{
    if (k <= 0 || !jitw_layout(e) || k + e > 250 || !coef)
        return -1;
    const size_t need = jitw_code_bytes(k, e, 1);
    if (!out || out_bytes < need)
        return (long long)need;
    uint64_t* o64 = reinterpret_cast<uint64_t*>(out);
    for (size_t i = 0; i < need / 8; ++i)
        o64[i] = (uint64_t)jit::S_NOP0 << 32 | jit::S_SETPC_82;
    for (int p = 0; p < jit::wide_passes(e); ++p) {  // passes of <= 64 rows (e > 64)
        const int r0 = jit::wide_pass_row0(e, p), rows = jit::wide_pass_rows(e, p);
        uint64_t* po = o64 + jitw_pass_offset(k, e, p) / 8;
        if (jitw_rows(rows) == 16)
            jitw_emit_host<jit::J16>(k, r0, rows, coef, po);
        else if (jitw_rows(rows) == 12)
            jitw_emit_host<jit::J12>(k, r0, rows, coef, po);
        else
            jitw_emit_host<jit::J10>(k, r0, rows, coef, po);
    }
    return (long long)need;
}

// Test hook (not in include/rsgpu.h): the host-built shared program of an
// e x k matrix in the two- or four-wave layout (16 < e <= 125; passes of <= 64
// rows above 64), built exactly as shared_program builds it, for the CPU suite
// to disassemble and interpret.  Returns the bytes needed, or -1; writes only
// when out_bytes is large enough; pass p's byte offset and chunk stride go to
// pass_off[p] / pass_stride[p] (p < max_passes), *npasses gets the count.
long long rsgpu_internal_jitw_matrix_code(int k, int e, const unsigned char* coef, unsigned char* out,
                                          size_t out_bytes, long long* pass_off, int* pass_stride, int max_passes,
                                          int* npasses, int max_ops)
{
    if (k <= 0 || k + e > 250 || !jitw_layout(e) || !coef || !pass_off || !pass_stride || !npasses)
        return -1;
    std::vector<std::pair<size_t, int>> passes;
    const std::vector<uint8_t> code = jit::build_matrix_code_wide_passes(coef, k, e, &passes, max_ops);
    if (code.empty() || (int)passes.size() > max_passes)
        return -1;
    *npasses = (int)passes.size();
    for (size_t p = 0; p < passes.size(); ++p) {
        pass_off[p] = (long long)passes[p].first;
        pass_stride[p] = passes[p].second;
    }
    if (out && out_bytes >= code.size())
        std::memcpy(out, code.data(), code.size());
    return (long long)code.size();
}

// Test hook (not part of include/rsgpu.h): the DEVICE emitter k_jitw_emit
// for `blocks` blocks of decode rows coef [blocks][e][k] (host memory), its
// code copied back into out (blocks x the bytes rsgpu_internal_jitw_emit
// returns for one block), so a GPU test compares it word for word with the
// host emitter the CPU suite interprets.  Returns the bytes, or -1.
long long rsgpu_internal_jitw_emit_device(rsgpu_ctx* ctx, int k, int e, size_t blocks,
                                          const unsigned char* coef, unsigned char* out, size_t out_bytes)
{
    if (!ctx || k <= 0 || !jitw_layout(e) || k + e > 250 || blocks == 0 || blocks > kMaxGridBlocks || !coef)
        return -1;
    const size_t need = jitw_code_bytes(k, e, (long long)blocks);
    if (!out || out_bytes < need)
        return (long long)need;
    uint8_t *d_coef = nullptr, *d_code = nullptr;
    int* d_status = nullptr;
    long long rc = -1;
    if (hipMalloc(&d_coef, blocks * e * k) == hipSuccess && hipMalloc(&d_code, need) == hipSuccess &&
        hipMalloc(&d_status, blocks * sizeof(int)) == hipSuccess &&
        hipMemcpyAsync(d_coef, coef, blocks * e * k, hipMemcpyHostToDevice, ctx->stream) == hipSuccess &&
        hipMemsetAsync(d_status, 0, blocks * sizeof(int), ctx->stream) == hipSuccess &&
        launch_jit_fill(d_code, need, ctx->stream) == hipSuccess &&
        launch_jitw_emit(k, e, (long long)blocks, d_coef, d_status, d_code, ctx->stream) == hipSuccess &&
        hipMemcpyAsync(out, d_code, need, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
        hipStreamSynchronize(ctx->stream) == hipSuccess)
        rc = (long long)need;
    (void)hipFree(d_coef);
    (void)hipFree(d_code);
    (void)hipFree(d_status);
    return rc;
}

}  // extern "C"
