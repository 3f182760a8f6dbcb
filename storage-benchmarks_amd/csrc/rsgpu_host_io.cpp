// rsgpu_host_io.cpp -- the host-resident form of the hot path
// (include/rsgpu.h rsgpu_encode_blocks_host / rsgpu_decode_blocks_host).
//
// The reference keeps its blocks in host memory (isa.cpp:46-58: m buffers
// from posix_memalign, filled with rand(); the decoder's own buffers,
// isa.cpp:158-167) and times encode_all / decode_all over them.  Here a batch
// in host memory streams through device staging slots in chunks of blocks,
// three stages on three streams so that chunk i+1 crosses the link towards
// the GPU while chunk i is encoded or decoded and chunk i-1 comes back:
//   io_in        host -> device copies of the rows a stage reads
//   ctx->stream  rsgpu_encode_blocks / rsgpu_decode_blocks on the slot
//   io_out       device -> host copies of the rows it wrote
// Each slot's three events order its reuse: a slot's input rows are
// overwritten only after the kernel of the chunk that last used it finished,
// its output rows only after they were copied out.  The calls are
// synchronous: every output byte is in host memory on return.
//
// With pinned host memory (rsgpu_host_alloc) the copies are DMA at the link
// rate and overlap; pageable memory works, but the runtime copies it
// synchronously, so the stages run in series.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsgpu.h"
#include "rsgpu_ctx.h"

namespace {

using rsgpu::fail;

constexpr int kSlots = 3;
constexpr size_t kChunkBytes = size_t(128) << 20;  // device bytes per chunk (target)
constexpr size_t kMaxChunkBlocks = 65535;          // one grid's worth
// the decoder ships survivors as runs of consecutive rows when rows are at
// least this long; shorter rows go as whole blocks in one copy per chunk
// (the erased rows cross the link too, the kernels still never read them)
constexpr size_t kRunMinBytes = size_t(64) << 10;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

size_t chunk_blocks(size_t bytes_per_block, size_t blocks)
{
    size_t nb = std::max<size_t>(1, kChunkBytes / std::max<size_t>(1, bytes_per_block));
    return std::min({nb, blocks, kMaxChunkBlocks});
}

// Streams, staging of `bytes` and 3 kSlots events.  Growing the staging
// waits for every earlier host-resident call (they all synchronised before
// returning, so nothing in flight reads it).
int io_setup(rsgpu_ctx* ctx, size_t bytes)
{
    if (!ctx->io_in)
        RS_HIP(ctx, rsgpu_ctx_stream_create(ctx, &ctx->io_in));
    if (!ctx->io_out)
        RS_HIP(ctx, rsgpu_ctx_stream_create(ctx, &ctx->io_out));
    if (ctx->io_bytes < bytes) {
        if (ctx->d_io) {  // no copy or kernel of an earlier call may still use it
            RS_HIP(ctx, hipStreamSynchronize(ctx->io_in));
            RS_HIP(ctx, hipStreamSynchronize(ctx->io_out));
            RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
            RS_HIP(ctx, hipFree(ctx->d_io));
            ctx->d_io = nullptr;
            ctx->io_bytes = 0;
        }
        RS_HIP(ctx, hipMalloc(&ctx->d_io, bytes));
        ctx->io_bytes = bytes;
    }
    while (ctx->io_evs.size() < 3 * kSlots) {
        hipEvent_t e = nullptr;
        RS_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->io_evs.push_back(e);
    }
    return RSGPU_OK;
}

// rows x len bytes between pitches (one 2D copy; a plain one when both
// pitches are equal)
hipError_t copy_rows(void* dst, size_t dpitch, const void* src, size_t spitch, size_t len, size_t rows,
                     hipMemcpyKind kind, hipStream_t st)
{
    if (rows == 0 || len == 0)
        return hipSuccess;
    if (dpitch == spitch)
        return hipMemcpyAsync(dst, src, (rows - 1) * spitch + len, kind, st);
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, len, rows, kind, st);
}

int finish_io(rsgpu_ctx* ctx)
{
    RS_HIP(ctx, hipStreamSynchronize(ctx->io_out));
    RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    RS_HIP(ctx, hipStreamSynchronize(ctx->io_in));
    return RSGPU_OK;
}

// Runs the pipeline body, then drains all three streams whatever it
// returned: no copy queued by the body may still move bytes into the
// caller's host buffers (or out of the staging) after the call returns.
template <class F>
int with_drain(rsgpu_ctx* ctx, F&& body)
{
    const int rc = body();
    const int rc2 = finish_io(ctx);
    return rc ? rc : rc2;
}

}  // namespace

extern "C" {

int rsgpu_host_alloc(rsgpu_ctx* ctx, void** hptr, size_t bytes)
{
    if (!ctx || !hptr)
        return RSGPU_ERR_ARG;
    if (hipHostMalloc(hptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return fail(ctx, RSGPU_ERR_NOMEM, "hipHostMalloc failed");
    return RSGPU_OK;
}

int rsgpu_host_free(rsgpu_ctx* ctx, void* hptr)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipHostFree(hptr));
    return RSGPU_OK;
}

int rsgpu_encode_blocks_host(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                             const unsigned char* h_src, unsigned char* h_parity,
                             const unsigned char* coef)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    if (k <= 0 || e < 0 || k + e > 255 || len > pitch || (blocks && (!h_src || !h_parity)))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_encode_blocks_host: bad arguments");
    if (e == 0 || len == 0 || blocks == 0)
        return RSGPU_OK;
    const size_t pd = align_up(len, 256);  // device rows: aligned for the fast kernels
    const size_t nb = chunk_blocks((size_t)(k + e) * pd, blocks);
    const size_t src_b = nb * k * pd, par_b = nb * e * pd, slot_b = src_b + par_b;
    int rc = io_setup(ctx, kSlots * slot_b);
    if (rc)
        return rc;
    const size_t nch = (blocks + nb - 1) / nb;
    return with_drain(ctx, [&]() -> int {
    for (size_t i = 0; i < nch; ++i) {
        const int s = (int)(i % kSlots);
        const size_t b0 = i * nb, n = std::min(nb, blocks - b0);
        unsigned char* d_src = (unsigned char*)ctx->d_io + s * slot_b;
        unsigned char* d_par = d_src + src_b;
        hipEvent_t ev_in = ctx->io_evs[3 * s], ev_cmp = ctx->io_evs[3 * s + 1], ev_out = ctx->io_evs[3 * s + 2];
        if (i >= kSlots)  // the slot's sources were read by chunk i - kSlots
            RS_HIP(ctx, hipStreamWaitEvent(ctx->io_in, ev_cmp, 0));
        RS_HIP(ctx, copy_rows(d_src, pd, h_src + b0 * k * pitch, pitch, len, n * k, hipMemcpyHostToDevice,
                              ctx->io_in));
        RS_HIP(ctx, hipEventRecord(ev_in, ctx->io_in));
        RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev_in, 0));
        if (i >= kSlots)  // its parity rows were copied out
            RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev_out, 0));
        const int rk = rsgpu_encode_blocks(ctx, k, e, len, pd, n, d_src, d_par, coef);
        if (rk)
            return rk;
        RS_HIP(ctx, hipEventRecord(ev_cmp, ctx->stream));
        RS_HIP(ctx, hipStreamWaitEvent(ctx->io_out, ev_cmp, 0));
        RS_HIP(ctx, copy_rows(h_parity + b0 * e * pitch, pitch, d_par, pd, len, n * e, hipMemcpyDeviceToHost,
                              ctx->io_out));
        RS_HIP(ctx, hipEventRecord(ev_out, ctx->io_out));
    }
    return RSGPU_OK;
    });
}

int rsgpu_decode_blocks_host(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                             const unsigned char* h_src, const unsigned char* h_parity,
                             const unsigned char* h_err, unsigned char* h_out, int* h_status)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    if (k <= 0 || e < 0 || e > k || k + e > 255 || len > pitch ||
        (blocks && e && (!h_src || !h_parity || !h_err || !h_out)))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_blocks_host: bad arguments");
    if (e == 0 || blocks == 0) {
        if (h_status)
            std::fill(h_status, h_status + blocks, 0);
        return RSGPU_OK;
    }
    const size_t pd = align_up(std::max<size_t>(len, 1), 256);
    const size_t nb = chunk_blocks((size_t)(k + 2 * e) * pd, blocks);
    const size_t ws_b = align_up(rsgpu_decode_workspace_bytes(k, e, nb), 256);
    const size_t src_b = nb * k * pd, par_b = nb * e * pd, out_b = nb * e * pd;
    const size_t slot_b = src_b + par_b + out_b + ws_b;
    // after the slots: every block's erasure list and status (one upload and
    // one download for the whole batch: no pageable copy inside the pipeline)
    const size_t err_off = kSlots * slot_b, st_off = align_up(err_off + blocks * e, 256);
    int rc = io_setup(ctx, st_off + blocks * sizeof(int));
    if (rc)
        return rc;
    unsigned char* d_err = (unsigned char*)ctx->d_io + err_off;
    int* d_status = (int*)((unsigned char*)ctx->d_io + st_off);
    const bool runs = len >= kRunMinBytes;
    std::vector<char> erased(k);
    const size_t nch = (blocks + nb - 1) / nb;
    rc = with_drain(ctx, [&]() -> int {
    RS_HIP(ctx, hipMemcpyAsync(d_err, h_err, blocks * e, hipMemcpyHostToDevice, ctx->io_in));
    for (size_t i = 0; i < nch; ++i) {
        const int s = (int)(i % kSlots);
        const size_t b0 = i * nb, n = std::min(nb, blocks - b0);
        unsigned char* d_src = (unsigned char*)ctx->d_io + s * slot_b;
        unsigned char* d_par = d_src + src_b;
        unsigned char* d_out = d_par + par_b;
        void* d_ws = d_out + out_b;
        hipEvent_t ev_in = ctx->io_evs[3 * s], ev_cmp = ctx->io_evs[3 * s + 1], ev_out = ctx->io_evs[3 * s + 2];
        if (i >= kSlots)
            RS_HIP(ctx, hipStreamWaitEvent(ctx->io_in, ev_cmp, 0));
        if (runs) {
            // what isa_decoder reads (isa.cpp:193-197): the surviving
            // originals, as runs of consecutive rows, and the parity rows
            for (size_t b = 0; b < n; ++b) {
                std::fill(erased.begin(), erased.end(), 0);
                for (int t = 0; t < e; ++t)
                    if (h_err[(b0 + b) * e + t] < k)
                        erased[h_err[(b0 + b) * e + t]] = 1;
                for (int j = 0; j < k;) {
                    if (erased[j]) {
                        ++j;
                        continue;
                    }
                    int j1 = j;
                    while (j1 < k && !erased[j1])
                        ++j1;
                    RS_HIP(ctx, copy_rows(d_src + (b * k + j) * pd, pd, h_src + ((b0 + b) * k + j) * pitch, pitch,
                                          len, (size_t)(j1 - j), hipMemcpyHostToDevice, ctx->io_in));
                    j = j1;
                }
            }
        } else {
            RS_HIP(ctx, copy_rows(d_src, pd, h_src + b0 * k * pitch, pitch, len, n * k, hipMemcpyHostToDevice,
                                  ctx->io_in));
        }
        RS_HIP(ctx, copy_rows(d_par, pd, h_parity + b0 * e * pitch, pitch, len, n * e, hipMemcpyHostToDevice,
                              ctx->io_in));
        RS_HIP(ctx, hipEventRecord(ev_in, ctx->io_in));
        RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev_in, 0));
        if (i >= kSlots)
            RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev_out, 0));
        const int rk = rsgpu_decode_blocks(ctx, k, e, len, pd, n, d_src, d_par, d_err + b0 * e, d_out, d_ws,
                                           d_status + b0);
        if (rk)
            return rk;
        RS_HIP(ctx, hipEventRecord(ev_cmp, ctx->stream));
        RS_HIP(ctx, hipStreamWaitEvent(ctx->io_out, ev_cmp, 0));
        RS_HIP(ctx, copy_rows(h_out + b0 * e * pitch, pitch, d_out, pd, len, n * e, hipMemcpyDeviceToHost,
                              ctx->io_out));
        RS_HIP(ctx, hipEventRecord(ev_out, ctx->io_out));
    }
    return RSGPU_OK;
    });
    if (rc)
        return rc;
    if (h_status)
        RS_HIP(ctx, hipMemcpy(h_status, d_status, blocks * sizeof(int), hipMemcpyDeviceToHost));
    return RSGPU_OK;
}

}  // extern "C"
