// rsgpu_ctx.h -- the context behind include/rsgpu.h's opaque rsgpu_ctx
// (internal to librsgpu): its stream, grow-only device scratch, generated-code
// memory, the host-resident pipeline's streams and staging, and timing.
#pragma once
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <string>
#include <vector>

#include "../../include/rsgpu.h"

struct rsgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // cross-stream ordering events (rsgpu_set_stream), recycled round-robin
    std::vector<hipEvent_t> sync_evs;
    size_t sync_next = 0;
    // threaded-code kernel (rs_tc.hip): device table of the handler
    // addresses [slot][coefficient]; tc_state 0 = not probed, 1 = ready,
    // -1 = unavailable (k_dot_generic serves instead)
    unsigned long long* d_tc_table = nullptr;
    unsigned long long h_tc_table[2048] = {};
    unsigned long long tc_base = 0;  // first handler (the table is tc_base + i * stride)
    int tc_state = 0;
    int decode_kernel = RSGPU_DECODE_AUTO;
    int jitw_tpw = 0;  // k_rs_jitw column tiles per workgroup (0: by geometry)
    int jitw_prefetch = -1;  // k_rs_jitw code prefetch into L2 (-1: by geometry)
    int jitw_rot = -1;       // k_rs_jitw chunk rotation period, ticks (-1: by geometry, 0: off)
    // wave priority of k_rs_bs / k_rs_jitw / k_rs_jit from a chunk's transposes
    // to its barrier (0: off, the A/B hooks set it)
    int bs_prio = 2;
    int jitw_prio = 2;
    // short-row generated decode: prepare + emission on `aux` beside the
    // decode, in decode_pipe slices (-1: by geometry, 0 / 1: off)
    int decode_pipe = -1;
    hipStream_t aux = nullptr;
    // executable device memory for the generated decode code (rs_jit.h):
    // grow-only; jit_state 0 = not probed, 1 = pool found, -1 = unavailable
    void* d_jit = nullptr;
    size_t jit_bytes = 0;
    int jit_state = 0;
    // the code in d_jit belongs to ONE prepare: its key, and a generation
    // bumped by every emission and reallocation, checked by the apply
    unsigned long long jit_gen = 0;
    struct {
        int k = 0, e = 0;
        size_t blocks = 0;
        const void* ws = nullptr;
        unsigned long long gen = 0;
    } jit_key;
    hsa_amd_memory_pool_t jit_pool{};
    // host-built code of shared coefficient matrices (jit_prog.h), a small
    // LRU cache: key (k, rows, layout, coefficients), executable copy, chunk
    // stride, the wide layout's passes (rows > 64: code offset, chunk stride
    // each); the ordinary device buffer the code is staged through
    int encode_kernel = RSGPU_ENCODE_AUTO;
    struct SharedProg {
        std::vector<uint8_t> key;
        void* code = nullptr;
        size_t bytes = 0;
        int chunk_stride = 0;
        std::vector<std::pair<size_t, int>> passes;
        unsigned long long last = 0;
    };
    std::vector<SharedProg> progs;
    unsigned long long prog_tick = 0;
    void* d_code_stage = nullptr;
    size_t code_stage_bytes = 0;
    std::string err;
    // grow-only device scratch for pointer tables / coefficient tables
    void* d_scratch = nullptr;
    size_t scratch_bytes = 0;
    // pinned host staging for small uploads, guarded by an event
    void* h_stage = nullptr;
    size_t stage_bytes = 0;
    hipEvent_t stage_done = nullptr;
    bool stage_pending = false;
    // timing instrumentation
    bool timing = false;
    struct Rec {
        const char* name;
        hipEvent_t a, b;
        size_t blocks;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> ev_pool;
    // host-resident calls (rsgpu_encode_blocks_host / _decode_blocks_host):
    // copy-in and copy-out streams beside `stream`, grow-only device staging
    // slots, and the events that chain the three stages
    hipStream_t io_in = nullptr, io_out = nullptr;
    void* d_io = nullptr;
    size_t io_bytes = 0;
    std::vector<hipEvent_t> io_evs;
};


namespace rsgpu {

inline int fail(rsgpu_ctx* ctx, int code, const std::string& msg)
{
    if (ctx)
        ctx->err = msg;
    return code;
}

}  // namespace rsgpu

// a stream of the context's device, whatever device the calling thread has
// current (the thread's choice is restored)
inline hipError_t rsgpu_ctx_stream_create(const rsgpu_ctx* ctx, hipStream_t* s)
{
    int cur = -1;
    hipError_t e = hipGetDevice(&cur);
    if (e != hipSuccess)
        return e;
    if (cur != ctx->device && (e = hipSetDevice(ctx->device)) != hipSuccess)
        return e;
    e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    if (cur != ctx->device)
        (void)hipSetDevice(cur);
    return e;
}

#define RS_HIP(ctx, call)                                                                     \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return ::rsgpu::fail((ctx), RSGPU_ERR_HIP,                                        \
                                 std::string(#call) + ": " + hipGetErrorString(e_));          \
    } while (0)
