// rsgpu_capi.cpp -- C ABI of librsgpu (include/rsgpu.h): host GF helpers with
// ISA-L semantics, context/stream management, and the launch sequences of the
// batched encode / decode hot path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.h"
#include "rs_kernels.h"
#include "rs_synth.h"

struct rsgpu_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // second stream for the pipelined decode (syndrome chunk i+1 overlaps the
    // solve of chunk i); created on first use, joined back into `stream`
    hipStream_t aux = nullptr;
    int decode_chunks = 1;
    std::vector<hipEvent_t> sync_evs;
    size_t sync_next = 0;
    // threaded-code solve (rs_tc.hip): device table of the 256 handler
    // addresses; tc_state 0 = not probed, 1 = ready, -1 = unavailable
    unsigned long long* d_tc_table = nullptr;
    unsigned long long h_tc_table[2048] = {};  // [slot][coefficient]
    int tc_state = 0;
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
};

static bool use_tc(rsgpu_ctx* ctx, int e);

namespace {

using namespace rsgpu;

const GfTables& host_gf()
{
    static GfTables t = [] {
        GfTables x{};
        gf_build_tables(x);
        return x;
    }();
    return t;
}

inline uint8_t hmul(uint8_t a, uint8_t b)
{
    const GfTables& t = host_gf();
    return (a && b) ? t.exp[t.log[a] + t.log[b]] : 0;
}

int fail(rsgpu_ctx* ctx, int code, const std::string& msg)
{
    if (ctx)
        ctx->err = msg;
    return code;
}

#define RS_HIP(ctx, call)                                                                     \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail((ctx), RSGPU_ERR_HIP,                                                 \
                        std::string(#call) + ": " + hipGetErrorString(e_));                   \
    } while (0)

int ensure_scratch(rsgpu_ctx* ctx, size_t bytes)
{
    if (ctx->scratch_bytes >= bytes)
        return RSGPU_OK;
    if (ctx->d_scratch) {
        RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
        RS_HIP(ctx, hipFree(ctx->d_scratch));
        ctx->d_scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
    RS_HIP(ctx, hipMalloc(&ctx->d_scratch, want));
    ctx->scratch_bytes = want;
    return RSGPU_OK;
}

// Returns a pinned staging pointer of >= bytes, after the previous upload
// from it has completed.
int get_stage(rsgpu_ctx* ctx, size_t bytes, void** out)
{
    if (ctx->stage_pending) {
        RS_HIP(ctx, hipEventSynchronize(ctx->stage_done));
        ctx->stage_pending = false;
    }
    if (ctx->stage_bytes < bytes) {
        if (ctx->h_stage)
            RS_HIP(ctx, hipHostFree(ctx->h_stage));
        size_t want = bytes < (1u << 20) ? (1u << 20) : bytes;
        RS_HIP(ctx, hipHostMalloc(&ctx->h_stage, want));
        ctx->stage_bytes = want;
    }
    *out = ctx->h_stage;
    return RSGPU_OK;
}

int upload(rsgpu_ctx* ctx, void* d_dst, size_t bytes)
{
    RS_HIP(ctx, hipMemcpyAsync(d_dst, ctx->h_stage, bytes, hipMemcpyHostToDevice, ctx->stream));
    RS_HIP(ctx, hipEventRecord(ctx->stage_done, ctx->stream));
    ctx->stage_pending = true;
    return RSGPU_OK;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

hipEvent_t pool_event(rsgpu_ctx* ctx)
{
    if (!ctx->ev_pool.empty()) {
        hipEvent_t e = ctx->ev_pool.back();
        ctx->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

// Cross-stream ordering events (timing disabled), recycled round-robin: an
// event may be re-recorded once the stream that waits on it has been handed
// the wait, which hipStreamWaitEvent captures at enqueue time.
hipEvent_t sync_event(rsgpu_ctx* ctx)
{
    if (ctx->sync_evs.size() < 32) {
        hipEvent_t e = nullptr;
        (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        ctx->sync_evs.push_back(e);
        return e;
    }
    hipEvent_t e = ctx->sync_evs[ctx->sync_next];
    ctx->sync_next = (ctx->sync_next + 1) % ctx->sync_evs.size();
    return e;
}

// Number of block chunks for the two-stream decode: 1 (no overlap) for small
// batches; RSGPU_DECODE_CHUNKS overrides for experiments.
size_t decode_chunk_count(rsgpu_ctx* ctx, size_t blocks)
{
    size_t want = (size_t)ctx->decode_chunks;
    if (const char* v = std::getenv("RSGPU_DECODE_CHUNKS"))
        want = (size_t)std::max(1, std::atoi(v));
    const size_t by_size = blocks / 32;  // keep >= 32 blocks per chunk
    return std::max<size_t>(1, std::min(want, by_size));
}

// Brackets one kernel launch with events when timing is enabled.
struct KTimer {
    rsgpu_ctx* ctx;
    hipStream_t s;
    rsgpu_ctx::Rec rec{};
    KTimer(rsgpu_ctx* c, const char* name, size_t blocks, hipStream_t st = nullptr)
        : ctx(c), s(st ? st : c->stream)
    {
        if (!ctx->timing)
            return;
        rec.name = name;
        rec.blocks = blocks;
        rec.a = pool_event(ctx);
        rec.b = pool_event(ctx);
        (void)hipEventRecord(rec.a, s);
    }
    ~KTimer()
    {
        if (!ctx->timing)
            return;
        (void)hipEventRecord(rec.b, s);
        ctx->recs.push_back(rec);
    }
};

size_t tc_table_bytes(int k, int rows);
void tc_fill_addr(const rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, unsigned long long* h);
int tc_launch_shared(rsgpu_ctx* ctx, const unsigned long long* d_addr, int k, int rows, long long len,
                     long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                     const char* timer_name);

// Runtime-coefficient dot product through the threaded-code kernel: host
// coefficients coef[rows][k] become one handler-address table [k][slots]
// shared by every block (uploaded to scratch at tab_off); rows <= 32, len %
// 32 == 0, 16-byte aligned rows behind the device pointer tables.
int tc_from_host_coef(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, long long len,
                      long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                      size_t tab_off, const char* timer_name);

// Fill host tables [k][rows_pad] for coefficient matrix coef[rows][k]
// (coef row r column j at coef[r*k + j]).
void fill_tables(const uint8_t* coef, int k, int rows, int rows_pad, uint4* t4, uint32_t* tc)
{
    for (int j = 0; j < k; ++j)
        for (int r = 0; r < rows_pad; ++r) {
            uint32_t t[5] = {0, 0, 0, 0, 0};
            if (r < rows)
                perm_tables(coef[(size_t)r * k + j], t);
            t4[(size_t)j * rows_pad + r] = make_uint4(t[0], t[1], t[2], t[3]);
            tc[(size_t)j * rows_pad + r] = t[4];
        }
}

int rows_pad_for(int rows)
{
    const int R = generic_rows_per_pass(rows);
    return (rows + R - 1) / R * R;
}

// Generic dot product launch from HOST coefficients coef[rows][k] over
// device pointer tables already in place (d_srcs [blocks][k], d_dsts
// [blocks][rows]).  Uploads the tables into scratch at offset `tab_off`.
int generic_from_host_coef(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, long long len,
                           long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                           size_t tab_off, bool bytewise)
{
    const int rows_pad = rows_pad_for(rows);
    const size_t n = (size_t)k * rows_pad;
    const size_t bytes4 = n * sizeof(uint4), bytesc = n * sizeof(uint32_t);
    void* stage;
    int rc = get_stage(ctx, bytes4 + bytesc, &stage);
    if (rc)
        return rc;
    uint4* t4 = (uint4*)stage;
    uint32_t* tc = (uint32_t*)((char*)stage + bytes4);
    fill_tables(coef, k, rows, rows_pad, t4, tc);
    char* d = (char*)ctx->d_scratch + tab_off;
    rc = upload(ctx, d, bytes4 + bytesc);
    if (rc)
        return rc;
    DotArgs a{};
    a.srcs = d_srcs;
    a.dsts = d_dsts;
    a.tabs4 = (const uint4*)d;
    a.ctab = (const uint32_t*)(d + bytes4);
    a.tab_block_stride = 0;
    a.k = k;
    a.rows = rows;
    a.rows_pad = rows_pad;
    a.len = len;
    a.blocks = blocks;
    a.status = nullptr;
    a.bytewise = bytewise;
    {
        KTimer kt(ctx, "k_dot_generic", (size_t)blocks);
        RS_HIP(ctx, launch_dot_generic(a, ctx->stream));
    }
    return RSGPU_OK;
}

}  // namespace

extern "C" {

const char* rsgpu_version(void) { return "0.1.0"; }

int rsgpu_create(int device, rsgpu_ctx** out)
{
    if (!out)
        return RSGPU_ERR_ARG;
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess)
        return RSGPU_ERR_HIP;
    rsgpu_ctx* c = new rsgpu_ctx();
    c->device = device;
    if (hipEventCreateWithFlags(&c->stage_done, hipEventDisableTiming) != hipSuccess) {
        delete c;
        return RSGPU_ERR_HIP;
    }
    *out = c;
    return RSGPU_OK;
}

int rsgpu_destroy(rsgpu_ctx* ctx)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->aux) {
        (void)hipStreamSynchronize(ctx->aux);
        (void)hipStreamDestroy(ctx->aux);
    }
    if (ctx->d_scratch)
        (void)hipFree(ctx->d_scratch);
    if (ctx->h_stage)
        (void)hipHostFree(ctx->h_stage);
    if (ctx->stage_done)
        (void)hipEventDestroy(ctx->stage_done);
    for (auto& r : ctx->recs) {
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    for (auto e : ctx->ev_pool)
        (void)hipEventDestroy(e);
    for (auto e : ctx->sync_evs)
        (void)hipEventDestroy(e);
    if (ctx->d_tc_table)
        (void)hipFree(ctx->d_tc_table);
    delete ctx;
    return RSGPU_OK;
}

int rsgpu_set_stream(rsgpu_ctx* ctx, void* s)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    ctx->stream = (hipStream_t)s;
    return RSGPU_OK;
}

void* rsgpu_get_stream(rsgpu_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int rsgpu_synchronize(rsgpu_ctx* ctx)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RSGPU_OK;
}

const char* rsgpu_last_error(rsgpu_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int rsgpu_timing_enable(rsgpu_ctx* ctx, int on)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    ctx->timing = on != 0;
    return RSGPU_OK;
}

int rsgpu_timing_read(rsgpu_ctx* ctx, const char** names, float* ms, size_t* blocks, int max)
{
    if (!ctx || max < 0)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->aux)
        RS_HIP(ctx, hipStreamSynchronize(ctx->aux));
    int n = 0;
    for (auto& r : ctx->recs) {
        if (n < max) {
            float t = 0;
            (void)hipEventElapsedTime(&t, r.a, r.b);
            if (names)
                names[n] = r.name;
            if (ms)
                ms[n] = t;
            if (blocks)
                blocks[n] = r.blocks;
            ++n;
        }
        ctx->ev_pool.push_back(r.a);
        ctx->ev_pool.push_back(r.b);
    }
    ctx->recs.clear();
    return n;
}

int rsgpu_malloc(rsgpu_ctx* ctx, void** p, size_t bytes)
{
    if (!ctx || !p)
        return RSGPU_ERR_ARG;
    if (hipMalloc(p, bytes ? bytes : 1) != hipSuccess)
        return fail(ctx, RSGPU_ERR_NOMEM, "hipMalloc failed");
    return RSGPU_OK;
}

int rsgpu_free(rsgpu_ctx* ctx, void* p)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipFree(p));
    return RSGPU_OK;
}

int rsgpu_memcpy_h2d(rsgpu_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RSGPU_OK;
}

int rsgpu_memcpy_d2h(rsgpu_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    RS_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return RSGPU_OK;
}

// ---- host GF helpers -------------------------------------------------------

unsigned char rsgpu_gf_mul(unsigned char a, unsigned char b) { return hmul(a, b); }

unsigned char rsgpu_gf_inv(unsigned char a)
{
    const GfTables& t = host_gf();
    return a ? t.exp[255 - t.log[a]] : 0;
}

void rsgpu_gf_gen_rs_matrix(unsigned char* a, int m, int k)
{
    std::memset(a, 0, (size_t)m * k);
    for (int i = 0; i < k; ++i)
        a[(size_t)k * i + i] = 1;
    uint8_t gen = 1;
    for (int i = k; i < m; ++i) {
        uint8_t p = 1;
        for (int j = 0; j < k; ++j) {
            a[(size_t)k * i + j] = p;
            p = hmul(p, gen);
        }
        gen = hmul(gen, 2);
    }
}

void rsgpu_gf_gen_cauchy1_matrix(unsigned char* a, int m, int k)
{
    std::memset(a, 0, (size_t)m * k);
    for (int i = 0; i < k; ++i)
        a[(size_t)k * i + i] = 1;
    unsigned char* p = a + (size_t)k * k;
    for (int i = k; i < m; ++i)
        for (int j = 0; j < k; ++j)
            *p++ = rsgpu_gf_inv((unsigned char)(i ^ j));
}

int rsgpu_gf_invert_matrix(unsigned char* in, unsigned char* out, const int n)
{
    std::memset(out, 0, (size_t)n * n);
    for (int i = 0; i < n; ++i)
        out[(size_t)i * n + i] = 1;
    for (int i = 0; i < n; ++i) {
        if (in[(size_t)i * n + i] == 0) {
            int j = i + 1;
            while (j < n && in[(size_t)j * n + i] == 0)
                ++j;
            if (j == n)
                return -1;
            for (int c = 0; c < n; ++c) {
                std::swap(in[(size_t)i * n + c], in[(size_t)j * n + c]);
                std::swap(out[(size_t)i * n + c], out[(size_t)j * n + c]);
            }
        }
        const uint8_t piv = rsgpu_gf_inv(in[(size_t)i * n + i]);
        for (int c = 0; c < n; ++c) {
            in[(size_t)i * n + c] = hmul(in[(size_t)i * n + c], piv);
            out[(size_t)i * n + c] = hmul(out[(size_t)i * n + c], piv);
        }
        for (int r = 0; r < n; ++r) {
            if (r == i)
                continue;
            const uint8_t f = in[(size_t)r * n + i];
            if (!f)
                continue;
            for (int c = 0; c < n; ++c) {
                out[(size_t)r * n + c] ^= hmul(f, out[(size_t)i * n + c]);
                in[(size_t)r * n + c] ^= hmul(f, in[(size_t)i * n + c]);
            }
        }
    }
    return 0;
}

void rsgpu_gf_vect_mul_init(unsigned char c, unsigned char* tbl)
{
    for (int x = 0; x < 16; ++x) {
        tbl[x] = hmul(c, (uint8_t)x);
        tbl[16 + x] = hmul(c, (uint8_t)(x << 4));
    }
}

void rsgpu_ec_init_tables(int k, int rows, unsigned char* a, unsigned char* g)
{
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < k; ++j) {
            rsgpu_gf_vect_mul_init(*a++, g);
            g += 32;
        }
}

// ---- device, ISA-L-shaped ----------------------------------------------------

int rsgpu_ec_encode_data(rsgpu_ctx* ctx, int len, int k, int rows, const unsigned char* gftbls,
                         unsigned char** data, unsigned char** coding)
{
    if (!ctx || len < 0 || k <= 0 || rows < 0 || k > RSGPU_MAX_SOURCES || rows > 255 ||
        (rows > 0 && (!gftbls || !data || !coding)))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_ec_encode_data: bad arguments");
    if (rows == 0 || len == 0)
        return RSGPU_OK;
    // coefficient = tbl[1] of each 32-byte table (isa/ec_base.c:300)
    std::vector<uint8_t> coef((size_t)rows * k);
    for (int r = 0; r < rows; ++r)
        for (int j = 0; j < k; ++j)
            coef[(size_t)r * k + j] = gftbls[((size_t)r * k + j) * 32 + 1];
    bool aligned = true;
    for (int j = 0; j < k; ++j)
        aligned &= ((uintptr_t)data[j] & 15) == 0;
    for (int r = 0; r < rows; ++r)
        aligned &= ((uintptr_t)coding[r] & 15) == 0;
    const size_t ptr_bytes = align_up(sizeof(void*) * (size_t)(k + rows), 256);
    const int rows_pad = rows_pad_for(rows);
    const bool tcp = aligned && len % 32 == 0 && use_tc(ctx, rows);
    const size_t tab_bytes = tcp ? tc_table_bytes(k, rows)
                                 : (size_t)k * rows_pad * (sizeof(uint4) + sizeof(uint32_t));
    int rc = ensure_scratch(ctx, ptr_bytes + tab_bytes);
    if (rc)
        return rc;
    // pointer tables go through the same staging buffer after the tables:
    // stage layout [ptrs | tables] keeps one upload per call
    void* stage;
    rc = get_stage(ctx, ptr_bytes + tab_bytes, &stage);
    if (rc)
        return rc;
    void** hp = (void**)stage;
    for (int j = 0; j < k; ++j)
        hp[j] = data[j];
    for (int r = 0; r < rows; ++r)
        hp[k + r] = coding[r];
    if (tcp) {
        // bit-sliced threaded-code kernel (rs_tc.hip): any coefficient matrix
        tc_fill_addr(ctx, coef.data(), k, rows, (unsigned long long*)((char*)stage + ptr_bytes));
        rc = upload(ctx, ctx->d_scratch, ptr_bytes + tab_bytes);
        if (rc)
            return rc;
        char* d = (char*)ctx->d_scratch;
        return tc_launch_shared(ctx, (const unsigned long long*)(d + ptr_bytes), k, rows, len, 1,
                                (const uint8_t* const*)d, (uint8_t* const*)(d + sizeof(void*) * k),
                                "k_rs_tc(ec_encode_data)");
    }
    uint4* t4 = (uint4*)((char*)stage + ptr_bytes);
    uint32_t* tc = (uint32_t*)((char*)t4 + (size_t)k * rows_pad * sizeof(uint4));
    fill_tables(coef.data(), k, rows, rows_pad, t4, tc);
    rc = upload(ctx, ctx->d_scratch, ptr_bytes + tab_bytes);
    if (rc)
        return rc;
    char* d = (char*)ctx->d_scratch;
    DotArgs a{};
    a.srcs = (const uint8_t* const*)d;
    a.dsts = (uint8_t* const*)(d + sizeof(void*) * k);
    a.tabs4 = (const uint4*)(d + ptr_bytes);
    a.ctab = (const uint32_t*)(d + ptr_bytes + (size_t)k * rows_pad * sizeof(uint4));
    a.tab_block_stride = 0;
    a.k = k;
    a.rows = rows;
    a.rows_pad = rows_pad;
    a.len = len;
    a.blocks = 1;
    a.status = nullptr;
    a.bytewise = !aligned;
    RS_HIP(ctx, launch_dot_generic(a, ctx->stream));
    return RSGPU_OK;
}

int rsgpu_ec_encode_data_update(rsgpu_ctx* ctx, int len, int k, int rows, int vec_i,
                                const unsigned char* gftbls, unsigned char* data,
                                unsigned char** coding)
{
    if (!ctx || len < 0 || k <= 0 || rows < 0 || vec_i < 0 || vec_i >= k || rows > 255 ||
        (rows > 0 && (!gftbls || !data || !coding)))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_ec_encode_data_update: bad arguments");
    if (rows == 0 || len == 0)
        return RSGPU_OK;
    const size_t ptr_bytes = align_up(sizeof(void*) * (size_t)rows, 256);
    const size_t tab_bytes = (size_t)rows * (sizeof(uint4) + sizeof(uint32_t));
    int rc = ensure_scratch(ctx, ptr_bytes + tab_bytes);
    if (rc)
        return rc;
    void* stage;
    rc = get_stage(ctx, ptr_bytes + tab_bytes, &stage);
    if (rc)
        return rc;
    void** hp = (void**)stage;
    for (int r = 0; r < rows; ++r)
        hp[r] = coding[r];
    uint4* t4 = (uint4*)((char*)stage + ptr_bytes);
    uint32_t* tc = (uint32_t*)((char*)t4 + (size_t)rows * sizeof(uint4));
    for (int r = 0; r < rows; ++r) {
        uint32_t t[5];
        // coefficient of (row r, column vec_i): tbl[1] (isa/ec_base.c:316)
        perm_tables(gftbls[((size_t)r * k + vec_i) * 32 + 1], t);
        t4[r] = make_uint4(t[0], t[1], t[2], t[3]);
        tc[r] = t[4];
    }
    rc = upload(ctx, ctx->d_scratch, ptr_bytes + tab_bytes);
    if (rc)
        return rc;
    char* d = (char*)ctx->d_scratch;
    RS_HIP(ctx, launch_update(data, (uint8_t* const*)d, (const uint4*)(d + ptr_bytes),
                              (const uint32_t*)(d + ptr_bytes + (size_t)rows * sizeof(uint4)),
                              rows, len, ctx->stream));
    return RSGPU_OK;
}

// ---- device, batched -----------------------------------------------------------

static int check_geom(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    if (k <= 0 || e < 0 || k + e > RSGPU_MAX_SOURCES || pitch < len || blocks == 0)
        return fail(ctx, RSGPU_ERR_ARG, "bad geometry (k, e, len, pitch, blocks)");
    return RSGPU_OK;
}

int rsgpu_encode_blocks(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char* d_src, unsigned char* d_parity,
                        const unsigned char* coef)
{
    int rc = check_geom(ctx, k, e, len, pitch, blocks);
    if (rc)
        return rc;
    if (e == 0 || len == 0)
        return RSGPU_OK;
    const bool aligned = ((uintptr_t)d_src % 16 == 0) && ((uintptr_t)d_parity % 16 == 0) &&
                         (pitch % 16 == 0);
    // Fast paths: the gf_gen_rs_matrix code with compile-time coefficients,
    // bit-sliced (len % 32 == 0) or nibble-table (len % 4 == 0).
    if (!coef && aligned && len % 32 == 0 && rs_bitsliced_available(k, e)) {
        KTimer kt(ctx, "k_rs_bs(encode)", blocks);
        RS_HIP(ctx, launch_rs_bitsliced(k, e, d_src, nullptr, d_parity, (long long)pitch,
                                        (long long)len, (long long)blocks, nullptr, ctx->stream));
        return RSGPU_OK;
    }
    if (!coef && aligned && len % 4 == 0 && rs_encode_specialized_available(k, e)) {
        KTimer kt(ctx, "k_rs_encode_lh", blocks);
        RS_HIP(ctx, launch_rs_encode_specialized(k, e, d_src, d_parity, (long long)pitch,
                                                 (long long)len, (long long)blocks, ctx->stream));
        return RSGPU_OK;
    }
    std::vector<uint8_t> c((size_t)e * k);
    if (coef) {
        std::memcpy(c.data(), coef, c.size());
    } else {
        std::vector<uint8_t> a((size_t)(k + e) * k);
        rsgpu_gf_gen_rs_matrix(a.data(), k + e, k);
        std::memcpy(c.data(), a.data() + (size_t)k * k, c.size());
    }
    const size_t src_ptr_bytes = align_up(sizeof(void*) * (size_t)k * blocks, 256);
    const size_t dst_ptr_bytes = align_up(sizeof(void*) * (size_t)e * blocks, 256);
    const int rows_pad = rows_pad_for(e);
    const size_t tab_bytes = std::max((size_t)k * rows_pad * (sizeof(uint4) + sizeof(uint32_t)),
                                      tc_table_bytes(k, e));
    rc = ensure_scratch(ctx, src_ptr_bytes + dst_ptr_bytes + tab_bytes);
    if (rc)
        return rc;
    char* d = (char*)ctx->d_scratch;
    RS_HIP(ctx, launch_row_ptrs(d_src, (long long)pitch, k, (long long)blocks,
                                (const uint8_t**)d, ctx->stream));
    RS_HIP(ctx, launch_row_ptrs(d_parity, (long long)pitch, e, (long long)blocks,
                                (const uint8_t**)(d + src_ptr_bytes), ctx->stream));
    if (aligned && len % 32 == 0 && use_tc(ctx, e))
        return tc_from_host_coef(ctx, c.data(), k, e, (long long)len, (long long)blocks,
                                 (const uint8_t* const*)d, (uint8_t* const*)(d + src_ptr_bytes),
                                 src_ptr_bytes + dst_ptr_bytes, "k_rs_tc(encode)");
    return generic_from_host_coef(ctx, c.data(), k, e, (long long)len, (long long)blocks,
                                  (const uint8_t* const*)d, (uint8_t* const*)(d + src_ptr_bytes),
                                  src_ptr_bytes + dst_ptr_bytes, !aligned);
}

// Locate the handler table of k_rs_tc once per context: the query kernel
// reports the table's first and end addresses; the layout must be exactly
// tc_handler_count() handlers of tc_handler_stride() bytes, otherwise the
// threaded-code path stays off (and k_dot_generic solves).  The address
// table has 2048 entries: [slot][coefficient], each the handler copy that
// serves the slot (tc_slot_copy).
static int tc_init(rsgpu_ctx* ctx)
{
    if (ctx->tc_state != 0)
        return ctx->tc_state;
    ctx->tc_state = -1;
    unsigned long long* d = nullptr;
    if (hipMalloc((void**)&d, 2050 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    unsigned long long se[2] = {0, 0};
    if (tc_query_handlers(d + 2048, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(se, d + 2048, sizeof se, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
        (void)hipFree(d);
        return -1;
    }
    const unsigned long long stride = (unsigned long long)tc_handler_stride();
    const unsigned long long count = (unsigned long long)tc_handler_count();
    if (se[0] == 0 || se[1] - se[0] != count * stride || count % 256 != 0 || count > 2048) {
        std::fprintf(stderr, "rsgpu: threaded-code handler table has an unexpected layout "
                             "(%#llx..%#llx); using k_dot_generic\n", se[0], se[1]);
        (void)hipFree(d);
        return -1;
    }
    unsigned long long h[2048];
    for (int s = 0; s < 8; ++s)
        for (int c = 0; c < 256; ++c)
            h[s * 256 + c] = se[0] + (unsigned long long)(tc_slot_copy(s) * 256 + c) * stride;
    if (hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return -1;
    }
    std::memcpy(ctx->h_tc_table, h, sizeof h);
    ctx->d_tc_table = d;
    ctx->tc_state = 1;
    return 1;
}

namespace {

size_t tc_table_bytes(int k, int rows)
{
    return sizeof(unsigned long long) * (size_t)k * tc_rows_per_pass(rows);
}

void tc_fill_addr(const rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, unsigned long long* h)
{
    const int slots = tc_rows_per_pass(rows);
    for (int j = 0; j < k; ++j)
        for (int s = 0; s < slots; ++s)
            h[(size_t)j * slots + s] = ctx->h_tc_table[(s & 7) * 256 + (s < rows ? coef[(size_t)s * k + j] : 0)];
}

int tc_launch_shared(rsgpu_ctx* ctx, const unsigned long long* d_addr, int k, int rows, long long len,
                     long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                     const char* timer_name)
{
    TcArgs t{};
    t.srcs = d_srcs;
    t.dsts = d_dsts;
    t.addr = d_addr;
    t.addr_stride = 0;
    t.k = k;
    t.rows = rows;
    t.len = len;
    t.status = nullptr;
    KTimer kt(ctx, timer_name, (size_t)blocks);
    RS_HIP(ctx, launch_rs_tc(t, blocks, ctx->stream));
    return RSGPU_OK;
}

int tc_from_host_coef(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, long long len,
                      long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                      size_t tab_off, const char* timer_name)
{
    const size_t bytes = tc_table_bytes(k, rows);
    void* stage;
    int rc = get_stage(ctx, bytes, &stage);
    if (rc)
        return rc;
    tc_fill_addr(ctx, coef, k, rows, (unsigned long long*)stage);
    char* d = (char*)ctx->d_scratch + tab_off;
    rc = upload(ctx, d, bytes);
    if (rc)
        return rc;
    return tc_launch_shared(ctx, (const unsigned long long*)d, k, rows, len, blocks, d_srcs, d_dsts,
                            timer_name);
}

}  // namespace

// The threaded-code solve serves e <= 32 on the syndrome path.  Decided once
// per context (RSGPU_NO_TC=1 at first use selects k_dot_generic instead, for
// comparison), so prepare and apply always agree on the workspace contents.
static bool use_tc(rsgpu_ctx* ctx, int e)
{
    if (e > 32)
        return false;
    if (ctx->tc_state == 0) {
        const char* v = std::getenv("RSGPU_NO_TC");
        if (v && v[0] == '1')
            ctx->tc_state = -1;
    }
    return tc_init(ctx) == 1;
}

// Decode kernels of the syndrome path once threaded code is available
// (RSGPU_DECODE, read once per process):
//   direct (default)  one matrix: k_rs_tc over the k - e survivors and the e
//                     parity rows with the e x k decode rows (one pass, HBM
//                     traffic (k + e) L per block)
//   fused             k_rs_decode_fused: syndromes + e x e solve per tile
//                     (the default for k 100, e 20, where it measured faster)
//                     (instantiated codes only)
//   split             k_rs_bs syndromes to HBM, then the in-place k_rs_tc solve
// RSGPU_NO_FUSED=1 (older switch) means split.
enum class DecodeMode { direct, fused, split };

static DecodeMode decode_mode(int k, int e)
{
    // -1: no override, per-code default below
    static const int forced = [] {
        const char* v = std::getenv("RSGPU_DECODE");
        const char* nf = std::getenv("RSGPU_NO_FUSED");
        if (v && std::strcmp(v, "fused") == 0)
            return (int)DecodeMode::fused;
        if ((v && std::strcmp(v, "split") == 0) || (nf && nf[0] == '1'))
            return (int)DecodeMode::split;
        if (v && std::strcmp(v, "direct") == 0)
            return (int)DecodeMode::direct;
        return -1;
    }();
    DecodeMode m = DecodeMode::direct;
    if (forced >= 0)
        m = (DecodeMode)forced;
    else if (k == 100 && e == 20)
        m = DecodeMode::fused;  // measured 2 % faster there (BASELINE C5)
    if (m == DecodeMode::fused && !rs_decode_fused_available(k, e))
        return DecodeMode::split;
    return m;
}

static bool use_fused(rsgpu_ctx*, int k, int e) { return decode_mode(k, e) == DecodeMode::fused; }
static bool use_direct(rsgpu_ctx*, int k, int e) { return decode_mode(k, e) == DecodeMode::direct; }

// Syndrome decode (bit-sliced syndromes + runtime e x e in place) applies to
// the instantiated codes with 32-byte-multiple rows; otherwise the direct
// k x k inversion + e x k dot product.
static bool use_syn_path(int k, int e, size_t len, size_t pitch, const void* src, const void* par,
                         const void* out)
{
    return rs_bitsliced_available(k, e) && len % 32 == 0 && pitch % 16 == 0 &&
           (uintptr_t)src % 16 == 0 && (uintptr_t)par % 16 == 0 && (uintptr_t)out % 16 == 0;
}

// General decode (k x k inversion) through k_rs_tc: e <= 32 with 32-byte
// multiple, 16-byte aligned rows (RSGPU_NO_TC=1 keeps k_dot_generic).
static bool use_tc_general(rsgpu_ctx* ctx, int e, size_t len, size_t pitch, const void* src,
                           const void* par, const void* out)
{
    return len % 32 == 0 && pitch % 16 == 0 && (uintptr_t)src % 16 == 0 && (uintptr_t)par % 16 == 0 &&
           (uintptr_t)out % 16 == 0 && use_tc(ctx, e);
}

static void decode_ws_layout(int k, int e, size_t blocks, size_t* off_surv, size_t* off_out,
                             size_t* off_t4, size_t* off_tc, size_t* off_tca, size_t* off_sa,
                             size_t* total)
{
    const int rows_pad = rows_pad_for(e);
    size_t o = 16 * blocks;  // emask [blocks][2] u64 at offset 0
    o = align_up(o, 256);
    *off_surv = o;
    o = align_up(o + sizeof(void*) * (size_t)k * blocks, 256);
    *off_out = o;
    o = align_up(o + sizeof(void*) * (size_t)e * blocks, 256);
    *off_t4 = o;
    o = align_up(o + sizeof(uint4) * (size_t)k * rows_pad * blocks, 256);
    *off_tc = o;
    o = align_up(o + sizeof(uint32_t) * (size_t)k * rows_pad * blocks, 256);
    // k_rs_tc handler addresses: [blocks][e][tc_rows] (split / fused solve)
    // or, for the one-matrix decode, [blocks][k][tc_rows] spanning this
    // region and the next one
    *off_tca = o;
    o = align_up(o + sizeof(unsigned long long) * (size_t)e * tc_rows_per_pass(e) * blocks, 256);
    *off_sa = o;  // fused decode: syndrome-phase handler addresses [blocks][k-e][tc_rows]
    o = align_up(o + sizeof(unsigned long long) * (size_t)(k > e ? k - e : 0) * tc_rows_per_pass(e) *
                         blocks,
                 256);
    *total = o;
}

size_t rsgpu_decode_workspace_bytes(int k, int e, size_t blocks)
{
    if (k <= 0 || e <= 0)
        return 256;
    size_t a, b, c, d, x, y, t;
    decode_ws_layout(k, e, blocks, &a, &b, &c, &d, &x, &y, &t);
    return t;
}

int rsgpu_decode_prepare(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                         const unsigned char* d_src, const unsigned char* d_parity,
                         const unsigned char* d_err, unsigned char* d_out, void* d_workspace,
                         int* d_status)
{
    int rc = check_geom(ctx, k, e, len, pitch, blocks);
    if (rc)
        return rc;
    if (e == 0)
        return RSGPU_OK;
    if (e > k || !d_err || !d_workspace || !d_status)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_prepare: bad arguments");
    size_t o_surv, o_out, o_t4, o_tc, o_tca, o_sa, total;
    decode_ws_layout(k, e, blocks, &o_surv, &o_out, &o_t4, &o_tc, &o_tca, &o_sa, &total);
    char* ws = (char*)d_workspace;
    const int rows_pad = rows_pad_for(e);
    if (use_syn_path(k, e, len, pitch, d_src, d_parity, d_out)) {
        const bool tcp = use_tc(ctx, e);
        KTimer kt(ctx, "k_decode_prepare_syn", blocks);
        RS_HIP(ctx, launch_decode_prepare_syn(
                        k, e, rows_pad, (long long)blocks, d_err, d_out, (long long)pitch,
                        (const uint8_t**)(ws + o_surv), (uint8_t**)(ws + o_out),
                        tcp ? nullptr : (uint4*)(ws + o_t4), tcp ? nullptr : (uint32_t*)(ws + o_tc),
                        (long long)e * rows_pad, tcp ? ctx->d_tc_table : nullptr,
                        tcp ? (unsigned long long*)(ws + o_tca) : nullptr, tc_rows_per_pass(e),
                        (unsigned long long*)ws, d_status,
                        tcp && use_fused(ctx, k, e) ? (unsigned long long*)(ws + o_sa) : nullptr,
                        d_src, d_parity,
                        tcp && use_direct(ctx, k, e) ? (unsigned long long*)(ws + o_tca) : nullptr,
                        ctx->stream));
        return RSGPU_OK;
    }
    PrepArgs p{};
    p.k = k;
    p.e = e;
    p.rows_pad = rows_pad;
    p.blocks = (long long)blocks;
    p.err = d_err;
    p.src = d_src;
    p.src_pitch = (long long)pitch;
    p.par = d_parity;
    p.par_pitch = (long long)pitch;
    p.out = d_out;
    p.out_pitch = (long long)pitch;
    p.surv_ptrs = (const uint8_t**)(ws + o_surv);
    p.out_ptrs = (uint8_t**)(ws + o_out);
    p.tabs4 = (uint4*)(ws + o_t4);
    p.ctab = (uint32_t*)(ws + o_tc);
    p.tab_block_stride = (long long)k * rows_pad;
    p.status = d_status;
    if (use_tc_general(ctx, e, len, pitch, d_src, d_parity, d_out)) {
        // [blocks][k][tc_rows] spans the tca and sa regions (k >= e)
        p.tc_table = ctx->d_tc_table;
        p.tc_addr = (unsigned long long*)(ws + o_tca);
        p.tc_rows = tc_rows_per_pass(e);
        p.tabs4 = nullptr;
        p.ctab = nullptr;
    }
    KTimer kt(ctx, "k_decode_prepare", blocks);
    RS_HIP(ctx, launch_decode_prepare(p, ctx->stream));
    return RSGPU_OK;
}

int rsgpu_decode_apply(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                       const unsigned char* d_src, const unsigned char* d_parity,
                       unsigned char* d_out, void* d_workspace, const int* d_status)
{
    int rc = check_geom(ctx, k, e, len, pitch, blocks);
    if (rc)
        return rc;
    if (e == 0 || len == 0)
        return RSGPU_OK;
    if (e > k || !d_workspace || !d_status)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_apply: bad arguments");
    size_t o_surv, o_out, o_t4, o_tc, o_tca, o_sa, total;
    decode_ws_layout(k, e, blocks, &o_surv, &o_out, &o_t4, &o_tc, &o_tca, &o_sa, &total);
    char* ws = (char*)d_workspace;
    const int rows_pad = rows_pad_for(e);
    if (use_syn_path(k, e, len, pitch, d_src, d_parity, d_out)) {
        // Syndromes into out (bit-sliced, memory-latency bound), then the
        // in-place e x e solve (VALU bound; blocks with a bad status are
        // skipped).  The blocks are cut into chunks and the two kernels run
        // on two streams so that the syndromes of chunk i+1 overlap the solve
        // of chunk i.
        const bool tcp = use_tc(ctx, e);
        if (tcp && use_direct(ctx, k, e)) {
            // one pass, one matrix (prepared by k_decode_prepare_syn)
            TcArgs t{};
            t.srcs = (const uint8_t* const*)(ws + o_surv);
            t.dsts = (uint8_t* const*)(ws + o_out);
            t.addr = (const unsigned long long*)(ws + o_tca);
            t.addr_stride = (long long)k * tc_rows_per_pass(e);
            t.k = k;
            t.rows = e;
            t.len = (long long)len;
            t.status = d_status;
            KTimer kt(ctx, "k_rs_tc(decode)", blocks);
            RS_HIP(ctx, launch_rs_tc(t, (long long)blocks, ctx->stream));
            return RSGPU_OK;
        }
        if (tcp && use_fused(ctx, k, e)) {
            // one pass: syndromes + solve per column tile (rs_decode_fused.hip)
            KTimer kt(ctx, "k_rs_decode_fused", blocks);
            RS_HIP(ctx, launch_rs_decode_fused(k, e, d_src, d_parity, d_out, (long long)pitch,
                                               (long long)len, (long long)blocks,
                                               (const uint64_t*)ws,
                                               (const unsigned long long*)(ws + o_tca),
                                               (const unsigned long long*)(ws + o_sa), d_status,
                                               ctx->stream));
            return RSGPU_OK;
        }
        const size_t chunks = decode_chunk_count(ctx, blocks);
        hipStream_t solve_stream = ctx->stream;
        if (chunks > 1) {
            if (!ctx->aux)
                RS_HIP(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
            solve_stream = ctx->aux;
        }
        const size_t per = (blocks + chunks - 1) / chunks;
        const long long tstride = (long long)e * rows_pad;
        for (size_t b0 = 0; b0 < blocks; b0 += per) {
            const size_t nb = std::min(per, blocks - b0);
            {
                KTimer kt(ctx, "k_rs_bs(syndrome)", nb);
                RS_HIP(ctx, launch_rs_bitsliced(k, e, d_src + b0 * k * pitch, d_parity + b0 * e * pitch,
                                                d_out + b0 * e * pitch, (long long)pitch,
                                                (long long)len, (long long)nb,
                                                (const uint64_t*)ws + 2 * b0, ctx->stream));
            }
            if (chunks > 1) {
                hipEvent_t ev = sync_event(ctx);
                RS_HIP(ctx, hipEventRecord(ev, ctx->stream));
                RS_HIP(ctx, hipStreamWaitEvent(solve_stream, ev, 0));
            }
            if (tcp) {
                TcArgs t{};
                t.srcs = (const uint8_t* const*)(ws + o_surv) + b0 * e;
                t.dsts = (uint8_t* const*)(ws + o_out) + b0 * e;
                t.addr = (const unsigned long long*)(ws + o_tca) + b0 * e * tc_rows_per_pass(e);
                t.addr_stride = (long long)e * tc_rows_per_pass(e);
                t.k = e;
                t.rows = e;
                t.len = (long long)len;
                t.status = d_status + b0;
                KTimer kt(ctx, "k_rs_tc(solve)", nb, solve_stream);
                RS_HIP(ctx, launch_rs_tc(t, (long long)nb, solve_stream));
                continue;
            }
            DotArgs a{};
            a.srcs = (const uint8_t* const*)(ws + o_surv) + b0 * e;
            a.dsts = (uint8_t* const*)(ws + o_out) + b0 * e;
            a.tabs4 = (const uint4*)(ws + o_t4) + b0 * tstride;
            a.ctab = (const uint32_t*)(ws + o_tc) + b0 * tstride;
            a.tab_block_stride = tstride;
            a.k = e;
            a.rows = e;
            a.rows_pad = rows_pad;
            a.len = (long long)len;
            a.blocks = (long long)nb;
            a.status = d_status + b0;
            a.bytewise = false;
            KTimer kt(ctx, "k_dot_generic(solve)", nb, solve_stream);
            RS_HIP(ctx, launch_dot_generic(a, solve_stream));
        }
        if (chunks > 1) {
            hipEvent_t ev = sync_event(ctx);
            RS_HIP(ctx, hipEventRecord(ev, solve_stream));
            RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ev, 0));
        }
        return RSGPU_OK;
    }
    if (use_tc_general(ctx, e, len, pitch, d_src, d_parity, d_out)) {
        // any geometry, e <= 32, 32-byte-multiple aligned rows: the rows of
        // inv(b) through the threaded-code kernel (prepared by k_decode_prepare)
        TcArgs t{};
        t.srcs = (const uint8_t* const*)(ws + o_surv);
        t.dsts = (uint8_t* const*)(ws + o_out);
        t.addr = (const unsigned long long*)(ws + o_tca);
        t.addr_stride = (long long)k * tc_rows_per_pass(e);
        t.k = k;
        t.rows = e;
        t.len = (long long)len;
        t.status = d_status;
        KTimer kt(ctx, "k_rs_tc(decode)", blocks);
        RS_HIP(ctx, launch_rs_tc(t, (long long)blocks, ctx->stream));
        return RSGPU_OK;
    }
    const bool aligned = ((uintptr_t)d_src % 16 == 0) && ((uintptr_t)d_parity % 16 == 0) &&
                         ((uintptr_t)d_out % 16 == 0) && (pitch % 16 == 0);
    DotArgs a{};
    a.srcs = (const uint8_t* const*)(ws + o_surv);
    a.dsts = (uint8_t* const*)(ws + o_out);
    a.tabs4 = (const uint4*)(ws + o_t4);
    a.ctab = (const uint32_t*)(ws + o_tc);
    a.tab_block_stride = (long long)k * rows_pad;
    a.k = k;
    a.rows = e;
    a.rows_pad = rows_pad;
    a.len = (long long)len;
    a.blocks = (long long)blocks;
    a.status = d_status;
    a.bytewise = !aligned;
    KTimer kt(ctx, "k_dot_generic(decode)", blocks);
    RS_HIP(ctx, launch_dot_generic(a, ctx->stream));
    return RSGPU_OK;
}

int rsgpu_decode_blocks(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char* d_src, const unsigned char* d_parity,
                        const unsigned char* d_err, unsigned char* d_out, void* d_workspace,
                        int* d_status)
{
    int rc = rsgpu_decode_prepare(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_err, d_out,
                                  d_workspace, d_status);
    if (rc)
        return rc;
    return rsgpu_decode_apply(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out, d_workspace,
                              d_status);
}

int rsgpu_verify_blocks(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char* d_src, const unsigned char* d_out,
                        const unsigned char* d_err, unsigned long long* d_mismatch)
{
    int rc = check_geom(ctx, k, e, len, pitch, blocks);
    if (rc)
        return rc;
    if (e == 0 || len == 0)
        return RSGPU_OK;
    RS_HIP(ctx, launch_compare_rows(d_src, (long long)pitch, k, d_out, (long long)pitch, e, d_err,
                                    (long long)len, (long long)blocks, d_mismatch, ctx->stream));
    return RSGPU_OK;
}

int rsgpu_fill_synthetic(rsgpu_ctx* ctx, unsigned char* d_rows, size_t rows, size_t len,
                         size_t pitch, uint64_t seed, uint64_t row0)
{
    if (!ctx || pitch < len)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_fill_synthetic: bad arguments");
    if (rows == 0 || len == 0)
        return RSGPU_OK;
    RS_HIP(ctx, launch_fill_synth(d_rows, (long long)rows, (long long)len, (long long)pitch, seed,
                                  row0, ctx->stream));
    return RSGPU_OK;
}

int rsgpu_erasure_patterns(uint64_t seed, uint64_t blk0, size_t blocks, int k, int e,
                           unsigned char* h_err)
{
    if (!h_err || k <= 0 || e < 0 || e > k || k > 256)
        return RSGPU_ERR_ARG;
    for (size_t b = 0; b < blocks; ++b)
        erasure_pattern(seed, blk0 + b, k, e, h_err + b * (size_t)e);
    return RSGPU_OK;
}

}  // extern "C"
