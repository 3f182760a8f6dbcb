// rsgpu_capi.cpp -- C ABI of librsgpu (include/rsgpu.h): host GF helpers with
// ISA-L semantics, context/stream management, and the launch sequences of the
// batched encode / decode hot path.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsgpu.h"
#include "gf256.h"
#include "rsgpu_ctx.h"
#include "jit_prog.h"
#include "rs_jit.h"
#include "rs_kernels.h"
#include "rs_synth.h"

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

// Grow the scratch buffer.  Every kernel that may still read the old buffer
// was enqueued on the context stream, or on an earlier stream the current
// one waits on (rsgpu_set_stream), so synchronising the current stream
// retires them all before the free.
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

// Brackets one kernel launch with events when timing is enabled.
struct KTimer {
    rsgpu_ctx* ctx;
    hipStream_t s;
    rsgpu_ctx::Rec rec{};
    KTimer(rsgpu_ctx* c, const char* name, size_t blocks) : KTimer(c, name, blocks, c->stream) {}
    KTimer(rsgpu_ctx* c, const char* name, size_t blocks, hipStream_t st) : ctx(c), s(st)
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

// Locate the handler table of k_rs_tc once per context: the query kernel
// reports the table's first and end addresses; the layout must be exactly
// tc_handler_count() handlers of tc_handler_stride() bytes, otherwise the
// threaded-code path stays off (and k_dot_generic serves).  The address
// table has 2048 entries: [slot][coefficient], each the handler copy that
// serves the slot (tc_slot_copy).
int tc_init(rsgpu_ctx* ctx)
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
    ctx->tc_base = se[0];
    ctx->d_tc_table = d;
    ctx->tc_state = 1;
    return 1;
}

bool tc_ready(rsgpu_ctx* ctx) { return tc_init(ctx) == 1; }

hsa_status_t pick_coarse_pool(hsa_amd_memory_pool_t p, void* out)
{
    hsa_amd_segment_t seg;
    if (hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && alloc) {
        *(hsa_amd_memory_pool_t*)out = p;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

// The device's coarse-grained pool, found through the owner of a hipMalloc'd
// probe (the HSA agent behind this HIP device): executable allocations for
// the generated decode code come from it.
int jit_probe(rsgpu_ctx* ctx)
{
    if (ctx->jit_state != 0)
        return ctx->jit_state;
    ctx->jit_state = -1;
    void* probe = nullptr;
    if (hipMalloc(&probe, 256) != hipSuccess)
        return -1;
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    const bool ok = hsa_amd_pointer_info(probe, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS;
    (void)hipFree(probe);
    if (!ok)
        return -1;
    hsa_amd_memory_pool_t pool{};
    pool.handle = 0;
    hsa_amd_agent_iterate_memory_pools(info.agentOwner, pick_coarse_pool, &pool);
    if (!pool.handle)
        return -1;
    ctx->jit_pool = pool;
    ctx->jit_state = 1;
    return 1;
}

// >= bytes of executable device memory, filled with returns when (re)made.
// Every kernel that may still execute the old code was enqueued on the
// context stream (or one it waits on): synchronising it retires them.
int jit_ensure(rsgpu_ctx* ctx, size_t bytes)
{
    if (ctx->jit_bytes >= bytes)
        return RSGPU_OK;
    if (jit_probe(ctx) != 1)
        return fail(ctx, RSGPU_ERR_UNSUPPORTED, "no executable device memory pool");
    if (ctx->d_jit) {
        RS_HIP(ctx, hipStreamSynchronize(ctx->stream));
        hsa_amd_memory_pool_free(ctx->d_jit);
        ctx->d_jit = nullptr;
        ctx->jit_bytes = 0;
    }
    const size_t want = std::max<size_t>(bytes, 1u << 20);
    void* p = nullptr;
    if (hsa_amd_memory_pool_allocate(ctx->jit_pool, want, HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, &p) !=
            HSA_STATUS_SUCCESS || !p)
        return fail(ctx, RSGPU_ERR_NOMEM, "executable device allocation failed");
    ctx->d_jit = p;
    ctx->jit_bytes = want;
    ++ctx->jit_gen;
    RS_HIP(ctx, launch_jit_fill(p, want, ctx->stream));
    return RSGPU_OK;
}

// The shared program of a matrix (jit_prog.h, composites by greedy cover):
// for 16 < rows <= 64 in the two- / four-wave layout of the decode (k_rs_jitw: a
// source's composites built twice or four times per tile), above 64 rows in
// passes of <= 64 in that layout (one program per pass, concatenated), else
// the 8-row layout (k_rs_jit).  Built on the host (~50 us for one row of 32
// sources, ~0.3 ms for 32 x 32) and kept in a per-context LRU cache of up to
// kProgCacheEntries programs / kProgCacheBytes, so a caller cycling through a
// few matrices (isa_arithmetic's one-output-per-call loop: 32 rows) builds
// each once.  Each program has its own executable buffer; an eviction waits
// for the context's stream first (a kernel in flight may run that code).
constexpr size_t kProgCacheEntries = 64;
constexpr size_t kProgCacheBytes = 256u << 20;

const rsgpu_ctx::SharedProg* shared_program(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, int* rc_out)
{
    *rc_out = RSGPU_OK;
    const bool wide = jitw_layout(rows);
    std::vector<uint8_t> key(9 + (size_t)k * rows);
    std::memcpy(key.data(), &k, 4);
    std::memcpy(key.data() + 4, &rows, 4);
    key[8] = wide ? 1 : 0;
    std::memcpy(key.data() + 9, coef, (size_t)k * rows);
    for (auto& pr : ctx->progs)
        if (pr.key == key) {
            pr.last = ++ctx->prog_tick;
            return &pr;
        }
    auto err = [&](int code, const char* msg) -> const rsgpu_ctx::SharedProg* {
        *rc_out = fail(ctx, code, msg);
        return nullptr;
    };
    if (jit_probe(ctx) != 1)
        return err(RSGPU_ERR_UNSUPPORTED, "no executable device memory pool");
    int stride = 0;
    std::vector<uint8_t> code;
    std::vector<std::pair<size_t, int>> passes;
    if (wide) {
        code = jit::build_matrix_code_wide_passes(coef, k, rows, &passes);
        if (code.empty())
            return err(RSGPU_ERR_UNSUPPORTED, "shared program: rows exceed the layout");
    } else {
        code = jit::build_matrix_code(coef, k, rows, &stride);
    }
    // room: least recently used programs out, after the stream has drained
    size_t used = 0;
    for (const auto& pr : ctx->progs)
        used += pr.bytes;
    if (!ctx->progs.empty() &&
        (ctx->progs.size() >= kProgCacheEntries || used + code.size() > kProgCacheBytes)) {
        if (hipStreamSynchronize(ctx->stream) != hipSuccess)
            return err(RSGPU_ERR_HIP, "shared program: draining the stream before an eviction");
        while (!ctx->progs.empty() &&
               (ctx->progs.size() >= kProgCacheEntries || used + code.size() > kProgCacheBytes)) {
            auto lru = std::min_element(ctx->progs.begin(), ctx->progs.end(),
                                        [](const auto& a, const auto& b) { return a.last < b.last; });
            used -= lru->bytes;
            hsa_amd_memory_pool_free(lru->code);
            ctx->progs.erase(lru);
        }
    }
    if (ctx->code_stage_bytes < code.size()) {
        if (hipStreamSynchronize(ctx->stream) != hipSuccess)
            return err(RSGPU_ERR_HIP, "shared program: draining the stream before regrowing the stage");
        if (ctx->d_code_stage)
            (void)hipFree(ctx->d_code_stage);
        ctx->d_code_stage = nullptr;
        ctx->code_stage_bytes = 0;
        if (hipMalloc(&ctx->d_code_stage, code.size()) != hipSuccess)
            return err(RSGPU_ERR_NOMEM, "shared program: code stage allocation failed");
        ctx->code_stage_bytes = code.size();
    }
    rsgpu_ctx::SharedProg pr;
    if (hsa_amd_memory_pool_allocate(ctx->jit_pool, code.size(), HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG,
                                     &pr.code) != HSA_STATUS_SUCCESS || !pr.code)
        return err(RSGPU_ERR_NOMEM, "executable device allocation failed");
    pr.bytes = code.size();
    void* stage;
    int rc = get_stage(ctx, code.size(), &stage);
    if (!rc) {
        std::memcpy(stage, code.data(), code.size());
        rc = upload(ctx, ctx->d_code_stage, code.size());
    }
    if (!rc && launch_jit_copy(pr.code, ctx->d_code_stage, code.size(), ctx->stream) != hipSuccess)
        rc = fail(ctx, RSGPU_ERR_HIP, "shared program: copy into executable memory");
    if (rc) {
        hsa_amd_memory_pool_free(pr.code);
        *rc_out = rc;
        return nullptr;
    }
    pr.key = std::move(key);
    pr.chunk_stride = stride;
    pr.passes = std::move(passes);
    pr.last = ++ctx->prog_tick;
    ctx->progs.push_back(std::move(pr));
    return &ctx->progs.back();
}

// dsts[b][i] = sum_j coef[i][j] srcs[b][j] through the shared generated code,
// in passes of <= 32 rows (aligned rows, len % 32 == 0)
int shared_program_launch(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, long long len,
                          long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                          const char* name)
{
    int rc = RSGPU_OK;
    const rsgpu_ctx::SharedProg* pg = shared_program(ctx, coef, k, rows, &rc);
    if (!pg)
        return rc;
    if (jitw_layout(rows)) {  // the two- / four-wave kernel, every block on the same code
        for (int p = 0; p < jit::wide_passes(rows); ++p) {  // one pass up to 64 rows
            JitArgs j{};
            j.srcs = d_srcs;
            j.dsts = d_dsts + jit::wide_pass_row0(rows, p);
            j.code = (const uint8_t*)pg->code + pg->passes[p].first;
            j.chunk_stride = pg->passes[p].second;
            j.block_stride = 0;
            j.k = k;
            j.rows = jit::wide_pass_rows(rows, p);
            j.dst_stride = rows;
            j.len = len;
            j.status = nullptr;
            j.tiles_per_wg = ctx->jitw_tpw ? ctx->jitw_tpw : 2;
            // every block on the same code: the start-time chunk rotation
            // (k_rs_jitw) lines up the workgroups of a CU pair on one chunk
            // (same-process ABBA x6, profiles/r05_rot/shared/: C5 encode 12.96
            // -> 12.37 ms, step -2.7 %; (48, 24) step -0.7 %; C3's generated
            // encode 22.65 -> 21.73 ms, still 1.7 % behind k_rs_bs)
            j.chunk_rot_ticks = ctx->jitw_rot >= 0 ? ctx->jitw_rot : jitw_rot_ticks(j.rows);
            j.prio = ctx->jitw_prio;
            KTimer kt(ctx, name, (size_t)blocks);
            RS_HIP(ctx, launch_rs_jitw(j, blocks, ctx->stream));
        }
        return RSGPU_OK;
    }
    const int nch = (k + 7) / 8;
    for (int p = 0; p * 32 < rows; ++p) {
        JitArgs j{};
        j.srcs = d_srcs;
        j.dsts = d_dsts + 32 * p;
        j.code = (const uint8_t*)pg->code + (size_t)p * 4 * nch * pg->chunk_stride;
        j.chunk_stride = pg->chunk_stride;
        j.block_stride = 0;
        j.k = k;
        j.rows = std::min(32, rows - 32 * p);
        j.dst_stride = rows;
        j.len = len;
        j.status = nullptr;
        // no wave priority for the shared 8-row program: (32, 8)'s encode
        // measured 15.25 -> 17.06 ms with it, (8, 2)'s +1 % (same process
        // ABBA x6, profiles/r06_prio/r06_prio_small_e/); the per-block 8-row
        // decode keeps it (16, 4) -1.4 %, (64, 16) -3.2 %
        j.prio = 0;
        KTimer kt(ctx, name, (size_t)blocks);
        RS_HIP(ctx, launch_rs_jit(j, blocks, ctx->stream));
    }
    return RSGPU_OK;
}

// Host-side handler addresses of coefficient matrix coef[rows][k] in the
// pass layout (rs_kernels.h tc_elem): pass p, source j, slot s -> row 32p + s.
void tc_fill_addr(const rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, unsigned long long* h)
{
    for (int p = 0; p < tc_passes(rows); ++p) {
        const int pr = tc_pass_rows(rows, p), slots = tc_rows_per_pass(pr);
        unsigned long long* hp = h + tc_pass_offset(k, p);
        for (int j = 0; j < k; ++j)
            for (int s = 0; s < slots; ++s)
                hp[(size_t)j * slots + s] =
                    ctx->h_tc_table[(s & 7) * 256 + (s < pr ? coef[(size_t)(32 * p + s) * k + j] : 0)];
    }
}

// k_rs_tc over `rows` output rows as passes of <= 32 rows: d_srcs [B][k],
// d_dsts [B][rows] device row-pointer tables, d_addr the pass-layout
// handler addresses, addr_stride elements between blocks' tables (0: one
// table shared by every block).
// (block, 2 KB tile) pairs below which a threaded-code pass of <= 8 rows
// splits each tile's sources over four waves (k_rs_tc_split): one wave per
// tile leaves most of the 1024 SIMDs idle and walks every source in series
// (C2: one block, 489 tiles)
constexpr long long kTcSplitMaxWork = 2048;

int tc_launch(rsgpu_ctx* ctx, const char* name, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
              const unsigned long long* d_addr, long long addr_stride, int k, int rows, long long len,
              long long blocks, const int* d_status)
{
    if (rows <= 8 && k >= 4 && (len + 2047) / 2048 * blocks < kTcSplitMaxWork) {
        TcArgs t{};
        t.srcs = d_srcs;
        t.dsts = d_dsts;
        t.dst_stride = rows;
        t.addr = d_addr;
        t.addr_stride = addr_stride;
        t.k = k;
        t.rows = rows;
        t.len = len;
        t.status = d_status;
        KTimer kt(ctx, name, (size_t)blocks);
        RS_HIP(ctx, launch_rs_tc_split(t, blocks, ctx->stream));
        return RSGPU_OK;
    }
    for (int p = 0; p < tc_passes(rows); ++p) {
        TcArgs t{};
        t.srcs = d_srcs;
        t.dsts = d_dsts + 32 * p;
        t.dst_stride = rows;
        t.addr = d_addr + tc_pass_offset(k, p);
        t.addr_stride = addr_stride;
        t.k = k;
        t.rows = tc_pass_rows(rows, p);
        t.len = len;
        t.status = d_status;
        KTimer kt(ctx, name, (size_t)blocks);
        RS_HIP(ctx, launch_rs_tc(t, blocks, ctx->stream));
    }
    return RSGPU_OK;
}

// Fill host v_perm tables [k][rows_pad] for coefficient matrix coef[rows][k]
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

// Runtime-coefficient dot product from HOST coefficients coef[rows][k] over
// device pointer tables (d_srcs [blocks][k], d_dsts [blocks][rows]), one
// coefficient table shared by every block, uploaded into scratch at
// tab_off: k_rs_tc for aligned 32-byte-multiple rows, otherwise
// k_dot_generic.  `pre` (pre_bytes <= tab_off, optional) goes to the start
// of scratch in the same upload (the pointer tables of ec_encode_data).
int dot_from_host_coef(rsgpu_ctx* ctx, const uint8_t* coef, int k, int rows, long long len,
                       long long blocks, const uint8_t* const* d_srcs, uint8_t* const* d_dsts,
                       size_t tab_off, bool aligned, const char* tc_name, const char* jit_name,
                       const void* pre = nullptr, size_t pre_bytes = 0)
{
    const bool tcp = aligned && len % 32 == 0 && tc_ready(ctx);
    if (aligned && len % 32 == 0 && ctx->encode_kernel != RSGPU_ENCODE_THREADED && jit_probe(ctx) == 1) {
        if (pre && pre_bytes <= sizeof(PutArgs::w) && pre_bytes % 8 == 0) {
            // a few row pointers (isa_arithmetic's per-row calls): through the
            // kernel arguments, no staging round trip
            RS_HIP(ctx, launch_put_words(ctx->d_scratch, pre, pre_bytes, ctx->stream));
        } else if (pre) {  // the row pointers the caller staged with the table upload
            void* stage;
            int rc = get_stage(ctx, pre_bytes, &stage);
            if (rc)
                return rc;
            std::memcpy(stage, pre, pre_bytes);
            rc = upload(ctx, ctx->d_scratch, pre_bytes);
            if (rc)
                return rc;
        }
        return shared_program_launch(ctx, coef, k, rows, len, blocks, d_srcs, d_dsts, jit_name);
    }
    const int rows_pad = rows_pad_for(rows);
    const size_t n = (size_t)k * rows_pad;
    const size_t bytes = tcp ? sizeof(unsigned long long) * (size_t)tc_table_elems(k, rows)
                             : n * (sizeof(uint4) + sizeof(uint32_t));
    const size_t skip = pre ? tab_off : 0;  // staging offset of the table
    void* stage;
    int rc = get_stage(ctx, skip + bytes, &stage);
    if (rc)
        return rc;
    if (pre)
        std::memcpy(stage, pre, pre_bytes);
    char* tab = (char*)stage + skip;
    char* d = (char*)ctx->d_scratch + tab_off;
    char* d_up = pre ? (char*)ctx->d_scratch : d;
    if (tcp) {
        tc_fill_addr(ctx, coef, k, rows, (unsigned long long*)tab);
        rc = upload(ctx, d_up, skip + bytes);
        if (rc)
            return rc;
        return tc_launch(ctx, tc_name, d_srcs, d_dsts, (const unsigned long long*)d, 0, k, rows, len,
                         blocks, nullptr);
    }
    uint4* t4 = (uint4*)tab;
    uint32_t* tc = (uint32_t*)(tab + n * sizeof(uint4));
    fill_tables(coef, k, rows, rows_pad, t4, tc);
    rc = upload(ctx, d_up, skip + bytes);
    if (rc)
        return rc;
    DotArgs a{};
    a.srcs = d_srcs;
    a.dsts = d_dsts;
    a.tabs4 = (const uint4*)d;
    a.ctab = (const uint32_t*)(d + n * sizeof(uint4));
    a.tab_block_stride = 0;
    a.k = k;
    a.rows = rows;
    a.rows_pad = rows_pad;
    a.len = len;
    a.blocks = blocks;
    a.status = nullptr;
    a.bytewise = !aligned;
    KTimer kt(ctx, "k_dot_generic", (size_t)blocks);
    RS_HIP(ctx, launch_dot_generic(a, ctx->stream));
    return RSGPU_OK;
}

// scratch bytes dot_from_host_coef needs for its table (either kernel)
size_t dot_table_bytes(int k, int rows)
{
    return std::max(sizeof(unsigned long long) * (size_t)tc_table_elems(k, rows),
                    (size_t)k * rows_pad_for(rows) * (sizeof(uint4) + sizeof(uint32_t)));
}

}  // namespace

extern "C" {

const char* rsgpu_version(void) { return "0.2.0"; }

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
    if (ctx->d_jit)
        hsa_amd_memory_pool_free(ctx->d_jit);
    for (auto& pr : ctx->progs)
        hsa_amd_memory_pool_free(pr.code);
    if (ctx->d_code_stage)
        (void)hipFree(ctx->d_code_stage);
    for (hipStream_t st : {ctx->io_in, ctx->io_out, ctx->aux})
        if (st) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    if (ctx->d_io)
        (void)hipFree(ctx->d_io);
    for (auto e : ctx->io_evs)
        (void)hipEventDestroy(e);
    delete ctx;
    return RSGPU_OK;
}

int rsgpu_set_stream(rsgpu_ctx* ctx, void* s)
{
    if (!ctx)
        return RSGPU_ERR_ARG;
    hipStream_t ns = (hipStream_t)s;
    if (ns == ctx->stream)
        return RSGPU_OK;
    // everything enqueued on the old stream (kernels reading the scratch
    // tables among them) is ordered before the new stream's work.  The
    // context moves to the new stream even when that cannot be arranged (an
    // old stream already destroyed): it is never left bound to a dead one;
    // the error is reported after the move.
    hipEvent_t ev = sync_event(ctx);
    hipError_t e = hipEventRecord(ev, ctx->stream);
    if (e == hipSuccess)
        e = hipStreamWaitEvent(ns, ev, 0);
    ctx->stream = ns;
    if (e != hipSuccess)
        return fail(ctx, RSGPU_ERR_HIP, std::string("rsgpu_set_stream: ordering against the old stream: ") +
                                            hipGetErrorString(e));
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
    int n = 0;
    for (auto& r : ctx->recs) {
        if (n < max) {
            float t = 0;
            (void)hipEventSynchronize(r.b);  // recorded on an earlier stream, possibly
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
    int rc = ensure_scratch(ctx, ptr_bytes + dot_table_bytes(k, rows));
    if (rc)
        return rc;
    // the row pointers go up in the same upload as the coefficient table
    std::vector<void*> hp((size_t)(k + rows));
    for (int j = 0; j < k; ++j)
        hp[j] = data[j];
    for (int r = 0; r < rows; ++r)
        hp[k + r] = coding[r];
    char* d = (char*)ctx->d_scratch;
    return dot_from_host_coef(ctx, coef.data(), k, rows, len, 1, (const uint8_t* const*)d,
                              (uint8_t* const*)(d + sizeof(void*) * k), ptr_bytes, aligned,
                              "k_rs_tc(ec_encode_data)", "k_rs_jit(ec_encode_data)", hp.data(),
                              sizeof(void*) * hp.size());
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

int rsgpu_gf_vect_dot_prod(rsgpu_ctx* ctx, int len, int vlen, const unsigned char* gftbls, unsigned char** src,
                           unsigned char* dest)
{
    if (!ctx || len < 0 || vlen <= 0 || !gftbls || !src || !dest)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_gf_vect_dot_prod: bad arguments");
    unsigned char* coding[1] = {dest};
    return rsgpu_ec_encode_data(ctx, len, vlen, 1, gftbls, src, coding);
}

int rsgpu_gf_vect_mad(rsgpu_ctx* ctx, int len, int vec, int vec_i, const unsigned char* gftbls, unsigned char* src,
                      unsigned char* dest)
{
    if (!ctx || len < 0 || vec <= 0 || vec_i < 0 || vec_i >= vec || !gftbls || !src || !dest)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_gf_vect_mad: bad arguments");
    unsigned char* coding[1] = {dest};
    return rsgpu_ec_encode_data_update(ctx, len, vec, 1, vec_i, gftbls, src, coding);
}

int rsgpu_gf_vect_mul(rsgpu_ctx* ctx, int len, const unsigned char* gftbl, void* src, void* dest)
{
    if (!ctx || len < 0 || len % 32 != 0 || !gftbl || !src || !dest)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_gf_vect_mul: len must be a multiple of 32 (gf_vect_mul.h:96-101)");
    unsigned char* data[1] = {(unsigned char*)src};
    unsigned char* coding[1] = {(unsigned char*)dest};
    return rsgpu_ec_encode_data(ctx, len, 1, 1, gftbl, data, coding);
}

// ---- device, batched -----------------------------------------------------------

// Most kernels put the block index in grid.y (or z), whose limit is 65535:
// the block-batched entry points run larger batches as consecutive slices.
constexpr size_t kMaxGridBlocks = 65535;

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
    if (blocks > kMaxGridBlocks) {
        for (size_t b0 = 0; b0 < blocks; b0 += kMaxGridBlocks) {
            rc = rsgpu_encode_blocks(ctx, k, e, len, pitch, std::min(kMaxGridBlocks, blocks - b0),
                                     d_src + b0 * k * pitch, d_parity + b0 * e * pitch, coef);
            if (rc)
                return rc;
        }
        return RSGPU_OK;
    }
    const bool aligned = ((uintptr_t)d_src % 16 == 0) && ((uintptr_t)d_parity % 16 == 0) &&
                         (pitch % 16 == 0);
    // Fast paths: the gf_gen_rs_matrix code with compile-time coefficients,
    // bit-sliced (len % 32 == 0) or nibble-table (len % 4 == 0).
    const bool compiled_ok = ctx->encode_kernel == RSGPU_ENCODE_AUTO || ctx->encode_kernel == RSGPU_ENCODE_COMPILED;
    if (compiled_ok && !coef && aligned && len % 32 == 0 && rs_bitsliced_split_available(k, e) &&
        (long long)((len + 2047) / 2048 * blocks) < kTcSplitMaxWork) {
        KTimer kt(ctx, "k_rs_bs_split(encode)", blocks);
        RS_HIP(ctx, launch_rs_bitsliced_split(k, e, d_src, d_parity, (long long)pitch, (long long)len,
                                              (long long)blocks, ctx->stream));
        return RSGPU_OK;
    }
    // AUTO leaves the compiled kernel when its waves own fewer than 8 rows and
    // the two-wave generated layout covers e (16 < e <= 32): (100, 20) builds
    // every source's composites per 5 rows there, per 10 rows in k_rs_jitw --
    // C5 encode 12.8-13.0 vs 14.4 ms (profiles/r03_ab/wide_encode/)
    const bool compiled_pays = ctx->encode_kernel == RSGPU_ENCODE_COMPILED ||
                               rs_bitsliced_rows_per_wave(k, e) >= 8 || !jitw_rows(e) ||
                               !(len % 32 == 0 && jit_probe(ctx) == 1);
    if (compiled_ok && compiled_pays && !coef && aligned && len % 32 == 0 && rs_bitsliced_available(k, e)) {
        KTimer kt(ctx, "k_rs_bs(encode)", blocks);
        RS_HIP(ctx, launch_rs_bitsliced(k, e, d_src, d_parity, (long long)pitch, (long long)len,
                                        (long long)blocks, ctx->stream, ctx->bs_prio));
        return RSGPU_OK;
    }
    if (compiled_ok && !coef && aligned && len % 4 == 0 && len % 32 != 0 &&
        rs_encode_specialized_available(k, e)) {
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
    rc = ensure_scratch(ctx, src_ptr_bytes + dst_ptr_bytes + dot_table_bytes(k, e));
    if (rc)
        return rc;
    char* d = (char*)ctx->d_scratch;
    RS_HIP(ctx, launch_row_ptrs(d_src, (long long)pitch, k, (long long)blocks,
                                (const uint8_t**)d, ctx->stream));
    RS_HIP(ctx, launch_row_ptrs(d_parity, (long long)pitch, e, (long long)blocks,
                                (const uint8_t**)(d + src_ptr_bytes), ctx->stream));
    return dot_from_host_coef(ctx, c.data(), k, e, (long long)len, (long long)blocks,
                              (const uint8_t* const*)d, (uint8_t* const*)(d + src_ptr_bytes),
                              src_ptr_bytes + dst_ptr_bytes, aligned, "k_rs_tc(encode)",
                              "k_rs_jit(encode)");
}

int rsgpu_set_encode_kernel(rsgpu_ctx* ctx, int kernel)
{
    if (!ctx || kernel < RSGPU_ENCODE_AUTO || kernel > RSGPU_ENCODE_THREADED)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_set_encode_kernel: unknown kernel");
    ctx->encode_kernel = kernel;
    return RSGPU_OK;
}

int rsgpu_set_decode_kernel(rsgpu_ctx* ctx, int kernel)
{
    if (!ctx || kernel < RSGPU_DECODE_AUTO || kernel > RSGPU_DECODE_GENERATED)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_set_decode_kernel: unknown kernel");
    // the retired FUSED choice runs ONE_MATRIX (the same bytes; rsgpu.h)
    ctx->decode_kernel = kernel == RSGPU_DECODE_FUSED ? RSGPU_DECODE_ONE_MATRIX : kernel;
    return RSGPU_OK;
}

}  // extern "C"

namespace {

// How rsgpu_decode_blocks runs for a geometry (prepare and apply agree as
// long as the context's decode kernel setting does not change in between).
enum class Plan {
    generated,   // k_decode_prepare_syn (closed form, writes code) + k_rs_jit
    one_matrix,  // k_decode_prepare_syn (closed form) + k_rs_tc
    general_tc,   // k_decode_prepare (k x k inversion) + k_rs_tc passes
    general_jit,  // k_decode_prepare + per-block generated code, passes of 32 rows
    general_dot   // k_decode_prepare + k_dot_generic (unaligned / odd lengths)
};

// column tiles (2 KB) per block from which AUTO decodes through generated
// code, every layout: the two-wave layouts (16 < e <= 32, two tiles per
// workgroup) pay from 16 tiles (C4 14.07 + 0.86 emission vs 15.44 ms
// threaded per 16384 blocks, profiles/r03_ab/c4_gen_vs_tc/), and so does the
// 8-row layout in XCD-contiguous order (per 16384 / 8192 blocks of 16 tiles,
// profiles/r03_ab/autoshort/: (64, 16) 10.69 + 0.54 vs 12.06 ms, (128, 16)
// 9.90 + 0.52 vs 11.82; round 2 measured 48 tiles, before that order); below
// kJitXcdTiles the 8-row decode runs in XCD-contiguous order
constexpr size_t kJitMinTiles = 16;
constexpr size_t kJitwMinTiles = 16;
// the general (k x k) decode through generated code in passes of 32 rows:
// no A/B below 48 tiles was made for it (round 2's threshold stays)
constexpr size_t kGeneralJitMinTiles = 48;
constexpr size_t kJitXcdTiles = 128;

size_t jit_min_tiles(int e) { return jitw_layout(e) ? kJitwMinTiles : kJitMinTiles; }
size_t decode_code_bytes(int k, int e, size_t blocks);
// generated code pays for a block of `tiles` column tiles: enough tiles to
// amortise its code (every tile's workgroup fetches all of it), or, below
// that, code small enough per tile.  (16, 8) has 10 KB per block: at 8 tiles
// (1.25 KB per tile) 3.46 + 0.15 ms emission against 3.84 threaded, at 4
// tiles (2.5 KB) 3.71 + 0.29 against 3.90, per 16 GB of sources
// (profiles/r03_ab/fewtiles/)
constexpr size_t kJitCodePerTile = 2048;
bool jit_pays(int k, int e, size_t tiles)
{
    return tiles >= jit_min_tiles(e) || decode_code_bytes(k, e, 1) <= kJitCodePerTile * tiles;
}
// (block, tile) pairs per call from which AUTO pays the emission launch
// (~10 us whatever the batch) for the ~4 ns per pair the generated code saves
// over threaded code: C2 (one block, 489 tiles) decodes 16 us threaded
// against 10 + 11 us emitted + generated (profiles/r02_ab/c2_*.json)
constexpr size_t kJitMinWork = 4096;

bool rows_aligned(size_t len, size_t pitch, const void* a, const void* b, const void* c)
{
    return len % 32 == 0 && pitch % 16 == 0 && (uintptr_t)a % 16 == 0 && (uintptr_t)b % 16 == 0 &&
           (uintptr_t)c % 16 == 0;
}

// the k x k general decode on aligned rows: generated code where the rows
// are long enough to amortise it (as decode_plan's AUTO), threaded code else
Plan general_plan(rsgpu_ctx* ctx, size_t len)
{
    if ((len + 2047) / 2048 >= kGeneralJitMinTiles && ctx->decode_kernel != RSGPU_DECODE_ONE_MATRIX &&
        jit_probe(ctx) == 1)
        return Plan::general_jit;
    return Plan::general_tc;
}

Plan decode_plan(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks, const void* src,
                 const void* par, const void* out)
{
    if (!rows_aligned(len, pitch, src, par, out) || !tc_ready(ctx))
        return Plan::general_dot;
    const int want = ctx->decode_kernel;
    // the closed-form rows serve every e (Lambda's e + 1 coefficients in one
    // wave up to e = 63, in LDS above); the threaded-code kernel takes e <= 32
    const bool gen_ok = jit_probe(ctx) == 1 && want != RSGPU_DECODE_ONE_MATRIX &&
                        want != RSGPU_DECODE_GENERAL &&
                        (want == RSGPU_DECODE_GENERATED || jit_pays(k, e, (len + 2047) / 2048));
    if (e > 32 && gen_ok)
        return Plan::generated;
    if (want == RSGPU_DECODE_GENERAL || e > 32)
        return general_plan(ctx, len);
    if (want == RSGPU_DECODE_ONE_MATRIX || jit_probe(ctx) != 1)
        return Plan::one_matrix;
    // AUTO: generated code only when a block has enough column tiles to
    // amortise its ~160 KB of code (every tile's workgroup fetches all of
    // it): C3 / C5 (489 tiles) 25.2 / 15.0 ms vs 27 / 17.7 threaded; L =
    // 128000 (63 tiles) 3.79 vs 3.94 ms (8-row layout, profiles/r02_ab); C4
    // (16 tiles) with two tiles per workgroup, above
    if (want == RSGPU_DECODE_AUTO &&
        (!jit_pays(k, e, (len + 2047) / 2048) || (len + 2047) / 2048 * blocks < kJitMinWork))
        return Plan::one_matrix;
    return Plan::generated;
}

// Workspace: [survivor ptrs B x k | output ptrs B x e | coefficient region],
// the region sized for the largest consumer: k_rs_tc handler addresses (pass
// layout), the v_perm tables, or the generated decode's e x k rows.
struct WsLayout {
    size_t surv, outp, tab, total;
};

WsLayout ws_layout(int k, int e, size_t blocks)
{
    WsLayout w{};
    size_t o = 0;
    w.surv = o;
    o = align_up(o + sizeof(void*) * (size_t)k * blocks, 256);
    w.outp = o;
    o = align_up(o + sizeof(void*) * (size_t)e * blocks, 256);
    w.tab = o;
    const size_t tc_bytes = sizeof(unsigned long long) * (size_t)tc_table_elems(k, e) * blocks;
    const size_t dot_bytes = (sizeof(uint4) + sizeof(uint32_t)) * (size_t)k * rows_pad_for(e) * blocks;
    const size_t jit_bytes = (size_t)e * k * blocks;
    w.total = align_up(o + std::max({tc_bytes, dot_bytes, jit_bytes}), 256);
    return w;
}

// Generated decode code of a call: two waves of 16 rows for 24 < e <= 32, of
// 12 for 20 < e <= 24, of 10 for 16 < e <= 20 (rs_jit.h Wide: the composites of a source
// built twice per tile instead of 4 or 3 times), else waves of 8 rows in
// passes of 32.  k_rs_jit16 measured on the same boxes (round 2's A/B build,
// profiles/r02_ab/jit_rows16): 10 % fewer VALU instructions, 40 % fewer
// instruction-cache misses, 3 % more cycles at 3 waves per SIMD; with the
// XCD-contiguous order 3.7 % faster than the 8-row kernel.
size_t decode_code_bytes(int k, int e, size_t blocks)
{
    return jitw_layout(e) ? jitw_code_bytes(k, e, (long long)blocks) : jit_code_bytes(k, e, (long long)blocks);
}

// k_jit_emit / k_jitw_emit: the code of every block from its decode rows
// coef [B][e][k] into the context's executable memory, which from now on
// belongs to this (k, e, blocks, workspace) prepare
int emit_decode_code(rsgpu_ctx* ctx, int k, int e, size_t blocks, const uint8_t* coef, const int* d_status,
                     const void* ws)
{
    ctx->jit_key.k = k;
    ctx->jit_key.e = e;
    ctx->jit_key.blocks = blocks;
    ctx->jit_key.ws = ws;
    ctx->jit_key.gen = ++ctx->jit_gen;
    if (jitw_layout(e)) {
        const int r = jitw_rows(jit::wide_pass_rows(e, 0));
        KTimer ke(ctx, r == 16 ? "k_jit16_emit" : r == 12 ? "k_jit12_emit" : "k_jit10_emit", blocks);
        RS_HIP(ctx, launch_jitw_emit(k, e, (long long)blocks, coef, d_status, (uint8_t*)ctx->d_jit, ctx->stream));
    } else {
        KTimer ke(ctx, "k_jit_emit", blocks);
        RS_HIP(ctx, launch_jit_emit(k, e, (long long)blocks, coef, d_status, (uint8_t*)ctx->d_jit, ctx->stream));
    }
    return RSGPU_OK;
}

// k_rs_jitw over `blocks` blocks whose code starts at `code` (the block
// stride jitw_code_bytes(k, e, 1)), one launch per pass of <= 64 rows (one
// pass for e <= 64), on stream st
int jitw_launch(rsgpu_ctx* ctx, int k, int e, size_t len, size_t blocks, const uint8_t* const* d_srcs,
                uint8_t* const* d_dsts, const uint8_t* code, const int* d_status, hipStream_t st)
{
    // one launch per pass of <= 64 rows (one pass for e <= 64)
    const size_t bs = jitw_code_bytes(k, e, 1);
    for (int p = 0; p < jit::wide_passes(e); ++p) {
        const int r0 = jit::wide_pass_row0(e, p), rows = jit::wide_pass_rows(e, p);
        JitArgs j{};
        j.srcs = d_srcs;
        j.dsts = d_dsts + r0;
        j.code = code + jitw_pass_offset(k, e, p);
        j.chunk_stride = (long long)jitw_chunk_stride(rows);
        j.block_stride = (long long)bs;
        j.k = k;
        j.rows = rows;
        j.dst_stride = e;
        j.len = (long long)len;
        j.status = d_status;
        // each XCD a contiguous range of (block, tile): a block's code is
        // fetched into one L2, not eight -- 3.7 % faster at C3 for the
        // 16-row kernel (23.3 vs 24.2 ms, profiles/r02_ab/jit_rows16/xcd_*.log),
        // where the 8-row kernel measured 1 % slower
        j.xcd_order = 1;
        // two column tiles per workgroup: the waves with the same rows share
        // their code's instruction-cache lines (C4 13.7 vs 14.2 ms per 16384
        // blocks, C3 23.2-23.3 vs 23.4-23.5, C5 12.7-12.8 vs 12.8-12.9;
        // three tiles: 20-30 % slower; profiles/r03_ab/tpw/)
        j.tiles_per_wg = jit::wide_waves(rows) == 4 ? 1 : ctx->jitw_tpw ? ctx->jitw_tpw : 2;
        // short rows: the block's few workgroups pull its code into L2 before
        // the instruction fetch misses on it line by line (C4: 12.8 vs 13.7
        // ms per 16384 blocks; C3, 245 workgroups per block, unchanged:
        // profiles/r03_ab/prefetch/)
        {
            const long long wgs = ((long long)((len + 2047) / 2048) + j.tiles_per_wg - 1) / j.tiles_per_wg;
            const long long lines = (long long)jitw_pass_bytes(k, rows) / 128;
            j.code_prefetch = ctx->jitw_prefetch >= 0 ? ctx->jitw_prefetch : lines >= 32 * wgs;
        }
        // chunk order rotated by each workgroup's start time, so the
        // workgroups sharing a CU pair's instruction cache walk their block's
        // code in step (k_rs_jitw).  Not for short rows: a block's few
        // workgroups run its code once each, and the rotation measured +0.5 %
        // on the C4 step (same-process ABBA x6, profiles/r05_rot/shared/)
        j.chunk_rot_ticks = ctx->jitw_rot >= 0 ? ctx->jitw_rot : j.code_prefetch ? 0 : jitw_rot_ticks(rows);
        j.prio = ctx->jitw_prio;
        const int r = jitw_rows(rows);
        KTimer kt(ctx,
                  e > 64  ? "k_rs_jitw_passes(decode)"
                  : e > 32 ? (r == 16 ? "k_rs_jit16x4(decode)" : r == 12 ? "k_rs_jit12x4(decode)" : "k_rs_jit10x4(decode)")
                  : r == 16 ? "k_rs_jit16(decode)"
                  : r == 12 ? "k_rs_jit12(decode)"
                            : "k_rs_jit10(decode)",
                  blocks, st);
        RS_HIP(ctx, launch_rs_jitw(j, (long long)blocks, st));
    }
    return RSGPU_OK;
}

// The per-block generated decode (rs_jit.hip) over rows e of every block:
// k_rs_jitw in one launch (decode_code_bytes), or k_rs_jit in passes of
// <= 32 rows: block b, pass p, wave w, chunk ch at d_jit + b block_stride +
// ((4 p + w) nch + ch) chunk_stride (k_jit_emit's layout).
int jit_decode_launch(rsgpu_ctx* ctx, int k, int e, size_t len, size_t blocks, const void* ws,
                      const uint8_t* const* d_srcs, uint8_t* const* d_dsts, const int* d_status)
{
    if (!ctx->d_jit || ctx->jit_bytes < decode_code_bytes(k, e, blocks))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_apply: no prepared decode code");
    // the code must be the one this workspace's prepare emitted, untouched
    // since: another prepare, a decode_general or a regrow rewrites it
    if (ctx->jit_key.gen != ctx->jit_gen || ctx->jit_key.k != k || ctx->jit_key.e != e ||
        ctx->jit_key.blocks != blocks || ctx->jit_key.ws != ws)
        return fail(ctx, RSGPU_ERR_ARG,
                    "rsgpu_decode_apply: the generated code belongs to another prepare "
                    "(re-run rsgpu_decode_prepare for this workspace)");
    if (jitw_layout(e))
        return jitw_launch(ctx, k, e, len, blocks, d_srcs, d_dsts, (const uint8_t*)ctx->d_jit, d_status,
                           ctx->stream);
    const int nch = (k + 7) / 8, nwt = (e + 7) / 8;
    for (int p = 0; p * 32 < e; ++p) {
        JitArgs j{};
        j.srcs = d_srcs;
        j.dsts = d_dsts + 32 * p;
        j.code = (const uint8_t*)ctx->d_jit + (size_t)4 * p * nch * jit::chunk_stride(8);
        j.chunk_stride = jit::chunk_stride(8);
        j.block_stride = (long long)nwt * nch * jit::chunk_stride(8);
        j.k = k;
        j.rows = std::min(32, e - 32 * p);
        j.dst_stride = e;
        j.len = (long long)len;
        j.status = d_status;
        // few tiles per block: keep each block's code in one XCD's L2
        j.xcd_order = (len + 2047) / 2048 < kJitXcdTiles;
        j.prio = ctx->jitw_prio;
        KTimer kt(ctx, "k_rs_jit(decode)", blocks);
        RS_HIP(ctx, launch_rs_jit(j, (long long)blocks, ctx->stream));
    }
    return RSGPU_OK;
}

// k_decode_prepare launch for the general plans (enc: device m x k matrix
// or nullptr for gf_gen_rs_matrix)
int general_prepare(rsgpu_ctx* ctx, Plan plan, int k, int m, int nerrs, bool originals_only,
                    size_t pitch, size_t blocks, const uint8_t* enc, const unsigned char* d_src,
                    const unsigned char* d_parity, const unsigned char* d_err, unsigned char* d_out,
                    void* d_workspace, int* d_status)
{
    const WsLayout w = ws_layout(k, nerrs, blocks);
    char* ws = (char*)d_workspace;
    PrepArgs p{};
    p.k = k;
    p.m = m;
    p.nerrs = nerrs;
    p.rows_pad = rows_pad_for(nerrs);
    p.blocks = (long long)blocks;
    p.err = d_err;
    p.enc = enc;
    p.originals_only = originals_only ? 1 : 0;
    p.src = d_src;
    p.src_pitch = (long long)pitch;
    p.par = d_parity;
    p.par_pitch = (long long)pitch;
    p.out = d_out;
    p.out_pitch = (long long)pitch;
    p.surv_ptrs = (const uint8_t**)(ws + w.surv);
    p.out_ptrs = (uint8_t**)(ws + w.outp);
    p.status = d_status;
    if (plan == Plan::general_jit) {
        p.coef_out = (uint8_t*)(ws + w.tab);  // [B][nerrs][k] decode rows
        const int rc = jit_ensure(ctx, decode_code_bytes(k, nerrs, blocks));
        if (rc)
            return rc;
    } else if (plan == Plan::general_tc) {
        p.tc_table = ctx->d_tc_table;
        p.tc_addr = (unsigned long long*)(ws + w.tab);
        p.tc_block_stride = tc_table_elems(k, nerrs);
    } else {
        p.tabs4 = (uint4*)(ws + w.tab);
        p.ctab = (uint32_t*)(ws + w.tab + sizeof(uint4) * (size_t)k * p.rows_pad * blocks);
        p.tab_block_stride = (long long)k * p.rows_pad;
    }
    {
        KTimer kt(ctx, "k_decode_prepare", blocks);
        RS_HIP(ctx, launch_decode_prepare(p, ctx->stream));
    }
    if (plan == Plan::general_jit)
        return emit_decode_code(ctx, k, nerrs, blocks, p.coef_out, d_status, d_workspace);
    return RSGPU_OK;
}

int general_apply(rsgpu_ctx* ctx, Plan plan, int k, int nerrs, size_t len, size_t pitch,
                  size_t blocks, bool aligned, void* d_workspace, const int* d_status)
{
    const WsLayout w = ws_layout(k, nerrs, blocks);
    char* ws = (char*)d_workspace;
    if (plan == Plan::general_jit)
        return jit_decode_launch(ctx, k, nerrs, len, blocks, ws, (const uint8_t* const*)(ws + w.surv),
                                 (uint8_t* const*)(ws + w.outp), d_status);
    if (plan == Plan::general_tc)
        return tc_launch(ctx, "k_rs_tc(decode)", (const uint8_t* const*)(ws + w.surv),
                         (uint8_t* const*)(ws + w.outp), (const unsigned long long*)(ws + w.tab),
                         tc_table_elems(k, nerrs), k, nerrs, (long long)len, (long long)blocks,
                         d_status);
    const int rows_pad = rows_pad_for(nerrs);
    DotArgs a{};
    a.srcs = (const uint8_t* const*)(ws + w.surv);
    a.dsts = (uint8_t* const*)(ws + w.outp);
    a.tabs4 = (const uint4*)(ws + w.tab);
    a.ctab = (const uint32_t*)(ws + w.tab + sizeof(uint4) * (size_t)k * rows_pad * blocks);
    a.tab_block_stride = (long long)k * rows_pad;
    a.k = k;
    a.rows = nerrs;
    a.rows_pad = rows_pad;
    a.len = (long long)len;
    a.blocks = (long long)blocks;
    a.status = d_status;
    a.bytewise = !aligned;
    (void)pitch;
    KTimer kt(ctx, "k_dot_generic(decode)", blocks);
    RS_HIP(ctx, launch_dot_generic(a, ctx->stream));
    return RSGPU_OK;
}

// Short-row batches of the generated decode (C4: 16 column tiles per block,
// 16384 blocks per call): run first on the context's stream, the prepare and
// the code emission of the whole batch (0.26 + 0.63 ms per C4 batch) hide
// behind no kernel.  Here the batch goes in `parts` slices of whole blocks:
// every slice's prepare and emission run on a second stream, and the context's
// stream waits for a slice's code just before that slice's decode launch, so
// the later slices' emission runs beside the earlier slices' decode.  Each
// slice's code has its place in the batch's code (block b at b x the block
// stride) and the workspace's key is the batch's: the result and the state
// left behind are those of prepare + apply.
constexpr size_t kPipeMinBlocks = 2048;
constexpr size_t kPipeMaxTiles = 64;
constexpr int kPipeParts = 4;

int decode_parts(const rsgpu_ctx* ctx, int e, size_t len, size_t blocks)
{
    if (!jitw_layout(e) || blocks < 4)
        return 1;
    if (ctx->decode_pipe >= 0)
        return std::max(1, std::min(ctx->decode_pipe, (int)(blocks / 2)));
    return (len + 2047) / 2048 <= kPipeMaxTiles && blocks >= kPipeMinBlocks ? kPipeParts : 1;
}

int decode_slices(rsgpu_ctx* ctx, int parts, int k, int e, size_t len, size_t pitch, size_t blocks,
                  const unsigned char* d_src, const unsigned char* d_parity, const unsigned char* d_err,
                  unsigned char* d_out, void* d_workspace, int* d_status);

int decode_pipelined(rsgpu_ctx* ctx, int parts, int k, int e, size_t len, size_t pitch, size_t blocks,
                     const unsigned char* d_src, const unsigned char* d_parity, const unsigned char* d_err,
                     unsigned char* d_out, void* d_workspace, int* d_status)
{
    const int rc = jit_ensure(ctx, decode_code_bytes(k, e, blocks));
    if (rc)
        return rc;
    if (!ctx->aux)
        RS_HIP(ctx, rsgpu_ctx_stream_create(ctx, &ctx->aux));
    const int rs = decode_slices(ctx, parts, k, e, len, pitch, blocks, d_src, d_parity, d_err, d_out,
                                 d_workspace, d_status);
    if (rs)
        ctx->jit_key.gen = 0;  // a failed call leaves no prepare behind for an apply to trust
    // whatever the outcome, nothing enqueued on the second stream outlives
    // the context's stream order (a failed launch leaves no emission behind
    // that later work on the same code or workspace could race)
    hipEvent_t done = sync_event(ctx);
    if (hipEventRecord(done, ctx->aux) != hipSuccess || hipStreamWaitEvent(ctx->stream, done, 0) != hipSuccess) {
        (void)hipStreamSynchronize(ctx->aux);
        return rs ? rs : fail(ctx, RSGPU_ERR_HIP, "rsgpu_decode_blocks: joining the emission stream");
    }
    return rs;
}

int decode_slices(rsgpu_ctx* ctx, int parts, int k, int e, size_t len, size_t pitch, size_t blocks,
                  const unsigned char* d_src, const unsigned char* d_parity, const unsigned char* d_err,
                  unsigned char* d_out, void* d_workspace, int* d_status)
{
    int rc = RSGPU_OK;
    const WsLayout w = ws_layout(k, e, blocks);
    char* ws = (char*)d_workspace;
    const uint8_t** surv = (const uint8_t**)(ws + w.surv);
    uint8_t** outp = (uint8_t**)(ws + w.outp);
    uint8_t* coef = (uint8_t*)(ws + w.tab);
    uint8_t* code = (uint8_t*)ctx->d_jit;
    const size_t bs = jitw_code_bytes(k, e, 1);
    const int r = jitw_rows(jit::wide_pass_rows(e, 0));
    const char* emit_name = r == 16 ? "k_jit16_emit" : r == 12 ? "k_jit12_emit" : "k_jit10_emit";
    ctx->jit_key.k = k;
    ctx->jit_key.e = e;
    ctx->jit_key.blocks = blocks;
    ctx->jit_key.ws = d_workspace;
    ctx->jit_key.gen = ++ctx->jit_gen;
    // the second stream starts behind everything enqueued on the context's
    // stream so far (the erasure lists, the code memory's fill, the kernels
    // of the last call that read this workspace and code)
    hipEvent_t start = sync_event(ctx);
    RS_HIP(ctx, hipEventRecord(start, ctx->stream));
    RS_HIP(ctx, hipStreamWaitEvent(ctx->aux, start, 0));
    // slices of an even number of blocks: a slice's code starts on a 128-byte line
    const size_t per = ((blocks + parts - 1) / parts + 1) / 2 * 2;
    for (size_t b0 = 0; b0 < blocks; b0 += per) {
        const size_t nb = std::min(per, blocks - b0);
        {
            KTimer kt(ctx, "k_decode_prepare_syn", nb, ctx->aux);
            RS_HIP(ctx, launch_decode_prepare_syn(k, e, (long long)nb, d_err + b0 * e, d_out + b0 * e * pitch,
                                                  (long long)pitch, surv + b0 * k, outp + b0 * e, ctx->d_tc_table,
                                                  d_status + b0, d_src + b0 * k * pitch, d_parity + b0 * e * pitch,
                                                  nullptr, coef + b0 * e * k, ctx->aux));
        }
        {
            KTimer kt(ctx, emit_name, nb, ctx->aux);
            RS_HIP(ctx, launch_jitw_emit(k, e, (long long)nb, coef + b0 * e * k, d_status + b0, code + b0 * bs,
                                         ctx->aux));
        }
        hipEvent_t ready = sync_event(ctx);
        RS_HIP(ctx, hipEventRecord(ready, ctx->aux));
        RS_HIP(ctx, hipStreamWaitEvent(ctx->stream, ready, 0));
        rc = jitw_launch(ctx, k, e, len, nb, surv + b0 * k, outp + b0 * e, code + b0 * bs, d_status + b0,
                         ctx->stream);
        if (rc)
            return rc;
    }
    return RSGPU_OK;
}

}  // namespace

extern "C" {

size_t rsgpu_decode_workspace_bytes(int k, int e, size_t blocks)
{
    if (k <= 0 || e <= 0)
        return 256;
    return ws_layout(k, e, blocks).total;
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
    if (blocks > kMaxGridBlocks)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_prepare: at most 65535 blocks per call "
                                        "(rsgpu_decode_blocks slices larger batches)");
    const Plan plan = decode_plan(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out);
    if (plan == Plan::one_matrix || plan == Plan::generated) {
        const WsLayout w = ws_layout(k, e, blocks);
        char* ws = (char*)d_workspace;
        const bool gen = plan == Plan::generated;
        if (gen) {
            rc = jit_ensure(ctx, decode_code_bytes(k, e, blocks));
            if (rc)
                return rc;
        }
        {
            KTimer kt(ctx, "k_decode_prepare_syn", blocks);
            RS_HIP(ctx, launch_decode_prepare_syn(
                            k, e, (long long)blocks, d_err, d_out, (long long)pitch,
                            (const uint8_t**)(ws + w.surv), (uint8_t**)(ws + w.outp), ctx->d_tc_table,
                            d_status, d_src, d_parity, gen ? nullptr : (unsigned long long*)(ws + w.tab),
                            gen ? (uint8_t*)(ws + w.tab) : nullptr, ctx->stream));
        }
        if (gen)  // the decode rows [B][e][k] sit in the coefficient region
            return emit_decode_code(ctx, k, e, blocks, (const uint8_t*)(ws + w.tab), d_status, ws);
        return RSGPU_OK;
    }
    return general_prepare(ctx, plan, k, k + e, e, true, pitch, blocks, nullptr, d_src, d_parity,
                           d_err, d_out, d_workspace, d_status);
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
    if (blocks > kMaxGridBlocks)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_apply: at most 65535 blocks per call "
                                        "(rsgpu_decode_blocks slices larger batches)");
    const Plan plan = decode_plan(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out);
    const WsLayout w = ws_layout(k, e, blocks);
    char* ws = (char*)d_workspace;
    if (plan == Plan::generated)
        // one matrix, the block's generated code (rs_jit.hip), passes of 32 rows
        return jit_decode_launch(ctx, k, e, len, blocks, ws, (const uint8_t* const*)(ws + w.surv),
                                 (uint8_t* const*)(ws + w.outp), d_status);
    if (plan == Plan::one_matrix)
        // one pass, one matrix over the k - e survivors and the e parity rows
        return tc_launch(ctx, "k_rs_tc(decode)", (const uint8_t* const*)(ws + w.surv),
                         (uint8_t* const*)(ws + w.outp), (const unsigned long long*)(ws + w.tab),
                         (long long)k * tc_rows_per_pass(e), k, e, (long long)len,
                         (long long)blocks, d_status);
    const bool aligned = ((uintptr_t)d_src % 16 == 0) && ((uintptr_t)d_parity % 16 == 0) &&
                         ((uintptr_t)d_out % 16 == 0) && (pitch % 16 == 0);
    return general_apply(ctx, plan, k, e, len, pitch, blocks, aligned, d_workspace, d_status);
}

int rsgpu_decode_blocks(rsgpu_ctx* ctx, int k, int e, size_t len, size_t pitch, size_t blocks,
                        const unsigned char* d_src, const unsigned char* d_parity,
                        const unsigned char* d_err, unsigned char* d_out, void* d_workspace,
                        int* d_status)
{
    // argument checks before any plan is made (decode_plan reads the context)
    int rc = check_geom(ctx, k, e, len, pitch, blocks);
    if (rc)
        return rc;
    if (e > 0 && (e > k || !d_err || !d_status))
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_blocks: bad arguments");
    if (blocks > kMaxGridBlocks) {
        // slices in stream order, each through the start of the workspace
        // (a slice's layout is no larger than the whole batch's)
        for (size_t b0 = 0; b0 < blocks; b0 += kMaxGridBlocks) {
            const int rc = rsgpu_decode_blocks(
                ctx, k, e, len, pitch, std::min(kMaxGridBlocks, blocks - b0), d_src + b0 * k * pitch,
                d_parity + b0 * e * pitch, d_err ? d_err + b0 * e : nullptr, d_out + b0 * e * pitch,
                d_workspace, d_status ? d_status + b0 : nullptr);
            if (rc)
                return rc;
        }
        return RSGPU_OK;
    }
    // A small batch of the one-matrix decode with few rows (C2: one block of
    // (16, 4, 1e6)): the decode rows are built inside the decode kernel, one
    // launch instead of prepare + apply (k_rs_tc_fused)
    if (e > 0 && e <= 8 && k <= 64 && len > 0 && blocks > 0 &&
        decode_plan(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out) == Plan::one_matrix &&
        (long long)((len + 2047) / 2048 * blocks) < kTcSplitMaxWork) {
        // AUTO, and a code with a compiled single-chunk program (C2's (16, 4)):
        // syndromes through the compiled programs, the e x e solve in the same
        // launch (k_rs_syn_split); otherwise the threaded-code one-launch decode
        if (ctx->decode_kernel == RSGPU_DECODE_AUTO && rs_bitsliced_split_available(k, e)) {
            SynArgs y{};
            y.src = d_src;
            y.par = d_parity;
            y.out = d_out;
            y.err = d_err;
            y.status = d_status;
            y.pitch = (long long)pitch;
            y.len = (long long)len;
            KTimer kt(ctx, "k_rs_syn_split(decode)", blocks);
            RS_HIP(ctx, launch_rs_syn_split(k, e, y, (long long)blocks, ctx->stream));
            return RSGPU_OK;
        }
        TcFusedArgs f{};
        f.k = k;
        f.e = e;
        f.len = (long long)len;
        f.pitch = (long long)pitch;
        f.blocks = (long long)blocks;
        f.err = d_err;
        f.src = d_src;
        f.par = d_parity;
        f.out = d_out;
        f.status = d_status;
        f.map_base = ctx->tc_base;
        f.map_stride = tc_handler_stride();
        for (int sl = 0; sl < 8; ++sl)
            f.map_copy[sl] = tc_slot_copy(sl);
        KTimer kt(ctx, "k_rs_tc_fused(decode)", blocks);
        RS_HIP(ctx, launch_rs_tc_fused(f, ctx->stream));
        return RSGPU_OK;
    }
    // short rows, many blocks: prepare and emission beside the decode
    if (e > 0 && len > 0 && blocks > 0 && d_workspace &&
        decode_plan(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out) == Plan::generated)
        if (const int parts = decode_parts(ctx, e, len, blocks); parts > 1)
            return decode_pipelined(ctx, parts, k, e, len, pitch, blocks, d_src, d_parity, d_err, d_out,
                                    d_workspace, d_status);
    rc = rsgpu_decode_prepare(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_err, d_out,
                              d_workspace, d_status);
    if (rc)
        return rc;
    return rsgpu_decode_apply(ctx, k, e, len, pitch, blocks, d_src, d_parity, d_out, d_workspace,
                              d_status);
}

size_t rsgpu_decode_general_workspace_bytes(int k, int m, int nerrs, size_t blocks)
{
    if (k <= 0 || m < k || nerrs <= 0)
        return 256;
    return ws_layout(k, nerrs, blocks).total;
}

int rsgpu_decode_general(rsgpu_ctx* ctx, int k, int m, size_t len, size_t pitch, size_t blocks,
                         const unsigned char* encode_matrix, const unsigned char* d_src,
                         const unsigned char* d_parity, const unsigned char* d_err, int nerrs,
                         unsigned char* d_out, void* d_workspace, int* d_status)
{
    int rc = check_geom(ctx, k, m - k, len, pitch, blocks);
    if (rc)
        return rc;
    if (nerrs < 0 || nerrs > m - k)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_general: nerrs must be in [0, m - k]");
    if (nerrs == 0)
        return RSGPU_OK;
    if (!d_err || !d_workspace || !d_status || !d_out)
        return fail(ctx, RSGPU_ERR_ARG, "rsgpu_decode_general: bad arguments");
    if (blocks > kMaxGridBlocks) {
        for (size_t b0 = 0; b0 < blocks; b0 += kMaxGridBlocks) {
            rc = rsgpu_decode_general(ctx, k, m, len, pitch, std::min(kMaxGridBlocks, blocks - b0),
                                      encode_matrix, d_src + b0 * k * pitch, d_parity + b0 * (m - k) * pitch,
                                      d_err + b0 * nerrs, nerrs, d_out + b0 * nerrs * pitch, d_workspace,
                                      d_status + b0);
            if (rc)
                return rc;
        }
        return RSGPU_OK;
    }
    const bool tcp = rows_aligned(len, pitch, d_src, d_parity, d_out) && tc_ready(ctx);
    const Plan plan = tcp ? general_plan(ctx, len) : Plan::general_dot;
    const uint8_t* d_enc = nullptr;
    if (encode_matrix) {
        const size_t bytes = (size_t)m * k;
        rc = ensure_scratch(ctx, bytes);
        if (rc)
            return rc;
        void* stage;
        rc = get_stage(ctx, bytes, &stage);
        if (rc)
            return rc;
        std::memcpy(stage, encode_matrix, bytes);
        rc = upload(ctx, ctx->d_scratch, bytes);
        if (rc)
            return rc;
        d_enc = (const uint8_t*)ctx->d_scratch;
    }
    rc = general_prepare(ctx, plan, k, m, nerrs, false, pitch, blocks, d_enc, d_src, d_parity, d_err,
                         d_out, d_workspace, d_status);
    if (rc || len == 0)
        return rc;
    const bool aligned = ((uintptr_t)d_src % 16 == 0) && ((uintptr_t)d_parity % 16 == 0) &&
                         ((uintptr_t)d_out % 16 == 0) && (pitch % 16 == 0);
    return general_apply(ctx, plan, k, nerrs, len, pitch, blocks, aligned, d_workspace, d_status);
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
    if (blocks > kMaxGridBlocks) {
        for (size_t b0 = 0; b0 < blocks; b0 += kMaxGridBlocks) {
            rc = rsgpu_verify_blocks(ctx, k, e, len, pitch, std::min(kMaxGridBlocks, blocks - b0),
                                     d_src + b0 * k * pitch, d_out + b0 * e * pitch, d_err + b0 * e,
                                     d_mismatch + b0);
            if (rc)
                return rc;
        }
        return RSGPU_OK;
    }
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
