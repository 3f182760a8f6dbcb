// gpu_plugin.hpp -- gpu_encoder / gpu_decoder: MI355X peers of isa_encoder /
// isa_decoder (benchmark/isa_throughput/isa.cpp:29-259) over the C ABI of
// librsgpu (include/rsgpu.h).  One object carries `blocks` independent blocks
// resident in HBM; blocks == 1 is exactly the reference's shape.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "rsgpu.h"

namespace sbamd {

struct gpu_session {
    rsgpu_ctx* ctx = nullptr;
    explicit gpu_session(int device)
    {
        if (rsgpu_create(device, &ctx) != RSGPU_OK)
            throw std::runtime_error("rsgpu_create failed (no HIP device?)");
    }
    ~gpu_session() { rsgpu_destroy(ctx); }
    void check(int rc, const char* what) const
    {
        if (rc != RSGPU_OK)
            throw std::runtime_error(std::string(what) + ": " + rsgpu_last_error(ctx));
    }
};

inline size_t row_pitch(uint32_t symbol_size) { return (symbol_size + 255u) / 256u * 256u; }

// Process-wide session for the reference-shaped constructors (device from
// RSGPU_DEVICE, default 0): throughput_benchmark.hpp:173-176 builds plugins
// with (symbols, symbol_size, erased_symbols) only.
inline std::shared_ptr<gpu_session> default_session()
{
    static std::shared_ptr<gpu_session> s = [] {
        const char* d = std::getenv("RSGPU_DEVICE");
        return std::make_shared<gpu_session>(d ? std::atoi(d) : 0);
    }();
    return s;
}

// Seed of the reference-shaped constructors (isa.cpp:55-58 uses rand(); the
// erasure sets, isa.cpp:137-146, are drawn from the same seed here).
inline uint64_t default_seed()
{
    const char* v = std::getenv("RSGPU_SEED");
    return v ? std::strtoull(v, nullptr, 10) : 20240611ull;
}

// Where a plugin's blocks live between calls.  DEVICE: in HBM (the timed
// regions are the kernels).  HOST: in page-locked host memory, as the
// reference's buffers (isa.cpp:46-58): encode_all / decode_all then include
// the copies across the link (rsgpu_encode_blocks_host /
// rsgpu_decode_blocks_host: chunked, copies overlapped with the kernels).
enum class resident { device, host };

struct gpu_encoder {
    gpu_encoder(std::shared_ptr<gpu_session> s, uint32_t symbols, uint32_t symbol_size,
                uint32_t encoded_symbols, uint32_t blocks, uint64_t seed, uint64_t block0,
                resident where = resident::device)
        : m_s(std::move(s)), k(symbols), e(encoded_symbols), L(symbol_size), B(blocks),
          pitch(row_pitch(symbol_size)), where(where)
    {
        const size_t src_b = (size_t)B * k * pitch, par_b = (size_t)B * (e ? e : 1) * pitch;
        if (where == resident::device) {
            m_s->check(rsgpu_malloc(m_s->ctx, (void**)&src, src_b), "alloc src");
            m_s->check(rsgpu_malloc(m_s->ctx, (void**)&par, par_b), "alloc parity");
            // isa.cpp:55-58 fills originals with rand(); the seeded stream here
            m_s->check(rsgpu_fill_synthetic(m_s->ctx, src, (size_t)B * k, L, pitch, seed, block0 * k),
                       "fill");
        } else {
            m_s->check(rsgpu_host_alloc(m_s->ctx, (void**)&src, src_b), "host alloc src");
            m_s->check(rsgpu_host_alloc(m_s->ctx, (void**)&par, par_b), "host alloc parity");
            // the same seeded stream, generated on the device a block at a
            // time and brought into host memory (untimed, like isa.cpp's ctor)
            unsigned char* tmp = nullptr;
            m_s->check(rsgpu_malloc(m_s->ctx, (void**)&tmp, (size_t)k * pitch), "alloc fill");
            for (uint32_t b = 0; b < B; ++b) {
                m_s->check(rsgpu_fill_synthetic(m_s->ctx, tmp, k, L, pitch, seed, (block0 + b) * k), "fill");
                m_s->check(rsgpu_memcpy_d2h(m_s->ctx, src + (size_t)b * k * pitch, tmp, (size_t)k * pitch),
                           "fill d2h");
            }
            rsgpu_free(m_s->ctx, tmp);
        }
        m_s->check(rsgpu_synchronize(m_s->ctx), "sync");
    }
    // Drop-in form of isa_encoder(symbols, symbol_size, encoded_symbols)
    // (isa.cpp:31): one block, synchronous calls -- like the CPU library, the
    // work is finished when encode_all() returns, so the reference harness's
    // own timer measures it.
    gpu_encoder(uint32_t symbols, uint32_t symbol_size, uint32_t encoded_symbols)
        : gpu_encoder(default_session(), symbols, symbol_size, encoded_symbols, 1, default_seed(), 0)
    {
        synchronous = true;
    }
    ~gpu_encoder()
    {
        if (where == resident::device) {
            rsgpu_free(m_s->ctx, src);
            rsgpu_free(m_s->ctx, par);
        } else {
            rsgpu_host_free(m_s->ctx, src);
            rsgpu_host_free(m_s->ctx, par);
        }
    }
    // isa.cpp:69-79: gf_gen_rs_matrix + ec_init_tables + ec_encode_data
    void encode_all()
    {
        if (where == resident::host) {  // synchronous: parity in host memory on return
            m_s->check(rsgpu_encode_blocks_host(m_s->ctx, (int)k, (int)e, L, pitch, B, src, par, nullptr),
                       "rsgpu_encode_blocks_host");
            return;
        }
        m_s->check(rsgpu_encode_blocks(m_s->ctx, (int)k, (int)e, L, pitch, B, src, par, nullptr),
                   "rsgpu_encode_blocks");
        if (synchronous)
            finish();
    }
    void finish() { m_s->check(rsgpu_synchronize(m_s->ctx), "sync"); }
    uint32_t block_size() const { return k * L; }
    uint32_t symbol_size() const { return L; }
    uint32_t payload_size() const { return L; }
    uint32_t payload_count() const { return e; }
    uint32_t blocks() const { return B; }

    std::shared_ptr<gpu_session> m_s;
    uint32_t k, e, L, B;
    size_t pitch;
    resident where;
    unsigned char* src = nullptr;  // device or (pinned) host rows, per `where`
    unsigned char* par = nullptr;
    bool synchronous = false;
};

struct gpu_decoder {
    gpu_decoder(std::shared_ptr<gpu_session> s, uint32_t symbols, uint32_t symbol_size,
                uint32_t encoded_symbols, uint32_t blocks, uint64_t seed, uint64_t block0,
                resident where = resident::device)
        : m_s(std::move(s)), k(symbols), e(encoded_symbols), L(symbol_size), B(blocks),
          pitch(row_pitch(symbol_size)), where(where)
    {
        // isa.cpp:133-156: erasure choice is part of the (untimed) constructor
        std::vector<unsigned char> h_err((size_t)B * (e ? e : 1));
        m_s->check(rsgpu_erasure_patterns(seed, block0, B, (int)k, (int)e, h_err.data()),
                   "erasure patterns");
        h_list = h_err;
        h_status.assign(B, -1);
        const size_t out_b = (size_t)B * (e ? e : 1) * pitch;
        if (where == resident::host) {
            m_s->check(rsgpu_host_alloc(m_s->ctx, (void**)&out, out_b), "host alloc out");
            return;
        }
        ws_bytes = rsgpu_decode_workspace_bytes((int)k, (int)e, B);
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&err, h_err.size()), "alloc err");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&out, out_b), "alloc out");
        m_s->check(rsgpu_malloc(m_s->ctx, &ws, ws_bytes), "alloc ws");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&status, sizeof(int) * B), "alloc status");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&mism, sizeof(unsigned long long) * B), "alloc");
        m_s->check(rsgpu_memcpy_h2d(m_s->ctx, err, h_err.data(), h_err.size()), "upload err");
    }
    // Drop-in form of isa_decoder(symbols, symbol_size, erased_symbols)
    // (isa.cpp:110): one block, synchronous, status fetched by decode_all.
    gpu_decoder(uint32_t symbols, uint32_t symbol_size, uint32_t erased_symbols)
        : gpu_decoder(default_session(), symbols, symbol_size, erased_symbols, 1, default_seed(), 0)
    {
        synchronous = true;
    }
    ~gpu_decoder()
    {
        if (where == resident::host) {
            rsgpu_host_free(m_s->ctx, out);
            return;
        }
        rsgpu_free(m_s->ctx, err);
        rsgpu_free(m_s->ctx, out);
        rsgpu_free(m_s->ctx, ws);
        rsgpu_free(m_s->ctx, status);
        rsgpu_free(m_s->ctx, mism);
    }
    // isa.cpp:169-213.  The synchronous (reference-shaped) decoder knows the
    // outcome on return: 0 when a block's matrix was singular or its
    // erasure list malformed, as decode_all returns 0 on "BAD MATRIX"
    // (isa.cpp:185-190).  Batched decoders return the payload count and
    // report failures through is_complete() after finish().
    uint32_t decode_all(const std::shared_ptr<gpu_encoder>& enc)
    {
        if (where == resident::host) {
            // the survivors and parity cross the link, the recovered rows
            // come back, statuses with them: synchronous
            if (enc->where != resident::host)
                throw std::runtime_error("host-resident decoder needs a host-resident encoder");
            m_s->check(rsgpu_decode_blocks_host(m_s->ctx, (int)k, (int)e, L, pitch, B, enc->src, enc->par,
                                                h_list.data(), out, h_status.data()),
                       "rsgpu_decode_blocks_host");
            m_decoded = true;
            if (synchronous && !is_complete())
                return 0;
            return enc->payload_count();
        }
        m_s->check(rsgpu_decode_blocks(m_s->ctx, (int)k, (int)e, L, pitch, B, enc->src, enc->par,
                                       err, out, ws, status),
                   "rsgpu_decode_blocks");
        m_decoded = true;
        if (synchronous) {
            finish();
            if (!is_complete())
                return 0;
        }
        return enc->payload_count();
    }
    // Replace the erasure lists ([blocks][e], ascending originals) drawn by
    // the constructor, e.g. with a malformed list to exercise the failure
    // path (test hook; the reference draws them in its constructor only).
    void set_erasures(const std::vector<unsigned char>& h_err)
    {
        if (h_err.size() != (size_t)B * e)
            throw std::runtime_error("set_erasures: want blocks x erased entries");
        if (where == resident::device)
            m_s->check(rsgpu_memcpy_h2d(m_s->ctx, err, h_err.data(), h_err.size()), "upload err");
        h_list = h_err;
    }
    const std::vector<unsigned char>& erasures() const { return h_list; }
    void finish()
    {
        if (where == resident::device)
            m_s->check(rsgpu_memcpy_d2h(m_s->ctx, h_status.data(), status, sizeof(int) * B), "status");
    }
    // isa.cpp:231 (complete iff every block's matrix inverted)
    bool is_complete() const
    {
        if (!m_decoded)
            return false;
        for (int st : h_status)
            if (st != 0)
                return false;
        return true;
    }
    // isa.cpp:215-229: on the device, or on the host for host-resident blocks
    bool verify_data(const std::shared_ptr<gpu_encoder>& enc)
    {
        if (where == resident::host) {
            for (uint32_t b = 0; b < B; ++b)
                for (uint32_t i = 0; i < e; ++i) {
                    const unsigned char* want = enc->src + ((size_t)b * k + h_list[(size_t)b * e + i]) * pitch;
                    if (std::memcmp(out + ((size_t)b * e + i) * pitch, want, L) != 0)
                        return false;
                }
            return true;
        }
        std::vector<unsigned long long> h(B, 0);
        m_s->check(rsgpu_memcpy_h2d(m_s->ctx, mism, h.data(), sizeof(unsigned long long) * B),
                   "zero");
        m_s->check(rsgpu_verify_blocks(m_s->ctx, (int)k, (int)e, L, pitch, B, enc->src, out, err,
                                       mism),
                   "verify");
        m_s->check(rsgpu_memcpy_d2h(m_s->ctx, h.data(), mism, sizeof(unsigned long long) * B),
                   "mismatch");
        for (auto v : h)
            if (v)
                return false;
        return true;
    }
    uint32_t block_size() const { return k * L; }

    std::shared_ptr<gpu_session> m_s;
    uint32_t k, e, L, B;
    size_t pitch, ws_bytes = 0;
    resident where;
    unsigned char* err = nullptr;  // device lists (device-resident decoders)
    unsigned char* out = nullptr;  // device or (pinned) host rows, per `where`
    void* ws = nullptr;
    int* status = nullptr;
    unsigned long long* mism = nullptr;
    std::vector<int> h_status;
    std::vector<unsigned char> h_list;  // erasure lists [blocks][e] (host copy)
    bool m_decoded = false;
    bool synchronous = false;
};

}  // namespace sbamd
