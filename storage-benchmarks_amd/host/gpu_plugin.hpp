// gpu_plugin.hpp -- gpu_encoder / gpu_decoder: MI355X peers of isa_encoder /
// isa_decoder (benchmark/isa_throughput/isa.cpp:29-259) over the C ABI of
// librsgpu (include/rsgpu.h).  One object carries `blocks` independent blocks
// resident in HBM; blocks == 1 is exactly the reference's shape.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

struct gpu_encoder {
    gpu_encoder(std::shared_ptr<gpu_session> s, uint32_t symbols, uint32_t symbol_size,
                uint32_t encoded_symbols, uint32_t blocks, uint64_t seed, uint64_t block0)
        : m_s(std::move(s)), k(symbols), e(encoded_symbols), L(symbol_size), B(blocks),
          pitch(row_pitch(symbol_size))
    {
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&src, (size_t)B * k * pitch), "alloc src");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&par, (size_t)B * (e ? e : 1) * pitch),
                   "alloc parity");
        // isa.cpp:55-58 fills originals with rand(); the seeded stream here
        m_s->check(rsgpu_fill_synthetic(m_s->ctx, src, (size_t)B * k, L, pitch, seed, block0 * k),
                   "fill");
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
        rsgpu_free(m_s->ctx, src);
        rsgpu_free(m_s->ctx, par);
    }
    // isa.cpp:69-79: gf_gen_rs_matrix + ec_init_tables + ec_encode_data
    void encode_all()
    {
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
    unsigned char* src = nullptr;
    unsigned char* par = nullptr;
    bool synchronous = false;
};

struct gpu_decoder {
    gpu_decoder(std::shared_ptr<gpu_session> s, uint32_t symbols, uint32_t symbol_size,
                uint32_t encoded_symbols, uint32_t blocks, uint64_t seed, uint64_t block0)
        : m_s(std::move(s)), k(symbols), e(encoded_symbols), L(symbol_size), B(blocks),
          pitch(row_pitch(symbol_size))
    {
        // isa.cpp:133-156: erasure choice is part of the (untimed) constructor
        std::vector<unsigned char> h_err((size_t)B * (e ? e : 1));
        m_s->check(rsgpu_erasure_patterns(seed, block0, B, (int)k, (int)e, h_err.data()),
                   "erasure patterns");
        ws_bytes = rsgpu_decode_workspace_bytes((int)k, (int)e, B);
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&err, h_err.size()), "alloc err");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&out, (size_t)B * (e ? e : 1) * pitch), "alloc out");
        m_s->check(rsgpu_malloc(m_s->ctx, &ws, ws_bytes), "alloc ws");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&status, sizeof(int) * B), "alloc status");
        m_s->check(rsgpu_malloc(m_s->ctx, (void**)&mism, sizeof(unsigned long long) * B), "alloc");
        m_s->check(rsgpu_memcpy_h2d(m_s->ctx, err, h_err.data(), h_err.size()), "upload err");
        h_list = h_err;
        h_status.assign(B, -1);
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
        m_s->check(rsgpu_memcpy_h2d(m_s->ctx, err, h_err.data(), h_err.size()), "upload err");
        h_list = h_err;
    }
    const std::vector<unsigned char>& erasures() const { return h_list; }
    void finish()
    {
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
    // isa.cpp:215-229
    bool verify_data(const std::shared_ptr<gpu_encoder>& enc)
    {
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
    unsigned char* err = nullptr;
    unsigned char* out = nullptr;
    void* ws = nullptr;
    int* status = nullptr;
    unsigned long long* mism = nullptr;
    std::vector<int> h_status;
    std::vector<unsigned char> h_list;  // erasure lists [blocks][e] (host copy)
    bool m_decoded = false;
    bool synchronous = false;
};

}  // namespace sbamd
