// throughput_benchmark.hpp -- the runner slice of steinwurf/storage-benchmarks'
// benchmark/throughput_benchmark.hpp, restated without gauge/boost (both are
// network-fetched and absent here).  Same Encoder/Decoder concept, same
// configuration cross-product (get_options :126-163), same timed regions
// (run_encode :199-206, run_decode :209-220) and the same goodput accounting
// (measurement :37-67: output bytes per iteration / microseconds = MB/s),
// same acceptance rule (accept_measurement :99-119).
//
// Encoder concept: Encoder(symbols, symbol_size, encoded_symbols, extra...),
//   encode_all(), payload_count(), block_size(), blocks(), finish()
// Decoder concept: Decoder(symbols, symbol_size, erased, extra...),
//   decode_all(std::shared_ptr<Encoder>), is_complete(),
//   verify_data(std::shared_ptr<Encoder>), finish()
// finish() waits for enqueued device work (a CPU plugin makes it a no-op);
// blocks() is the number of independent blocks one plugin object carries.
#pragma once

#include <cassert>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace sbamd {

struct config_set {
    uint32_t symbols = 16;
    uint32_t symbol_size = 1000000;
    double loss_rate = 0.5;
    std::string type = "encoder";
    uint32_t erased_symbols = 8;
};

struct options {
    std::vector<uint32_t> symbols{16};
    std::vector<double> loss_rate{0.5};
    std::vector<uint32_t> symbol_size{1000000};
    std::vector<std::string> types{"encoder", "decoder"};
    uint32_t runs = 1;  // BENCHMARK_F_INLINE(isa_throughput, ISA, ErasureCode, 1)
};

struct result_row {
    config_set cs;
    uint32_t run = 0;
    double goodput = 0;  // MB/s (1e6 B/s)
    double seconds = 0;
    uint64_t bytes = 0;
    bool accepted = false;
};

// get_options: symbols x loss_rate x symbol_size x type, erased = ceil(s*r)
inline std::vector<config_set> expand(const options& o)
{
    std::vector<config_set> out;
    for (uint32_t s : o.symbols)
        for (double r : o.loss_rate)
            for (uint32_t p : o.symbol_size) {
                assert(p % 64 == 0);  // throughput_benchmark.hpp:145
                for (const auto& t : o.types) {
                    config_set cs;
                    cs.symbols = s;
                    cs.symbol_size = p;
                    cs.loss_rate = r;
                    cs.type = t;
                    cs.erased_symbols = (uint32_t)std::ceil(s * r);
                    out.push_back(cs);
                }
            }
    return out;
}

template <class Encoder, class Decoder>
struct throughput_benchmark {
    using factory_enc = std::function<std::shared_ptr<Encoder>(const config_set&)>;
    using factory_dec = std::function<std::shared_ptr<Decoder>(const config_set&)>;

    throughput_benchmark(factory_enc fe, factory_dec fd) : m_fe(std::move(fe)), m_fd(std::move(fd)) {}

    // setup :165-177
    void setup(const config_set& cs)
    {
        m_cs = cs;
        m_encoder = m_fe(cs);
        m_decoder = m_fd(cs);
        m_encoded_symbols = m_recovered_symbols = m_processed_symbols = 0;
    }

    // encode_payloads :179-183
    void encode_payloads()
    {
        m_encoder->encode_all();
        m_encoded_symbols += (uint64_t)m_encoder->payload_count() * m_encoder->blocks();
    }

    // decode_payloads :185-196
    void decode_payloads()
    {
        m_processed_symbols += (uint64_t)m_decoder->decode_all(m_encoder) * m_encoder->blocks();
        m_decoder->finish();
        if (m_decoder->is_complete())
            m_recovered_symbols += (uint64_t)m_cs.erased_symbols * m_encoder->blocks();
    }

    // Called right before each timed region: the multi-GPU runner's barrier,
    // so every GPU's thread starts its region together.
    std::function<void()> before_timed;

    double run_timed(const std::function<void()>& f)
    {
        if (before_timed)
            before_timed();
        auto t0 = std::chrono::steady_clock::now();
        f();
        auto t1 = std::chrono::steady_clock::now();
        return std::chrono::duration<double>(t1 - t0).count();
    }

    // run_benchmark :222-240 -> returns one measured row
    result_row run(uint32_t run_index)
    {
        result_row row;
        row.cs = m_cs;
        row.run = run_index;
        double t = 0;
        if (m_cs.type == "encoder") {
            // RUN { encode_payloads(); } -- device work is part of the region
            t = run_timed([&] {
                encode_payloads();
                m_encoder->finish();
            });
            row.bytes = m_encoded_symbols * m_cs.symbol_size;
        } else if (m_cs.type == "decoder") {
            encode_payloads();  // untimed parity, :212-213
            m_encoder->finish();
            t = run_timed([&] { decode_payloads(); });
            row.bytes = m_recovered_symbols * m_cs.symbol_size;
        } else {
            assert(0);
        }
        row.seconds = t;
        row.goodput = (double)row.bytes / (t * 1e6);  // bytes / us = MB/s
        row.accepted = accept_measurement();
        return row;
    }

    // accept_measurement :99-119
    bool accept_measurement()
    {
        if (m_cs.type == "decoder") {
            if (!m_decoder->is_complete())
                return false;
            const bool ok = m_decoder->verify_data(m_encoder);
            assert(ok);
            if (!ok)
                return false;
        }
        return true;
    }

    std::shared_ptr<Encoder> m_encoder;
    std::shared_ptr<Decoder> m_decoder;
    config_set m_cs;
    uint64_t m_encoded_symbols = 0, m_recovered_symbols = 0, m_processed_symbols = 0;

private:
    factory_enc m_fe;
    factory_dec m_fd;
};

}  // namespace sbamd
