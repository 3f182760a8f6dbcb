// plugin_dropin_test.cpp -- exercises gpu_encoder / gpu_decoder exactly as the
// reference harness drives isa_encoder / isa_decoder
// (benchmark/throughput_benchmark.hpp:165-196): reference-shaped constructors,
// synchronous encode_all / decode_all, is_complete, verify_data and the
// goodput accounting (:37-67), for the configurations given on the command
// line as  symbols:symbol_size:erased ...
//
//   --decode-kernel K   rsgpu_set_decode_kernel: auto | generated |
//                       one_matrix | general
//   --poison            after encode_all, overwrite every erased original row
//                       on the device with 0xA5 (keeping a host copy): the
//                       reference's decoder never reads them (isa.cpp:193-
//                       197), so neither may ours.  The recovered rows are
//                       compared with the saved originals, then the rows are
//                       restored and verify_data runs as usual.
//   --malformed M       replace the erasure list with a malformed one (dup:
//                       a repeated index, unsorted: descending, range: an
//                       index >= symbols): decode_all must return 0,
//                       is_complete() must be false, and the harness
//                       (throughput_benchmark<>::accept_measurement) must
//                       reject the measurement.
// Exit status 0 iff every decode is complete and verified (or, with
// --malformed, every one is rejected).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "gpu_plugin.hpp"
#include "throughput_benchmark.hpp"

using Encoder = sbamd::gpu_encoder;
using Decoder = sbamd::gpu_decoder;

namespace {

std::vector<unsigned char> malformed_list(const std::vector<unsigned char>& good, unsigned k,
                                          const std::string& how)
{
    std::vector<unsigned char> bad = good;
    const size_t e = bad.size();
    if (how == "dup" && e >= 2) {
        bad[1] = bad[0];
    } else if (how == "unsorted" && e >= 2) {
        for (size_t i = 0; i < e; ++i)
            bad[i] = good[e - 1 - i];
    } else {  // range (also the fallback for e == 1)
        bad[e - 1] = (unsigned char)k;
    }
    return bad;
}

// Overwrite the erased originals of block 0 (the reference-shaped objects
// hold one block) with 0xA5; returns their original bytes.
std::vector<unsigned char> poison_erased(Encoder& enc, const Decoder& dec)
{
    std::vector<unsigned char> saved((size_t)dec.e * enc.L), bytes(enc.L, 0xA5);
    for (unsigned i = 0; i < dec.e; ++i) {
        unsigned char* row = enc.src + (size_t)dec.erasures()[i] * enc.pitch;
        enc.m_s->check(rsgpu_memcpy_d2h(enc.m_s->ctx, saved.data() + (size_t)i * enc.L, row, enc.L),
                       "save erased row");
        enc.m_s->check(rsgpu_memcpy_h2d(enc.m_s->ctx, row, bytes.data(), enc.L), "poison row");
    }
    return saved;
}

void restore_erased(Encoder& enc, const Decoder& dec, const std::vector<unsigned char>& saved)
{
    for (unsigned i = 0; i < dec.e; ++i)
        enc.m_s->check(rsgpu_memcpy_h2d(enc.m_s->ctx, enc.src + (size_t)dec.erasures()[i] * enc.pitch,
                                        saved.data() + (size_t)i * enc.L, enc.L),
                       "restore row");
}

bool recovered_equal(const Decoder& dec, const std::vector<unsigned char>& saved)
{
    std::vector<unsigned char> got((size_t)dec.e * dec.L);
    for (unsigned i = 0; i < dec.e; ++i)
        dec.m_s->check(rsgpu_memcpy_d2h(dec.m_s->ctx, got.data() + (size_t)i * dec.L,
                                        dec.out + (size_t)i * dec.pitch, dec.L),
                       "read recovered");
    return std::memcmp(got.data(), saved.data(), got.size()) == 0;
}

}  // namespace

int main(int argc, char** argv)
{
    bool poison = false;
    std::string malformed;
    std::vector<std::string> cfgs;
    int kernel = RSGPU_DECODE_AUTO;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--poison") {
            poison = true;
        } else if (a == "--malformed" && i + 1 < argc) {
            malformed = argv[++i];
        } else if (a == "--decode-kernel" && i + 1 < argc) {
            const std::string k = argv[++i];
            kernel = k == "one_matrix" ? RSGPU_DECODE_ONE_MATRIX
                   : k == "general"    ? RSGPU_DECODE_GENERAL
                   : k == "generated"  ? RSGPU_DECODE_GENERATED
                                       : RSGPU_DECODE_AUTO;
        } else {
            cfgs.push_back(a);
        }
    }
    // every configuration is checked before the GPU is touched
    for (const auto& c : cfgs) {
        unsigned k = 0, L = 0, e = 0;
        if (std::sscanf(c.c_str(), "%u:%u:%u", &k, &L, &e) != 3) {
            std::fprintf(stderr, "bad config %s (want symbols:symbol_size:erased)\n", c.c_str());
            return 2;
        }
    }
    sbamd::default_session()->check(rsgpu_set_decode_kernel(sbamd::default_session()->ctx, kernel),
                                     "decode kernel");
    int bad = 0;
    for (const auto& c : cfgs) {
        unsigned k = 0, L = 0, e = 0;
        std::sscanf(c.c_str(), "%u:%u:%u", &k, &L, &e);
        // setup() (:165-177)
        auto enc = std::make_shared<Encoder>(k, L, e);
        auto dec = std::make_shared<Decoder>(k, L, e);
        if (!malformed.empty()) {
            // the reference-shaped decoder: decode_all -> 0, not complete
            dec->set_erasures(malformed_list(dec->erasures(), k, malformed));
            enc->encode_all();
            const uint32_t processed = dec->decode_all(enc);
            const bool complete = dec->is_complete();
            // the harness: the measurement is rejected (accept_measurement)
            sbamd::throughput_benchmark<Encoder, Decoder> tb(
                [&](const sbamd::config_set&) { return std::make_shared<Encoder>(k, L, e); },
                [&](const sbamd::config_set&) {
                    auto d = std::make_shared<Decoder>(k, L, e);
                    d->set_erasures(malformed_list(d->erasures(), k, malformed));
                    return d;
                });
            sbamd::config_set cs;
            cs.symbols = k;
            cs.symbol_size = L;
            cs.loss_rate = (double)e / k;
            cs.type = "decoder";
            cs.erased_symbols = e;
            tb.setup(cs);
            const sbamd::result_row row = tb.run(0);
            const bool rejected = processed == 0 && !complete && !row.accepted && row.bytes == 0;
            std::printf("symbols=%u symbol_size=%u erased=%u malformed=%s processed=%u complete=%d "
                        "accepted=%d rejected=%d\n",
                        k, L, e, malformed.c_str(), processed, complete, row.accepted, rejected);
            bad += !rejected;
            continue;
        }
        // run_encode / run_decode timed regions (:179-196)
        auto t0 = std::chrono::steady_clock::now();
        enc->encode_all();
        auto t1 = std::chrono::steady_clock::now();
        std::vector<unsigned char> saved;
        if (poison)
            saved = poison_erased(*enc, *dec);
        auto t2 = std::chrono::steady_clock::now();
        uint32_t processed = dec->decode_all(enc);
        auto t3 = std::chrono::steady_clock::now();
        const bool complete = dec->is_complete();
        bool poison_ok = true;
        if (poison) {
            poison_ok = complete && recovered_equal(*dec, saved);
            restore_erased(*enc, *dec, saved);
        }
        const bool ok = complete && poison_ok && dec->verify_data(enc);
        const double us_e = std::chrono::duration<double, std::micro>(t1 - t0).count();
        const double us_d = std::chrono::duration<double, std::micro>(t3 - t2).count();
        // goodput as measurement() (:37-67): payload bytes per microsecond = MB/s
        std::printf("symbols=%u symbol_size=%u erased=%u payload_count=%u processed=%u "
                    "encoder=%.1f MB/s decoder=%.1f MB/s poisoned=%d complete=%d verified=%d\n",
                    k, L, e, enc->payload_count(), processed,
                    (double)enc->payload_count() * L / us_e, (double)e * L / us_d, poison ? 1 : 0,
                    complete, ok);
        bad += !ok || processed != e || enc->payload_count() != e || enc->block_size() != k * L;
    }
    return bad ? 1 : 0;
}
