// plugin_dropin_test.cpp -- exercises gpu_encoder / gpu_decoder exactly as the
// reference harness drives isa_encoder / isa_decoder
// (benchmark/throughput_benchmark.hpp:165-196): reference-shaped constructors,
// synchronous encode_all / decode_all, is_complete, verify_data and the
// goodput accounting (:37-67), for the configurations given on the command
// line as  symbols:symbol_size:erased ...  Exit status 0 iff every decode is
// complete and verified.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "gpu_plugin.hpp"

using Encoder = sbamd::gpu_encoder;
using Decoder = sbamd::gpu_decoder;

int main(int argc, char** argv)
{
    int bad = 0;
    for (int i = 1; i < argc; ++i) {
        unsigned k = 0, L = 0, e = 0;
        if (std::sscanf(argv[i], "%u:%u:%u", &k, &L, &e) != 3) {
            std::fprintf(stderr, "bad config %s (want symbols:symbol_size:erased)\n", argv[i]);
            return 2;
        }
        // setup() (:165-177)
        auto enc = std::make_shared<Encoder>(k, L, e);
        auto dec = std::make_shared<Decoder>(k, L, e);
        // run_encode / run_decode timed regions (:179-196)
        auto t0 = std::chrono::steady_clock::now();
        enc->encode_all();
        auto t1 = std::chrono::steady_clock::now();
        uint32_t processed = dec->decode_all(enc);
        auto t2 = std::chrono::steady_clock::now();
        const bool complete = dec->is_complete();
        const bool ok = complete && dec->verify_data(enc);
        const double us_e = std::chrono::duration<double, std::micro>(t1 - t0).count();
        const double us_d = std::chrono::duration<double, std::micro>(t2 - t1).count();
        // goodput as measurement() (:37-67): payload bytes per microsecond = MB/s
        std::printf("symbols=%u symbol_size=%u erased=%u payload_count=%u processed=%u "
                    "encoder=%.1f MB/s decoder=%.1f MB/s complete=%d verified=%d\n",
                    k, L, e, enc->payload_count(), processed,
                    (double)enc->payload_count() * L / us_e, (double)e * L / us_d, complete, ok);
        bad += !ok || processed != e || enc->payload_count() != e || enc->block_size() != k * L;
    }
    return bad ? 1 : 0;
}
