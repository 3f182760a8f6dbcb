// rs_arithmetic.cpp -- command-line peer of benchmark/isa_arithmetic
// (isa_arithmetic.cpp:31-447) running the MI355X engine: GF(2^8) dot-product
// throughput of `vectors` outputs over `vectors` sources of `size` bytes,
// device-resident, through the ISA-L-shaped C ABI (rsgpu_ec_encode_data).
//
// Benchmarks (the reference's names, ISA/<name>):
//   dot_product1        one output per call, `vectors` calls (rsgpu_gf_vect_dot_prod)
//                       (gf_vect_dot_prod loop, isa_arithmetic.cpp:121-138)
//   dot_product2        two outputs per call (gf_2vect_dot_prod_avx2 passes, :176-205)
//   dot_product4        four outputs per call, 3/2/1 tail (gf_4vect_dot_prod_avx2, :221-257)
//   dot_product_encode  all outputs in one call (ec_encode_data, :275-292)
// The timed region holds ec_init_tables and the calls, as RUN{} does there;
// throughput = size * vectors / time in MB/s (10^6 B/s, :40-54).
//
// Coefficients: the reference calls gf_gen_rs_matrix(a, vectors, vectors) and
// then builds tables from &a[vectors * vectors] (isa_arithmetic.cpp:118, :130),
// rows that were never generated; here a = gf_gen_rs_matrix(2 vectors,
// vectors) so those rows are the RS parity rows the code intends.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "rsgpu.h"

namespace {

void usage()
{
    std::printf(
        "rs_arithmetic [--size BYTES...] [--vectors N...] [--runs N] [--device D]\n"
        "              [--csv_file F] [--json_file F]\n");
}

#define CHECK(call)                                                                   \
    do {                                                                              \
        int rc_ = (call);                                                             \
        if (rc_ != RSGPU_OK) {                                                        \
            std::fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_,                  \
                         rsgpu_last_error(ctx));                                      \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

struct Row {
    std::string name;
    uint32_t size, vectors, run;
    double seconds, throughput;
};

}  // namespace

int main(int argc, char** argv)
{
    std::vector<uint32_t> sizes{1000000}, vectors{8, 16, 32};
    uint32_t runs = 1;
    int device = 0;
    std::string csv, json;
    auto take = [&](int& i, std::vector<uint32_t>& out) {
        out.clear();
        while (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0)
            out.push_back((uint32_t)std::atoi(argv[++i]));
    };
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--size")
            take(i, sizes);
        else if (a == "--vectors")
            take(i, vectors);
        else if (a == "--runs" && i + 1 < argc)
            runs = (uint32_t)std::atoi(argv[++i]);
        else if (a == "--device" && i + 1 < argc)
            device = std::atoi(argv[++i]);
        else if (a == "--csv_file" && i + 1 < argc)
            csv = argv[++i];
        else if (a == "--json_file" && i + 1 < argc)
            json = argv[++i];
        else {
            usage();
            return a == "--help" ? 0 : 2;
        }
    }
    rsgpu_ctx* ctx = nullptr;
    if (rsgpu_create(device, &ctx) != RSGPU_OK) {
        std::fprintf(stderr, "rsgpu_create(%d) failed\n", device);
        return 1;
    }
    const char* names[4] = {"dot_product1", "dot_product2", "dot_product4", "dot_product_encode"};
    std::vector<Row> rows;
    for (uint32_t size : sizes) {
        for (uint32_t v : vectors) {
            if (v == 0 || 2 * v > RSGPU_MAX_SOURCES) {
                std::fprintf(stderr, "vectors=%u out of range\n", v);
                continue;
            }
            const size_t pitch = (size + 255) / 256 * 256;
            unsigned char *d_src = nullptr, *d_dst = nullptr;
            CHECK(rsgpu_malloc(ctx, (void**)&d_src, pitch * v));
            CHECK(rsgpu_malloc(ctx, (void**)&d_dst, pitch * v));
            CHECK(rsgpu_fill_synthetic(ctx, d_src, v, size, pitch, 1, 0));
            std::vector<unsigned char*> data(v), coding(v);
            for (uint32_t i = 0; i < v; ++i) {
                data[i] = d_src + i * pitch;
                coding[i] = d_dst + i * pitch;
            }
            std::vector<unsigned char> a((size_t)2 * v * v), g((size_t)32 * v * v);
            rsgpu_gf_gen_rs_matrix(a.data(), 2 * v, v);
            // every pass split must produce the same outputs (self-check)
            // (row padding past `size` is never written: start from zeros)
            std::vector<unsigned char> first, now((size_t)pitch * v, 0);
            CHECK(rsgpu_memcpy_h2d(ctx, d_dst, now.data(), now.size()));
            for (int bm = 0; bm < 4; ++bm) {
                const int per = bm == 0 ? 1 : bm == 1 ? 2 : bm == 2 ? 4 : (int)v;
                auto once = [&] {
                    rsgpu_ec_init_tables(v, v, &a[(size_t)v * v], g.data());
                    for (uint32_t r = 0; r < v; r += per) {
                        const int n = (int)std::min<uint32_t>(per, v - r);
                        if (per == 1)  // isa_arithmetic.cpp:134 gf_vect_dot_prod
                            CHECK(rsgpu_gf_vect_dot_prod(ctx, size, v, &g[(size_t)r * v * 32], data.data(),
                                                         coding[r]));
                        else
                            CHECK(rsgpu_ec_encode_data(ctx, size, v, n, &g[(size_t)r * v * 32], data.data(),
                                                       &coding[r]));
                    }
                    CHECK(rsgpu_synchronize(ctx));
                };
                once();  // warm-up (tables, code objects)
                for (uint32_t run = 0; run < runs; ++run) {
                    const auto t0 = std::chrono::steady_clock::now();
                    once();
                    const double s =
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    const double mbps = (double)size * v / s / 1e6;
                    std::printf("ISA/%-20s size=%u vectors=%u run=%u  %.3f ms  %.1f MB/s\n",
                                names[bm], size, v, run, s * 1e3, mbps);
                    rows.push_back({names[bm], size, v, run, s, mbps});
                }
                CHECK(rsgpu_memcpy_d2h(ctx, now.data(), d_dst, now.size()));
                if (bm == 0) {
                    first = now;
                } else if (now != first) {
                    std::fprintf(stderr, "ISA/%s outputs differ from dot_product1\n", names[bm]);
                    return 1;
                }
                std::fill(now.begin(), now.end(), 0);
                CHECK(rsgpu_memcpy_h2d(ctx, d_dst, now.data(), now.size()));
            }
            CHECK(rsgpu_free(ctx, d_src));
            CHECK(rsgpu_free(ctx, d_dst));
        }
    }
    if (!csv.empty()) {
        std::ofstream f(csv);
        f << "testcase,benchmark,size,vectors,run,seconds,throughput\n";
        for (const auto& r : rows)
            f << "ISA," << r.name << "," << r.size << "," << r.vectors << "," << r.run << ","
              << r.seconds << "," << r.throughput << "\n";
    }
    if (!json.empty()) {
        std::ofstream f(json);
        f << "[\n";
        for (size_t i = 0; i < rows.size(); ++i) {
            const auto& r = rows[i];
            f << "  {\"testcase\": \"ISA\", \"benchmark\": \"" << r.name << "\", \"size\": " << r.size
              << ", \"vectors\": " << r.vectors << ", \"run\": " << r.run << ", \"seconds\": "
              << r.seconds << ", \"throughput\": " << r.throughput << "}"
              << (i + 1 < rows.size() ? "," : "") << "\n";
        }
        f << "]\n";
    }
    rsgpu_destroy(ctx);
    return 0;
}
