// rs_throughput.cpp -- command-line peer of benchmark/isa_throughput
// (isa.cpp:261-330) running the MI355X engine.  Same options
// (--symbols, --loss_rate, --symbol_size, --type as multitoken lists, --runs),
// plus --blocks, --seed, --device.  Results print as a table and optionally
// as gauge-compatible CSV / JSON (columns: testcase, benchmark, symbols,
// symbol_size, loss_rate, type, erased_symbols, goodput -- the names
// plot_storage_benchmarks.py reads) with extra blocks/seconds columns.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "gpu_plugin.hpp"
#include "throughput_benchmark.hpp"

using namespace sbamd;

static void usage()
{
    std::printf(
        "rs_throughput [--symbols N...] [--loss_rate R...] [--symbol_size P...]\n"
        "              [--type encoder|decoder...] [--runs N] [--blocks B]\n"
        "              [--seed S] [--device D] [--csv_file F] [--json_file F]\n");
}

int main(int argc, char** argv)
{
    options o;
    uint32_t blocks = 1;
    uint64_t seed = 1;
    int device = 0;
    std::string csv, json;
    auto take = [&](int& i, auto fn) {
        while (i + 1 < argc && std::strncmp(argv[i + 1], "--", 2) != 0)
            fn(argv[++i]);
    };
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--symbols") {
            o.symbols.clear();
            take(i, [&](const char* v) { o.symbols.push_back((uint32_t)std::atoi(v)); });
        } else if (a == "--loss_rate") {
            o.loss_rate.clear();
            take(i, [&](const char* v) { o.loss_rate.push_back(std::atof(v)); });
        } else if (a == "--symbol_size") {
            o.symbol_size.clear();
            take(i, [&](const char* v) { o.symbol_size.push_back((uint32_t)std::atoi(v)); });
        } else if (a == "--type") {
            o.types.clear();
            take(i, [&](const char* v) { o.types.push_back(v); });
        } else if (a == "--runs" && i + 1 < argc) {
            o.runs = (uint32_t)std::atoi(argv[++i]);
        } else if (a == "--blocks" && i + 1 < argc) {
            blocks = (uint32_t)std::atoi(argv[++i]);
        } else if (a == "--seed" && i + 1 < argc) {
            seed = std::strtoull(argv[++i], nullptr, 10);
        } else if (a == "--device" && i + 1 < argc) {
            device = std::atoi(argv[++i]);
        } else if (a == "--csv_file" && i + 1 < argc) {
            csv = argv[++i];
        } else if (a == "--json_file" && i + 1 < argc) {
            json = argv[++i];
        } else {
            usage();
            return a == "--help" ? 0 : 2;
        }
    }
    auto session = std::make_shared<gpu_session>(device);
    std::vector<result_row> rows;
    uint64_t run_id = 0;
    for (const auto& cs : expand(o)) {
        throughput_benchmark<gpu_encoder, gpu_decoder> tb(
            [&](const config_set& c) {
                return std::make_shared<gpu_encoder>(session, c.symbols, c.symbol_size,
                                                     c.erased_symbols, blocks, seed, run_id * blocks);
            },
            [&](const config_set& c) {
                return std::make_shared<gpu_decoder>(session, c.symbols, c.symbol_size,
                                                     c.erased_symbols, blocks, seed, run_id * blocks);
            });
        for (uint32_t r = 0; r < o.runs; ++r, ++run_id) {
            tb.setup(cs);
            result_row row = tb.run(r);
            if (!row.accepted) {
                std::printf("measurement rejected (incomplete decode)\n");
                continue;
            }
            std::printf("symbols=%u symbol_size=%u loss_rate=%g type=%s erased=%u blocks=%u "
                        "run=%u goodput=%.1f MB/s (%.3f GiB/s, %.3f ms)\n",
                        cs.symbols, cs.symbol_size, cs.loss_rate, cs.type.c_str(),
                        cs.erased_symbols, blocks, r, row.goodput,
                        row.bytes / row.seconds / 1073741824.0, row.seconds * 1e3);
            rows.push_back(row);
        }
    }
    if (!csv.empty()) {
        std::ofstream f(csv);
        f << "testcase,benchmark,symbols,symbol_size,loss_rate,type,erased_symbols,blocks,run,"
             "seconds,goodput\n";
        for (const auto& r : rows)
            f << "MI355X,ErasureCode," << r.cs.symbols << "," << r.cs.symbol_size << ","
              << r.cs.loss_rate << "," << r.cs.type << "," << r.cs.erased_symbols << "," << blocks
              << "," << r.run << "," << r.seconds << "," << r.goodput << "\n";
    }
    if (!json.empty()) {
        std::ofstream f(json);
        f << "[\n";
        for (size_t i = 0; i < rows.size(); ++i) {
            const auto& r = rows[i];
            f << "  {\"testcase\": \"MI355X\", \"benchmark\": \"ErasureCode\", \"symbols\": "
              << r.cs.symbols << ", \"symbol_size\": " << r.cs.symbol_size
              << ", \"loss_rate\": " << r.cs.loss_rate << ", \"type\": \"" << r.cs.type
              << "\", \"erased_symbols\": " << r.cs.erased_symbols << ", \"blocks\": " << blocks
              << ", \"run\": " << r.run << ", \"seconds\": " << r.seconds
              << ", \"goodput\": " << r.goodput << "}" << (i + 1 < rows.size() ? "," : "")
              << "\n";
        }
        f << "]\n";
    }
    return 0;
}
