// rs_throughput.cpp -- command-line peer of benchmark/isa_throughput
// (isa.cpp:261-330) running the MI355X engine.  Same options
// (--symbols, --loss_rate, --symbol_size, --type as multitoken lists, --runs),
// plus --blocks, --seed, --device, and:
//   --resident device|host  where the blocks live between calls (host: the
//                           reference's layout, copies inside the timed
//                           regions; gpu_plugin.hpp `resident`)
//   --gpus N                one host thread per GPU (devices device ..
//                           device+N-1), each with its own context and its own
//                           `blocks` blocks (weak scaling, no exchange); the
//                           threads start every timed region on a barrier
//                           and a run's goodput is all GPUs' bytes over the
//                           slowest GPU's time
//   --same-device           every thread on `device` (tests the fan-out and
//                           the concurrent contexts on a one-GPU box)
// Results print as a table and optionally as gauge-compatible CSV / JSON
// (columns: testcase, benchmark, symbols, symbol_size, loss_rate, type,
// erased_symbols, goodput -- the names plot_storage_benchmarks.py reads) with
// extra blocks/gpus/seconds columns.
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "gpu_plugin.hpp"
#include "throughput_benchmark.hpp"

using namespace sbamd;

static void usage()
{
    std::printf(
        "rs_throughput [--symbols N...] [--loss_rate R...] [--symbol_size P...]\n"
        "              [--type encoder|decoder...] [--runs N] [--blocks B]\n"
        "              [--seed S] [--device D] [--resident device|host]\n"
        "              [--gpus N] [--same-device] [--csv_file F] [--json_file F] [--python_file F]\n");
}

// A reusable barrier for the per-GPU threads; a thread that fails breaks it
// so that the others stop waiting.
struct barrier {
    explicit barrier(int n) : n(n) {}
    void wait()
    {
        std::unique_lock<std::mutex> lk(m);
        if (broken)
            throw std::runtime_error("another GPU thread failed");
        const unsigned long long g = gen;
        if (++count == n) {
            count = 0;
            ++gen;
            cv.notify_all();
            return;
        }
        cv.wait(lk, [&] { return gen != g || broken; });
        if (broken)
            throw std::runtime_error("another GPU thread failed");
    }
    void brk()
    {
        std::lock_guard<std::mutex> lk(m);
        broken = true;
        cv.notify_all();
    }
    std::mutex m;
    std::condition_variable cv;
    int n, count = 0;
    unsigned long long gen = 0;
    bool broken = false;
};

int main(int argc0, char** argv0)
{
    // boost::program_options syntax as the reference's README invokes it
    // (README.rst:121, --symbols=100): "--opt=value" is "--opt value"
    std::vector<std::string> toks;
    for (int i = 0; i < argc0; ++i) {
        const std::string t = argv0[i];
        const size_t eq = t.find('=');
        if (i > 0 && t.rfind("--", 0) == 0 && eq != std::string::npos) {
            toks.push_back(t.substr(0, eq));
            toks.push_back(t.substr(eq + 1));
        } else {
            toks.push_back(t);
        }
    }
    std::vector<char*> av;
    for (auto& t : toks)
        av.push_back(t.data());
    const int argc = (int)av.size();
    char** argv = av.data();

    options o;
    uint32_t blocks = 1;
    uint64_t seed = 1;
    int device = 0, gpus = 1;
    bool same_device = false;
    resident where = resident::device;
    std::string csv, json, python;
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
        } else if (a == "--gpus" && i + 1 < argc) {
            gpus = std::atoi(argv[++i]);
        } else if (a == "--same-device") {
            same_device = true;
        } else if (a == "--resident" && i + 1 < argc) {
            const std::string v = argv[++i];
            if (v != "host" && v != "device")
                return usage(), 2;
            where = v == "host" ? resident::host : resident::device;
        } else if (a == "--csv_file" && i + 1 < argc) {
            csv = argv[++i];
        } else if (a == "--json_file" && i + 1 < argc) {
            json = argv[++i];
        } else if (a == "--python_file" && i + 1 < argc) {
            python = argv[++i];
        } else {
            usage();
            return a == "--help" ? 0 : 2;
        }
    }
    if (gpus < 1 || blocks < 1)
        return usage(), 2;
    // every (configuration, run) in order; each GPU thread runs all of them
    std::vector<std::pair<config_set, uint32_t>> plan;
    for (const auto& cs : expand(o))
        for (uint32_t r = 0; r < o.runs; ++r)
            plan.push_back({cs, r});
    std::vector<std::vector<result_row>> per(gpus, std::vector<result_row>(plan.size()));
    barrier bar(gpus);
    std::vector<std::string> errors(gpus);
    auto worker = [&](int t) {
        try {
            auto session = std::make_shared<gpu_session>(same_device ? device : device + t);
            for (size_t i = 0; i < plan.size(); ++i) {
                const config_set& cs = plan[i].first;
                // distinct blocks per (run, GPU): erasures and data follow the
                // global block index
                const uint64_t block0 = ((uint64_t)i * gpus + t) * blocks;
                throughput_benchmark<gpu_encoder, gpu_decoder> tb(
                    [&](const config_set& c) {
                        return std::make_shared<gpu_encoder>(session, c.symbols, c.symbol_size,
                                                             c.erased_symbols, blocks, seed, block0, where);
                    },
                    [&](const config_set& c) {
                        return std::make_shared<gpu_decoder>(session, c.symbols, c.symbol_size,
                                                             c.erased_symbols, blocks, seed, block0, where);
                    });
                if (gpus > 1)
                    tb.before_timed = [&] { bar.wait(); };
                tb.setup(cs);
                per[t][i] = tb.run(plan[i].second);
            }
        } catch (const std::exception& ex) {
            errors[t] = ex.what();
            bar.brk();
        }
    };
    if (gpus == 1) {
        worker(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < gpus; ++t)
            th.emplace_back(worker, t);
        for (auto& x : th)
            x.join();
    }
    int rc = 0;
    for (int t = 0; t < gpus; ++t)
        if (!errors[t].empty()) {
            std::fprintf(stderr, "gpu thread %d: %s\n", t, errors[t].c_str());
            rc = 1;
        }
    if (rc)
        return rc;
    std::vector<result_row> rows;
    for (size_t i = 0; i < plan.size(); ++i) {
        // the job's row: every GPU's bytes over the slowest GPU's time
        result_row row = per[0][i];
        row.bytes = 0;
        row.seconds = 0;
        for (int t = 0; t < gpus; ++t) {
            row.bytes += per[t][i].bytes;
            row.seconds = std::max(row.seconds, per[t][i].seconds);
            row.accepted = row.accepted && per[t][i].accepted;
        }
        row.goodput = (double)row.bytes / (row.seconds * 1e6);
        const config_set& cs = row.cs;
        if (!row.accepted) {
            std::printf("measurement rejected (incomplete decode)\n");
            rc = 3;
            continue;
        }
        std::printf("symbols=%u symbol_size=%u loss_rate=%g type=%s erased=%u blocks=%u gpus=%d "
                    "resident=%s run=%u goodput=%.1f MB/s (%.3f GiB/s, %.3f ms)\n",
                    cs.symbols, cs.symbol_size, cs.loss_rate, cs.type.c_str(), cs.erased_symbols, blocks, gpus,
                    where == resident::host ? "host" : "device", row.run, row.goodput,
                    row.bytes / row.seconds / 1073741824.0, row.seconds * 1e3);
        rows.push_back(row);
    }
    // gauge's printers (README.rst:109-113): the same columns as a CSV table,
    // a JSON document and a Python dictionary of columns
    const std::vector<std::string> cols = {"testcase", "benchmark", "symbols", "symbol_size", "loss_rate",
                                           "type", "erased_symbols", "blocks", "gpus", "resident",
                                           "run", "seconds", "goodput"};
    auto cells = [&](const result_row& r) {
        auto num = [](double v) {
            std::ostringstream o;
            o << v;
            return o.str();
        };
        return std::vector<std::pair<std::string, bool>>{  // (text, is a string)
            {"MI355X", true}, {"ErasureCode", true}, {num(r.cs.symbols), false},
            {num(r.cs.symbol_size), false}, {num(r.cs.loss_rate), false}, {r.cs.type, true},
            {num(r.cs.erased_symbols), false}, {num(blocks), false}, {num(gpus), false},
            {where == resident::host ? "host" : "device", true}, {num(r.run), false},
            {num(r.seconds), false}, {num(r.goodput), false}};
    };
    if (!csv.empty()) {
        std::ofstream f(csv);
        for (size_t c = 0; c < cols.size(); ++c)
            f << cols[c] << (c + 1 < cols.size() ? "," : "\n");
        for (const auto& r : rows) {
            const auto v = cells(r);
            for (size_t c = 0; c < v.size(); ++c)
                f << v[c].first << (c + 1 < v.size() ? "," : "\n");
        }
    }
    if (!json.empty()) {
        std::ofstream f(json);
        f << "[\n";
        for (size_t i = 0; i < rows.size(); ++i) {
            const auto v = cells(rows[i]);
            f << "  {";
            for (size_t c = 0; c < v.size(); ++c)
                f << "\"" << cols[c] << "\": " << (v[c].second ? "\"" + v[c].first + "\"" : v[c].first)
                  << (c + 1 < v.size() ? ", " : "");
            f << "}" << (i + 1 < rows.size() ? "," : "") << "\n";
        }
        f << "]\n";
    }
    if (!python.empty()) {
        std::ofstream f(python);
        f << "{\n";
        for (size_t c = 0; c < cols.size(); ++c) {
            f << "    '" << cols[c] << "': [";
            for (size_t i = 0; i < rows.size(); ++i) {
                const auto v = cells(rows[i])[c];
                f << (v.second ? "'" + v.first + "'" : v.first) << (i + 1 < rows.size() ? ", " : "");
            }
            f << "]" << (c + 1 < cols.size() ? "," : "") << "\n";
        }
        f << "}\n";
    }
    return rc;
}
