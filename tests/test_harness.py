"""Host-side harness logic (no GPU): the configuration cross-product and
erased-symbol count of throughput_benchmark::get_options
(benchmark/throughput_benchmark.hpp:126-163) as restated by
rsgpu.ThroughputBenchmark, and the C++ runner's option handling."""
import math
import os
import subprocess

import pytest

import rsgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = os.path.join(ROOT, "storage-benchmarks_amd", "bin", "rs_throughput")


def test_cross_product_order_and_erased():
    tb = rsgpu.ThroughputBenchmark(symbols=(16, 64), loss_rate=(0.5, 0.2),
                                   symbol_size=(32000, 1000000), types=("encoder", "decoder"))
    cfgs = tb.configurations()
    assert len(cfgs) == 2 * 2 * 2 * 2
    # nesting: symbols > loss_rate > symbol_size > type (hpp:137-160)
    assert [(c.symbols, c.loss_rate, c.symbol_size, c.type) for c in cfgs[:4]] == [
        (16, 0.5, 32000, "encoder"), (16, 0.5, 32000, "decoder"),
        (16, 0.5, 1000000, "encoder"), (16, 0.5, 1000000, "decoder")]
    for c in cfgs:
        assert c.erased_symbols == math.ceil(c.symbols * c.loss_rate)  # hpp:155


def test_reference_defaults():
    # isa.cpp:261-308 defaults: symbols=16, loss_rate=0.5, symbol_size=1e6, both types
    tb = rsgpu.ThroughputBenchmark()
    cfgs = tb.configurations()
    assert [(c.symbols, c.loss_rate, c.symbol_size, c.erased_symbols, c.type) for c in cfgs] == [
        (16, 0.5, 1000000, 8, "encoder"), (16, 0.5, 1000000, 8, "decoder")]


def test_symbol_size_must_be_multiple_of_64():
    tb = rsgpu.ThroughputBenchmark(symbol_size=(1000,))
    with pytest.raises(AssertionError):
        tb.configurations()


@pytest.mark.skipif(not os.path.exists(RUNNER), reason="runner not built")
def test_cpp_runner_usage():
    r = subprocess.run([RUNNER, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--symbols" in r.stdout
    r = subprocess.run([RUNNER, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 2


DROPIN = os.path.join(ROOT, "storage-benchmarks_amd", "bin", "plugin_dropin_test")


@pytest.mark.skipif(not os.path.exists(DROPIN), reason="drop-in test not built")
def test_dropin_rejects_bad_config_before_touching_the_gpu():
    r = subprocess.run([DROPIN, "16-64000-8"], capture_output=True, text=True)
    assert r.returncode == 2 and "symbols:symbol_size:erased" in r.stderr


@pytest.mark.parametrize("k,e,blocks,chunk", [(16, 8, 6, 4), (64, 32, 9, 2), (5, 4, 3, 4), (10, 0, 2, 1)])
def test_survivor_runs_cover_exactly_the_live_rows(k, e, blocks, chunk):
    """bench.survivor_runs (the pipelined host-IO path's decoder-side copies):
    the runs of each chunk are disjoint, lie inside the chunk's blocks and
    cover exactly the non-erased source rows."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    pitch = 256
    err = rsgpu.erasure_patterns(7, 0, blocks, k, e) if e else np.zeros((blocks, 0), np.uint8)
    runs = bench.survivor_runs(err, k, pitch, chunk)
    assert len(runs) == (blocks + chunk - 1) // chunk
    for i, rr in enumerate(runs):
        got = np.zeros(blocks * k, bool)
        for off, n in rr:
            assert off % pitch == 0 and n % pitch == 0 and n > 0
            rows = np.arange(off // pitch, (off + n) // pitch)
            assert not got[rows].any()
            got[rows] = True
        want = np.zeros(blocks * k, bool)
        for blk in range(i * chunk, min(blocks, (i + 1) * chunk)):
            live = np.ones(k, bool)
            live[np.asarray(err[blk], np.int64)] = False
            want[blk * k:(blk + 1) * k] = live
        assert (got == want).all()


def test_every_timed_kernel_has_algorithmic_bytes():
    """Each kernel the C-ABI times under an (encode)/(decode) name is priced
    in bench.alg_bytes: an unpriced one would print alg_GBps 0 and a zero
    roofline when it is the step's dominant kernel."""
    import re

    import bench
    src = open(os.path.join(ROOT, "storage-benchmarks_amd", "csrc", "rsgpu_capi.cpp")).read()
    names = set(re.findall(r'"(k_[a-z0-9_]+\((?:encode|decode)\))"', src))
    assert names, "no timed kernels found"
    priced = bench.alg_bytes(16, 4, 1000)
    missing = sorted(n for n in names if priced.get(n, 0.0) <= 0.0)
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libisal_ref.so")),
                    reason="oracle/_ref not built")
def test_bench_c1_cpu_line():
    """bench.py --config c1: BASELINE configs[0], the reference's CPU path at
    (16, 8, 64000) with the harness accounting (throughput_benchmark.hpp:37-67),
    host only -- the line must come out without a GPU and without loading
    the engine."""
    import json
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--c1-seconds", "0.05",
                        "--cpu-threads", "2"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["device"] == "cpu" and line["n_gpus"] == 0 and line["verified"]
    assert line["config"]["symbols"] == 16 and line["config"]["symbol_size"] == 64000
    assert line["config"]["erased"] == 8
    kinds = [(lg["kind"], lg["threads"]) for lg in line["legs"]]
    assert kinds == [("reference", 1), ("port", 1), ("reference", 2), ("port", 2)]
    for lg in line["legs"]:
        assert lg["failures"] == 0 and lg["encoder_goodput_MBps"] > 0 and lg["decoder_goodput_MBps"] > 0
    assert line["value"] == round(line["legs"][0]["goodput_GiBps"], 4) > 0
    assert line["cpu_baseline"]["kind"] == "reference" and line["cpu_baseline"]["cores"] == 1
    assert "rsgpu" not in r.stderr


def test_bench_c1_rejects_geometry_and_gpus():
    """--config c1 is the reference's fixed CPU case: custom geometry and
    --gpus > 1 (N ranks timing the CPU on shared cores) are refused."""
    import sys
    for extra in (["--symbols", "32"], ["--gpus", "2"], ["--blocks", "3"]):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1"] + extra,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 2 and "c1" in r.stderr, (extra, r.stderr)
