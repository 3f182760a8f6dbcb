"""C ABI of librsgpu.so on CPU: the library loads, exports every entry point
declared in include/rsgpu.h, and its HOST GF helpers (the ISA-L C ABI mirror,
no device work) match the oracle and the reference's golden vectors.
Device entry points are exercised by tests/test_gpu_parity.py (-m gpu).
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

import rsgpu
from oracle_lib import Oracle
from golden.synth import erasure_pattern

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rsgpu.h")
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(rsgpu_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    assert os.path.exists(rsgpu.LIB_PATH), "build librsgpu.so first (make -C storage-benchmarks_amd)"
    out = subprocess.run(["nm", "-D", "--defined-only", rsgpu.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (rsgpu_\w+)", out))
    declared = header_symbols()
    assert declared, "no declarations parsed"
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    # the Python binding table covers the header exactly
    assert rsgpu.EXPORTED_SYMBOLS == declared


def test_library_exports_nothing_beyond_the_header():
    """librsgpu.so's dynamic symbol table is exactly include/rsgpu.h (version
    script csrc/rsgpu.map): no test hooks, no C++ internals."""
    out = subprocess.run(["nm", "-D", "--defined-only", rsgpu.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    text = set(re.findall(r" [TWV] (\S+)", out))
    assert text == set(header_symbols()), sorted(text ^ set(header_symbols()))


def test_test_hooks_live_in_their_own_library():
    out = subprocess.run(["nm", "-D", "--defined-only", rsgpu.HOOKS_PATH], capture_output=True,
                         text=True, check=True).stdout
    hooks = set(re.findall(r" T (rsgpu_internal_\w+)", out))
    assert {"rsgpu_internal_jit_emit", "rsgpu_internal_jitw_emit", "rsgpu_internal_jit_matrix_code",
            "rsgpu_internal_jitw_matrix_code", "rsgpu_internal_jitw_emit_device",
            "rsgpu_internal_set_jitw_tiles", "rsgpu_internal_set_jitw_prefetch"} <= hooks


def test_decode_blocks_null_context_is_an_argument_error():
    """rsgpu_decode_blocks checks its arguments before planning
    (no device work: the call returns before touching the context)."""
    L = rsgpu.lib()
    assert L.rsgpu_decode_blocks(None, 16, 4, 1000000, 1000192, 1, None, None, None, None, None,
                                 None) == -1


def test_library_loads_and_binds():
    L = rsgpu.lib()
    assert L.rsgpu_version().decode().count(".") == 2


def test_host_gf_helpers_match_oracle():
    orc = Oracle()
    for a in range(256):
        assert rsgpu.gf_inv(a) == orc.gf_inv(a)
        for b in (0, 1, 2, 3, 0x1d, 0x80, 0xff, a):
            assert rsgpu.gf_mul(a, b) == orc.gf_mul(a, b)
    for m, k in ((9, 5), (20, 16), (96, 64), (120, 100), (250, 200)):
        assert (rsgpu.gf_gen_rs_matrix(m, k) == orc.gen_rs_matrix(m, k)).all()
        assert (rsgpu.gf_gen_cauchy1_matrix(m, k) == orc.gen_cauchy1_matrix(m, k)).all()
    for c in range(256):
        assert (rsgpu.gf_vect_mul_init(c) == orc.vect_mul_init(c)).all()
    rng = np.random.default_rng(3)
    coef = rng.integers(0, 256, (7, 13), dtype=np.uint8)
    assert (rsgpu.ec_init_tables(13, 7, coef) == orc.init_tables(13, 7, coef)).all()


def test_host_invert_kats():
    for name in ("test1", "test2", "test3", "test4_singular"):
        kat = GOLD["kat"][name]
        n = kat["n"]
        rc, inv = rsgpu.gf_invert_matrix(np.array(kat["in"], np.uint8).reshape(n, n))
        assert rc == kat["rc"]
        if rc == 0:
            assert inv.flatten().tolist() == kat["inv"]


def test_erasure_patterns_match_definition():
    for k, e in ((16, 4), (16, 8), (64, 32), (100, 20), (7, 7), (250, 1)):
        got = rsgpu.erasure_patterns(42, 5, 8, k, e)
        for b in range(8):
            exp = erasure_pattern(42, 5 + b, k, e)
            assert got[b].tolist() == exp.tolist()
            assert len(set(got[b].tolist())) == e and all(x < k for x in got[b])


def test_erasure_patterns_rejects_bad_args():
    with pytest.raises(rsgpu.RsGpuError):
        rsgpu.erasure_patterns(1, 0, 1, 4, 5)


def test_diagnostic_variants_need_the_diagnostic_build():
    """the timing-only variants (csrc/diag_variants.h,
    wrong outputs by design) enter a kernel only through kernel_hooks.h, and a
    stray -DRSGPU_DIAG_VARIANT without the diagnostic library's own flag
    (RSGPU_DIAG_CLOCK, `make diag`) does not compile; the product kernels
    name no variant."""
    csrc = os.path.join(ROOT, "storage-benchmarks_amd", "csrc")
    src = '#include "kernel_hooks.h"\nint main() { return rsgpu::Hooks::kVariant; }\n'
    r = subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-I", csrc, "-DRSGPU_DIAG_VARIANT=3", "-x", "c++",
                        "-"], input=src, capture_output=True, text=True)
    assert r.returncode != 0 and "only the diagnostic library" in r.stderr, r.stderr
    r = subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-I", csrc, "-DRSGPU_DIAG_VARIANT=3",
                        "-DRSGPU_DIAG_CLOCK", "-x", "c++", "-"], input=src, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    for f in ("rs_jit.hip", "rs_bitsliced.hip", "rs_jit.h"):
        text = open(os.path.join(csrc, f)).read()
        assert "RSGPU_DIAG_VAR" not in text and "DIAG_VARIANT" not in text, f
    mk = open(os.path.join(ROOT, "storage-benchmarks_amd", "Makefile")).read()
    product_flags = mk.split("HIPFLAGS ?=")[1].splitlines()[0]
    assert "DIAG" not in product_flags
