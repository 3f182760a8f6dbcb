"""Pin the CPU oracle (oracle/rs_oracle.c) to the reference.

1. Known-answer tests held by the reference's own tests
   (erasure_code/gf_inverse_test.c:124-179, gf_vect_mul_test.c:53-80) and the
   committed golden vectors generated from the reference's ISA-L base C
   (tests/golden/golden.json, gen_golden.py).
2. When oracle/_ref/libisal_ref.so is present (built from /root/reference in
   the build container), random cross-checks oracle vs reference.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_lib import Oracle, Reference, have_reference
from golden.synth import erasure_pattern, synth_block, synth_row

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def sha(b):
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def test_gf_inverse_kats(orc):
    for name in ("test1", "test2", "test3", "test4_singular"):
        kat = GOLD["kat"][name]
        n = kat["n"]
        rc, inv = orc.invert_matrix(np.array(kat["in"], np.uint8).reshape(n, n))
        assert rc == kat["rc"], name
        if rc == 0:
            assert inv.flatten().tolist() == kat["inv"], name


def test_gf_mul_inv_tables(orc):
    assert [int(orc.gf_mul(2, x)) for x in range(256)] == GOLD["kat"]["gf_mul_2"]
    assert [int(orc.gf_inv(x)) for x in range(256)] == GOLD["kat"]["gf_inv"]
    # field axioms on the whole table
    for a in range(1, 256):
        assert orc.gf_mul(a, orc.gf_inv(a)) == 1


def test_vect_mul_init_kat(orc):
    for c, tbl in GOLD["kat"]["vect_mul_init"].items():
        assert orc.vect_mul_init(int(c)).tolist() == tbl


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"k{c['k']}e{c['e']}L{c['len']}")
def test_golden_encode_decode(orc, case):
    k, e, L = case["k"], case["e"], case["len"]
    a = orc.gen_rs_matrix(k + e, k)
    assert a[k:].tobytes().hex() == case["parity_matrix_hex"]
    for b in case["blocks"]:
        data = list(synth_block(GOLD["seed"], b["blk"], k, L))
        assert [sha(d) for d in data] == b["src_sha"]
        par = orc.encode_block(data, e)
        assert [sha(p) for p in par] == b["parity_sha"]
        err = erasure_pattern(GOLD["seed"], b["blk"], k, e)
        assert err.tolist() == b["err"]
        assert orc.erasure_pattern(GOLD["seed"], b["blk"], k, e).tolist() == b["err"]
        rc, rec = orc.decode_block(data, par, err)
        assert rc == 0
        for i in range(e):
            assert (rec[i] == data[err[i]]).all()
        rc, c = orc.decode_matrix(k, e, err)
        assert rc == 0 and sha(c) == b["decode_rows_sha"]


def test_golden_cauchy(orc):
    g = GOLD["cauchy_9_5"]
    ca = orc.gen_cauchy1_matrix(9, 5)
    assert ca.tobytes().hex() == g["matrix_hex"]
    data = list(synth_block(GOLD["seed"], g["blk"], 5, g["len"]))
    tb = orc.init_tables(5, 4, ca[5:])
    par = [np.zeros(g["len"], np.uint8) for _ in range(4)]
    orc.encode_data(g["len"], 5, 4, tb, data, par)
    assert [p.tobytes().hex() for p in par] == g["parity_hex"]


def test_synth_matches_oracle(orc):
    for row in (0, 1, 77, 12345):
        for L in (1, 7, 8, 9, 1000):
            assert (orc.synth_row(99, row, L) == synth_row(99, row, L)).all()
    for blk in range(20):
        for k, e in ((16, 8), (64, 32), (100, 20), (5, 5)):
            assert (orc.erasure_pattern(3, blk, k, e) == erasure_pattern(3, blk, k, e)).all()


needs_ref = pytest.mark.skipif(not have_reference(), reason="oracle/_ref not built")


@needs_ref
def test_oracle_vs_reference_random():
    orc, ref = Oracle(), Reference()
    rng = np.random.default_rng(11)  # TEST_SEED of erasure_code_base_test.c:62
    for _ in range(30):
        k = int(rng.integers(1, 40))
        rows = int(rng.integers(1, 20))
        L = int(rng.integers(1, 700))
        coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
        g1, g2 = orc.init_tables(k, rows, coef), ref.init_tables(k, rows, coef)
        assert (g1 == g2).all()
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        o1 = [np.zeros(L, np.uint8) for _ in range(rows)]
        o2 = [np.zeros(L, np.uint8) for _ in range(rows)]
        orc.encode_data(L, k, rows, g1, data, o1)
        ref.encode_data(L, k, rows, g2, data, o2)
        assert all((x == y).all() for x, y in zip(o1, o2))
        # update path (ec_encode_data_update_base)
        vec_i = int(rng.integers(0, k))
        u1 = [x.copy() for x in o1]
        u2 = [x.copy() for x in o2]
        orc.encode_data_update(L, k, rows, vec_i, g1, data[vec_i], u1)
        ref.encode_data_update(L, k, rows, vec_i, g2, data[vec_i], u2)
        assert all((x == y).all() for x, y in zip(u1, u2))


@needs_ref
def test_invert_vs_reference_random():
    orc, ref = Oracle(), Reference()
    rng = np.random.default_rng(5)
    for _ in range(40):
        n = int(rng.integers(1, 60))
        mat = rng.integers(0, 256, (n, n), dtype=np.uint8)
        if rng.random() < 0.3:  # force singular: duplicate a row
            mat[n - 1] = mat[0]
        r1, i1 = orc.invert_matrix(mat)
        r2, i2 = ref.invert_matrix(mat)
        assert r1 == r2
        if r1 == 0:
            assert (i1 == i2).all()


@needs_ref
def test_rs_and_cauchy_matrices_vs_reference():
    orc, ref = Oracle(), Reference()
    for m, k in ((9, 5), (20, 16), (96, 64), (120, 100), (250, 200)):
        assert (orc.gen_rs_matrix(m, k) == ref.gen_rs_matrix(m, k)).all()
        assert (orc.gen_cauchy1_matrix(m, k) == ref.gen_cauchy1_matrix(m, k)).all()


@needs_ref
def test_avx2_port_equals_reference_base():
    """The CPU baseline's AVX2 data kernel (oracle/isal_avx2_port.c, a
    restatement of gf_{1..4}vect_dot_prod_avx2 + ec_encode_data_avx2) gives the
    reference base C's bytes, as ISA-L's own SIMD-vs-base tests require
    (gf_vect_dot_prod_avx_test.c:162-193): every 4/3/2/1-row pass split and
    lengths with an overlapped tail."""
    ref = Reference()
    if not ref.have_avx2:
        pytest.skip("host CPU has no AVX2")
    rng = np.random.default_rng(11)
    for k, e, L in ((16, 4, 4096), (64, 32, 4096), (100, 20, 1000), (5, 4, 33), (7, 3, 31),
                    (9, 5, 32), (13, 7, 8191), (3, 1, 100), (30, 2, 65)):
        data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        p_base = ref.encode_block(data, e)
        p_avx = ref.encode_block_avx2(data, e)
        assert all((x == y).all() for x, y in zip(p_base, p_avx)), (k, e, L)
        err = np.sort(rng.choice(k, size=min(e, k), replace=False)).astype(np.uint8)
        rc1, r1 = ref.decode_block(data, p_base, err)
        rc2, r2 = ref.decode_block_avx2(data, p_base, err)
        assert rc1 == rc2 == 0
        assert all((x == y).all() for x, y in zip(r1, r2))
        assert all((r2[i] == data[s]).all() for i, s in enumerate(err))


def _general_rows(orc, case):
    k, m, L = case["k"], case["m"], case["len"]
    enc = orc.gen_rs_matrix(m, k) if case["matrix"] == "rs" else orc.gen_cauchy1_matrix(m, k)
    data = list(synth_block(GOLD["seed"], case["blk"], k, L))
    g = orc.init_tables(k, m - k, enc[k:])
    par = [np.zeros(L, np.uint8) for _ in range(m - k)]
    orc.encode_data(L, k, m - k, g, data, par)
    return enc, data + par


@pytest.mark.parametrize("case", GOLD["general_decode"],
                         ids=lambda c: f"{c['matrix']}k{c['k']}m{c['m']}n{len(c['err'])}")
def test_golden_general_decode(orc, case):
    """gf_gen_decode_matrix restated (erasure_code_base_test.c:133-213) ==
    the reference's own function on the golden cases: status, survivor
    choice (including the singular-survivor retry and "BAD MATRIX"), decode
    matrix and recovered rows (data and parity erasures)."""
    enc, rows = _general_rows(orc, case)
    k = case["k"]
    assert [sha(p) for p in rows[k:]] == case["parity_sha"]
    rc, dm, idx = orc.gen_decode_matrix(enc, case["err"])
    assert rc == case["rc"]
    if rc != 0:
        return
    assert idx.tolist() == case["decode_index"]
    assert sha(dm) == case["decode_matrix_sha"]
    rc2, rec = orc.decode_general(enc, rows, case["err"])
    assert rc2 == 0
    assert [sha(r) for r in rec] == case["recovered_sha"]
    assert all((rec[i] == rows[j]).all() for i, j in enumerate(case["err"]))


@needs_ref
def test_general_decode_matrix_vs_reference_random():
    """Random RS / Cauchy codes and erasure lists over data and parity rows:
    the restatement equals the reference's gf_gen_decode_matrix (compiled
    from erasure_code_base_test.c by oracle/Makefile) in status, survivors
    and matrix."""
    orc, ref = Oracle(), Reference()
    rng = np.random.default_rng(13)
    for trial in range(400):
        k = int(rng.integers(1, 60))
        p = int(rng.integers(1, 24))
        m = k + p
        enc = orc.gen_rs_matrix(m, k) if trial % 2 else orc.gen_cauchy1_matrix(m, k)
        n = int(rng.integers(1, p + 1))
        err = np.sort(rng.choice(m, n, replace=False)).astype(np.uint8)
        a, b = orc.gen_decode_matrix(enc, err), ref.gen_decode_matrix(enc, err)
        assert a[0] == b[0]
        if a[0] == 0:
            assert (a[1] == b[1]).all() and (a[2] == b[2]).all()
