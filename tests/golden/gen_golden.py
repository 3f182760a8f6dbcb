"""Generate tests/golden/golden.json from the REFERENCE's own ISA-L 2.13 base C.

Run in the container where /root/reference exists (oracle/Makefile compiles the
reference sources into oracle/_ref/libisal_ref.so):

    make -C oracle && python tests/golden/gen_golden.py

The committed JSON holds data only -- inputs (seed, geometry, erasure lists,
fixed matrices) and the reference's outputs (matrices, tables, parity and
recovered bytes or their SHA-256) -- so the GPU box, where the reference is
absent, can check both the oracle and the engine against them.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from oracle_lib import Reference  # noqa: E402
from synth import erasure_pattern, synth_block  # noqa: E402

SEED = 20240611

# (k, e, len): SURVEY.md 8(c) fixture list + odd lengths
CASES = [
    (5, 4, 8192), (16, 4, 4096), (16, 8, 64000), (64, 32, 4096), (100, 20, 4096),
    (16, 8, 8191), (10, 4, 33), (10, 4, 17), (4, 2, 1), (20, 5, 1000),
]
BLOCKS = 2

# general decode cases: (matrix, k, m, len, block, erased rows ascending)
GENERAL = [
    ("cauchy", 5, 9, 256, 7, [1, 3, 6, 8]),
    ("rs", 10, 14, 4096, 1, [2, 4, 11, 13]),
    ("cauchy", 12, 20, 2048, 2, [12, 13, 14, 15, 16, 17, 18, 19]),
    ("rs", 64, 96, 4096, 3, [0, 5, 9, 17, 30, 31, 44, 63, 64, 70, 81, 95]),
    ("rs", 100, 120, 2048, 4, [3, 50, 99, 100, 119]),
    ("cauchy", 40, 72, 1024, 5, list(range(20, 52))),
    ("rs", 144, 163, 1024, 6, [12, 16, 41, 49, 58, 68, 73, 75, 95, 97, 110, 113, 115, 145, 156]),
    ("rs", 150, 177, 1024, 7, [1, 6, 34, 44, 46, 48, 51, 70, 83, 110, 111, 120, 130, 142, 157, 176]),
    ("rs", 121, 137, 1024, 8, [2, 25, 26, 38, 42, 43, 44, 47, 48, 63, 84, 89, 90, 113, 117, 129]),
]


def sha(b: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


def main() -> None:
    ref = Reference()
    out = {"generator": "tests/golden/gen_golden.py",
           "reference": "isa-l_open_src_2.13 isa/ec_base.c + isa/ec_highlevel_func.c "
                        "(compiled by oracle/Makefile), driven as benchmark/isa_throughput/isa.cpp",
           "seed": SEED, "cases": [], "kat": {}}

    for k, e, L in CASES:
        m = k + e
        a = ref.gen_rs_matrix(m, k)
        case = {"k": k, "e": e, "len": L, "blocks": []}
        case["parity_matrix_hex"] = a[k:].tobytes().hex()
        for blk in range(BLOCKS):
            data = [row for row in synth_block(SEED, blk, k, L)]
            par = ref.encode_block(data, e)
            err = erasure_pattern(SEED, blk, k, e)
            rc, rec = ref.decode_block(data, par, err)
            assert rc == 0
            assert all((rec[i] == data[err[i]]).all() for i in range(e))
            b = {"blk": blk, "err": err.tolist(),
                 "src_sha": [sha(d) for d in data],
                 "parity_sha": [sha(p) for p in par],
                 "parity_head_hex": [p[:32].tobytes().hex() for p in par]}
            # decode coefficient rows exactly as decode_all builds them
            in_err = np.zeros(m, bool)
            in_err[err] = True
            surv = [r for r in range(m) if not in_err[r]][:k]
            rcinv, inv = ref.invert_matrix(a[surv])
            assert rcinv == 0
            b["decode_rows_sha"] = sha(inv[err])
            if k * L <= 4096:
                b["parity_hex"] = [p.tobytes().hex() for p in par]
            case["blocks"].append(b)
        out["cases"].append(case)

    # Cauchy (erasure_code_base_test.c:333-399 uses gf_gen_cauchy1_matrix(9,5))
    ca = ref.gen_cauchy1_matrix(9, 5)
    data = [row for row in synth_block(SEED, 7, 5, 256)]
    g = ref.init_tables(5, 4, ca[5:])
    par = [np.zeros(256, np.uint8) for _ in range(4)]
    ref.encode_data(256, 5, 4, g, data, par)
    out["cauchy_9_5"] = {"matrix_hex": ca.tobytes().hex(), "blk": 7, "len": 256,
                         "parity_hex": [p.tobytes().hex() for p in par]}

    # General decode (erasure_code_base_test.c:133-213 gf_gen_decode_matrix,
    # the test's own static function compiled from the reference, and the
    # recovery of :299-308): erasures among data AND parity rows, RS and
    # Cauchy matrices; the two RS cases at k 144 / 150 take the singular-
    # survivor retry, the k 121 case ends in "BAD MATRIX".
    out["general_decode"] = []
    for kind, k, m, L, blk, err in GENERAL:
        enc = ref.gen_rs_matrix(m, k) if kind == "rs" else ref.gen_cauchy1_matrix(m, k)
        data = [row for row in synth_block(SEED, blk, k, L)]
        g = ref.init_tables(k, m - k, enc[k:])
        par = [np.zeros(L, np.uint8) for _ in range(m - k)]
        ref.encode_data(L, k, m - k, g, data, par)
        rows = data + par
        rc, dm, idx = ref.gen_decode_matrix(enc, err)
        case = {"matrix": kind, "k": k, "m": m, "len": L, "blk": blk, "err": err, "rc": rc,
                "parity_sha": [sha(p) for p in par]}
        if rc == 0:
            recov = [rows[i] for i in idx]
            gd = ref.init_tables(k, len(err), dm)
            rec = [np.zeros(L, np.uint8) for _ in err]
            ref.encode_data(L, k, len(err), gd, recov, rec)
            assert all((rec[i] == rows[err[i]]).all() for i in range(len(err)))
            case["decode_index"] = idx.tolist()
            case["decode_matrix_sha"] = sha(dm)
            case["recovered_sha"] = [sha(r) for r in rec]
        out["general_decode"].append(case)

    # KATs from erasure_code/gf_inverse_test.c:124-143, :172-179
    kat = {}
    mats = {"test1": [1, 1, 6, 1, 1, 1, 7, 1, 9], "test2": [0, 1, 6, 1, 0, 1, 0, 1, 9],
            "test3": [0, 0, 1, 1, 0, 0, 0, 1, 1],
            "test4_singular": [0, 1, 6, 7, 1, 1, 0, 0, 0, 1, 2, 3, 3, 2, 2, 3]}
    for name, v in mats.items():
        n = int(round(len(v) ** 0.5))
        rc, inv = ref.invert_matrix(np.array(v, np.uint8).reshape(n, n))
        kat[name] = {"n": n, "in": v, "rc": rc, "inv": inv.flatten().tolist() if rc == 0 else None}
    # gf_vect_mul_test.c:53-80: tables and x2 products
    kat["vect_mul_init"] = {str(c): ref.vect_mul_init(c).tolist() for c in (0, 1, 2, 3, 0x1d, 0x8e, 0xff)}
    kat["gf_mul_2"] = [int(ref.gf_mul(2, x)) for x in range(256)]
    kat["gf_inv"] = [int(ref.gf_inv(x)) for x in range(256)]
    out["kat"] = kat

    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
