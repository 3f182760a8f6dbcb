"""ctypes bindings for the parity checker under oracle/ (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  Two libraries:

* ``oracle/liboracle.so``        -- our CPU restatement (rs_oracle.c)
* ``oracle/_ref/libisal_ref.so`` -- the reference's own ISA-L 2.13 base C,
  compiled in place from /root/reference by oracle/Makefile (absent when the
  reference was never present; tests that need it skip).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libisal_ref.so")

u8p = C.c_void_p
vpp = C.POINTER(C.c_void_p)


def build() -> None:
    """Build oracle/liboracle.so (and _ref/ when the reference is present)."""
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def _ptrs(arrs):
    return (C.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])


class _Lib:
    def __init__(self, path: str, prefix: str):
        self.lib = C.CDLL(path)
        self.p = prefix

    def fn(self, name, restype, *argtypes):
        f = getattr(self.lib, self.p + name)
        f.restype = restype
        f.argtypes = list(argtypes)
        return f


class Oracle:
    """Our restatement (kind "port")."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build()
        L = _Lib(path, "orc_")
        self.gf_mul = L.fn("gf_mul", C.c_ubyte, C.c_ubyte, C.c_ubyte)
        self.gf_inv = L.fn("gf_inv", C.c_ubyte, C.c_ubyte)
        self._gen_rs = L.fn("gen_rs_matrix", None, u8p, C.c_int, C.c_int)
        self._gen_cauchy = L.fn("gen_cauchy1_matrix", None, u8p, C.c_int, C.c_int)
        self._inv = L.fn("invert_matrix", C.c_int, u8p, u8p, C.c_int)
        self._mul_init = L.fn("vect_mul_init", None, C.c_ubyte, u8p)
        self._init_tables = L.fn("init_tables", None, C.c_int, C.c_int, u8p, u8p)
        self._encode_data = L.fn("encode_data", None, C.c_int, C.c_int, C.c_int, u8p, vpp, vpp)
        self._update = L.fn("encode_data_update", None, C.c_int, C.c_int, C.c_int, C.c_int,
                            u8p, u8p, vpp)
        self._vect_mul = L.fn("vect_mul", None, C.c_int, u8p, u8p, u8p)
        self._enc_block = L.fn("encode_block", None, C.c_int, C.c_int, C.c_int, vpp, vpp)
        self._dec_block = L.fn("decode_block", C.c_int, C.c_int, C.c_int, C.c_int, u8p,
                               vpp, vpp, vpp)
        self._dec_matrix = L.fn("decode_matrix", C.c_int, C.c_int, C.c_int, u8p, u8p)
        self._gen_dec = L.fn("gen_decode_matrix", C.c_int, u8p, C.c_int, C.c_int, u8p, C.c_int,
                             u8p, u8p)
        self._dec_general = L.fn("decode_general", C.c_int, u8p, C.c_int, C.c_int, C.c_int, u8p,
                                 C.c_int, vpp, vpp)
        self.synth_word = L.fn("synth_word", C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64)
        self._synth_row = L.fn("synth_row", None, C.c_uint64, C.c_uint64, u8p, C.c_size_t)
        self._pattern = L.fn("erasure_pattern", None, C.c_uint64, C.c_uint64, C.c_int,
                             C.c_int, u8p)

    # -- ISA-L-shaped helpers ------------------------------------------------
    def gen_rs_matrix(self, m: int, k: int) -> np.ndarray:
        a = np.zeros(m * k, np.uint8)
        self._gen_rs(a.ctypes.data, m, k)
        return a.reshape(m, k)

    def gen_cauchy1_matrix(self, m: int, k: int) -> np.ndarray:
        a = np.zeros(m * k, np.uint8)
        self._gen_cauchy(a.ctypes.data, m, k)
        return a.reshape(m, k)

    def invert_matrix(self, mat: np.ndarray):
        n = mat.shape[0]
        inp = np.ascontiguousarray(mat, np.uint8).copy()
        out = np.zeros((n, n), np.uint8)
        rc = self._inv(inp.ctypes.data, out.ctypes.data, n)
        return rc, out

    def vect_mul_init(self, c: int) -> np.ndarray:
        t = np.zeros(32, np.uint8)
        self._mul_init(c, t.ctypes.data)
        return t

    def init_tables(self, k: int, rows: int, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, np.uint8)
        g = np.zeros(32 * k * max(rows, 1), np.uint8)
        self._init_tables(k, rows, a.ctypes.data, g.ctypes.data)
        return g

    def encode_data(self, length, k, rows, g, data, coding) -> None:
        self._encode_data(length, k, rows, g.ctypes.data, _ptrs(data), _ptrs(coding))

    def encode_data_update(self, length, k, rows, vec_i, g, data, coding) -> None:
        self._update(length, k, rows, vec_i, g.ctypes.data, data.ctypes.data, _ptrs(coding))

    def vect_mul(self, length, tbl, src, dest) -> None:
        self._vect_mul(length, tbl.ctypes.data, src.ctypes.data, dest.ctypes.data)

    # -- block helpers mirroring isa.cpp -------------------------------------
    def encode_block(self, data, e: int):
        k, L = len(data), data[0].shape[0]
        par = [np.zeros(L, np.uint8) for _ in range(e)]
        self._enc_block(k, e, L, _ptrs(data), _ptrs(par))
        return par

    def decode_block(self, data, parity, err_list):
        k, e, L = len(data), len(parity), data[0].shape[0]
        err = np.ascontiguousarray(err_list, np.uint8)
        out = [np.zeros(L, np.uint8) for _ in range(e)]
        rc = self._dec_block(k, e, L, err.ctypes.data, _ptrs(data), _ptrs(parity), _ptrs(out))
        return rc, out

    def decode_matrix(self, k: int, e: int, err_list):
        err = np.ascontiguousarray(err_list, np.uint8)
        c = np.zeros(k * max(e, 1), np.uint8)
        rc = self._dec_matrix(k, e, err.ctypes.data, c.ctypes.data)
        return rc, c[: k * e].reshape(e, k)

    def gen_decode_matrix(self, encode_matrix: np.ndarray, err_list):
        """erasure_code_base_test.c:133-213 -> (rc, decode_matrix [nerrs][k],
        decode_index [k]); rc -2 = NO_INVERT_MATRIX."""
        m, k = encode_matrix.shape
        enc = np.ascontiguousarray(encode_matrix, np.uint8)
        err = np.ascontiguousarray(err_list, np.uint8)
        dm = np.zeros(max(1, len(err)) * k, np.uint8)
        idx = np.zeros(k, np.int32)
        rc = self._gen_dec(enc.ctypes.data, k, m, err.ctypes.data, len(err), dm.ctypes.data,
                           idx.ctypes.data)
        return rc, dm[: len(err) * k].reshape(len(err), k), idx

    def decode_general(self, encode_matrix: np.ndarray, rows, err_list):
        """Recover rows err_list (data and parity) from the m rows `rows` (the
        erased ones are not read) -> (rc, [nerrs rows])."""
        m, k = encode_matrix.shape
        enc = np.ascontiguousarray(encode_matrix, np.uint8)
        err = np.ascontiguousarray(err_list, np.uint8)
        L = rows[0].shape[0]
        out = [np.zeros(L, np.uint8) for _ in range(len(err))]
        rc = self._dec_general(enc.ctypes.data, k, m, L, err.ctypes.data, len(err), _ptrs(rows),
                               _ptrs(out))
        return rc, out

    def synth_row(self, seed: int, row: int, length: int) -> np.ndarray:
        d = np.zeros(length, np.uint8)
        self._synth_row(seed, row, d.ctypes.data, length)
        return d

    def erasure_pattern(self, seed: int, blk: int, k: int, e: int) -> np.ndarray:
        err = np.zeros(max(e, 1), np.uint8)
        self._pattern(seed, blk, k, e, err.ctypes.data)
        return err[:e]


class Reference:
    """The reference's own ISA-L base C (kind "reference")."""

    def __init__(self, path: str = REF_SO):
        L = _Lib(path, "ref_")
        self.gf_mul = L.fn("gf_mul", C.c_ubyte, C.c_ubyte, C.c_ubyte)
        self.gf_inv = L.fn("gf_inv", C.c_ubyte, C.c_ubyte)
        self._gen_rs = L.fn("gf_gen_rs_matrix", None, u8p, C.c_int, C.c_int)
        self._gen_cauchy = L.fn("gf_gen_cauchy1_matrix", None, u8p, C.c_int, C.c_int)
        self._inv = L.fn("gf_invert_matrix", C.c_int, u8p, u8p, C.c_int)
        self._mul_init = L.fn("gf_vect_mul_init", None, C.c_ubyte, u8p)
        self._init_tables = L.fn("ec_init_tables", None, C.c_int, C.c_int, u8p, u8p)
        self._encode_data = L.fn("ec_encode_data", None, C.c_int, C.c_int, C.c_int, u8p, vpp,
                                 vpp)
        self._update = L.fn("ec_encode_data_update", None, C.c_int, C.c_int, C.c_int, C.c_int,
                            u8p, u8p, vpp)
        self._vect_mul = L.fn("gf_vect_mul", None, C.c_int, u8p, u8p, u8p)
        self._enc_block = L.fn("encode_block", None, C.c_int, C.c_int, C.c_int, vpp, vpp)
        self._dec_block = L.fn("decode_block", C.c_int, C.c_int, C.c_int, C.c_int, u8p,
                               vpp, vpp, vpp)
        self._bench = L.fn("cpu_bench_kernel", C.c_double, C.c_int, C.c_int, C.c_int, C.c_int,
                           C.c_int, C.c_uint64, C.c_int, C.POINTER(C.c_double),
                           C.POINTER(C.c_double), C.POINTER(C.c_double),
                           C.POINTER(C.c_int))
        # the AVX2 restatement of ISA-L's asm data kernel (isal_avx2_port.c)
        self._enc_avx2 = L.fn("encode_block_avx2", None, C.c_int, C.c_int, C.c_int, vpp, vpp)
        self._dec_avx2 = L.fn("decode_block_avx2", C.c_int, C.c_int, C.c_int, C.c_int, u8p,
                              vpp, vpp, vpp)
        self.have_avx2 = bool(L.fn("have_avx2", C.c_int)())
        # erasure_code_base_test.c's own static gf_gen_decode_matrix
        # (ref_decode_matrix.c)
        self._gen_dec = L.fn("gf_gen_decode_matrix", C.c_int, u8p, u8p, u8p, u8p, C.c_int,
                             C.c_int, C.c_int)

    def gen_decode_matrix(self, encode_matrix: np.ndarray, err_list):
        m, k = encode_matrix.shape
        enc = np.ascontiguousarray(encode_matrix, np.uint8).copy()
        err = np.ascontiguousarray(err_list, np.uint8).copy()
        dm = np.zeros(max(1, len(err)) * k, np.uint8)
        idx = np.zeros(k, np.uint32)
        rc = self._gen_dec(enc.ctypes.data, dm.ctypes.data, idx.ctypes.data, err.ctypes.data,
                           len(err), k, m)
        return rc, dm[: len(err) * k].reshape(len(err), k), idx.astype(np.int32)

    gen_rs_matrix = Oracle.gen_rs_matrix
    gen_cauchy1_matrix = Oracle.gen_cauchy1_matrix
    invert_matrix = Oracle.invert_matrix
    vect_mul_init = Oracle.vect_mul_init
    init_tables = Oracle.init_tables
    encode_data = Oracle.encode_data
    encode_data_update = Oracle.encode_data_update
    vect_mul = Oracle.vect_mul
    encode_block = Oracle.encode_block
    decode_block = Oracle.decode_block

    def encode_block_avx2(self, data, e: int):
        k, L = len(data), data[0].shape[0]
        par = [np.zeros(L, np.uint8) for _ in range(e)]
        self._enc_avx2(k, e, L, _ptrs(data), _ptrs(par))
        return par

    def decode_block_avx2(self, data, parity, err_list):
        k, e, L = len(data), len(parity), data[0].shape[0]
        err = np.ascontiguousarray(err_list, np.uint8)
        out = [np.zeros(L, np.uint8) for _ in range(e)]
        rc = self._dec_avx2(k, e, L, err.ctypes.data, _ptrs(data), _ptrs(parity), _ptrs(out))
        return rc, out

    def cpu_bench(self, k, e, length, threads, blocks_per_thread, seed=1, kernel=0):
        """kernel 0: the reference's ec_encode_data_base; 1: the AVX2 port."""
        es, ds, mx, f = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        wall = self._bench(k, e, length, threads, blocks_per_thread, seed, kernel, C.byref(es),
                           C.byref(ds), C.byref(mx), C.byref(f))
        return {"wall_s": wall, "enc_s": es.value, "dec_s": ds.value,
                "max_thread_s": mx.value, "failures": f.value}


def have_reference() -> bool:
    return os.path.exists(REF_SO)
