"""rsgpu -- Python host side of the MI355X Reed-Solomon engine (librsgpu.so).

Mirrors the plugin interface of steinwurf/storage-benchmarks'
``benchmark/isa_throughput`` over the C ABI declared in ``include/rsgpu.h``:

* :class:`GpuEncoder` / :class:`GpuDecoder` satisfy the Encoder/Decoder concept
  of ``throughput_benchmark<Encoder, Decoder>`` (benchmark/throughput_benchmark.hpp:
  165-196): ``encode_all()``, ``payload_count()``, ``block_size()``,
  ``decode_all(encoder)``, ``is_complete()``, ``verify_data(encoder)`` -- the
  same names, argument meaning and error behaviour as ``isa_encoder`` /
  ``isa_decoder`` (benchmark/isa_throughput/isa.cpp:29-259), extended with a
  ``blocks`` count: a GPU plugin object owns ``blocks`` independent
  (symbols x symbol_size) blocks, laid out contiguously in HBM.
* :class:`ThroughputBenchmark` restates the harness' configuration
  cross-product and goodput accounting (throughput_benchmark.hpp:37-163).
* Module-level functions mirror the ISA-L C ABI the plugin calls
  (isa-l_open_src_2.13/isa/erasure_code.h).

PyTorch is used only as plumbing: device buffers and the HIP stream.  There is
no CPU fallback: if the HIP library or a GPU is missing every device call
raises.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

__all__ = [
    "RsGpuError", "lib", "Context", "GpuEncoder", "GpuDecoder", "ThroughputBenchmark",
    "gf_mul", "gf_inv", "gf_gen_rs_matrix", "gf_gen_cauchy1_matrix", "gf_invert_matrix",
    "gf_vect_mul_init", "ec_init_tables", "erasure_patterns", "EXPORTED_SYMBOLS",
    "LIB_PATH",
]

HERE = os.path.dirname(os.path.abspath(__file__))
# RSGPU_LIB: another build of the same ABI (tools/bound_probe.py loads the
# diagnostic build, tools/diag/librsgpu_diag.so); the product is librsgpu.so
LIB_PATH = os.environ.get("RSGPU_LIB") or os.path.join(HERE, "librsgpu.so")

RSGPU_OK = 0
ERRORS = {-1: "RSGPU_ERR_ARG", -2: "RSGPU_ERR_HIP", -3: "RSGPU_ERR_SINGULAR",
          -4: "RSGPU_ERR_NOMEM", -5: "RSGPU_ERR_UNSUPPORTED"}
MAX_SOURCES = 250  # TEST_SOURCES, isa.cpp:25-27
# rsgpu_set_decode_kernel choices (include/rsgpu.h)
DECODE_KERNELS = {"auto": 0, "one_matrix": 1, "general": 3, "generated": 4,
                  "fused": 2}  # deprecated alias of one_matrix (rsgpu.h RSGPU_DECODE_FUSED)
# rsgpu_set_encode_kernel choices (include/rsgpu.h)
ENCODE_KERNELS = {"auto": 0, "compiled": 1, "generated": 2, "threaded": 3}

vp = C.c_void_p
sz = C.c_size_t

# name -> (restype, argtypes); must match include/rsgpu.h (checked by tests)
_SIGS = {
    "rsgpu_version": (C.c_char_p, []),
    "rsgpu_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "rsgpu_destroy": (C.c_int, [vp]),
    "rsgpu_set_stream": (C.c_int, [vp, vp]),
    "rsgpu_get_stream": (vp, [vp]),
    "rsgpu_synchronize": (C.c_int, [vp]),
    "rsgpu_last_error": (C.c_char_p, [vp]),
    "rsgpu_timing_enable": (C.c_int, [vp, C.c_int]),
    "rsgpu_timing_read": (C.c_int, [vp, C.POINTER(C.c_char_p), C.POINTER(C.c_float),
                                   C.POINTER(C.c_size_t), C.c_int]),
    "rsgpu_malloc": (C.c_int, [vp, C.POINTER(vp), sz]),
    "rsgpu_free": (C.c_int, [vp, vp]),
    "rsgpu_memcpy_h2d": (C.c_int, [vp, vp, vp, sz]),
    "rsgpu_memcpy_d2h": (C.c_int, [vp, vp, vp, sz]),
    "rsgpu_gf_mul": (C.c_ubyte, [C.c_ubyte, C.c_ubyte]),
    "rsgpu_gf_inv": (C.c_ubyte, [C.c_ubyte]),
    "rsgpu_gf_gen_rs_matrix": (None, [vp, C.c_int, C.c_int]),
    "rsgpu_gf_gen_cauchy1_matrix": (None, [vp, C.c_int, C.c_int]),
    "rsgpu_gf_invert_matrix": (C.c_int, [vp, vp, C.c_int]),
    "rsgpu_gf_vect_mul_init": (None, [C.c_ubyte, vp]),
    "rsgpu_ec_init_tables": (None, [C.c_int, C.c_int, vp, vp]),
    "rsgpu_ec_encode_data": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, C.POINTER(vp),
                                       C.POINTER(vp)]),
    "rsgpu_ec_encode_data_update": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp,
                                              C.POINTER(vp)]),
    "rsgpu_gf_vect_dot_prod": (C.c_int, [vp, C.c_int, C.c_int, vp, C.POINTER(vp), vp]),
    "rsgpu_gf_vect_mad": (C.c_int, [vp, C.c_int, C.c_int, C.c_int, vp, vp, vp]),
    "rsgpu_gf_vect_mul": (C.c_int, [vp, C.c_int, vp, vp, vp]),
    "rsgpu_encode_blocks": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp]),
    "rsgpu_decode_workspace_bytes": (sz, [C.c_int, C.c_int, sz]),
    "rsgpu_set_decode_kernel": (C.c_int, [vp, C.c_int]),
    "rsgpu_set_encode_kernel": (C.c_int, [vp, C.c_int]),
    "rsgpu_decode_general_workspace_bytes": (sz, [C.c_int, C.c_int, C.c_int, sz]),
    "rsgpu_decode_general": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp, C.c_int,
                                       vp, vp, vp]),
    "rsgpu_decode_blocks": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp, vp, vp]),
    "rsgpu_decode_prepare": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp, vp,
                                       vp]),
    "rsgpu_decode_apply": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp, vp]),
    "rsgpu_verify_blocks": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp]),
    "rsgpu_host_alloc": (C.c_int, [vp, C.POINTER(vp), sz]),
    "rsgpu_host_free": (C.c_int, [vp, vp]),
    "rsgpu_encode_blocks_host": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp]),
    "rsgpu_decode_blocks_host": (C.c_int, [vp, C.c_int, C.c_int, sz, sz, sz, vp, vp, vp, vp, vp]),
    "rsgpu_fill_synthetic": (C.c_int, [vp, vp, sz, sz, sz, C.c_uint64, C.c_uint64]),
    "rsgpu_erasure_patterns": (C.c_int, [C.c_uint64, C.c_uint64, sz, C.c_int, C.c_int, vp]),
}
EXPORTED_SYMBOLS = sorted(_SIGS)


class RsGpuError(RuntimeError):
    pass


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load librsgpu.so (built in-tree by storage-benchmarks_amd/Makefile)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RsGpuError(
                f"{LIB_PATH} is missing: build it with `make -C storage-benchmarks_amd` "
                "(there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


HOOKS_PATH = os.path.join(HERE, "librsgpu_testhooks.so")
_hooks: Optional[C.CDLL] = None


def testhooks() -> C.CDLL:
    """The test / A-B hook library (rsgpu_testhooks.cpp), NOT the product:
    host emitters of the generated code for the CPU suite, the device emitter
    and the generated decode's layout knobs (rsgpu_internal_*).  librsgpu.so
    itself exports only include/rsgpu.h."""
    global _hooks
    if _hooks is None:
        if not os.path.exists(HOOKS_PATH):
            raise RsGpuError(f"{HOOKS_PATH} is missing: build it with `make -C storage-benchmarks_amd`")
        _hooks = C.CDLL(HOOKS_PATH)
    return _hooks


def _ptr(x) -> int:
    """Raw address of a torch tensor, numpy array or int."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(type(x))


# ---- host GF helpers (ISA-L C ABI) -----------------------------------------

def gf_mul(a: int, b: int) -> int:
    return lib().rsgpu_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().rsgpu_gf_inv(a)


def gf_gen_rs_matrix(m: int, k: int) -> np.ndarray:
    a = np.zeros(m * k, np.uint8)
    lib().rsgpu_gf_gen_rs_matrix(a.ctypes.data, m, k)
    return a.reshape(m, k)


def gf_gen_cauchy1_matrix(m: int, k: int) -> np.ndarray:
    a = np.zeros(m * k, np.uint8)
    lib().rsgpu_gf_gen_cauchy1_matrix(a.ctypes.data, m, k)
    return a.reshape(m, k)


def gf_invert_matrix(mat: np.ndarray):
    """Returns (rc, inverse); rc = -1 for a singular matrix (ec_base.c:120)."""
    n = mat.shape[0]
    inp = np.ascontiguousarray(mat, np.uint8).copy()
    out = np.zeros((n, n), np.uint8)
    rc = lib().rsgpu_gf_invert_matrix(inp.ctypes.data, out.ctypes.data, n)
    return rc, out


def gf_vect_mul_init(c: int) -> np.ndarray:
    t = np.zeros(32, np.uint8)
    lib().rsgpu_gf_vect_mul_init(c, t.ctypes.data)
    return t


def ec_init_tables(k: int, rows: int, a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, np.uint8)
    g = np.zeros(32 * k * max(rows, 1), np.uint8)
    lib().rsgpu_ec_init_tables(k, rows, a.ctypes.data, g.ctypes.data)
    return g


def erasure_patterns(seed: int, blk0: int, blocks: int, k: int, e: int) -> np.ndarray:
    out = np.zeros((max(blocks, 1), max(e, 1)), np.uint8)
    rc = lib().rsgpu_erasure_patterns(seed, blk0, blocks, k, e, out.ctypes.data)
    if rc != RSGPU_OK:
        raise RsGpuError(f"rsgpu_erasure_patterns: {ERRORS.get(rc, rc)}")
    return out[:blocks, :e]


# ---- device context ---------------------------------------------------------

class Context:
    """One engine context per device (and per host thread / rank)."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        self._h = vp()
        rc = lib().rsgpu_create(device, C.byref(self._h))
        if rc != RSGPU_OK:
            raise RsGpuError(f"rsgpu_create(device={device}) failed: {ERRORS.get(rc, rc)}")
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            lib().rsgpu_destroy(self._h)
            self._h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str) -> None:
        if rc != RSGPU_OK:
            msg = lib().rsgpu_last_error(self._h)
            raise RsGpuError(f"{what}: {ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")

    def set_stream(self, stream: int) -> None:
        self.check(lib().rsgpu_set_stream(self._h, stream), "rsgpu_set_stream")

    def get_stream(self) -> int:
        return lib().rsgpu_get_stream(self._h) or 0

    def set_torch_stream(self) -> None:
        import torch
        self.set_stream(torch.cuda.current_stream().cuda_stream)

    def set_encode_kernel(self, kernel: str) -> None:
        """Encode kernel of encode_blocks / ec_encode_data: auto | compiled |
        generated | threaded (include/rsgpu.h rsgpu_set_encode_kernel)."""
        self.check(lib().rsgpu_set_encode_kernel(self._h, ENCODE_KERNELS[kernel]),
                   "rsgpu_set_encode_kernel")

    def set_decode_kernel(self, kernel: str) -> None:
        """Decode kernel of decode_blocks: auto | one_matrix | general |
        generated (include/rsgpu.h rsgpu_set_decode_kernel)."""
        self.check(lib().rsgpu_set_decode_kernel(self._h, DECODE_KERNELS[kernel]),
                   "rsgpu_set_decode_kernel")

    def timing_enable(self, on: bool = True) -> None:
        self.check(lib().rsgpu_timing_enable(self._h, 1 if on else 0), "rsgpu_timing_enable")

    def timing_read(self, max_records: int = 4096):
        """[(kernel name, ms, blocks)] of the kernels enqueued since the last read."""
        names = (C.c_char_p * max_records)()
        ms = (C.c_float * max_records)()
        blocks = (C.c_size_t * max_records)()
        n = lib().rsgpu_timing_read(self._h, names, ms, blocks, max_records)
        if n < 0:
            self.check(n, "rsgpu_timing_read")
        return [(names[i].decode(), float(ms[i]), int(blocks[i])) for i in range(n)]

    def synchronize(self) -> None:
        self.check(lib().rsgpu_synchronize(self._h), "rsgpu_synchronize")

    # ISA-L-shaped device calls
    def ec_encode_data(self, length: int, k: int, rows: int, gftbls: np.ndarray,
                       data: Sequence, coding: Sequence) -> None:
        dp = (vp * max(k, 1))(*[_ptr(d) for d in data])
        cp = (vp * max(rows, 1))(*[_ptr(c) for c in coding])
        g = np.ascontiguousarray(gftbls, np.uint8)
        self.check(lib().rsgpu_ec_encode_data(self._h, length, k, rows, g.ctypes.data, dp, cp),
                   "rsgpu_ec_encode_data")

    def ec_encode_data_update(self, length: int, k: int, rows: int, vec_i: int,
                              gftbls: np.ndarray, data, coding: Sequence) -> None:
        cp = (vp * max(rows, 1))(*[_ptr(c) for c in coding])
        g = np.ascontiguousarray(gftbls, np.uint8)
        self.check(lib().rsgpu_ec_encode_data_update(self._h, length, k, rows, vec_i,
                                                     g.ctypes.data, _ptr(data), cp),
                   "rsgpu_ec_encode_data_update")

    def gf_vect_dot_prod(self, length: int, vlen: int, gftbls: np.ndarray, src: Sequence, dest) -> None:
        """erasure_code.h gf_vect_dot_prod: dest = XOR_j c[j] * src[j]."""
        sp = (vp * max(vlen, 1))(*[_ptr(x) for x in src])
        g = np.ascontiguousarray(gftbls, np.uint8)
        self.check(lib().rsgpu_gf_vect_dot_prod(self._h, length, vlen, g.ctypes.data, sp, _ptr(dest)),
                   "rsgpu_gf_vect_dot_prod")

    def gf_vect_mad(self, length: int, vec: int, vec_i: int, gftbls: np.ndarray, src, dest) -> None:
        """erasure_code.h gf_vect_mad: dest ^= c[vec_i] * src."""
        g = np.ascontiguousarray(gftbls, np.uint8)
        self.check(lib().rsgpu_gf_vect_mad(self._h, length, vec, vec_i, g.ctypes.data, _ptr(src), _ptr(dest)),
                   "rsgpu_gf_vect_mad")

    def gf_vect_mul(self, length: int, gftbl: np.ndarray, src, dest) -> int:
        """gf_vect_mul.h gf_vect_mul: dest = c * src; returns the status
        (non-zero when length is not a multiple of 32, as ISA-L's)."""
        g = np.ascontiguousarray(gftbl, np.uint8)
        return lib().rsgpu_gf_vect_mul(self._h, length, g.ctypes.data, _ptr(src), _ptr(dest))

    # batched calls
    def encode_blocks(self, k, e, length, pitch, blocks, d_src, d_par, coef=None) -> None:
        cptr = None
        if coef is not None:
            coef = np.ascontiguousarray(coef, np.uint8)
            cptr = coef.ctypes.data
        self.check(lib().rsgpu_encode_blocks(self._h, k, e, length, pitch, blocks, _ptr(d_src),
                                             _ptr(d_par), cptr), "rsgpu_encode_blocks")

    def decode_blocks(self, k, e, length, pitch, blocks, d_src, d_par, d_err, d_out, d_ws,
                      d_status) -> None:
        self.check(lib().rsgpu_decode_blocks(self._h, k, e, length, pitch, blocks, _ptr(d_src),
                                             _ptr(d_par), _ptr(d_err), _ptr(d_out), _ptr(d_ws),
                                             _ptr(d_status)), "rsgpu_decode_blocks")

    def decode_prepare(self, k, e, length, pitch, blocks, d_src, d_par, d_err, d_out, d_ws,
                       d_status) -> None:
        self.check(lib().rsgpu_decode_prepare(self._h, k, e, length, pitch, blocks, _ptr(d_src),
                                              _ptr(d_par), _ptr(d_err), _ptr(d_out), _ptr(d_ws),
                                              _ptr(d_status)), "rsgpu_decode_prepare")

    def decode_apply(self, k, e, length, pitch, blocks, d_src, d_par, d_out, d_ws,
                     d_status) -> None:
        self.check(lib().rsgpu_decode_apply(self._h, k, e, length, pitch, blocks, _ptr(d_src),
                                            _ptr(d_par), _ptr(d_out), _ptr(d_ws), _ptr(d_status)),
                   "rsgpu_decode_apply")

    # host-resident calls (include/rsgpu.h): numpy arrays or pinned torch
    # CPU tensors; synchronous
    def encode_blocks_host(self, k, e, length, pitch, blocks, h_src, h_par, coef=None) -> None:
        cptr = None
        if coef is not None:
            coef = np.ascontiguousarray(coef, np.uint8)
            cptr = coef.ctypes.data
        self.check(lib().rsgpu_encode_blocks_host(self._h, k, e, length, pitch, blocks, _ptr(h_src),
                                                  _ptr(h_par), cptr), "rsgpu_encode_blocks_host")

    def decode_blocks_host(self, k, e, length, pitch, blocks, h_src, h_par, h_err, h_out,
                           h_status=None) -> None:
        self.check(lib().rsgpu_decode_blocks_host(self._h, k, e, length, pitch, blocks, _ptr(h_src),
                                                  _ptr(h_par), _ptr(h_err), _ptr(h_out),
                                                  None if h_status is None else _ptr(h_status)),
                   "rsgpu_decode_blocks_host")

    def decode_general(self, k, m, length, pitch, blocks, encode_matrix, d_src, d_par, d_err, nerrs,
                       d_out, d_ws, d_status) -> None:
        """gf_gen_decode_matrix + recovery (erasure_code_base_test.c:133-213)
        for any m x k encode matrix (None: gf_gen_rs_matrix) and erasures
        among data and parity rows."""
        mp = None
        if encode_matrix is not None:
            encode_matrix = np.ascontiguousarray(encode_matrix, np.uint8).reshape(m, k)
            mp = encode_matrix.ctypes.data
        self.check(lib().rsgpu_decode_general(self._h, k, m, length, pitch, blocks, mp, _ptr(d_src),
                                              _ptr(d_par), _ptr(d_err), nerrs, _ptr(d_out),
                                              _ptr(d_ws), _ptr(d_status)), "rsgpu_decode_general")

    def verify_blocks(self, k, e, length, pitch, blocks, d_src, d_out, d_err, d_mism) -> None:
        self.check(lib().rsgpu_verify_blocks(self._h, k, e, length, pitch, blocks, _ptr(d_src),
                                             _ptr(d_out), _ptr(d_err), _ptr(d_mism)),
                   "rsgpu_verify_blocks")

    def fill_synthetic(self, d_rows, rows, length, pitch, seed, row0=0) -> None:
        self.check(lib().rsgpu_fill_synthetic(self._h, _ptr(d_rows), rows, length, pitch, seed,
                                              row0), "rsgpu_fill_synthetic")


def decode_workspace_bytes(k: int, e: int, blocks: int) -> int:
    return int(lib().rsgpu_decode_workspace_bytes(k, e, blocks))


def decode_general_workspace_bytes(k: int, m: int, nerrs: int, blocks: int) -> int:
    return int(lib().rsgpu_decode_general_workspace_bytes(k, m, nerrs, blocks))


def row_pitch(symbol_size: int) -> int:
    """Row pitch in HBM: symbol_size rounded up to 256 B (16-B vector rows)."""
    return (symbol_size + 255) // 256 * 256


def _context(ctx: Optional[Context], device: int) -> Context:
    if ctx is not None:
        return ctx
    import torch
    if not torch.cuda.is_available():
        raise RsGpuError("no HIP device visible (there is no CPU fallback)")
    c = Context(device)
    c.set_torch_stream()
    return c


# ---- plugin: the Encoder / Decoder concept ----------------------------------

class GpuEncoder:
    """Peer of ``isa_encoder`` (isa.cpp:29-105) over ``blocks`` blocks in HBM.

    The constructor allocates k+e rows per block and fills the k source rows
    with the seeded synthetic stream (isa.cpp:43-58); ``encode_all`` is the
    timed parity generation (isa.cpp:69-79).
    """

    def __init__(self, symbols: int, symbol_size: int, encoded_symbols: int, blocks: int = 1,
                 seed: int = 1, ctx: Optional[Context] = None, device: int = 0,
                 block0: int = 0, pitch: Optional[int] = None):
        import torch
        if not (0 < symbols and 0 <= encoded_symbols and symbols + encoded_symbols <= MAX_SOURCES):
            raise ValueError("symbols + encoded_symbols must be in (0, 250]")
        self.k, self.e, self.L, self.B = symbols, encoded_symbols, symbol_size, blocks
        self.pitch = pitch if pitch is not None else row_pitch(symbol_size)
        self.seed, self.block0 = seed, block0
        self.ctx = _context(ctx, device)
        dev = torch.device("cuda", self.ctx.device)
        self.src = torch.empty(max(1, self.B * self.k * self.pitch), dtype=torch.uint8, device=dev)
        self.par = torch.empty(max(1, self.B * self.e * self.pitch), dtype=torch.uint8, device=dev)
        self.ctx.fill_synthetic(self.src, self.B * self.k, self.L, self.pitch, seed,
                                block0 * self.k)
        self.m_block_size = self.k * self.L
        self.m_payload_count = self.e

    def encode_all(self) -> None:
        self.ctx.encode_blocks(self.k, self.e, self.L, self.pitch, self.B, self.src, self.par)

    def block_size(self) -> int:
        return self.m_block_size

    def symbol_size(self) -> int:
        return self.L

    def payload_size(self) -> int:
        return self.L

    def payload_count(self) -> int:
        return self.m_payload_count

    # host copies for tests
    def source_rows(self, blk: int) -> np.ndarray:
        v = self.src.view(self.B, self.k, self.pitch)[blk, :, : self.L]
        return v.cpu().numpy()

    def parity_rows(self, blk: int) -> np.ndarray:
        v = self.par.view(self.B, self.e, self.pitch)[blk, :, : self.L]
        return v.cpu().numpy()


class GpuDecoder:
    """Peer of ``isa_decoder`` (isa.cpp:108-259).

    The constructor chooses each block's erasure set (untimed, isa.cpp:133-156);
    ``decode_all(encoder)`` is the timed reconstruction (isa.cpp:169-213),
    ``is_complete()`` and ``verify_data(encoder)`` keep their meaning
    (isa.cpp:215-231): complete only if every block's decode matrix inverted.
    """

    def __init__(self, symbols: int, symbol_size: int, encoded_symbols: int, blocks: int = 1,
                 seed: int = 1, ctx: Optional[Context] = None, device: int = 0,
                 block0: int = 0, pitch: Optional[int] = None,
                 erasures: Optional[np.ndarray] = None, synchronous: bool = False):
        import torch
        self.synchronous = synchronous
        if encoded_symbols > symbols:
            raise ValueError("erased symbols must be originals (<= symbols)")
        self.k, self.e, self.L, self.B = symbols, encoded_symbols, symbol_size, blocks
        self.pitch = pitch if pitch is not None else row_pitch(symbol_size)
        self.ctx = _context(ctx, device)
        dev = torch.device("cuda", self.ctx.device)
        if erasures is None:
            erasures = erasure_patterns(seed, block0, blocks, symbols, encoded_symbols)
        self.err_host = np.ascontiguousarray(erasures, np.uint8).reshape(blocks, encoded_symbols)
        self.err = torch.from_numpy(self.err_host.copy()).to(dev)
        self.out = torch.empty(max(1, self.B * self.e * self.pitch), dtype=torch.uint8, device=dev)
        self.ws = torch.empty(decode_workspace_bytes(self.k, self.e, self.B), dtype=torch.uint8,
                              device=dev)
        self.status = torch.full((max(1, self.B),), -1, dtype=torch.int32, device=dev)
        self.mism = torch.zeros((max(1, self.B),), dtype=torch.int64, device=dev)
        self.m_block_size = self.k * self.L
        self._decoded = False

    def decode_all(self, encoder: GpuEncoder) -> int:
        """Enqueue the decode of every block.  Returns the processed payload
        count; a synchronous decoder (the reference's shape) waits and returns
        0 when any block's matrix was singular or its erasure list malformed,
        as isa_decoder::decode_all does on "BAD MATRIX" (isa.cpp:185-190)."""
        assert encoder.payload_count() == self.e  # isa.cpp:171-172
        self.ctx.decode_blocks(self.k, self.e, self.L, self.pitch, self.B, encoder.src,
                               encoder.par, self.err, self.out, self.ws, self.status)
        self._decoded = True
        if self.synchronous and not (self.block_status() == 0).all():
            return 0
        return encoder.payload_count()

    def block_status(self) -> np.ndarray:
        return self.status[: self.B].cpu().numpy()

    def is_complete(self) -> bool:
        return self._decoded and bool((self.block_status() == 0).all())

    def verify_data(self, encoder: GpuEncoder) -> bool:
        assert self.m_block_size == encoder.block_size()  # isa.cpp:217
        self.mism.zero_()
        self.ctx.verify_blocks(self.k, self.e, self.L, self.pitch, self.B, encoder.src,
                               self.out, self.err, self.mism)
        return int(self.mism[: self.B].sum().item()) == 0

    def block_size(self) -> int:
        return self.m_block_size

    def symbol_size(self) -> int:
        return self.L

    def payload_size(self) -> int:
        return self.L

    def recovered_rows(self, blk: int) -> np.ndarray:
        return self.out.view(self.B, self.e, self.pitch)[blk, :, : self.L].cpu().numpy()


# ---- harness mirror -----------------------------------------------------------

@dataclass
class Config:
    symbols: int
    symbol_size: int
    loss_rate: float
    type: str
    erased_symbols: int


@dataclass
class ThroughputBenchmark:
    """Restatement of ``throughput_benchmark<Encoder, Decoder>``.

    ``configurations()`` is get_options' cross-product (throughput_benchmark.hpp:
    126-163, with erased = ceil(symbols*loss_rate)); ``run(cfg)`` performs
    setup (:165-177), the timed encode or decode (:199-220) and the
    goodput accounting of measurement() (:37-67) in MB/s (1e6 B/s) per
    iteration; ``accept`` mirrors accept_measurement (:99-119).
    """

    symbols: Sequence[int] = (16,)
    loss_rate: Sequence[float] = (0.5,)
    symbol_size: Sequence[int] = (1000000,)
    types: Sequence[str] = ("encoder", "decoder")
    blocks: int = 1
    seed: int = 1
    ctx: Optional[Context] = None
    # erasure lists [blocks][erased] replacing the drawn ones (a test hook:
    # e.g. a malformed list, whose measurement must be rejected)
    erasures: Optional[np.ndarray] = None
    results: List[Dict] = field(default_factory=list)

    def configurations(self) -> List[Config]:
        out = []
        for s in self.symbols:
            for r in self.loss_rate:
                for p in self.symbol_size:
                    assert p % 64 == 0  # throughput_benchmark.hpp:145
                    for t in self.types:
                        out.append(Config(s, p, r, t, int(math.ceil(s * r))))
        return out

    def run(self, cfg: Config) -> Dict:
        import torch
        ctx = _context(self.ctx, 0)
        self.ctx = ctx
        enc = GpuEncoder(cfg.symbols, cfg.symbol_size, cfg.erased_symbols, self.blocks,
                         self.seed, ctx)
        dec = GpuDecoder(cfg.symbols, cfg.symbol_size, cfg.erased_symbols, self.blocks,
                         self.seed, ctx, erasures=self.erasures)
        encoded = recovered = processed = 0
        torch.cuda.synchronize()
        if cfg.type == "encoder":
            t0 = time.perf_counter()
            enc.encode_all()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            encoded += enc.payload_count() * self.blocks
        elif cfg.type == "decoder":
            enc.encode_all()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            processed += dec.decode_all(enc) * self.blocks
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            # measurement() counts recovered bytes only for complete decodes
            # (throughput_benchmark.hpp:185-196)
            if dec.is_complete():
                recovered += cfg.erased_symbols * self.blocks
        else:
            raise ValueError(cfg.type)
        accepted = True
        if cfg.type == "decoder":
            accepted = dec.is_complete()
            if accepted:
                assert dec.verify_data(enc)
        total = (recovered if cfg.type == "decoder" else encoded) * cfg.symbol_size
        row = {"symbols": cfg.symbols, "symbol_size": cfg.symbol_size,
               "loss_rate": cfg.loss_rate, "type": cfg.type,
               "erased_symbols": cfg.erased_symbols, "blocks": self.blocks,
               "goodput": total / (t * 1e6), "time_s": t, "accepted": accepted}
        self.results.append(row)
        return row
