"""The generated decode code (storage-benchmarks_amd/csrc/rs_jit.h) checked on
the CPU: librsgpu's host emitter (the same functions the prepare kernel runs on
the GPU) writes one block's code, llvm-mc disassembles it, and an interpreter
runs it with LDS-resident bit planes.  Every accumulator must end as
sum_q c[row][q] * src_q over GF(2^8) (isa/ec_base.c:36-48 gf_mul), only the
allowed instructions may appear, the layout must not depend on the
coefficients, and no register may be read while an LDS load into it is
still outstanding."""
import ctypes as C
import os
import random
import re
import shutil
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "storage-benchmarks_amd", "csrc"))
import gen_tc_handlers as g  # noqa: E402
from test_codegen import planes, unplanes  # noqa: E402

LLVM_MC = shutil.which("llvm-mc") or "/opt/rocm/lib/llvm/bin/llvm-mc"
pytestmark = pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not available")

ALLOWED = {"v_bitop3_b32", "v_xor_b32_e32", "v_xor_b32_e64", "ds_read_b128", "s_waitcnt", "s_nop",
           "s_setpc_b64"}
CHUNK_STRIDE = 5056  # jit::chunk_stride(8): (16 + 8 * 624 + 8) rounded to 64


def emit(k, e, coef):
    import rsgpu
    f = rsgpu.testhooks().rsgpu_internal_jit_emit
    f.restype = C.c_longlong
    f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]
    coef = np.ascontiguousarray(coef, np.uint8)
    need = f(k, e, coef.ctypes.data, None, 0)
    out = np.zeros(need, np.uint8)
    assert f(k, e, coef.ctypes.data, out.ctypes.data, need) == need
    return out


def disasm(code: bytes):
    """[(byte offset, mnemonic, operand text)] via llvm-mc, instruction sizes
    from the encodings (VOP3 / DS: 8 bytes, SOPP / SOP1 / VOP2: 4)."""
    text = " ".join(f"0x{b:02x}" for b in code)
    r = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "--disassemble", "-show-encoding"],
                       input=text, capture_output=True, text=True, check=True)
    out, off = [], 0
    for ln in r.stdout.splitlines():
        ln = ln.strip()
        if not ln or ln.startswith("."):
            continue
        body, _, enc = ln.partition(";")
        n = enc.count("0x")
        assert n in (4, 8), ln
        mnem, _, ops = body.strip().partition(" ")
        out.append((off, mnem, ops.strip()))
        off += n
    assert off == len(code), (off, len(code))
    return out


def regs_of(op):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return [int(op[1:])]


def run_chunk(ins, regs, lds, pending, addr_reg="v20"):
    """Interpret one chunk up to its s_setpc; LDS loads land at issue but stay
    'pending' until an s_waitcnt retires them (reading one is a hazard)."""
    def rd(r):
        for p in pending:
            assert r not in p, f"v{r} read before its LDS load was waited for"
        return regs[r]

    for off, mnem, ops in ins:
        assert mnem in ALLOWED, mnem
        a = [x.strip() for x in ops.split(",")] if ops else []
        if mnem == "s_setpc_b64":
            return off
        if mnem == "s_nop":
            continue
        if mnem == "s_waitcnt":
            n = int(re.fullmatch(r"lgkmcnt\((\d+)\)", ops).group(1))
            del pending[: max(0, len(pending) - n)]
        elif mnem == "ds_read_b128":
            dst = regs_of(a[0])
            addr, _, rest = a[1].partition(" ")
            assert addr == addr_reg, ops
            o = int(rest.split(":")[1]) if rest else 0
            for i, r in enumerate(dst):
                regs[r] = lds[o + 4 * i]
            pending.append(set(dst))
        elif mnem.startswith("v_xor"):
            d, x, y = (regs_of(v)[0] for v in a)
            regs[d] = rd(x) ^ rd(y)
        elif mnem == "v_bitop3_b32":
            last, _, mod = a[3].partition(" ")
            assert mod == "bitop3:0x96", ops
            d, x, y, z = (regs_of(v)[0] for v in a[:3] + [last])
            regs[d] = rd(x) ^ rd(y) ^ rd(z)
    raise AssertionError("chunk without a return")


@pytest.mark.parametrize("k,e", [(64, 32), (20, 13), (9, 8), (100, 20), (3, 1)])
def test_generated_block_decodes(k, e):
    rng = random.Random(k * 100 + e)
    coef = np.array([[rng.randrange(256) for _ in range(k)] for _ in range(e)], np.uint8)
    coef[0, 0] = 0  # a zero coefficient: no-op rows
    code = emit(k, e, coef).tobytes()
    nw, nch = (e + 7) // 8, (k + 7) // 8
    assert len(code) == nw * nch * CHUNK_STRIDE
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(k)]
    for w in range(nw):
        regs = {r: 0 for r in range(256)}
        pending = []
        for ch in range(nch):
            base = (w * nch + ch) * CHUNK_STRIDE
            nt = min(8, k - 8 * ch)
            nslot = min(8, e - 8 * w)
            end = base + 16 + nt * (112 + 64 * nslot)
            ins = disasm(code[base:end + 4])
            lds = {}
            for t in range(nt):
                p = planes(src[8 * ch + t])
                for a in range(8):
                    lds[t * 2048 + (a // 4) * 1024 + 4 * (a % 4)] = p[a]
            ret = run_chunk(ins, regs, lds, pending)
            assert base + ret == end, "the return sits right after the last source"
            assert not pending, "a load left outstanding at the return"
        for s in range(min(8, e - 8 * w)):
            row = 8 * w + s
            want = [0] * 32
            for q in range(k):
                want = [x ^ g.gf_mul(int(coef[row, q]), y) for x, y in zip(want, src[q])]
            got = unplanes([regs[64 + 8 * s + b] for b in range(8)])
            assert got == want, (k, e, row)


def test_layout_independent_of_coefficients():
    """Instruction boundaries and kinds depend on (k, e) only: a block's code
    rewritten with other coefficients never puts an instruction boundary
    elsewhere (what a stale instruction-cache line would otherwise expose)."""
    k, e = 24, 17
    rng = np.random.default_rng(5)
    layouts = []
    for _ in range(3):
        coef = rng.integers(1, 256, (e, k), dtype=np.uint8)
        ins = disasm(emit(k, e, coef).tobytes())
        layouts.append([(off, m.startswith("v_") and m != "ds_read_b128") for off, m, _ in ins])
    assert layouts[0] == layouts[1] == layouts[2]


def matrix_code(k, e, coef, max_ops=22):
    import rsgpu
    f = rsgpu.testhooks().rsgpu_internal_jit_matrix_code
    f.restype = C.c_longlong
    f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.c_int]
    coef = np.ascontiguousarray(coef, np.uint8)
    stride = C.c_int()
    need = f(k, e, coef.ctypes.data, None, 0, C.byref(stride), max_ops)
    out = np.zeros(need, np.uint8)
    assert f(k, e, coef.ctypes.data, out.ctypes.data, need, C.byref(stride), max_ops) == need
    return out.tobytes(), stride.value


def rs_rows(k, e):
    """gf_gen_rs_matrix rows k..k+e-1 (isa/ec_base.c:62-79): 2^(r j)."""
    rows = []
    for r in range(e):
        gen, p, row = 1, 1, []
        for _ in range(r):
            gen = g.gf_mul(gen, 2)
        for _ in range(k):
            row.append(p)
            p = g.gf_mul(p, gen)
        rows.append(row)
    return np.array(rows, np.uint8)


@pytest.mark.parametrize("k,e,kind", [(64, 32, "rs"), (32, 16, "random"), (128, 64, "random"),
                                      (20, 13, "random"), (9, 40, "random"), (100, 20, "rs"),
                                      (24, 17, "capped")])
def test_shared_matrix_code(k, e, kind):
    """The GENERATED encode's host-built code (jit_prog.cpp): per (wave,
    source) only the composites a greedy cover needs, rows in passes of 32.
    Interpreted chunk by chunk, every accumulator must equal sum_q c[row][q]
    * src_q over GF(2^8); every register read after its LDS load was waited
    for; and the composites must average well under the 22 of the full
    tables."""
    rng = random.Random(k * 1000 + e)
    if kind == "rs":
        coef = rs_rows(k, e)
    else:
        coef = np.array([[rng.randrange(256) for _ in range(k)] for _ in range(e)], np.uint8)
        coef[0, 0] = 0
    # "capped": a cover limited to 6 composites cannot finish, so every source
    # falls back to the full four-Russians tables
    code, stride = matrix_code(k, e, coef, 6 if kind == "capped" else 22)
    nch = (k + 7) // 8
    assert len(code) == ((e + 31) // 32) * 4 * nch * stride
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(k)]
    n_comp = n_src = 0
    for p in range((e + 31) // 32):
        prow = min(32, e - 32 * p)
        for w in range((prow + 7) // 8):
            regs = {r: 0 for r in range(256)}
            pending = []
            for ch in range(nch):
                base = ((p * 4 + w) * nch + ch) * stride
                nt = min(8, k - 8 * ch)
                ins = disasm(code[base:base + stride])
                end = next(off for off, m, _ in ins if m == "s_setpc_b64")
                ins = [x for x in ins if x[0] <= end]
                n_comp += sum(1 for off, m, ops in ins if m in ("v_xor_b32_e32", "v_bitop3_b32")
                              and int(regs_of(ops.split(",")[0])[0]) < 64)
                n_src += nt
                lds = {}
                for t in range(nt):
                    pl = planes(src[8 * ch + t])
                    for a in range(8):
                        lds[t * 2048 + (a // 4) * 1024 + 4 * (a % 4)] = pl[a]
                run_chunk(ins, regs, lds, pending)
                assert not pending, "a load left outstanding at the return"
            for s in range(min(8, prow - 8 * w)):
                row = 32 * p + 8 * w + s
                want = [0] * 32
                for q in range(k):
                    want = [x ^ g.gf_mul(int(coef[row, q]), y) for x, y in zip(want, src[q])]
                got = unplanes([regs[64 + 8 * s + b] for b in range(8)])
                assert got == want, (k, e, row)
    if kind == "capped":  # all but covers finished within 6 composites are full tables
        assert n_comp / n_src > 18, n_comp / n_src
    else:
        assert n_comp / n_src < 18, n_comp / n_src


def wide_rows(e):
    """jitw_rows: accumulator rows per wave of the two- / four-wave layouts."""
    if e > 32:
        return 16 if e > 48 else 12 if e > 40 else 10
    return 16 if e > 24 else 12 if e > 20 else 10


def wide_waves(e):
    return 4 if e > 32 else 2


def wide_row0(e, w):
    """rs_jit.h wide_row0: wave w's first row (balanced split)."""
    return w * e // wide_waves(e)


def matrix_code_wide(k, e, coef, max_ops=22):
    """The shared program as rsgpu_capi.cpp shared_program builds it: the
    code and its passes [(byte offset, chunk stride)] (one pass up to 64
    rows, passes of <= 64 rows above)."""
    import rsgpu
    f = rsgpu.testhooks().rsgpu_internal_jitw_matrix_code
    f.restype = C.c_longlong
    f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.POINTER(C.c_longlong),
                  C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int), C.c_int]
    coef = np.ascontiguousarray(coef, np.uint8)
    offs, strides, n = (C.c_longlong * 4)(), (C.c_int * 4)(), C.c_int()
    need = f(k, e, coef.ctypes.data, None, 0, offs, strides, 4, C.byref(n), max_ops)
    assert need > 0
    out = np.zeros(need, np.uint8)
    assert f(k, e, coef.ctypes.data, out.ctypes.data, need, offs, strides, 4, C.byref(n), max_ops) == need
    return out.tobytes(), [(offs[p], strides[p]) for p in range(n.value)]


@pytest.mark.parametrize("k,e,kind", [(64, 32, "rs"), (100, 20, "rs"), (100, 25, "random"),
                                      (128, 32, "random"), (48, 24, "random"), (17, 17, "random"),
                                      (24, 17, "capped"), (218, 32, "rs"), (100, 50, "rs"),
                                      (128, 64, "random"), (60, 40, "random"), (40, 33, "capped"),
                                      (150, 100, "random"), (125, 125, "random"), (160, 65, "rs"),
                                      (90, 70, "capped")])
def test_shared_matrix_code_wide(k, e, kind):
    """The GENERATED encode's host-built code for 16 < e <= 125 in the
    decode's two- / four-wave layout (jit_prog.cpp build_matrix_code_wide_passes,
    what shared_program runs: planes v10..v17 from LDS at v9, covered
    composites from v18, accumulators from v40; passes of <= 64 rows above 64,
    each in the layout of its own rows, at its own offset and chunk stride):
    interpreted chunk by chunk, every accumulator equals sum_q c[row][q] *
    src_q over GF(2^8), registers stay in v9..v(40+8R-1), every register is
    read after its LDS load was waited for, and the covers average under the
    22 composites of the full tables."""
    rng = random.Random(k * 1000 + e)
    if kind == "rs":
        coef = rs_rows(k, e)
    else:
        coef = np.array([[rng.randrange(256) for _ in range(k)] for _ in range(e)], np.uint8)
        coef[0, 0] = 0
    code, passes = matrix_code_wide(k, e, coef, 6 if kind == "capped" else 22)
    npass = (e + 63) // 64 if e > 64 else 1
    assert len(passes) == npass
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(k)]
    n_comp = n_src = 0
    end_of = [o for o, _ in passes[1:]] + [len(code)]
    for p, (poff, stride) in enumerate(passes):
        pr0, pr = p * e // npass, (p + 1) * e // npass - p * e // npass  # rs_jit.h wide_pass_row0
        R, nv = wide_rows(pr), wide_waves(pr)
        cs = WIDE[R][0]
        nch = (k + cs - 1) // cs
        assert stride % 64 == 0 and end_of[p] - poff == nv * nch * stride
        nc, ns = interpret_wide_pass(code[poff:end_of[p]], stride, k, pr, R, nv, cs, nch,
                                     coef[pr0:pr0 + pr], src)
        n_comp += nc
        n_src += ns
    # per (wave, source): the capped covers fall back to the full tables
    if kind == "capped":
        assert n_comp / n_src > 18, n_comp / n_src
    else:
        assert n_comp / n_src < 20, n_comp / n_src


def interpret_wide_pass(code, stride, k, e, R, nv, cs, nch, coef, src):
    """Runs one pass of shared wide code (rows coef[0..e-1]) on the CPU and
    checks every accumulator; returns (composites, sources) seen."""
    n_comp = n_src = 0
    for w in range(nv):
        nslot = wide_row0(e, w + 1) - wide_row0(e, w)
        assert 0 < nslot <= R
        regs = {r: 0 for r in range(256)}
        pending = []
        for ch in range(nch):
            base = (w * nch + ch) * stride
            nt = min(cs, k - cs * ch)
            ins = disasm(code[base:base + stride])
            end = next(off for off, m, _ in ins if m == "s_setpc_b64")
            ins = [x for x in ins if x[0] <= end]
            n_comp += sum(1 for off, m, ops in ins if m in ("v_xor_b32_e32", "v_bitop3_b32")
                          and int(regs_of(ops.split(",")[0])[0]) < 40)
            n_src += nt
            used = [int(n) for _, _, ops in ins for n in re.findall(r"v\[?(\d+)", ops)]
            used += [int(n) for _, _, ops in ins for n in re.findall(r"v\[\d+:(\d+)\]", ops)]
            assert max(used) < 40 + 8 * R and min(used) >= 9
            lds = {}
            for t in range(nt):
                pl = planes(src[cs * ch + t])
                for a in range(8):
                    lds[t * 2048 + (a // 4) * 1024 + 4 * (a % 4)] = pl[a]
            run_chunk(ins, regs, lds, pending, addr_reg="v9")
            assert not pending, "a load left outstanding at the return"
        for s in range(nslot):
            row = wide_row0(e, w) + s
            want = [0] * 32
            for q in range(k):
                want = [x ^ g.gf_mul(int(coef[row, q]), y) for x, y in zip(want, src[q])]
            got = unplanes([regs[40 + 8 * s + b] for b in range(8)])
            assert got == want, (k, e, row)
    return n_comp, n_src


def emitw(k, e, coef):
    import rsgpu
    f = rsgpu.testhooks().rsgpu_internal_jitw_emit
    f.restype = C.c_longlong
    f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_size_t]
    coef = np.ascontiguousarray(coef, np.uint8)
    need = f(k, e, coef.ctypes.data, None, 0)
    assert need > 0
    out = np.zeros(need, np.uint8)
    assert f(k, e, coef.ctypes.data, out.ctypes.data, need) == need
    return out


# Wide<R, CS>::chunk_stride(): (CS * (112 + 64 R) + 8) rounded to 64
WIDE = {16: (6, 6848), 12: (6, 5312), 10: (5, 3776)}


def wide_passes(e):
    """rs_jit.h wide_passes: e > 64 rows as passes of <= 64, split evenly."""
    return (e + 63) // 64 if e > 64 else 1


def wide_pass_row0(e, p):
    return p * e // wide_passes(e)


def pass_bytes(k, rows):
    cs, stride = WIDE[wide_rows(rows)]
    return wide_waves(rows) * ((k + cs - 1) // cs) * stride


@pytest.mark.parametrize("k,e", [(64, 32), (25, 25), (100, 30), (13, 27), (218, 32),
                                 (100, 20), (17, 17), (64, 19), (230, 20), (48, 24), (21, 21), (226, 24),
                                 (100, 50), (128, 64), (186, 64), (60, 40), (70, 45), (40, 33),
                                 # e > 64: passes of <= 64 rows
                                 (150, 100), (125, 125), (185, 65), (130, 120), (160, 90)])
def test_generated_wide_block_decodes(k, e):
    """k_rs_jitw's code (rs_jit.h Wide: 2 waves x R rows for e <= 32, 4
    waves for 32 < e <= 64, rows split evenly, chunks of CS sources, each source
    loading its own planes, accumulators from v40; e > 64 as passes of <= 64
    rows, each in the layout of its own row count): every accumulator equals
    sum_q c[row][q] * src_q over GF(2^8), only the allowed instructions
    appear, every register is read after its LDS load was waited for, and
    each chunk returns right after its last source."""
    rng = random.Random(k * 7 + e)
    coef = np.array([[rng.randrange(256) for _ in range(k)] for _ in range(e)], np.uint8)
    coef[1, 2] = 0
    code = emitw(k, e, coef).tobytes()
    passes = [(wide_pass_row0(e, p), wide_pass_row0(e, p + 1) - wide_pass_row0(e, p))
              for p in range(wide_passes(e))]
    assert all(0 < rows <= 64 for _, rows in passes)
    assert len(code) == sum(pass_bytes(k, rows) for _, rows in passes)
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(k)]
    done = set()
    off = 0
    for prow0, rows in passes:
        R, nv = wide_rows(rows), wide_waves(rows)
        cs, stride = WIDE[R]
        nch = (k + cs - 1) // cs
        for w in range(nv):
            nslot = wide_row0(rows, w + 1) - wide_row0(rows, w)
            assert 0 < nslot <= R
            regs = {r: 0 for r in range(256)}
            pending = []
            for ch in range(nch):
                base = off + (w * nch + ch) * stride
                nt = min(cs, k - cs * ch)
                end = base + nt * (112 + 64 * nslot)
                ins = disasm(code[base:end + 4])
                lds = {}
                for t in range(nt):
                    p = planes(src[cs * ch + t])
                    for a in range(8):
                        lds[t * 2048 + (a // 4) * 1024 + 4 * (a % 4)] = p[a]
                ret = run_chunk(ins, regs, lds, pending, addr_reg="v9")
                assert base + ret == end, "the return sits right after the last source"
                assert not pending, "a load left outstanding at the return"
                used = [int(n) for _, _, ops in ins for n in re.findall(r"v\[?(\d+)", ops)]
                used += [int(n) for _, _, ops in ins for n in re.findall(r"v\[\d+:(\d+)\]", ops)]
                assert max(used) < 40 + 8 * R and min(used) >= 9, "register outside the kernel's v9..v(40+8R-1)"
            for s in range(nslot):
                row = prow0 + wide_row0(rows, w) + s
                want = [0] * 32
                for q in range(k):
                    want = [x ^ g.gf_mul(int(coef[row, q]), y) for x, y in zip(want, src[q])]
                got = unplanes([regs[40 + 8 * s + b] for b in range(8)])
                assert got == want, (k, e, row)
                done.add(row)
        off += pass_bytes(k, rows)
    assert done == set(range(e)), "every row in exactly one pass"
