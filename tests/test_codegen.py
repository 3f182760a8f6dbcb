"""The generated GF(2^8) asm (storage-benchmarks_amd/csrc/gen_tc_handlers.py)
checked on the CPU by interpreting its VALU instructions over bit-sliced
planes: the 256 threaded-code handlers, the chunk dispatch, and the encode's
per-source XOR programs and Horner twiddles (gen_enc_progs.py) must multiply
exactly as gf_mul (isa/ec_base.c:36-48) does.  No GPU needed: a wrong register or plane
in the generator shows up here before it can corrupt a decode."""
import os
import random
import re
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "storage-benchmarks_amd", "csrc"))
import gen_tc_handlers as g  # noqa: E402

INSN = re.compile(r"(\S+) v(\d+), v(\d+)(?:, v(\d+))?(?:, v(\d+))?")


def run(ins, regs):
    for i in ins:
        if i.startswith("s_"):
            continue
        m = INSN.match(i)
        assert m, i
        op, d = m.group(1), int(m.group(2))
        s = [int(x) for x in m.groups()[2:] if x]
        if op.startswith("v_mov"):
            regs[d] = regs[s[0]]
        elif op.startswith("v_xor"):
            regs[d] = regs[s[0]] ^ regs[s[1]]
        elif op.startswith("v_bitop3"):
            assert i.endswith("bitop3:0x96"), i
            regs[d] = regs[s[0]] ^ regs[s[1]] ^ regs[s[2]]
        else:
            raise AssertionError(i)


def planes(by):
    return [sum(((x >> a) & 1) << i for i, x in enumerate(by)) for a in range(8)]


def unplanes(p):
    return [sum(((p[a] >> i) & 1) << a for a in range(8)) for i in range(32)]


def load_tables(regs, by):
    """The four-Russians tables of one source: single-bit entries = planes,
    the rest built by the generator's own table code."""
    p = planes(by)
    for a, r in enumerate(g.PLANE_REG):
        regs[r] = p[a]
    run(g.tables(), regs)


@pytest.mark.parametrize("c", range(256))
def test_handler_multiplies(c):
    for copy in range(g.NCOPY):
        rng = random.Random(c)
        regs = {i: 0 for i in range(256)}
        src = [rng.randrange(256) for _ in range(32)]
        acc = [rng.randrange(256) for _ in range(32)]
        load_tables(regs, src)
        base = g.ACC + 8 * copy
        for a, v in enumerate(planes(acc)):
            regs[base + a] = v
        body = g.handler(c, copy)
        assert sum(4 if i.startswith("s_") else 8 for i in body) == g.STRIDE
        # copies before the last continue the chain, the last one returns
        ret = g.RA_LIST[copy] if copy < g.NCOPY - 1 else g.RET
        assert f"s_setpc_b64 s[{ret}:{ret + 1}]" in body
        run(body, regs)
        got = unplanes([regs[base + a] for a in range(8)])
        assert got == [x ^ g.gf_mul(c, y) for x, y in zip(acc, src)]


def test_handler_table_layout():
    tbl = g.handler_table()
    assert sum(4 if i.startswith("s_") else 8 for i in tbl) == g.NHANDLERS * g.STRIDE


DS = re.compile(r"ds_read_b128 v\[(\d+):(\d+)\], %\[la\] offset:(\d+)")
SLD = re.compile(r"s_load_dwordx16 s\[(\d+):(\d+)\], %\[pa\], (\S+)")
SWAP = re.compile(r"s_swappc_b64 s\[\d+:\d+\], s\[(\d+):\d+\]")
SMOV = re.compile(r"s_mov_b64 s\[(\d+):\d+\], s\[(\d+):\d+\]")
SETPC = re.compile(r"s_setpc_b64 s\[(\d+):\d+\]")


def generator(chain):
    """gen_tc_handlers imported afresh under RSGPU_TC_CHAIN=chain (its
    dispatch layout is fixed at import), or the default module for None."""
    if chain is None:
        return g
    import importlib.util
    old = os.environ.get("RSGPU_TC_CHAIN")
    os.environ["RSGPU_TC_CHAIN"] = str(chain)
    try:
        spec = importlib.util.spec_from_file_location("gen_tc_chain%d" % chain, g.__file__)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        if old is None:
            del os.environ["RSGPU_TC_CHAIN"]
        else:
            os.environ["RSGPU_TC_CHAIN"] = old
    assert mod.NCOPY == chain
    return mod


@pytest.mark.parametrize("chain", [None, 1, 2, 3, 4], ids=["default", "chain1", "chain2", "chain3", "chain4"])
@pytest.mark.parametrize("nt", range(1, g.C + 1))
def test_chunk_dispatch(nt, chain):
    """The per-part chunk asm (gen_tc_handlers.chunk) interpreted with its
    LDS reads, handler-address loads, GPR-index relocation and handler calls:
    every accumulator slot s must end as acc_s ^ sum_t c(t, s) * src_t.  The
    interpreter applies each load at issue, so a read that lands in a register
    still in use by the dispatch shows up as a wrong product.  Every
    generator chain layout (RSGPU_TC_CHAIN) is checked, not only the built one."""
    g = generator(chain)
    rng = random.Random(100 + nt)
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(nt)]
    coef = [[rng.randrange(256) for _ in range(8)] for _ in range(nt)]
    acc0 = [[rng.randrange(256) for _ in range(32)] for _ in range(8)]
    regs = {i: 0 for i in range(256)}
    for s in range(8):
        for a, v in enumerate(planes(acc0[s])):
            regs[g.ACC + 8 * s + a] = v
    sregs, idx = {}, None
    for i in g.chunk(nt):
        m = DS.match(i)
        if m:
            lo, hi, off = int(m.group(1)), int(m.group(2)), int(m.group(3))
            t, half = off // g.LDS_T, (off % g.LDS_T) // g.LDS_H
            p = planes(src[t])
            for q in range(hi - lo + 1):
                regs[lo + q] = p[4 * half + q]
            continue
        m = SLD.match(i)
        if m:
            base, off = int(m.group(1)), m.group(3)
            t = 0 if off == "0" else int(off[3:-1])
            for s in range(8):
                sregs[base + 2 * s] = (s, coef[t][s])
            continue
        if i.startswith("s_set_gpr_idx_on"):
            idx = int(i.split()[1].rstrip(","))
        elif i.startswith("s_set_gpr_idx_idx"):
            idx = int(i.split()[1])
        elif i.startswith("s_set_gpr_idx_off"):
            idx = None
        elif i.startswith("s_mov_b64"):
            m = SMOV.match(i)
            sregs[int(m.group(1))] = sregs[int(m.group(2))]
        elif i.startswith("s_swappc"):
            rel = idx or 0  # outside index mode the handler registers are absolute
            slot, c = sregs[int(SWAP.match(i).group(1))]
            copy = g.SLOT_COPY[slot]  # the prepared address names this copy
            while True:  # a handler, and in chained mode the ones it jumps to
                body = g.handler(c, copy)
                for h in body:
                    if h.startswith("s_"):
                        continue
                    mm = INSN.match(h)
                    op, d = mm.group(1), int(mm.group(2)) + rel
                    ops = [int(x) for x in mm.groups()[2:] if x]
                    ops[0] += rel  # gpr_idx(SRC0,DST)
                    val = 0
                    for o in ops:
                        val ^= regs[o]
                    assert op.startswith(("v_xor", "v_bitop3"))
                    regs[d] = val
                tgt = int(SETPC.search(" ".join(body)).group(1))
                if tgt == g.RET:
                    assert copy == g.NCOPY - 1
                    break
                assert tgt == g.RA_LIST[copy]
                slot, c = sregs[tgt]
                assert g.SLOT_COPY[slot] == copy + 1
                copy += 1
        elif not i.startswith("s_"):
            assert idx is None, i
            run([i], regs)
    for s in range(8):
        exp = list(acc0[s])
        for t in range(nt):
            exp = [x ^ g.gf_mul(coef[t][s], y) for x, y in zip(exp, src[t])]
        assert unplanes([regs[g.ACC + 8 * s + a] for a in range(8)]) == exp, (nt, s)



import gen_enc_progs as ge  # noqa: E402


def test_encode_programs_cover_every_output():
    """Every generated per-source XOR program of k_rs_bs (gen_enc_progs.py):
    each composite is an XOR of earlier values, and every output plane of
    every row equals the plane mask of 2^(r T) (gf_gen_rs_matrix
    coefficient) -- evaluated symbolically over the 8 source planes."""
    nblk = 0
    for K, E, C, NW in ge.PLANS:
        opw = (E + NW - 1) // NW
        for grp in range(NW):
            R0, NR = grp * opw, min(opw, E - grp * opw)
            for T in range(C):
                ops, vals, outs = ge.block(K, E, C, R0, NR, T)
                V = [1 << a for a in range(8)]
                for op in ops:
                    assert all(i < len(V) or i == ge.NONE for i in op)
                    x = 0
                    for i in op:
                        if i != ge.NONE:
                            x ^= V[i]
                    V.append(x)
                for o, (x, y) in enumerate(outs):
                    r, b = R0 + o // 8, o % 8
                    got = (V[x] if x != ge.NONE else 0) ^ (V[y] if y != ge.NONE else 0)
                    assert got == ge.mat_row(ge.gf_pow2(r * T), b), (K, E, C, R0, T, o)
                nblk += 1
    assert nblk == 233


def test_twiddle_programs():
    """The Horner twiddle programs of k_rs_bs (row r times 2^(C r), one per
    row of every plan), evaluated symbolically over the 8 accumulator planes."""
    n = 0
    for K, E, C, NW in ge.PLANS:
        for r in range(E):
            c = ge.gf_pow2(C * r)
            ops, outs = ge.twiddle(c)
            V = [1 << a for a in range(8)]
            for op in ops:
                assert all(i < len(V) or i == ge.NONE for i in op)
                x = 0
                for i in op:
                    if i != ge.NONE:
                        x ^= V[i]
                V.append(x)
            for b in range(8):
                assert V[outs[b]] == ge.mat_row(c, b), (K, E, C, r, b)
            n += 1
    assert n == sum(E for _, E, _, _ in ge.PLANS)


def test_encode_t0_pairing_chunk():
    """k_rs_bs with T0Pair (gen_enc_progs.py): a chunk's source 0 (coefficient
    1 on every row) adds no term of its own to an output that a later source
    adds together with its single value; over a whole chunk every output plane
    still equals sum_T 2^(r T) d_T, evaluated symbolically over the 8 C
    source planes of the chunk (bit 8 T + a = plane a of source T)."""
    npair = 0
    for K, E, C, NW in ge.PLANS:
        opw = (E + NW - 1) // NW
        for grp in range(NW):
            R0, NR = grp * opw, min(opw, E - grp * opw)
            part = ge.t0_partners(K, E, C, R0, NR)
            acc = [0] * (NR * 8)
            for T in range(C):
                ops, vals, outs = ge.block(K, E, C, R0, NR, T)
                V = [1 << (8 * T + a) for a in range(8)]
                for op in ops:
                    x = 0
                    for i in op:
                        if i != ge.NONE:
                            x ^= V[i]
                    V.append(x)
                for o, (x, y) in enumerate(outs):
                    if T == 0 and part[o]:
                        continue
                    if T and part[o] == T:
                        assert x != ge.NONE and y == ge.NONE
                        acc[o] ^= V[x] ^ (1 << (o % 8))  # source 0's plane b
                        npair += 1
                        continue
                    acc[o] ^= (V[x] if x != ge.NONE else 0) ^ (V[y] if y != ge.NONE else 0)
            for o in range(NR * 8):
                r, b = R0 + o // 8, o % 8
                exp = 0
                for T in range(C):
                    exp |= ge.mat_row(ge.gf_pow2(r * T), b) << (8 * T)
                assert acc[o] == exp, (K, E, C, R0, o)
    assert npair > 0


RDL = re.compile(r"v_readlane_b32 s(\d+), %\[av\], (\d+)")


@pytest.mark.parametrize("nt", range(1, 5))
def test_chunk_v_dispatch(nt):
    """gen_tc_handlers.chunk_v (the fused small-batch decode's chunk): the
    handler addresses come from lanes 16 t + i of one VGPR by v_readlane
    instead of a scalar load, into the bank the scalar load would fill; the
    chunk must accumulate the same products as chunk() (test_chunk_dispatch),
    and every address word must be read before its first use."""
    rng = random.Random(300 + nt)
    src = [[rng.randrange(256) for _ in range(32)] for _ in range(nt)]
    coef = [[rng.randrange(256) for _ in range(8)] for _ in range(nt)]
    acc0 = [[rng.randrange(256) for _ in range(32)] for _ in range(8)]
    regs = {i: 0 for i in range(256)}
    for s in range(8):
        for a, v in enumerate(planes(acc0[s])):
            regs[g.ACC + 8 * s + a] = v
    sregs, idx, banks = {}, None, (g.BANK[0], g.BANK[1])
    code = g.chunk_v(nt)
    assert not any(i.startswith("s_load") for i in code)
    for i in code:
        m = DS.match(i)
        if m:
            lo, hi, off = int(m.group(1)), int(m.group(2)), int(m.group(3))
            t, half = off // g.LDS_T, (off % g.LDS_T) // g.LDS_H
            p = planes(src[t])
            for q in range(hi - lo + 1):
                regs[lo + q] = p[4 * half + q]
            continue
        m = RDL.match(i)
        if m:
            sreg, lane = int(m.group(1)), int(m.group(2))
            t, word = lane // 16, lane % 16
            bank = banks[0] if sreg < banks[1] else banks[1]
            assert sreg - bank == word and t < nt
            if word % 2 == 0:  # low half of (slot word/2)'s address
                sregs[sreg] = (word // 2, coef[t][word // 2])
            continue
        if i.startswith("s_set_gpr_idx_on"):
            idx = int(i.split()[1].rstrip(","))
        elif i.startswith("s_set_gpr_idx_idx"):
            idx = int(i.split()[1])
        elif i.startswith("s_set_gpr_idx_off"):
            idx = None
        elif i.startswith("s_mov_b64"):
            m = SMOV.match(i)
            sregs[int(m.group(1))] = sregs[int(m.group(2))]
        elif i.startswith("s_swappc"):
            rel = idx or 0
            slot, c = sregs[int(SWAP.match(i).group(1))]
            copy = g.SLOT_COPY[slot]
            while True:
                body = g.handler(c, copy)
                for h in body:
                    if h.startswith("s_"):
                        continue
                    mm = INSN.match(h)
                    d = int(mm.group(2)) + rel
                    ops = [int(x) for x in mm.groups()[2:] if x]
                    ops[0] += rel
                    val = 0
                    for o in ops:
                        val ^= regs[o]
                    regs[d] = val
                tgt = int(SETPC.search(" ".join(body)).group(1))
                if tgt == g.RET:
                    break
                slot, c = sregs[tgt]
                copy += 1
        elif not i.startswith("s_"):
            assert idx is None, i
            run([i], regs)
    for s in range(8):
        exp = list(acc0[s])
        for t in range(nt):
            exp = [x ^ g.gf_mul(coef[t][s], y) for x, y in zip(exp, src[t])]
        assert unplanes([regs[g.ACC + 8 * s + a] for a in range(8)]) == exp, (nt, s)
