#!/usr/bin/env python3
"""Generate enc_progs.inc: per-source XOR programs of the compile-time
bit-sliced kernel k_rs_bs (rs_bitsliced.hip).

For one source at chunk position T and one wave's rows R0..R0+NR-1, output
plane b of row r needs the XOR of the source planes selected by m = row b of
the matrix of 2^(r T) (gf_gen_rs_matrix coefficient, isa/ec_base.c:71-78).
The four-Russians form builds all 22 composite XORs of the plane nibbles and
adds each output with one 3-input XOR, acc ^= L[m & 15] ^ H[m >> 4].  Only
the masks this (rows, T) block uses matter, though: a greedy cover picks the
composites such that every needed mask is the XOR of at most two available
values (planes or composites), each composite costing one 2- or 3-input XOR
of values already available.  On the (64, 32) plan that is 12.1 composites
per source instead of 22; the accumulation stays one instruction per output.

Also the Horner twiddles (row r times 2^(C r) between chunks) as XOR
programs over the row's 8 accumulator planes: TwProg<K, E, C, R> with NOPS,
ops (as below) and outs[8] = the value that becomes plane b.

Source T = 0 of every chunk has the coefficient 2^0 = 1 on every row, so
each of its outputs is a single plane.  T0Pair<K, E, C, R0, NR>::partner[o]
names the first later source of the chunk whose output o is a single value
too; that source adds both terms with one 3-input XOR (acc ^= V[x] ^ p0[b])
and source 0 skips output o (0 = no partner: source 0 adds its plane).  On
the (64, 32) plan 204 of the 256 source-0 outputs per chunk find a partner.

Output: C++ specializations EncProg<K, E, C, R0, NR, T> with
  NOPS, ops[NOPS][3]  value 8 + i = XOR of values ops[i][0..2] (255 = none)
  outs[NR * 8][2]     acc[s][b] ^= values outs[s*8+b][0] ^ outs[s*8+b][1]
Values 0..7 are the source planes, 255 is "no operand".

usage: gen_enc_progs.py OUT.inc
"""
import itertools
import sys

# (K, E, C, NW) of rs_bitsliced.hip launch_rs_bitsliced
PLANS = [(16, 4, 16, 1), (16, 8, 16, 1), (64, 32, 16, 4), (64, 16, 16, 2), (100, 20, 20, 4),
         (5, 4, 5, 1), (20, 7, 20, 1)]
NONE = 255
# plans whose kernel would spill with source 0's planes held across the chunk
# (k_rs_bs<100, 20>: 128 VGPRs + 2 spilled, 122 without pairing)
NO_T0_PAIR = {(100, 20, 20)}


def gf_mul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = ((a << 1) ^ (0x11D if a & 0x80 else 0)) & 0xFF
        b >>= 1
    return r


def gf_pow2(n: int) -> int:
    v = 1
    for _ in range(n % 255):
        v = gf_mul(v, 2)
    return v


def mat_row(c: int, b: int) -> int:
    """Row b of the matrix of x -> c x: bit a set iff bit b of c 2^a is set."""
    row = 0
    for a in range(8):
        if (gf_mul(c, 1 << a) >> b) & 1:
            row |= 1 << a
    return row


def program(masks):
    """Greedy cover: returns (ops, value masks, outs) for the set of masks."""
    vals = [1 << a for a in range(8)]          # value id -> mask
    have = {m: i for i, m in enumerate(vals)}
    have[0] = NONE
    ops = []

    def pair(m):
        if m in have:
            return (have[m], NONE)
        for x in list(have):
            if (m ^ x) in have:
                return (have[x], have[m ^ x])
        return None

    need = sorted({m for m in masks if pair(m) is None})
    while need:
        cands = {}
        avail = list(have)
        for x in need:
            for a in avail:
                c = x ^ a
                if c not in have:
                    cands[c] = None
        best, best_n, best_src = None, -1, None
        for c in sorted(cands):
            src = None
            for a in avail:          # one 2-input XOR of available values
                if a and (c ^ a) in have and (c ^ a) != 0:
                    src = (have[a], have[c ^ a], NONE)
                    break
            if src is None:          # or one 3-input XOR
                for a, b in itertools.combinations([v for v in avail if v], 2):
                    if (c ^ a ^ b) in have and (c ^ a ^ b) not in (0, a, b):
                        src = (have[a], have[b], have[c ^ a ^ b])
                        break
            if src is None:
                continue
            n = 0
            for x in need:
                if (x ^ c) in have or x == c:
                    n += 1
            if n > best_n:
                best, best_n, best_src = c, n, src
        assert best is not None
        have[best] = len(vals)
        vals.append(best)
        ops.append(best_src)
        need = [m for m in need if pair(m) is None]
    return ops, vals, pair


def twiddle(c):
    """XOR program of the in-register map x -> c x on 8 planes (a Horner
    twiddle): outputs are masks over the input planes; greedy: whenever an
    output is one 2- or 3-input XOR of available values, build it, else add
    the 3-input XOR that makes the most outputs reachable."""
    outs_m = [mat_row(c, b) for b in range(8)]
    vals = [1 << a for a in range(8)]
    have = {m: i for i, m in enumerate(vals)}
    ops = []

    def one_op(m):
        for a, b in itertools.combinations(list(have), 2):
            if a ^ b == m:
                return (have[a], have[b], NONE)
        for a, b, d in itertools.combinations(list(have), 3):
            if a ^ b ^ d == m:
                return (have[a], have[b], have[d])
        return None

    need = [m for m in dict.fromkeys(outs_m) if m not in have]
    while need:
        done = None
        for m in need:
            src = one_op(m)
            if src:
                done = (m, src)
                break
        if done is None:
            best, best_n, best_src = None, -1, None
            for a, b, d in itertools.combinations(list(have), 3):
                cnd = a ^ b ^ d
                if cnd in have:
                    continue
                have[cnd] = -1
                n = sum(1 for m in need if one_op(m))
                del have[cnd]
                if n > best_n:
                    best, best_n, best_src = cnd, n, (have[a], have[b], have[d])
            done = (best, best_src)
        m, src = done
        have[m] = len(vals)
        vals.append(m)
        ops.append(src)
        need = [x for x in need if x not in have]
    return ops, [have[m] for m in outs_m]


def block(K, E, C, R0, NR, T):
    rows = [[mat_row(gf_pow2(r * T), b) for b in range(8)] for r in range(R0, R0 + NR)]
    ops, vals, pair = program({m for row in rows for m in row})
    outs = [pair(m) for row in rows for m in row]
    return ops, vals, outs


def t0_partners(K, E, C, R0, NR):
    """partner[o] for T0Pair (see the module docstring); all zeros when a
    chunk may be partial (K % C != 0)."""
    part = [0] * (NR * 8)
    if K % C or (K, E, C) in NO_T0_PAIR:
        return part
    for T in range(1, C):
        _, _, outs = block(K, E, C, R0, NR, T)
        for o, (x, y) in enumerate(outs):
            if part[o] == 0 and x != NONE and y == NONE:
                part[o] = T
    return part


def main():
    out = ["// generated by gen_enc_progs.py -- do not edit"]
    total = nblk = 0
    for K, E, C, NW in PLANS:
        opw = (E + NW - 1) // NW
        for g in range(NW):
            R0 = g * opw
            NR = min(opw, E - R0)
            if NR <= 0:
                continue
            for T in range(C):
                ops, vals, outs = block(K, E, C, R0, NR, T)
                total += len(ops)
                nblk += 1
                o = ", ".join("{%d, %d, %d}" % op for op in ops) if ops else "{255, 255, 255}"
                w = ", ".join("{%d, %d}" % p for p in outs)
                out.append(f"template <> struct EncProg<{K}, {E}, {C}, {R0}, {NR}, {T}> {{")
                out.append(f"    static constexpr int NOPS = {len(ops)};")
                out.append(f"    static constexpr uint8_t ops[{max(1, len(ops))}][3] = {{{o}}};")
                out.append(f"    static constexpr uint8_t outs[{NR * 8}][2] = {{{w}}};")
                out.append("};")
            part = t0_partners(K, E, C, R0, NR)
            out.append(f"template <> struct T0Pair<{K}, {E}, {C}, {R0}, {NR}> {{")
            out.append(f"    static constexpr uint8_t partner[{NR * 8}] = {{{', '.join(map(str, part))}}};")
            out.append("};")
    out.append(f"// {nblk} blocks, {total / max(1, nblk):.2f} composite XORs per source on average")
    # Horner twiddles: row r of a plan with chunk C is multiplied by 2^(C r)
    tw_total = tw_n = 0
    for K, E, C, NW in PLANS:
        for r in range(E):
            ops, outs = twiddle(gf_pow2(C * r))
            tw_total += len(ops)
            tw_n += 1
            o = ", ".join("{%d, %d, %d}" % op for op in ops) if ops else "{255, 255, 255}"
            out.append(f"template <> struct TwProg<{K}, {E}, {C}, {r}> {{")
            out.append(f"    static constexpr int NOPS = {len(ops)};")
            out.append(f"    static constexpr uint8_t ops[{max(1, len(ops))}][3] = {{{o}}};")
            out.append(f"    static constexpr uint8_t outs[8] = {{{', '.join(map(str, outs))}}};")
            out.append("};")
    out.append(f"// {tw_n} twiddle rows, {tw_total / max(1, tw_n):.2f} XORs per row on average")
    with open(sys.argv[1], "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
