#!/usr/bin/env python3
"""karatsuba_price.py -- VERDICT r04 item 3, priced on the CPU only: would an
algebraic split of the C3 encode matrix cut the compiled encode's XOR work?

The code's parity rows are V[r][j] = 2^(r j) (gf_gen_rs_matrix, isa/ec_base.c:
62-79; C3: r < 32, j < 64).  Since r j = C(r+j, 2) - C(r, 2) - C(j, 2),
    V = D1 . H . D2,  H[r][j] = h(r + j) = 2^C(r+j, 2)  (Hankel),
    D1 = diag(2^-C(r, 2)),  D2 = diag(2^-C(j, 2)),
and a square Hankel block [[A, B], [B, C]] (A = h(r+j), B = h(r+j+m),
C = h(r+j+2m)) times [x1; x2] needs three half-size products instead of
four (Karatsuba):  P = B (x1 + x2),  y_top = P + (A + B) x1,
y_bot = P + (C + B) x2  (+ is XOR: GF(2^8) has characteristic 2).

Everything is counted in wave64 VALU instructions per C3 column tile (2 KB x
96 rows) under the bit-sliced four-Russians scheme of the product kernels
(rs_bitsliced.hip): per (wave, source) the greedy cover of gen_enc_progs.py
(the composites its masks need), one instruction per nonzero output mask,
8 per vector addition, the greedy XOR program of gen_enc_progs.twiddle per
constant scaling (single-value outputs are renames), 36 per bit transpose.
Every split is checked on random bytes against V itself first.

What the counts do not show, and why the encode is not built this way
(DESIGN §4): every Karatsuba form shares a product (X = B (x1 + x2)) between
the top and the bottom output rows, which live in different waves.  A wave
owns ONE set of 8-row accumulators and its sources arrive as a stream, so
its share of X can reach the other wave only as a pure snapshot, which
exists only if the wave finishes X before it starts its own Q rows -- and
Q's sources (x1) are then streamed past it again (+25 % source traffic), or
it holds X and Q in two accumulator sets (+64 VGPRs: 3 waves per SIMD, and
the compiled 16-row encode already spills 416 VGPRs at that budget).  With
the measured prices (profiles/r05_energy/: 1 KB of LDS per tile ~ 2.75
VALU) neither leaves the >= 8 % the verdict asked for.

usage: python3 tools/karatsuba_price.py [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd", "csrc"))
import gen_enc_progs as G  # noqa: E402  (program, twiddle, mat_row, gf_mul, gf_pow2)

K, E = 64, 32
TR8 = 36          # VALU per tr8 (24 v_bitop3 + 12 64-bit shifts, tools/tr8_codegen.sh)
VADD = 8          # one vector (8 planes) XORed into another


def gpow(n: int) -> int:
    return G.gf_pow2(n % 255)


def c2(n: int) -> int:
    return n * (n - 1) // 2


EXP = [gpow(i) for i in range(255)]
LOG = {v: i for i, v in enumerate(EXP)}


def inv(c: int) -> int:
    return EXP[(255 - LOG[c]) % 255]


# ---- arithmetic on vectors of bytes (a source row: a list of byte values) --
MUL = [[G.gf_mul(a, b) for b in range(256)] for a in range(256)]


def vmul(c, x):
    t = MUL[c]
    return [t[v] for v in x]


def vadd(x, y):
    return [a ^ b for a, b in zip(x, y)]


def matvec(M, xs):
    out = []
    for row in M:
        acc = [0] * len(xs[0])
        for c, x in zip(row, xs):
            if c:
                acc = vadd(acc, vmul(c, x))
        out.append(acc)
    return out


# ---- costs ------------------------------------------------------------------
_prog_cache = {}


def source_cost(coefs):
    """One (wave, source): the cover of the masks of coefficients `coefs`
    (one per row of the wave) and one instruction per nonzero output mask."""
    key = tuple(coefs)
    if key not in _prog_cache:
        masks = [G.mat_row(c, b) for c in coefs for b in range(8)]
        ops, _, _ = G.program(set(masks))
        _prog_cache[key] = (len(ops), sum(1 for m in masks if m))
    return _prog_cache[key]


def product_cost(M):
    """A wave computing all rows of M (rows x sources) over its sources."""
    comp = mac = 0
    for s in range(len(M[0])):
        c, m = source_cost([row[s] for row in M])
        comp += c
        mac += m
    return comp, mac


_scale_cache = {}


def scale_cost(c: int) -> int:
    if c == 1:
        return 0
    if c not in _scale_cache:
        ops, _ = G.twiddle(c)
        _scale_cache[c] = len(ops)
    return _scale_cache[c]


# ---- the matrices -------------------------------------------------------------
V = [[gpow(r * j) for j in range(K)] for r in range(E)]


def h(n: int) -> int:
    return gpow(c2(n))


def check_hankel():
    for r in range(E):
        for j in range(K):
            assert MUL[MUL[gpow(-c2(r))][h(r + j)]][gpow(-c2(j))] == V[r][j], (r, j)


def hblock(off: int, m: int):
    """m x m Hankel block h(r + j + off)."""
    return [[h(r + j + off) for j in range(m)] for r in range(m)]


def madd(A, B):
    return [[a ^ b for a, b in zip(ra, rb)] for ra, rb in zip(A, B)]


def rows(M, r0, n):
    return M[r0:r0 + n]


# ---- the current kernel: k_rs_bs<64, 32, 16, 4> ---------------------------------
def current():
    C, NW, OPW = 16, 4, 8
    comp = mac = 0
    for g in range(NW):
        for T in range(C):
            c, m = source_cost([gpow(r * T) for r in range(g * OPW, (g + 1) * OPW)])
            comp += c
            mac += m
    comp *= K // C
    mac *= K // C
    # source 0 of a chunk (coefficient 1): 204 of its 256 single-plane
    # outputs per chunk ride in a later source's 3-input XOR (T0Pair)
    t0 = 204 * (K // C)
    tw = sum(scale_cost(gpow(C * r)) for r in range(E)) * (K // C - 1)
    tr = (K + E) * TR8
    total = comp + mac - t0 + tw + tr
    return {"composites": comp, "macs": mac, "t0pair_saved": t0, "twiddles": tw, "transposes": tr,
            "total": total}


# ---- one Karatsuba level on each 32 x 32 Hankel half, no Horner ------------------
def karatsuba1(check=True):
    m = 16
    halves = []
    for base in (0, 32):  # H_a = h(r + j), H_b = h(r + j + 32)
        A, B, Cc = hblock(base, m), hblock(base + m, m), hblock(base + 2 * m, m)
        halves.append({"P": B, "Q1": madd(A, B), "Q2": madd(Cc, B)})
    if check:
        rng = random.Random(5)
        d = [[rng.randrange(256) for _ in range(6)] for _ in range(K)]
        x = [vmul(gpow(-c2(j)), d[j]) for j in range(K)]
        y = [[0] * 6 for _ in range(E)]
        for hv, base in zip(halves, (0, 32)):
            x1, x2 = x[base:base + m], x[base + m:base + 2 * m]
            s = [vadd(a, b) for a, b in zip(x1, x2)]
            P = matvec(hv["P"], s)
            for r, (p, q) in enumerate(zip(P, matvec(hv["Q1"], x1))):
                y[r] = vadd(y[r], vadd(p, q))
            for r, (p, q) in enumerate(zip(P, matvec(hv["Q2"], x2))):
                y[m + r] = vadd(y[m + r], vadd(p, q))
        y = [vmul(gpow(-c2(r)), y[r]) for r in range(E)]
        assert y == matvec(V, d), "Karatsuba split disagrees with V"
    comp = mac = 0
    per = {}
    for name in ("P", "Q1", "Q2"):
        for hv in halves:
            for r0 in (0, 8):  # 8-row halves (a wave's accumulators)
                c, mm = product_cost(rows(hv[name], r0, 8))
                comp += c
                mac += mm
                per.setdefault(name, [0, 0])
                per[name][0] += c
                per[name][1] += mm
    # X = P_a + P_b computed once per 8 rows (waves 0, 1), shared through LDS
    # with the waves of the bottom rows (2, 3): the virtual sources
    # x1 + x2 of both halves formed by waves 0 and 1 each (32 x 8 x 2), the
    # readers' XOR of X (2 x 64)
    virt = 2 * 32 * VADD
    share = 2 * 64
    d2 = sum(scale_cost(gpow(-c2(j))) for j in range(K))
    d1 = sum(scale_cost(gpow(-c2(r))) for r in range(E))
    tr = (K + E) * TR8
    total = comp + mac + virt + share + d1 + d2 + tr
    return {"composites": comp, "macs": mac, "by_product": per, "virtual_sources": virt,
            "x_share": share, "d1": d1, "d2": d2, "transposes": tr, "total": total,
            "lds_extra_bytes_per_tile": 2 * 2 * 16 * 1024,
            "per_wave": {"waves 0,1 (P_a, P_b, Q1_a, Q1_b half-products)": None,
                         "waves 2,3 (Q2_a, Q2_b, + X)": None}}


# ---- one Karatsuba level, the balanced four-wave layout -----------------------
def karatsuba1_balanced(check=True):
    """y = H_a x_a + H_b x_b with 16 x 16 blocks A..E = h(r + j + 16 i):
    X = B (x1 + x2) + D (x3 + x4),  Q1 = (A + B) x1 + (C + D) x3,
    Q2 = (C + B) x2 + (E + D) x4,  y_top = X + Q1,  y_bot = X + Q2.
    Waves: w (rows 8 h .. 8 h + 7 of y_top or y_bot, h = w & 1, bottom =
    w >> 1) computes X rows over HALF of the 32 virtual sources (top waves
    x1 + x2, bottom waves x3 + x4) and its own Q rows over 32 sources, writes
    its X part (a snapshot, 16 KB) to LDS and adds its partner's: 48
    (wave, source) programs of 8 rows per wave, 384 coefficient
    applications each, balanced; LDS reads 48 sources per wave instead of 64
    plus one 16 KB snapshot, the same bytes as k_rs_bs."""
    m = 16
    A, B, Cc, D, Ee = (hblock(16 * i, m) for i in range(5))
    X = [rb + rd for rb, rd in zip(B, D)]                 # 16 x 32 over [s_a; s_b]
    Q1 = [a + c for a, c in zip(madd(A, B), madd(Cc, D))]  # over [x1; x3]
    Q2 = [a + c for a, c in zip(madd(Cc, B), madd(Ee, D))]  # over [x2; x4]
    if check:
        rng = random.Random(9)
        d = [[rng.randrange(256) for _ in range(6)] for _ in range(K)]
        x = [vmul(gpow(-c2(j)), d[j]) for j in range(K)]
        x1, x2, x3, x4 = x[0:16], x[16:32], x[32:48], x[48:64]
        s = [vadd(a, b) for a, b in zip(x1, x2)] + [vadd(a, b) for a, b in zip(x3, x4)]
        xv = matvec(X, s)
        top = [vadd(a, b) for a, b in zip(xv, matvec(Q1, x1 + x3))]
        bot = [vadd(a, b) for a, b in zip(xv, matvec(Q2, x2 + x4))]
        y = [vmul(gpow(-c2(r)), v) for r, v in enumerate(top + bot)]
        assert y == matvec(V, d), "balanced Karatsuba layout disagrees with V"
    waves = []
    for w in range(4):
        h, bottom = w & 1, w >> 1
        rx = [row[16 * bottom:16 * bottom + 16] for row in X[8 * h:8 * h + 8]]  # X over its half
        rq = (Q2 if bottom else Q1)[8 * h:8 * h + 8]
        cx, mx = product_cost(rx)
        cq, mq = product_cost(rq)
        waves.append({"composites": cx + cq, "macs": mx + mq, "virtual_sources": 16 * VADD,
                      "snapshot_xor": 64})
    d2 = sum(scale_cost(gpow(-c2(j))) for j in range(K))
    d1 = sum(scale_cost(gpow(-c2(r))) for r in range(E))
    tr = (K + E) * TR8
    total = sum(sum(w.values()) for w in waves) + d1 + d2 + tr
    per_wave = [sum(w.values()) + (d1 + d2 + tr) / 4 for w in waves]
    return {"waves": waves, "d1": d1, "d2": d2, "transposes": tr, "total": total,
            "per_wave_total": [round(v) for v in per_wave],
            "lds_read_sources_per_wave": 48, "lds_snapshot_bytes_per_tile": 4 * 2 * 16 * 1024}


# ---- the same algebra, recursively, without any layout (a lower bound) ---------
def karatsuba_rec(levels: int):
    """Products of (32 / 2^levels)-square Hankel blocks, every output row in
    one place (no wave split, no sharing cost): the algebraic floor."""
    def rec(off, n, lv):
        # returns (composites+macs, adds) for an n x n Hankel h(r+j+off)
        if lv == 0:
            c, m = product_cost(hblock(off, n))
            return c + m, 0
        mm = n // 2
        # P = h(off + m) block, Q1 = h(off) + h(off+m), Q2 = h(off+2m) + h(off+m)
        cP, aP = rec(off + mm, mm, lv - 1)
        A, B, Cc = hblock(off, mm), hblock(off + mm, mm), hblock(off + 2 * mm, mm)
        q1 = madd(A, B)
        q2 = madd(Cc, B)
        c1 = sum(product_cost(q1)) if lv == 1 else None
        c2_ = sum(product_cost(q2)) if lv == 1 else None
        if lv > 1:  # Q1, Q2 are not Hankel-shifted copies: count them directly
            c1 = sum(product_cost(q1))
            c2_ = sum(product_cost(q2))
        adds = aP + mm * VADD + 2 * mm * VADD  # x1 + x2; P into both outputs
        return cP + c1 + c2_, adds
    tot = 0
    adds = 0
    for base in (0, 32):
        w, a = rec(base, 32, levels)
        tot += w
        adds += a
    d2 = sum(scale_cost(gpow(-c2(j))) for j in range(K))
    d1 = sum(scale_cost(gpow(-c2(r))) for r in range(E))
    return {"levels": levels, "products": tot, "adds": adds, "d1": d1, "d2": d2,
            "transposes": (K + E) * TR8, "total": tot + adds + d1 + d2 + (K + E) * TR8}


# ---- Karatsuba inside ONE wave's rows ---------------------
# A wave owns R output rows r in [R w, R w + R) of a Horner chunk of C = 16
# sources; its R x R blocks of the Hankel form (g(n) = h(R w + j0 + n)) split
# into top / bottom row halves and a source pair (x1, x2) of m = R / 2 each:
#   P = B (x1 + x2),  top += P + (A + B) x1,  bottom += P + (C + B) x2,
# all three Hankel again, so the split recurses.  P reaches both halves with
# no second accumulator set: top ^= bottom; bottom += P; top ^= bottom (two
# vector additions, 16 m VALU).  Real sources keep the D2 scaling folded into
# their coefficients; a virtual source x1 s1 + x2 s2 is formed explicitly
# (16 VALU from the two sources' tables, 8 for two virtual ones); D1 once per
# row and tile at the end (the Horner twiddle 2^(C r) is unchanged).
def inwave_cost(g, m, srcs, lv):
    """VALU of y[r] = sum_q g[r + q] src_q, r < m, inside one wave; srcs are
    the folded scales of real sources (None: a virtual source)."""
    if lv == 0 or m < 4:
        tot = 0
        for q, s in enumerate(srcs):
            c, mm = source_cost([MUL[g[r + q]][s] if s is not None else g[r + q] for r in range(m)])
            tot += c + mm
        return tot, {"leaf": tot}
    hm = m // 2
    x1, x2 = srcs[:hm], srcs[hm:]
    virt = sum(VADD if a is None and b is None else 2 * VADD for a, b in zip(x1, x2))
    gB = [g[n + hm] for n in range(2 * hm - 1)]
    gQ1 = [g[n] ^ g[n + hm] for n in range(2 * hm - 1)]
    gQ2 = [g[n + 2 * hm] ^ g[n + hm] for n in range(2 * hm - 1)]
    cP, _ = inwave_cost(gB, hm, [None] * hm, lv - 1)
    cQ1, _ = inwave_cost(gQ1, hm, x1, lv - 1)
    cQ2, _ = inwave_cost(gQ2, hm, x2, lv - 1)
    tb = 2 * VADD * hm
    return cP + cQ1 + cQ2 + virt + tb, {"P": cP, "Q1": cQ1, "Q2": cQ2, "virtual_sources": virt,
                                        "P_into_both_halves": tb}


def inwave_eval(g, m, xs, lv):
    """The same recursion on byte vectors (xs already scaled by D2)."""
    if lv == 0 or m < 4:
        return [matvec([[g[r + q] for q in range(m)]], xs)[0] for r in range(m)]
    hm = m // 2
    x1, x2 = xs[:hm], xs[hm:]
    v = [vadd(a, b) for a, b in zip(x1, x2)]
    P = inwave_eval([g[n + hm] for n in range(2 * hm - 1)], hm, v, lv - 1)
    Q1 = inwave_eval([g[n] ^ g[n + hm] for n in range(2 * hm - 1)], hm, x1, lv - 1)
    Q2 = inwave_eval([g[n + 2 * hm] ^ g[n + hm] for n in range(2 * hm - 1)], hm, x2, lv - 1)
    return [vadd(p, q) for p, q in zip(P, Q1)] + [vadd(p, q) for p, q in zip(P, Q2)]


def inwave_tile(R: int, lv: int, C: int = 16, check=True):
    """One C3 column tile with E / R waves of R rows, Horner chunks of C."""
    tot, parts = 0, {}
    rng = random.Random(R * 10 + lv)
    for w in range(E // R):
        for j0 in range(0, C, R):
            g = [h(R * w + j0 + n) for n in range(2 * R - 1)]
            if check:
                d = [[rng.randrange(256) for _ in range(4)] for _ in range(R)]
                y = inwave_eval(g, R, [vmul(gpow(-c2(j0 + q)), d[q]) for q in range(R)], lv)
                for r in range(R):
                    row = R * w + r
                    want = matvec([[gpow(row * (j0 + q)) for q in range(R)]], d)[0]
                    assert vmul(gpow(c2(row)), want) == y[r], ("in-wave split disagrees with V", R, lv, row)
            c, p = inwave_cost(g, R, [gpow(-c2(j0 + q)) for q in range(R)], lv)
            tot += c
            for key, v in p.items():
                parts[key] = parts.get(key, 0) + v
    tot *= K // C
    parts = {key: v * (K // C) for key, v in parts.items()}
    tw = sum(scale_cost(gpow(C * r)) for r in range(E)) * (K // C - 1)
    d1 = sum(scale_cost(gpow(-c2(r))) for r in range(E))
    tr = (K + E) * TR8
    return {"rows_per_wave": R, "levels": lv, "products_and_adds": tot, "parts": parts, "twiddles": tw,
            "d1": d1, "transposes": tr, "total": tot + tw + d1 + tr,
            "vgprs": "accumulators 8 R + planes 8 + composites <= 22 + one virtual source's 8 planes"}


def direct_rows(R: int, C: int = 16):
    """The plain compiled encode with R rows per wave (no split): R = 8 is
    k_rs_bs<64, 32, 16, 4> without T0Pair, R = 16 round 4's two-wave layout."""
    comp = mac = 0
    for g in range(E // R):
        for T in range(C):
            c, m = source_cost([gpow(r * T) for r in range(g * R, (g + 1) * R)])
            comp += c
            mac += m
    comp *= K // C
    mac *= K // C
    tw = sum(scale_cost(gpow(C * r)) for r in range(E)) * (K // C - 1)
    tr = (K + E) * TR8
    return {"rows_per_wave": R, "composites": comp, "macs": mac, "twiddles": tw, "transposes": tr,
            "total": comp + mac + tw + tr}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    check_hankel()
    cur = current()
    k1 = karatsuba1()
    rec1 = karatsuba_rec(1)
    bal = karatsuba1_balanced()
    res = {"workload": "C3 encode (64, 32), one 2 KB column tile, wave64 VALU",
           "measured_k_rs_bs_valu_per_tile": round(1.201e10 / (489 * 1024), 1),
           "current_model": cur, "karatsuba_1level_layout": k1, "karatsuba_1level_balanced": bal,
           "karatsuba_1level_floor": rec1}
    res["in_wave"] = {"direct_R8": direct_rows(8), "direct_R16": direct_rows(16)}
    for R, lv in ((16, 1), (16, 2), (8, 1)):
        res["in_wave"][f"karatsuba_R{R}_levels{lv}"] = inwave_tile(R, lv)
    res["in_wave_cut_vs_model"] = {key: round(1 - v["total"] / cur["total"], 4)
                                   for key, v in res["in_wave"].items()}
    res["cut_vs_model"] = {"karatsuba_1level_layout": round(1 - k1["total"] / cur["total"], 4),
                           "karatsuba_1level_balanced": round(1 - bal["total"] / cur["total"], 4),
                           "karatsuba_1level_floor": round(1 - rec1["total"] / cur["total"], 4)}
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
