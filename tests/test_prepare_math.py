"""The one-matrix decode's prepare algebra (k_decode_prepare_syn, closed form)
restated in Python and checked against the oracle's decode rows, i.e. the
rows of inv(b) that isa.cpp:177-204 applies (oracle/rs_oracle.c
orc_decode_matrix, Gauss-Jordan of ec_base.c:99-152).  CPU only.

Kernel algorithm (rs_kernels.hip): points a_i = 2^(j_i) of the erased
originals, b_q = 2^(j_q) of the survivors (ascending), Lambda(z) = prod (z + a_l)
built one linear factor at a time, w_i = prod_{l != i} (a_i + a_l);
  row i, survivor q:  Lambda(b_q) / ((b_q + a_i) w_i)
  row i, parity p:    [z^p] (Lambda(z) / (z + a_i)) / w_i   (synthetic division)
"""
import random

import numpy as np
import pytest

from oracle_lib import Oracle

EXP = [0] * 512
LOG = [0] * 256
_v = 1
for _i in range(255):
    EXP[_i] = EXP[_i + 255] = _v
    LOG[_v] = _i
    _v <<= 1
    if _v & 0x100:
        _v ^= 0x11D


def mul(x, y):
    return EXP[LOG[x] + LOG[y]] if x and y else 0


def div(x, y):
    return EXP[(LOG[x] + 255 - LOG[y]) % 255] if x else 0


def closed_form(k, e, err):
    a = [EXP[j] for j in err]
    live = [j for j in range(k) if j not in set(err)]
    lam = [1]  # coefficient of z^m at index m
    for al in a:  # times (z + a_l), as the wave-parallel loop does
        lam = [(lam[m - 1] if m else 0) ^ (mul(al, lam[m]) if m < len(lam) else 0)
               for m in range(len(lam) + 1)]
    w = []
    for i, ai in enumerate(a):
        p = 1
        for l, al in enumerate(a):
            if l != i:
                p = mul(p, ai ^ al)
        w.append(p)
    rows = np.zeros((e, k), np.uint8)
    for i, ai in enumerate(a):
        for q, j in enumerate(live):
            bq = EXP[j]
            lb = 1
            for al in a:
                lb = mul(lb, bq ^ al)
            rows[i, q] = div(div(lb, bq ^ ai), w[i])
        qm = lam[e]  # synthetic division, q_{e-1} down to q_0
        for m in range(e - 1, -1, -1):
            rows[i, len(live) + m] = div(qm, w[i])
            if m:
                qm = lam[m] ^ mul(ai, qm)
    return rows


@pytest.fixture(scope="module")
def orc():
    return Oracle()


@pytest.mark.parametrize("k,e", [(64, 32), (16, 4), (100, 20), (20, 7), (5, 4), (64, 16), (9, 9), (40, 1),
                                 # e >= 64: Lambda's e + 1 coefficients built through LDS
                                 (186, 64), (150, 100), (125, 125), (160, 65)])
def test_closed_form_equals_inverse_rows(orc, k, e):
    rng = random.Random(k * 100 + e)
    for _ in range(6):
        err = sorted(rng.sample(range(k), e))
        rc, ref = orc.decode_matrix(k, e, err)
        assert rc == 0  # Vandermonde in distinct points: never singular
        assert (closed_form(k, e, err) == ref).all(), (k, e, err)
