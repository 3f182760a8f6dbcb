"""GPU parity over randomly drawn geometries (fixed seeds, so every run draws
the same cases): k, e, row length (32-multiples and odd lengths, short and
long rows), batch size, encode kernel, decode kernel and the short-row
decode's slicing all vary together, as no hand-picked list combines them.

Each case: encode the batch (parity of block 0 against the oracle's
ec_encode_data_base on the reference's gf_gen_rs_matrix rows), overwrite
every erased original of every block (0xA5) while the decode runs, then
compare each recovered row with the saved original.  isa.cpp:108-229 is the
flow; the erasure patterns are the reference's (isa.cpp:133-156, through
rsgpu.erasure_patterns).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import rsgpu  # noqa: E402
from oracle_lib import Oracle  # noqa: E402
from test_gpu_decode import decode_poisoned, run_general  # noqa: E402

ENC = ["auto", "generated", "threaded"]
DEC = ["auto", "generated", "one_matrix", "general"]


def draw(seed):
    """One case from its seed: (k, e, L, B, encode kernel, decode kernel,
    slicing knob)."""
    r = np.random.default_rng(seed)
    k = int(r.choice([2, 3, 5, 8, 13, 16, 20, 31, 32, 33, 48, 64, 65, 100, 127, 160, 200]))
    e = int(r.integers(1, min(k, 250 - k) + 1))
    if r.random() < 0.7:
        L = 32 * int(r.integers(1, 2048))            # aligned, up to 64 KB
    else:
        L = int(r.integers(1, 20000))                 # any length
    B = int(r.integers(1, 7))
    return k, e, L, B, ENC[seed % 3], DEC[(seed // 3) % 4], int(r.choice([-1, 0, 2, 3]))


# RSGPU_FUZZ_N widens the draw for a one-off extended run (default 48 cases)
CASES = [draw(s) for s in range(1000, 1000 + int(os.environ.get("RSGPU_FUZZ_N", "48")))]


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    c = rsgpu.Context(0)
    c.set_torch_stream()
    yield c
    torch.cuda.synchronize()
    c.close()


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def set_pipeline(ctx, n):
    import ctypes
    f = rsgpu.testhooks().rsgpu_internal_set_decode_pipeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert f(ctx._h, n) == 0


@pytest.mark.parametrize("case", CASES, ids=lambda c: "k{}e{}L{}B{}-{}-{}-p{}".format(*c))
def test_random_geometry_round_trip(ctx, orc, case):
    k, e, L, B, enc_k, dec_k, pipe = case
    ctx.set_encode_kernel(enc_k)
    ctx.set_decode_kernel(dec_k)
    set_pipeline(ctx, pipe)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=k * 1000 + e, ctx=ctx)
        enc.encode_all()
        torch.cuda.synchronize()
        ref = orc.encode_block(list(enc.source_rows(0)), e)
        got = enc.parity_rows(0)
        assert all((got[p] == ref[p]).all() for p in range(e)), "parity differs from ec_encode_data_base"
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=k * 1000 + e, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
    finally:
        set_pipeline(ctx, -1)
        ctx.set_encode_kernel("auto")
        ctx.set_decode_kernel("auto")


def draw_general(seed):
    """A general-decode case: an RS or Cauchy m x k code, erasures among data
    AND parity rows, rows long enough (>= 48 column tiles) for the generated
    general decode or short for the threaded / v_perm kernels."""
    r = np.random.default_rng(seed)
    k = int(r.integers(2, 120))
    p = int(r.integers(1, min(64, 250 - k) + 1))
    n = int(r.integers(1, p + 1))
    L = int(r.choice([131072, 98304 + 32 * int(r.integers(0, 512)), 4096, 4093]))
    kind = "rs" if seed % 2 else "cauchy"
    return k, p, n, L, kind


GENERAL = [draw_general(s) for s in range(2000, 2000 + int(os.environ.get("RSGPU_FUZZ_GENERAL_N", "16")))]


@pytest.mark.parametrize("case", GENERAL, ids=lambda c: "k{}p{}n{}L{}-{}".format(*c))
def test_random_general_decode(ctx, orc, case):
    """rsgpu_decode_general (gf_gen_decode_matrix semantics,
    erasure_code_base_test.c:133-213) over drawn codes and erasure lists of
    data and parity rows, erased rows poisoned, against the oracle's
    decode_general; a singular draw must report status -1 as the reference's
    -1 return."""
    k, p, n, L, kind = case
    m = k + p
    rng = np.random.default_rng(k * 7 + p)
    enc_m = orc.gen_rs_matrix(m, k) if kind == "rs" else orc.gen_cauchy1_matrix(m, k)
    err = np.sort(rng.choice(m, n, replace=False)).tolist()
    enc = rsgpu.GpuEncoder(k, L, p, blocks=1, seed=k + p, ctx=ctx)
    ctx.encode_blocks(k, p, L, enc.pitch, 1, enc.src, enc.par, coef=enc_m[k:])
    torch.cuda.synchronize()
    rows = list(enc.src.view(k, enc.pitch)[:, :L].cpu().numpy()) + \
        list(enc.par.view(p, enc.pitch)[:, :L].cpu().numpy())
    rc, ref = orc.decode_general(enc_m, [np.ascontiguousarray(x) for x in rows], err)
    st, rec = run_general(ctx, enc_m, enc, err, k, m, L)
    assert st == (0 if rc == 0 else -1), (k, m, err)
    if rc == 0:
        assert all((rec[i] == ref[i]).all() for i in range(n)), (k, m, err)


def draw_pointer_api(seed):
    r = np.random.default_rng(seed)
    k = int(r.integers(1, 65))
    rows = int(r.integers(1, 41))
    length = int(r.choice([32 * int(r.integers(1, 2200)), int(r.integers(1, 70000))]))
    aligned = bool(r.integers(0, 2))
    return k, rows, length, aligned


POINTER_API = [draw_pointer_api(s) for s in range(3000, 3000 + int(os.environ.get("RSGPU_FUZZ_API_N", "16")))]


@pytest.mark.parametrize("case", POINTER_API, ids=lambda c: "k{}r{}len{}-{}".format(
    c[0], c[1], c[2], "aligned" if c[3] else "offset"))
def test_random_ec_encode_data(ctx, orc, case):
    """rsgpu_ec_encode_data (erasure_code.h:98, the ISA-L argument list) over
    drawn k, rows and lengths, with each row either 16-byte aligned or at a
    drawn byte offset, then ec_encode_data_update of one source into the
    same outputs: equal to the oracle's ec_encode_data_base and
    ec_encode_data_update_base."""
    k, rows, length, aligned = case
    rng = np.random.default_rng(k * 100 + rows)
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    g = orc.init_tables(k, rows, coef)
    data = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(k)]
    pool = torch.zeros((k + rows) * (length + 64), dtype=torch.uint8, device="cuda")
    offs = [0 if aligned else int(rng.integers(0, 16)) for _ in range(k + rows)]
    views = [pool[i * (length + 64) + offs[i]: i * (length + 64) + offs[i] + length] for i in range(k + rows)]
    for i in range(k):
        views[i].copy_(torch.from_numpy(data[i]))
    d_data, d_out = views[:k], views[k:]
    ctx.ec_encode_data(length, k, rows, g, d_data, d_out)
    ref = [np.zeros(length, np.uint8) for _ in range(rows)]
    orc.encode_data(length, k, rows, g, data, ref)
    torch.cuda.synchronize()
    assert all((d_out[r].cpu().numpy() == ref[r]).all() for r in range(rows))
    vec_i = int(rng.integers(0, k))
    upd = rng.integers(0, 256, length, dtype=np.uint8)
    d_upd = torch.from_numpy(upd).cuda()
    ctx.ec_encode_data_update(length, k, rows, vec_i, g, d_upd, d_out)
    orc.encode_data_update(length, k, rows, vec_i, g, upd, ref)
    torch.cuda.synchronize()
    assert all((d_out[r].cpu().numpy() == ref[r]).all() for r in range(rows))
