"""GPU encode parity for every encode kernel (include/rsgpu.h
rsgpu_set_encode_kernel): the matrix compiled into the kernel, the
generated code built on the host once per matrix and shared by every block,
and the threaded-code kernel.  Parity rows must equal the oracle's
ec_encode_data_base restatement (isa/ec_base.c:290-305) for the
gf_gen_rs_matrix code, for caller matrices (Cauchy, random) and through the
ISA-L pointer API, including more than 32 rows (passes) and a matrix change
between calls (the cached code must be rebuilt)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import rsgpu  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

KERNELS = ["auto", "compiled", "generated", "threaded"]


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU test needs a HIP device"
    c = rsgpu.Context(0)
    c.set_torch_stream()
    yield c
    torch.cuda.synchronize()
    c.set_encode_kernel("auto")
    c.close()


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def encode_and_check(ctx, orc, k, e, L, B, coef=None, seed=5, pitch=None):
    """encode_blocks over B synthetic blocks; parity of every block against
    the oracle with the same matrix."""
    dev = torch.device("cuda", 0)
    pitch = pitch or (L + 255) // 256 * 256
    src = torch.empty(B * k * pitch, dtype=torch.uint8, device=dev)
    par = torch.full((B * e * pitch,), 0x5A, dtype=torch.uint8, device=dev)
    ctx.fill_synthetic(src, B * k, L, pitch, seed, 0)
    ctx.encode_blocks(k, e, L, pitch, B, src, par, coef=coef)
    torch.cuda.synchronize()
    a = orc.gen_rs_matrix(k + e, k)[k:] if coef is None else np.asarray(coef, np.uint8)
    s = src.view(B, k, pitch)[:, :, :L].cpu().numpy()
    pv = par.view(B, e, pitch)[:, :, :L].cpu().numpy()
    for b in range(B):
        want = [np.zeros(L, np.uint8) for _ in range(e)]
        orc.encode_data(L, k, e, orc.init_tables(k, e, a), list(s[b]), want)
        for i in range(e):
            assert (pv[b, i] == want[i]).all(), (k, e, L, b, i)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("k,e,L,B", [(64, 32, 65536, 3), (16, 4, 32000, 2), (100, 20, 8192, 2),
                                     (32, 16, 4096, 5), (128, 64, 2048, 2), (9, 40, 1024, 2),
                                     (20, 13, 96, 3), (250 - 37, 37, 64, 2),
                                     # more than 64 rows: passes of <= 64 in the wide layout
                                     (150, 100, 4096, 2), (125, 125, 2048, 2), (160, 65, 8192, 2),
                                     # the other compiled codes (k_rs_bs, source 0 pairing)
                                     (16, 8, 8192, 2), (64, 16, 4096, 2), (5, 4, 2048, 3), (20, 7, 4096, 2)],
                         ids=str)
def test_encode_kernels_rs(ctx, orc, kernel, k, e, L, B):
    ctx.set_encode_kernel(kernel)
    try:
        encode_and_check(ctx, orc, k, e, L, B)
    finally:
        ctx.set_encode_kernel("auto")


@pytest.mark.parametrize("kernel", ["auto", "generated", "threaded"])
def test_encode_caller_matrices(ctx, orc, kernel):
    """Cauchy and random caller matrices, back to back with the RS code: each
    call whose matrix differs from the last rebuilds the shared program."""
    ctx.set_encode_kernel(kernel)
    try:
        rng = np.random.default_rng(7)
        k, e, L, B = 24, 12, 8192, 2
        cauchy = orc.gen_cauchy1_matrix(k + e, k)[k:]
        rand = rng.integers(0, 256, (e, k), dtype=np.uint8)
        for coef in (cauchy, rand, None, cauchy, rand):
            encode_and_check(ctx, orc, k, e, L, B, coef=coef)
    finally:
        ctx.set_encode_kernel("auto")


def test_compiled_equals_generated_at_size(ctx):
    """The C3 code (64, 32) at full row length: the compiled kernel and the
    generated program write identical parity."""
    dev = torch.device("cuda", 0)
    k, e, L, B = 64, 32, 1000000, 4
    pitch = (L + 255) // 256 * 256
    src = torch.empty(B * k * pitch, dtype=torch.uint8, device=dev)
    ctx.fill_synthetic(src, B * k, L, pitch, 9, 0)
    outs = []
    for kernel in ("compiled", "generated"):
        ctx.set_encode_kernel(kernel)
        par = torch.zeros(B * e * pitch, dtype=torch.uint8, device=dev)
        ctx.encode_blocks(k, e, L, pitch, B, src, par)
        outs.append(par)
    ctx.set_encode_kernel("auto")
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("k,e", [(64, 32), (16, 4), (100, 20), (64, 16)])
@pytest.mark.parametrize("L,B", [(32, 67), (96, 5), (1056, 3), (2080, 2), (32000, 3), (63488 + 32, 2)])
def test_compiled_encode_short_rows_flat(ctx, orc, k, e, L, B):
    """Short rows with a partial last tile run the compiled encode with the
    tiles laid over all blocks' rows end to end (rs_bitsliced.hip tile_pos:
    one tile's lanes may belong to consecutive blocks, up to 64 of them at
    L = 32): every block's parity equals the oracle's and the row padding
    beyond L is left as it was."""
    ctx.set_encode_kernel("compiled")
    try:
        encode_and_check(ctx, orc, k, e, L, B)
        dev = torch.device("cuda", 0)
        pitch = (L + 255) // 256 * 256
        src = torch.empty(B * k * pitch, dtype=torch.uint8, device=dev)
        par = torch.full((B * e * pitch,), 0x5A, dtype=torch.uint8, device=dev)
        ctx.fill_synthetic(src, B * k, L, pitch, 3, 0)
        ctx.encode_blocks(k, e, L, pitch, B, src, par)
        torch.cuda.synchronize()
        assert (par.view(B, e, pitch)[:, :, L:] == 0x5A).all()
    finally:
        ctx.set_encode_kernel("auto")


@pytest.mark.parametrize("k,e,L,B,pitch", [(64, 32, 32, 67, 1 << 20), (16, 4, 96, 130, 1 << 22)], ids=str)
def test_compiled_encode_short_rows_wide_pitch(ctx, orc, k, e, L, B, pitch):
    """Short rows in a widely pitched buffer: a flat tile's lanes address
    their rows from the tile's first block with a 32-bit offset, which at
    L = 32, pitch 1 MiB reaches 64 blocks x 64 rows x 1 MiB = 4 GiB -- the
    launch keeps such geometries on per-block tiles,
    and every block's parity equals the oracle's."""
    ctx.set_encode_kernel("compiled")
    try:
        encode_and_check(ctx, orc, k, e, L, B, pitch=pitch)
    finally:
        ctx.set_encode_kernel("auto")


@pytest.mark.parametrize("k,e,name", [(100, 20, "k_rs_jit(encode)"), (64, 32, "k_rs_bs(encode)"),
                                      (64, 16, "k_rs_bs(encode)")])
def test_auto_encode_kernel_choice(ctx, orc, k, e, name):
    """AUTO keeps a compiled kernel whose waves own >= 8 rows and takes the
    two-wave generated program (composites per 10 rows) over (100, 20)'s
    compiled kernel (composites per 5 rows); parity equals the oracle's."""
    ctx.set_encode_kernel("auto")
    ctx.timing_read()
    ctx.timing_enable(True)
    try:
        encode_and_check(ctx, orc, k, e, 8192, 3)
        names = [n for n, _, _ in ctx.timing_read()]
    finally:
        ctx.timing_enable(False)
    assert names and names[-1] == name, names
