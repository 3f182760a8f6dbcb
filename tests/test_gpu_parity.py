"""GPU parity: the HIP path through the C ABI vs the oracle and the reference's
golden vectors (bit-exact: all work is byte arithmetic).

Small sizes are compared byte-for-byte with the CPU oracle; the benchmark
sizes (symbol_size 1e6, 16..100 symbols) are checked through the
size-independent round trip encode -> erase -> decode -> verify on the device,
plus every byte of one block per geometry against the oracle.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import rsgpu  # noqa: E402
from oracle_lib import Oracle  # noqa: E402
from golden.synth import erasure_pattern, synth_block, synth_row  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def sha(b):
    return hashlib.sha256(np.ascontiguousarray(b).tobytes()).hexdigest()


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


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_fill_synthetic_matches_definition(ctx):
    for L, pitch in ((1000, 1024), (8191, 8192), (17, 32), (64, 64)):
        rows = 5
        buf = torch.zeros(rows * pitch, dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic(buf, rows, L, pitch, 77, 10)
        got = buf.view(rows, pitch).cpu().numpy()
        for r in range(rows):
            assert (got[r, :L] == synth_row(77, 10 + r, L)).all()
            assert (got[r, L:] == 0).all()


def test_fill_synthetic_many_rows_and_odd_base(ctx):
    """More rows than one grid dimension holds (the fill's row loop), and a
    destination that is not 8-byte aligned (bytewise stores)."""
    rows, L, pitch = 70000, 24, 32
    buf = torch.zeros(rows * pitch + 8, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic(buf, rows, L, pitch, 5, 3)
    got = buf[:rows * pitch].view(rows, pitch).cpu().numpy()
    for r in (0, 1, 65534, 65535, 65536, rows - 1):
        assert (got[r, :L] == synth_row(5, 3 + r, L)).all()
    odd = buf[1:]
    ctx.fill_synthetic(odd, 3, 21, 29, 6, 0)
    g = odd[:3 * 29].view(3, 29).cpu().numpy()
    for r in range(3):
        assert (g[r, :21] == synth_row(6, r, 21)).all()


@pytest.mark.parametrize("L", [32000, 1000, 4099])
def test_verify_counts_each_differing_byte(ctx, L):
    """rsgpu_verify_blocks (isa.cpp:215-229 on the device) counts every
    differing byte of a recovered row, in the 16-byte body and the tail."""
    k, e, B = 8, 3, 4
    pitch = (L + 255) // 256 * 256
    rng = np.random.default_rng(L)
    src = torch.from_numpy(rng.integers(0, 256, (B, k, pitch), dtype=np.uint8)).cuda()
    err = np.array([[1, 4, 6]] * B, np.uint8)
    out = src[:, [1, 4, 6], :].clone()
    for b in range(1, B):
        pos = rng.choice(L, size=5 * b, replace=False)
        for p in pos:
            r = int(rng.integers(0, e))
            out[b, r, int(p)] ^= int(rng.integers(1, 256))
        # several bytes of one dword, and the last byte
        out[b, 0, 16:20] ^= 0xFF
        out[b, 2, L - 1] ^= 1
    # count what actually differs (a random position may repeat a fixed one)
    ref = (out.cpu().numpy()[:, :, :L] != src.cpu().numpy()[:, [1, 4, 6], :L]).sum(axis=(1, 2))
    mism = torch.zeros(B, dtype=torch.int64, device="cuda")
    ctx.verify_blocks(k, e, L, pitch, B, src, out, dev(err), mism)
    torch.cuda.synchronize()
    assert mism.cpu().numpy().tolist() == ref.tolist()
    assert int(mism[0]) == 0 and (ref[1:] > 0).all()


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"k{c['k']}e{c['e']}L{c['len']}")
def test_golden_batched_encode_decode(ctx, case):
    """Batched encode (specialized or generic) + device decode vs the
    reference's golden parity hashes and recovered bytes."""
    k, e, L = case["k"], case["e"], case["len"]
    B = len(case["blocks"])
    seed = GOLD["seed"]
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    assert dec.decode_all(enc) == e
    torch.cuda.synchronize()
    assert dec.is_complete()
    assert dec.verify_data(enc)
    for b in case["blocks"]:
        blk = b["blk"]
        src = enc.source_rows(blk)
        assert [sha(r) for r in src] == b["src_sha"]
        par = enc.parity_rows(blk)
        assert [sha(p) for p in par] == b["parity_sha"], "parity differs from ISA-L"
        assert dec.err_host[blk].tolist() == b["err"]
        rec = dec.recovered_rows(blk)
        for i, s in enumerate(b["err"]):
            assert (rec[i] == src[s]).all()


@pytest.mark.parametrize("k,e,L", [(16, 4, 4096), (64, 32, 4096), (100, 20, 4096), (7, 3, 1024),
                                   (16, 8, 64000), (33, 31, 2048)])
def test_generic_encode_equals_specialized_and_oracle(ctx, orc, k, e, L):
    B = 3
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=5, ctx=ctx)
    enc.encode_all()
    spec = enc.par.clone()
    a = rsgpu.gf_gen_rs_matrix(k + e, k)
    # explicit coefficients force the runtime-coefficient kernel
    ctx.encode_blocks(k, e, L, enc.pitch, B, enc.src, enc.par, coef=a[k:])
    torch.cuda.synchronize()
    assert torch.equal(spec, enc.par)
    for blk in range(B):
        data = list(enc.source_rows(blk))
        ref = orc.encode_block(data, e)
        got = enc.parity_rows(blk)
        for p in range(e):
            assert (got[p] == ref[p]).all()


def test_cauchy_encode_golden(ctx):
    g = GOLD["cauchy_9_5"]
    ca = np.frombuffer(bytes.fromhex(g["matrix_hex"]), np.uint8).reshape(9, 5)
    L = g["len"]
    enc = rsgpu.GpuEncoder(5, L, 4, blocks=1, seed=GOLD["seed"], ctx=ctx, block0=g["blk"])
    ctx.encode_blocks(5, 4, L, enc.pitch, 1, enc.src, enc.par, coef=ca[5:])
    par = enc.parity_rows(0)
    assert [p.tobytes().hex() for p in par] == g["parity_hex"]


@pytest.mark.parametrize("length", [0, 1, 15, 16, 17, 33, 100, 4095, 8191, 65537])
def test_ec_encode_data_pointer_api_any_length(ctx, orc, length):
    """rsgpu_ec_encode_data == ec_encode_data_base for odd lengths
    (erasure_code_base_test.c:687-760 sweeps odd lengths)."""
    rng = np.random.default_rng(length)
    k, rows = 11, 6
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    g = orc.init_tables(k, rows, coef)
    data = [rng.integers(0, 256, max(length, 1), dtype=np.uint8) for _ in range(k)]
    d_data = [dev(d) for d in data]
    d_out = [torch.zeros(max(length, 1), dtype=torch.uint8, device="cuda") for _ in range(rows)]
    ctx.ec_encode_data(length, k, rows, g, d_data, d_out)
    torch.cuda.synchronize()
    ref = [np.zeros(max(length, 1), np.uint8) for _ in range(rows)]
    if length:
        orc.encode_data(length, k, rows, g, data, ref)
    for r in range(rows):
        assert (d_out[r].cpu().numpy()[:length] == ref[r][:length]).all()


def test_ec_encode_data_misaligned_pointers(ctx, orc):
    """Random pointer misalignment (erasure_code_base_test.c:566-685)."""
    rng = np.random.default_rng(9)
    k, rows, L = 9, 5, 3001
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    g = orc.init_tables(k, rows, coef)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    pool = torch.zeros((k + rows) * (L + 64), dtype=torch.uint8, device="cuda")
    offs = [int(rng.integers(0, 32)) + i * (L + 64) for i in range(k + rows)]
    for j in range(k):
        pool[offs[j]: offs[j] + L] = dev(data[j])
    base = pool.data_ptr()
    ctx.ec_encode_data(L, k, rows, g, [base + offs[j] for j in range(k)],
                       [base + offs[k + r] for r in range(rows)])
    torch.cuda.synchronize()
    ref = [np.zeros(L, np.uint8) for _ in range(rows)]
    orc.encode_data(L, k, rows, g, data, ref)
    host = pool.cpu().numpy()
    for r in range(rows):
        o = offs[k + r]
        assert (host[o: o + L] == ref[r]).all()
        # pad bytes after the output untouched
        assert (host[o + L: o + L + 16] == 0).all()


@pytest.mark.parametrize("length", [1, 64, 1000, 4096, 70001])
def test_ec_encode_data_update(ctx, orc, length):
    rng = np.random.default_rng(length + 1)
    k, rows = 8, 5
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    g = orc.init_tables(k, rows, coef)
    data = rng.integers(0, 256, length, dtype=np.uint8)
    start = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(rows)]
    d_out = [dev(s) for s in start]
    ctx.ec_encode_data_update(length, k, rows, 3, g, dev(data), d_out)
    torch.cuda.synchronize()
    ref = [s.copy() for s in start]
    orc.encode_data_update(length, k, rows, 3, g, data, ref)
    for r in range(rows):
        assert (d_out[r].cpu().numpy() == ref[r]).all()


@pytest.mark.parametrize("k,rows", [(8, 1), (32, 1), (20, 3), (40, 24)])
def test_shared_program_cache_cycles_matrices(ctx, orc, k, rows):
    """rsgpu_ec_encode_data through the cached host-built programs: 70
    different coefficient matrices (more than the 64-entry cache holds), then
    the first ten again (rebuilt after eviction) and the last ten (cache hits),
    each against the oracle's ec_encode_data_base on the same sources."""
    rng = np.random.default_rng(k * 100 + rows)
    length = 8192
    src = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(k)]
    d_src = [dev(x) for x in src]
    d_out = [torch.empty(length, dtype=torch.uint8, device="cuda") for _ in range(rows)]
    mats = [rng.integers(0, 256, (rows, k), dtype=np.uint8) for _ in range(70)]
    for i in list(range(70)) + list(range(10)) + list(range(60, 70)):
        g = orc.init_tables(k, rows, mats[i])
        ctx.ec_encode_data(length, k, rows, g, d_src, d_out)
        ref = [np.zeros(length, np.uint8) for _ in range(rows)]
        orc.encode_data(length, k, rows, g, src, ref)
        torch.cuda.synchronize()
        for r in range(rows):
            assert (d_out[r].cpu().numpy() == ref[r]).all(), (i, r)


@pytest.mark.parametrize("length", [32, 64, 1000, 4096, 70016])
def test_single_vector_isal_entry_points(ctx, orc, length):
    """gf_vect_dot_prod (erasure_code.h:637, ec_base.c:264-276), gf_vect_mad
    (:664, ec_base.c:278-288) and gf_vect_mul (gf_vect_mul.h:108,
    ec_base.c:323-329) through the C ABI, against the oracle's base C; the
    multiply refuses a length that is not a multiple of 32 as ISA-L's
    dispatched function does."""
    rng = np.random.default_rng(length + 7)
    vlen = 9
    coef = rng.integers(0, 256, (1, vlen), dtype=np.uint8)
    g = orc.init_tables(vlen, 1, coef)
    src = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(vlen)]
    d_src = [dev(x) for x in src]
    d_dst = torch.full((length,), 0x5A, dtype=torch.uint8, device="cuda")
    ctx.gf_vect_dot_prod(length, vlen, g, d_src, d_dst)
    ref = [np.zeros(length, np.uint8)]
    orc.encode_data(length, vlen, 1, g, src, ref)
    torch.cuda.synchronize()
    assert (d_dst.cpu().numpy() == ref[0]).all()
    # multiply-accumulate of source 4 into a random destination
    start = rng.integers(0, 256, length, dtype=np.uint8)
    d_acc = dev(start)
    ctx.gf_vect_mad(length, vlen, 4, g, d_src[4], d_acc)
    want = [start.copy()]
    orc.encode_data_update(length, vlen, 1, 4, g, src[4], want)
    torch.cuda.synchronize()
    assert (d_acc.cpu().numpy() == want[0]).all()
    # dest = c * src
    tbl = orc.vect_mul_init(0x8E)
    d_mul = torch.zeros(length, dtype=torch.uint8, device="cuda")
    if length % 32:
        assert ctx.gf_vect_mul(length, tbl, d_src[0], d_mul) != 0
        return
    assert ctx.gf_vect_mul(length, tbl, d_src[0], d_mul) == 0
    want = np.zeros(length, np.uint8)
    orc.vect_mul(length, tbl, src[0], want)
    torch.cuda.synchronize()
    assert (d_mul.cpu().numpy() == want).all()
    assert ctx.gf_vect_mul(length + 1, tbl, d_src[0], d_mul) != 0


@pytest.mark.parametrize("k,e,L,B", [(16, 4, 1000000, 2), (64, 32, 1000000, 2),
                                     (100, 20, 1000000, 2), (64, 32, 32000, 64),
                                     (16, 8, 64000, 8)])
def test_benchmark_sizes_round_trip(ctx, orc, k, e, L, B):
    """Configs of BASELINE.json at full symbol size: encode -> erase -> decode ->
    device verify for every block; block 0's parity rows sampled vs oracle."""
    seed = 1234
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    assert dec.is_complete()
    assert dec.verify_data(enc)
    # sampled bytes vs the oracle on a 4 KiB window of block B-1
    blk = B - 1
    src = enc.source_rows(blk)
    win = slice(L // 2, L // 2 + 4096) if L >= 8192 else slice(0, L)
    data = [np.ascontiguousarray(s[win]) for s in src]
    ref = orc.encode_block(data, e)
    par = enc.parity_rows(blk)
    for p in range(e):
        assert (par[p][win] == ref[p]).all()
    # the erasures are the ones the definition picks
    assert dec.err_host[blk].tolist() == erasure_pattern(seed, blk, k, e).tolist()


@pytest.mark.parametrize("k,e", [(16, 4), (64, 32), (100, 20)])
def test_full_rows_byte_for_byte_vs_oracle(ctx, orc, k, e):
    """BASELINE's full symbol size (1e6 bytes), every byte of one block: all e
    parity rows against the oracle's ec_encode_data, and all e recovered rows
    against the oracle's decode (gf_invert_matrix + ec_encode_data over the
    survivors, isa.cpp:169-213) of the GPU's own parity."""
    L, B, seed = 1000000, 2, 4321
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    assert dec.is_complete()
    blk = B - 1
    data = [np.ascontiguousarray(s) for s in enc.source_rows(blk)]
    par = enc.parity_rows(blk)
    ref = orc.encode_block(data, e)
    for p in range(e):
        assert (par[p] == ref[p]).all(), p
    rc, rec = orc.decode_block(data, list(par), dec.err_host[blk])
    assert rc == 0
    got = dec.recovered_rows(blk)
    for i in range(e):
        assert (got[i] == rec[i]).all(), i
        assert (got[i] == data[dec.err_host[blk][i]]).all(), i


@pytest.mark.parametrize("k,e,L,B", [(64, 32, 1000000, 256), (100, 20, 1000000, 96)])
def test_full_occupancy_repeated_round_trips(ctx, k, e, L, B):
    """Enough blocks to fill every CU with several workgroups, encode + decode
    repeated back to back with a device verify after each: workgroup-level
    races (a missing barrier between a phase's last LDS reads and the next
    phase's writes) only show when co-resident workgroups run out of step,
    which the small-batch parity tests do not provoke."""
    seed = 99
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
    for _ in range(3):
        enc.encode_all()
        dec.decode_all(enc)
        torch.cuda.synchronize()
        assert dec.is_complete()
        assert dec.verify_data(enc)


def test_decode_matches_oracle_decode_rows(ctx, orc):
    """Decoding also recovers from a parity buffer that was produced by the
    oracle (cross-implementation), and recovers garbage-free bytes."""
    k, e, L, B = 20, 7, 2048, 3
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=8, ctx=ctx)
    pv = enc.par.view(B, e, enc.pitch)
    for blk in range(B):
        data = list(synth_block(8, blk, k, L))
        ref = orc.encode_block(data, e)
        for p in range(e):
            pv[blk, p, :L] = dev(ref[p])
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=8, ctx=ctx)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    assert dec.is_complete() and dec.verify_data(enc)


@pytest.mark.parametrize("k,e,L,B", [(40, 20, 8192, 3), (100, 30, 4096, 2), (200, 32, 2048, 2),
                                     (33, 1, 64, 2), (9, 9, 32, 3)])
def test_general_geometry_decode_tc(ctx, orc, k, e, L, B):
    """Codes without compile-time kernels (k x k inversion in k_decode_prepare,
    then the decode rows through the threaded-code kernel): parity from the
    oracle, decode, device verify of every recovered byte."""
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=31, ctx=ctx)
    pv = enc.par.view(B, e, enc.pitch)
    for blk in range(B):
        ref = orc.encode_block(list(synth_block(31, blk, k, L)), e)
        for p in range(e):
            pv[blk, p, :L] = dev(ref[p])
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=31, ctx=ctx)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    assert dec.is_complete() and dec.verify_data(enc)
    # and the device encode of the same code equals the oracle parity
    enc2 = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=31, ctx=ctx)
    enc2.encode_all()
    torch.cuda.synchronize()
    p2 = enc2.par.view(B, e, enc2.pitch)
    assert torch.equal(p2[:, :, :L], pv[:, :, :L])


def test_all_erasure_counts_small(ctx):
    """Every erasure count 1..k for small k (edge: e == k, only parity left)."""
    k, L = 12, 512
    for e in range(1, k + 1):
        enc = rsgpu.GpuEncoder(k, L, e, blocks=2, seed=e, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=2, seed=e, ctx=ctx)
        dec.decode_all(enc)
        torch.cuda.synchronize()
        assert dec.is_complete() and dec.verify_data(enc), e


def test_throughput_benchmark_mirror(ctx):
    tb = rsgpu.ThroughputBenchmark(symbols=(16,), loss_rate=(0.5,), symbol_size=(64000,),
                                   blocks=4, ctx=ctx)
    cfgs = tb.configurations()
    assert [c.type for c in cfgs] == ["encoder", "decoder"]
    for c in cfgs:
        row = tb.run(c)
        assert row["accepted"] and row["goodput"] > 0


def test_cpp_runner_end_to_end(tmp_path):
    """The C++ plugin + harness (storage-benchmarks_amd/host) on the GPU, with
    gauge-compatible CSV output columns."""
    import subprocess
    runner = os.path.join(os.path.dirname(HERE), "storage-benchmarks_amd", "bin", "rs_throughput")
    csv_path = tmp_path / "out.csv"
    r = subprocess.run([runner, "--symbols", "16", "64", "--symbol_size", "64000",
                        "--loss_rate", "0.5", "--blocks", "4", "--runs", "2",
                        "--csv_file", str(csv_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = csv_path.read_text().strip().splitlines()
    assert lines[0].startswith("testcase,benchmark,symbols,symbol_size,loss_rate,type,erased_symbols")
    assert len(lines) == 1 + 2 * 2 * 2  # symbols x type x runs
    for ln in lines[1:]:
        assert float(ln.split(",")[-1]) > 0


@pytest.mark.gpu
def test_plugin_dropin_reference_shape():
    """gpu_encoder / gpu_decoder driven exactly as throughput_benchmark.hpp
    drives isa_encoder / isa_decoder (3-argument constructors, synchronous
    encode_all / decode_all, is_complete, verify_data)."""
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "storage-benchmarks_amd", "bin", "plugin_dropin_test")
    r = subprocess.run([exe, "16:64000:8", "16:1000000:4", "64:1000000:32", "100:64000:20",
                        "10:4096:4", "5:8192:4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("complete=1 verified=1") == 6, r.stdout


@pytest.mark.parametrize("mode", ["generated", "one_matrix", "general"])
def test_decode_modes_end_to_end(mode):
    """Every decode kernel choice (rsgpu_set_decode_kernel): the one-matrix
    k_rs_tc decode, the per-block generated code and the general k x k
    inversion, through the reference-shaped plugin with device
    verification of every recovered byte."""
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "storage-benchmarks_amd", "bin", "plugin_dropin_test")
    r = subprocess.run([exe, "--decode-kernel", mode, "16:64000:8", "64:1000000:32", "100:64000:20",
                        "64:32000:32", "20:4096:7"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("complete=1 verified=1") == 5, r.stdout


@pytest.mark.parametrize("k,e,L,B,kind", [
    (32, 8, 4096, 3, "all256"),   # coefficient (r*32 + j) & 255: every value 0..255 once
    (13, 20, 2048, 2, "random"),  # partial LDS chunks (13 = 8 + 5), 3 wave groups
    (40, 32, 8192, 2, "random"),  # 5 chunks, 4 wave groups
    (3, 1, 64, 1, "random"),      # smallest shapes
])
def test_runtime_coefficient_encode_tc(ctx, orc, k, e, L, B, kind):
    """Arbitrary coefficient matrices through the threaded-code kernel
    (k_rs_tc: len % 32 == 0, aligned rows) == the oracle's ec_encode_data_base."""
    rng = np.random.default_rng(k * 1000 + e)
    if kind == "all256":
        coef = ((np.arange(e)[:, None] * k + np.arange(k)[None, :]) & 255).astype(np.uint8)
    else:
        coef = rng.integers(0, 256, (e, k), dtype=np.uint8)
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=9, ctx=ctx)
    ctx.encode_blocks(k, e, L, enc.pitch, B, enc.src, enc.par, coef=coef)
    torch.cuda.synchronize()
    g = orc.init_tables(k, e, coef)
    for blk in range(B):
        data = list(enc.source_rows(blk))
        ref = [np.zeros(L, np.uint8) for _ in range(e)]
        orc.encode_data(L, k, e, g, data, ref)
        got = enc.parity_rows(blk)
        for p in range(e):
            assert (got[p] == ref[p]).all(), (blk, p)


@pytest.mark.parametrize("kernel,name", [("auto", "k_rs_jit(ec_encode_data)"),
                                         ("threaded", "k_rs_tc(ec_encode_data)")])
def test_ec_encode_data_pointer_api_tc(ctx, orc, kernel, name):
    """rsgpu_ec_encode_data with 32-multiple lengths and aligned rows takes the
    generated code (default) or the threaded-code kernel; same bytes as
    ec_encode_data_base."""
    ctx.set_encode_kernel(kernel)
    rng = np.random.default_rng(77)
    k, rows, length = 17, 11, 32 * 1001
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    g = orc.init_tables(k, rows, coef)
    data = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(k)]
    d_data = [dev(d) for d in data]
    d_out = [torch.zeros(length, dtype=torch.uint8, device="cuda") for _ in range(rows)]
    ctx.timing_read()
    ctx.timing_enable(True)
    ctx.ec_encode_data(length, k, rows, g, d_data, d_out)
    names = [n for n, _, _ in ctx.timing_read()]
    ctx.timing_enable(False)
    ctx.set_encode_kernel("auto")
    assert names == [name], names
    ref = [np.zeros(length, np.uint8) for _ in range(rows)]
    orc.encode_data(length, k, rows, g, data, ref)
    for r in range(rows):
        assert (d_out[r].cpu().numpy() == ref[r]).all()


@pytest.mark.parametrize("k,e,pattern", [
    (64, 32, list(range(32))),                # bit 31 set, sources 32..63 all live
    (64, 32, list(range(1, 64, 2))),          # odd sources: bits 31 and 63 set
    (100, 20, [31, 63] + list(range(64, 82))),  # both 32-bit halves' sign bits + em1
    (100, 20, list(range(80, 100))),          # only the high mask word
])
def test_syndrome_decode_sign_bit_masks(ctx, k, e, pattern):
    """Erasure masks whose 32-bit halves have the sign bit set (a mask
    sign-extended when made wave-uniform marked every higher source erased)."""
    L, B = 4096, 2
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=4, ctx=ctx)
    enc.encode_all()
    errs = np.array([pattern] * B, np.uint8)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=4, ctx=ctx, erasures=errs)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    assert dec.is_complete()
    assert dec.verify_data(enc)


def test_isa_arithmetic_peer():
    """bin/rs_arithmetic (peer of benchmark/isa_arithmetic) runs every
    benchmark of the reference's sweep and checks that the 1/2/4/all-row pass
    splits give identical outputs (the runner exits non-zero otherwise)."""
    import subprocess
    exe = os.path.join(os.path.dirname(HERE), "storage-benchmarks_amd", "bin", "rs_arithmetic")
    out = subprocess.run([exe, "--size", "65536", "1000", "--vectors", "8", "13", "32"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("ISA/")]
    assert len(lines) == 2 * 3 * 4
    for name in ("dot_product1", "dot_product2", "dot_product4", "dot_product_encode"):
        assert sum(name + " " in ln for ln in lines) == 6


@pytest.mark.parametrize("length", [1000, 1024, 992, 100, 65536])
@pytest.mark.parametrize("per", [1, 2, 4, 8])
def test_ec_encode_data_row_passes(ctx, orc, length, per):
    """ec_encode_data called in passes of `per` output rows, as
    ec_encode_data_avx2 splits them (ec_highlevel_func.c:106-135) and
    isa_arithmetic's dot_product1/2/4 drive them, back to back on one
    stream: every pass equals the oracle."""
    rng = np.random.default_rng(length * 10 + per)
    k = rows = 8
    a = orc.gen_rs_matrix(2 * k, k)
    g = orc.init_tables(k, rows, a[k:])
    data = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(k)]
    d_data = [dev(d) for d in data]
    d_out = [torch.zeros(length, dtype=torch.uint8, device="cuda") for _ in range(rows)]
    for r in range(0, rows, per):
        ctx.ec_encode_data(length, k, per, g[r * k * 32:], d_data, d_out[r:r + per])
    torch.cuda.synchronize()
    ref = [np.zeros(length, np.uint8) for _ in range(rows)]
    orc.encode_data(length, k, rows, g, data, ref)
    bad = [r for r in range(rows) if not (d_out[r].cpu().numpy() == ref[r]).all()]
    assert not bad, f"rows {bad} differ"


def test_host_io_ragged_chunks(ctx):
    """bench.host_io_pipelined (the library's host-resident calls): 70 C4-shaped
    blocks go through device staging in chunks (42 blocks of (64, 32, 32000)
    per chunk: a ragged last chunk); the recovered rows that came back equal
    the originals and the parity equals the device path's.  The serial
    host_io_rate verifies too."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    r = bench.host_io_pipelined(rsgpu, ctx, 64, 32, 32000, 70, seed=3, reps=1)
    assert r["verified"] and r["blocks"] == 70
    s = bench.host_io_rate(rsgpu, ctx, 16, 8, 64000, 6, seed=3, reps=1)
    assert s["verified"] and s["poisoned"]


@pytest.mark.parametrize("k,e,L,B,chunk", [(64, 32, 32000, 11, 4), (16, 4, 1000000, 3, 2), (20, 7, 8192, 7, 3)])
def test_host_io_session(ctx, k, e, L, B, chunk):
    """bench.host_io_session (data crosses the link once each way: sources
    in, parity and recovered rows out, three streams over three device slots):
    ragged last chunk, slots reused; the parity equals the device path's and
    the recovered rows the originals."""
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    r = bench.host_io_session(rsgpu, ctx, k, e, L, B, seed=5, chunk=chunk, reps=1)
    assert r["verified"] and r["blocks"] == B


@pytest.mark.parametrize("k,e,kernel", [(64, 32, "generated"), (64, 32, "auto"), (100, 20, "generated"),
                                        (16, 4, "auto")])
def test_full_row_every_byte_vs_oracle(ctx, orc, k, e, kernel):
    """One block of a BASELINE geometry at its full 1 MB rows, EVERY byte of
    the parity and of the recovered rows against the CPU oracle (the round
    trips above compare the whole batch with the originals on the device and
    a 4 KiB window with the oracle).  The decode runs with the erased rows
    poisoned, through the generated code (two tiles per workgroup) or AUTO's
    choice for the call (threaded code; the one-launch small decode at
    (16, 4))."""
    L, B, seed = 1000000, 2, 4242
    ctx.set_decode_kernel(kernel)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=seed, ctx=ctx)
        torch.cuda.synchronize()
        blk = 1
        data = [np.ascontiguousarray(s) for s in enc.source_rows(blk)]
        ref = orc.encode_block(data, e)
        par = enc.parity_rows(blk)
        for p in range(e):
            assert (par[p] == ref[p]).all(), p
        src = enc.src.view(B, k, enc.pitch)
        for b in range(B):
            for j in dec.err_host[b]:
                src[b, int(j), :L] = 0xA5
        dec.decode_all(enc)
        torch.cuda.synchronize()
        assert dec.is_complete()
        rc, rec = orc.decode_block(data, [np.ascontiguousarray(x) for x in par], dec.err_host[blk])
        assert rc == 0
        got = dec.recovered_rows(blk)
        for i, j in enumerate(dec.err_host[blk]):
            assert (got[i] == rec[i]).all() and (got[i] == data[int(j)]).all(), (i, int(j))
    finally:
        ctx.set_decode_kernel("auto")
