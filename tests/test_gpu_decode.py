"""GPU decode parity, adversarial: the erased rows are poisoned before every
decode, malformed erasure lists must fail the block, and the general decode
(gf_gen_decode_matrix: data AND parity erasures, RS and Cauchy) must match
the reference's golden vectors.

isa_decoder reads only the survivors (benchmark/isa_throughput/isa.cpp:193-
197): its data[] pointer array skips every erased row.  A GPU decoder whose
tables picked an erased row would still pass a test that leaves the erased
originals in place, so here they hold 0xA5 while the decode runs and the
recovered rows are compared with copies saved beforehand.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import rsgpu  # noqa: E402
from oracle_lib import Oracle  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))
BIN = os.path.join(ROOT, "storage-benchmarks_amd", "bin")
KERNELS = ["auto", "generated", "one_matrix", "general"]


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


def poison_rows(view, rows, L):
    """view: [B][R][pitch] device rows; rows: per block the indices to poison.
    Returns the saved originals {(b, r): tensor}."""
    saved = {}
    for b, rr in enumerate(rows):
        for r in rr:
            saved[(b, int(r))] = view[b, int(r), :L].clone()
            view[b, int(r), :L] = 0xA5
    return saved


def restore_rows(view, saved, L):
    for (b, r), t in saved.items():
        view[b, r, :L] = t


def decode_poisoned(ctx, enc, dec):
    """decode_all with every erased original of every block overwritten;
    returns True iff each recovered row equals the saved original."""
    src = enc.src.view(enc.B, enc.k, enc.pitch)
    saved = poison_rows(src, dec.err_host, enc.L)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    out = dec.out.view(dec.B, dec.e, dec.pitch)
    ok = dec.is_complete()
    for b in range(dec.B):
        for i, j in enumerate(dec.err_host[b]):
            ok = ok and torch.equal(out[b, i, :dec.L], saved[(b, int(j))])
    restore_rows(src, saved, enc.L)
    return ok


GEOMS = [(16, 4, 1000000, 2), (64, 32, 1000000, 2), (100, 20, 1000000, 2), (16, 8, 64000, 4),
         (64, 32, 32000, 16), (40, 20, 8192, 3), (200, 32, 2048, 2), (128, 64, 4096, 2),
         (12, 12, 512, 2), (33, 1, 64, 2),
         # 32 < e <= 64: closed-form rows (e <= 63) or the k x k inversion,
         # generated code in four waves per tile (k_rs_jit{10,12,16}x4)
         (96, 48, 131072, 2), (187, 63, 4096, 2), (40, 33, 98304, 2), (100, 50, 131072, 2),
         (128, 64, 131072, 2), (70, 45, 65536, 3),
         # 24 < e <= 32: 16 rows per wave (k_rs_jit16) when generated;
         # 16 < e <= 20: 10 rows per wave (k_rs_jit10)
         (50, 25, 98304, 3), (31, 31, 4096, 2), (218, 32, 2048, 2),
         (17, 17, 65536, 2), (64, 19, 4096, 3), (230, 20, 2048, 2),
         # 20 < e <= 24: 12 rows per wave (k_rs_jit12)
         (48, 24, 65536, 2), (21, 21, 4096, 3), (226, 24, 2048, 2),
         # e > 64 (k + e <= 250 allows 125): closed-form rows through LDS,
         # generated code in passes of <= 64 rows, four waves per tile
         (150, 100, 65536, 2), (125, 125, 32768, 2), (160, 65, 65536, 2), (186, 64, 65536, 2),
         (130, 120, 4096, 2)]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("k,e,L,B", GEOMS, ids=lambda v: str(v))
def test_poisoned_decode_every_kernel(ctx, kernel, k, e, L, B):
    """Every decode kernel (one-matrix closed form, generated code, the
    general k x k inversion, and the automatic choice) recovers the
    originals with the erased rows poisoned, at the BASELINE geometries
    (C2, C3, C5, C1 golden, C4) and general codes (k up to 200, e up to 64
    in four waves per tile, e == k)."""
    ctx.set_decode_kernel(kernel)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=17, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=17, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
        assert dec.verify_data(enc)
    finally:
        ctx.set_decode_kernel("auto")


@pytest.mark.parametrize("kernel", ["auto", "general"])
def test_poisoned_decode_unaligned_lengths(ctx, kernel):
    """Odd symbol sizes go through k_dot_generic (v_perm tables): same
    guarantee with the erased rows poisoned."""
    ctx.set_decode_kernel(kernel)
    try:
        for k, e, L in ((10, 4, 33), (16, 8, 8191), (20, 5, 1000)):
            enc = rsgpu.GpuEncoder(k, L, e, blocks=2, seed=5, ctx=ctx)
            enc.encode_all()
            dec = rsgpu.GpuDecoder(k, L, e, blocks=2, seed=5, ctx=ctx)
            assert decode_poisoned(ctx, enc, dec), (k, e, L)
    finally:
        ctx.set_decode_kernel("auto")


def test_poisoned_host_io_pipelined(ctx):
    """bench.host_io_pipelined poisons the erased rows in host memory before
    its decode leg: the library ships only the survivors (full-length rows:
    runs of consecutive survivors)."""
    sys.path.insert(0, ROOT)
    import bench
    r = bench.host_io_pipelined(rsgpu, ctx, 16, 8, 200000, 6, seed=3, reps=1)
    assert r["verified"] and r["blocks"] == 6 and r["poisoned"]


def malformed(err, k, how):
    bad = err.copy()
    if how == "dup":
        bad[:, 1] = bad[:, 0]
    elif how == "unsorted":
        bad = bad[:, ::-1].copy()
    else:  # index >= k
        bad[:, -1] = k
    return bad


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("how", ["dup", "unsorted", "range"])
def test_malformed_erasure_list_fails_block(ctx, kernel, how):
    """A malformed list (duplicate, unsorted, index >= k) gives that block
    status -2 under every kernel; the other blocks decode; the synchronous
    decoder returns 0 and is not complete (isa.cpp:185-190)."""
    k, e, L, B = 64, 32, 32000, 3
    ctx.set_decode_kernel(kernel)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=2, ctx=ctx)
        enc.encode_all()
        err = rsgpu.erasure_patterns(2, 0, B, k, e)
        err[1] = malformed(err[1:2], k, how)[0]
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=2, ctx=ctx, erasures=err, synchronous=True)
        assert dec.decode_all(enc) == 0
        st = dec.block_status()
        assert st.tolist() == [0, -2, 0], st
        assert not dec.is_complete()
        out = dec.out.view(B, e, dec.pitch)
        src = enc.src.view(B, k, enc.pitch)
        for b in (0, 2):
            for i, j in enumerate(err[b]):
                assert torch.equal(out[b, i, :L], src[b, int(j), :L])
    finally:
        ctx.set_decode_kernel("auto")


@pytest.mark.parametrize("how", ["dup", "unsorted", "range"])
def test_malformed_rejected_by_python_harness(ctx, how):
    """ThroughputBenchmark (the throughput_benchmark.hpp mirror) rejects the
    measurement and counts no recovered bytes (:99-119, :185-196)."""
    k, e = 16, 8
    err = malformed(rsgpu.erasure_patterns(1, 0, 2, k, e), k, how)
    tb = rsgpu.ThroughputBenchmark(symbols=(k,), loss_rate=(0.5,), symbol_size=(64000,),
                                   types=("decoder",), blocks=2, ctx=ctx, erasures=err)
    row = tb.run(tb.configurations()[0])
    assert not row["accepted"] and row["goodput"] == 0


@pytest.mark.parametrize("how", ["dup", "unsorted", "range"])
def test_malformed_rejected_by_cpp_harness(how):
    """gpu_decoder through the C++ harness (host/throughput_benchmark.hpp):
    decode_all returns 0, is_complete() is false, accept_measurement()
    rejects."""
    r = subprocess.run([os.path.join(BIN, "plugin_dropin_test"), "--malformed", how, "16:64000:8",
                        "64:32000:32", "5:8192:4"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("rejected=1") == 3, r.stdout


@pytest.mark.parametrize("kernel", KERNELS)
def test_dropin_poisoned_every_kernel(kernel):
    """The reference-shaped plugin (3-argument constructors, synchronous
    calls) with the erased rows poisoned, for every decode kernel."""
    r = subprocess.run([os.path.join(BIN, "plugin_dropin_test"), "--poison", "--decode-kernel",
                        kernel, "16:64000:8", "16:1000000:4", "64:1000000:32", "100:64000:20",
                        "64:32000:32", "20:4096:7", "5:8192:4"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("poisoned=1 complete=1 verified=1") == 7, r.stdout


def general_setup(ctx, orc, case):
    """Device rows of a golden general-decode case: synthetic data, parity
    from the device encode with the case's matrix."""
    k, m, L = case["k"], case["m"], case["len"]
    enc_m = orc.gen_rs_matrix(m, k) if case["matrix"] == "rs" else orc.gen_cauchy1_matrix(m, k)
    enc = rsgpu.GpuEncoder(k, L, m - k, blocks=1, seed=GOLD["seed"], ctx=ctx, block0=case["blk"])
    ctx.encode_blocks(k, m - k, L, enc.pitch, 1, enc.src, enc.par, coef=enc_m[k:])
    torch.cuda.synchronize()
    return enc_m, enc


def run_general(ctx, enc_m, enc, err, k, m, L, poison=True, matrix_arg=True):
    n = len(err)
    dev = enc.src.device
    d_err = torch.tensor(np.asarray(err, np.uint8), device=dev)
    out = torch.zeros(max(1, n * enc.pitch), dtype=torch.uint8, device=dev)
    ws = torch.empty(rsgpu.decode_general_workspace_bytes(k, m, n, 1), dtype=torch.uint8,
                     device=dev)
    status = torch.full((1,), 7, dtype=torch.int32, device=dev)
    src = enc.src.view(1, k, enc.pitch)
    par = enc.par.view(1, m - k, enc.pitch)
    saved_s = poison_rows(src, [[j for j in err if j < k]], L) if poison else {}
    saved_p = poison_rows(par, [[j - k for j in err if j >= k]], L) if poison else {}
    ctx.decode_general(k, m, L, enc.pitch, 1, enc_m if matrix_arg else None, enc.src, enc.par,
                       d_err, n, out, ws, status)
    torch.cuda.synchronize()
    restore_rows(src, saved_s, L)
    restore_rows(par, saved_p, L)
    rec = out.view(max(1, n), enc.pitch)[:n, :L].cpu().numpy()
    return int(status.item()), rec


@pytest.mark.parametrize("case", GOLD["general_decode"],
                         ids=lambda c: f"{c['matrix']}k{c['k']}m{c['m']}n{len(c['err'])}")
def test_general_decode_golden(ctx, orc, case):
    """rsgpu_decode_general == the reference's gf_gen_decode_matrix +
    recovery (erasure_code_base_test.c:133-213, :299-308) on the golden
    cases: erased data and parity rows (poisoned during the decode), RS and
    Cauchy, the singular-survivor retry and "BAD MATRIX" (status -1)."""
    k, m, L = case["k"], case["m"], case["len"]
    enc_m, enc = general_setup(ctx, orc, case)
    par = enc.par.view(m - k, enc.pitch)[:, :L].cpu().numpy()
    assert [sha(p) for p in par] == case["parity_sha"]
    st, rec = run_general(ctx, enc_m, enc, case["err"], k, m, L)
    if case["rc"] != 0:
        assert st == -1
        return
    assert st == 0
    assert [sha(r) for r in rec] == case["recovered_sha"]
    if case["matrix"] == "rs":  # NULL matrix argument = gf_gen_rs_matrix
        st2, rec2 = run_general(ctx, enc_m, enc, case["err"], k, m, L, matrix_arg=False)
        assert st2 == 0 and (rec2 == rec).all()


@pytest.mark.parametrize("L", [4096, 4095, 33])
def test_general_decode_random_vs_oracle(ctx, orc, L):
    """Random codes and erasure lists (data and parity rows, up to 40
    erasures: more than one k_rs_tc row pass) through the threaded-code
    kernel (aligned 32-byte multiples) or k_dot_generic (odd lengths), equal
    to the oracle's decode_general."""
    rng = np.random.default_rng(L)
    for trial in range(6):
        k = int(rng.integers(2, 80))
        p = int(rng.integers(1, 48))
        m = k + p
        kind = "rs" if trial % 2 else "cauchy"
        enc_m = orc.gen_rs_matrix(m, k) if kind == "rs" else orc.gen_cauchy1_matrix(m, k)
        n = int(rng.integers(1, p + 1))
        err = np.sort(rng.choice(m, n, replace=False)).tolist()
        enc = rsgpu.GpuEncoder(k, L, p, blocks=1, seed=trial, ctx=ctx)
        ctx.encode_blocks(k, p, L, enc.pitch, 1, enc.src, enc.par, coef=enc_m[k:])
        torch.cuda.synchronize()
        rows = list(enc.src.view(k, enc.pitch)[:, :L].cpu().numpy()) + \
            list(enc.par.view(p, enc.pitch)[:, :L].cpu().numpy())
        rc, ref = orc.decode_general(enc_m, [np.ascontiguousarray(r) for r in rows], err)
        st, rec = run_general(ctx, enc_m, enc, err, k, m, L)
        assert st == (0 if rc == 0 else -1), (k, m, err)
        if rc == 0:
            assert all((rec[i] == ref[i]).all() for i in range(n)), (k, m, err)


def test_general_decode_malformed_status(ctx, orc):
    k, m, L = 8, 12, 4096
    enc_m = orc.gen_cauchy1_matrix(m, k)
    enc = rsgpu.GpuEncoder(k, L, m - k, blocks=1, seed=1, ctx=ctx)
    for bad in ([3, 3], [5, 2], [1, 12]):
        st, _ = run_general(ctx, enc_m, enc, bad, k, m, L, poison=False)
        assert st == -2, bad
    with pytest.raises(rsgpu.RsGpuError):
        run_general(ctx, enc_m, enc, [0, 1, 2, 3, 4], k, m, L, poison=False)  # > m - k


@pytest.mark.parametrize("rows", [33, 40, 64, 100])
def test_runtime_encode_row_passes(ctx, orc, rows):
    """More than 32 output rows through the threaded-code kernel in passes
    of 32 (encode with a caller matrix and the ISA-L pointer API)."""
    k, L = 24, 8192
    rng = np.random.default_rng(rows)
    coef = rng.integers(0, 256, (rows, k), dtype=np.uint8)
    enc = rsgpu.GpuEncoder(k, L, rows, blocks=2, seed=rows, ctx=ctx)
    ctx.encode_blocks(k, rows, L, enc.pitch, 2, enc.src, enc.par, coef=coef)
    torch.cuda.synchronize()
    g = orc.init_tables(k, rows, coef)
    for blk in range(2):
        data = list(enc.source_rows(blk))
        ref = [np.zeros(L, np.uint8) for _ in range(rows)]
        orc.encode_data(L, k, rows, g, data, ref)
        got = enc.parity_rows(blk)
        assert all((got[r] == ref[r]).all() for r in range(rows))
    d_data = [torch.from_numpy(d.copy()).cuda() for d in enc.source_rows(0)]
    d_out = [torch.zeros(L, dtype=torch.uint8, device="cuda") for _ in range(rows)]
    ctx.ec_encode_data(L, k, rows, g, d_data, d_out)
    torch.cuda.synchronize()
    assert all((d_out[r].cpu().numpy() == enc.parity_rows(0)[r]).all() for r in range(rows))


def test_stream_switch_orders_scratch_reuse(ctx, orc):
    """rsgpu_set_stream: a runtime-coefficient encode enqueued on one stream,
    the context moved to another, a second encode with other coefficients
    (re-uploading the scratch tables) enqueued there at once: the first
    result must still use its own coefficients."""
    k, rows, L, B = 16, 8, 1 << 20, 8
    rng = np.random.default_rng(3)
    c1 = rng.integers(1, 256, (rows, k), dtype=np.uint8)
    c2 = rng.integers(1, 256, (rows, k), dtype=np.uint8)
    enc = rsgpu.GpuEncoder(k, L, rows, blocks=B, seed=4, ctx=ctx)
    par2 = torch.empty_like(enc.par)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    prev = ctx.get_stream()
    try:
        ctx.set_stream(s1.cuda_stream)
        ctx.encode_blocks(k, rows, L, enc.pitch, B, enc.src, enc.par, coef=c1)
        ctx.set_stream(s2.cuda_stream)
        ctx.encode_blocks(k, rows, L, enc.pitch, B, enc.src, par2, coef=c2)
    finally:
        ctx.set_stream(prev)
    torch.cuda.synchronize()
    for coef, par in ((c1, enc.par), (c2, par2)):
        g = orc.init_tables(k, rows, coef)
        data = list(enc.source_rows(B - 1))
        ref = [np.zeros(L, np.uint8) for _ in range(rows)]
        orc.encode_data(L, k, rows, g, data, ref)
        got = par.view(B, rows, enc.pitch)[B - 1, :, :L].cpu().numpy()
        assert all((got[r] == ref[r]).all() for r in range(rows))


def run_bench(args, timeout=600):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes (here
    both on device 0) on the DEFAULT backend (gloo):
    disjoint contiguous shards, erasure lists drawn from the global block
    index, n_gpus 2, verified."""
    line = run_bench(["--gpus", "2", "--same-device", "--config", "c3",
                      "--blocks", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    assert line["n_gpus"] == 2 and line["verified"]
    assert line["config"]["dist_backend"] == "gloo"
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [(r["block0"], r["blocks"]) for r in ranks] == [(0, 4), (4, 4)]
    for r in ranks:
        err = rsgpu.erasure_patterns(1, r["block0"], r["blocks"], 64, 32)
        assert r["err_sha"] == hashlib.sha256(err.tobytes()).hexdigest()


def test_bench_under_torch_distributed_run():
    """The driver's scaling launch: `python -m torch.distributed.run
    --nproc-per-node 2 ... bench.py --gpus 2` (ranks from WORLD_SIZE/RANK in
    the environment, no self-spawn), here both ranks on device 0 on the
    default backend (gloo)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device",
           "--config", "c3", "--blocks", "4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified"]
    ranks = sorted(line["ranks"], key=lambda q: q["rank"])
    assert [(q["block0"], q["blocks"]) for q in ranks] == [(0, 4), (4, 4)]


def test_rccl_path_single_rank():
    """The collectives bench.py runs between ranks (barrier, all_reduce MAX of
    the timed region, all_gather_object of the shards, all_reduce of the
    mismatch count) on the optional `nccl` backend (--dist-backend nccl), i.e. RCCL, in a world of
    one rank on this GPU: the only RCCL run a one-GPU box allows (two ranks
    cannot share a device under RCCL).  A subprocess owns the process group."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    code = (
        "import os, sys, torch, torch.distributed as dist\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "torch.cuda.set_device(0)\n"
        "dist.init_process_group('nccl', init_method='env://')\n"
        "dev = torch.device('cuda', 0)\n"
        "dist.barrier()\n"
        "t = bench.reduce_max_time(1.25, 2, dev)\n"
        "info = [None]\n"
        "dist.all_gather_object(info, {'rank': 0, 'blocks': 7})\n"
        "bad = torch.tensor([3.0], dtype=torch.float64, device=dev)\n"
        "dist.all_reduce(bad)\n"
        "torch.cuda.synchronize()\n"
        "assert t == 1.25 and info[0]['blocks'] == 7 and bad.item() == 3.0, (t, info, bad)\n"
        "print('backend', dist.get_backend())\n"
        "dist.destroy_process_group()\n" % ROOT)
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "backend nccl" in r.stdout


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_bench_c4_streams_ragged_batches():
    """The streamed C4 path: 3 batches with a ragged tail (2500 blocks in
    batches of 1024), every batch verified on the device."""
    line = run_bench(["--config", "c4", "--blocks", "2500", "--batch", "1024", "--warmup", "1",
                      "--no-cpu-baseline"])
    assert line["verified"]
    st = line["streamed"]
    assert st["batches"] == 3 and st["blocks_total"] == 2500 and st["mismatch_bytes"] == 0
    assert "blocks=2500" in line["config"]["workload"]


def test_bench_c2_line_prices_its_kernels():
    """The C2 line (one block: split encode + one-launch decode): verified,
    its roofline kernel the one-launch decode, every timed kernel priced
    (a kernel missing from bench.alg_bytes used to report 0 GB/s)."""
    line = run_bench(["--config", "c2", "--steps", "20", "--warmup", "2", "--no-cpu-baseline"])
    assert line["verified"]
    assert set(line["kernels"]) == {"k_rs_bs_split(encode)", "k_rs_syn_split(decode)"}
    assert all(v["alg_GBps"] > 0 for v in line["kernels"].values())
    rf = line["roofline"]
    assert rf["kernel"] in line["kernels"] and rf["achieved"] > 0 and 0 < rf["frac"] < 1
    la = line["launch"]  # one launch per op, and what a launch costs on the stream
    assert la["launches_per_step"] == 2 and la["empty_kernel_us_device"] > 0 and la["step_us"] > 0


@pytest.mark.parametrize("kernel", ["auto", "generated", "one_matrix"])
@pytest.mark.parametrize("k,e", [(6, 3), (24, 20)])
def test_batch_beyond_grid_limit(ctx, orc, kernel, k, e):
    """70000 blocks in one call (more than the 65535 a grid dimension holds):
    encode, decode (erased rows poisoned) and verify run as consecutive
    slices (for (24, 20) generated, each grid slice is decoded in the four
    prepare + emission slices of the short-row path as well); every block is
    verified on the device and sampled blocks on either side of the slice
    boundary are compared with the oracle."""
    L, B = 64, 70000
    ctx.set_decode_kernel(kernel)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=11, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=11, ctx=ctx)
        src = enc.src.view(B, k, enc.pitch)
        keep = src[:, :, :L].clone()
        # poison every erased original of every block (vectorised)
        errs = torch.from_numpy(dec.err_host.astype(np.int64)).to(src.device)
        src.scatter_(1, errs[:, :, None].expand(B, e, enc.pitch), 0xA5)
        dec.decode_all(enc)
        torch.cuda.synchronize()
        src[:, :, :L] = keep
        assert dec.is_complete() and dec.verify_data(enc)
        out = dec.out.view(B, e, dec.pitch)
        for b in (0, 1, 65534, 65535, 65536, B - 1):
            data = [keep[b, j].cpu().numpy() for j in range(k)]
            par = enc.parity_rows(b)
            ref = orc.encode_block(data, e)
            assert all((par[i] == ref[i]).all() for i in range(e)), b
            rc, rec = orc.decode_block(data, list(par), dec.err_host[b])
            assert rc == 0
            got = out[b, :, :L].cpu().numpy()
            assert all((got[i] == rec[i]).all() for i in range(e)), b
    finally:
        ctx.set_decode_kernel("auto")


@pytest.mark.parametrize("blocks,name", [(1, "k_rs_syn_split(decode)"), (9, "k_rs_jit(decode)")])
def test_auto_decode_kernel_by_batch_work(ctx, blocks, name):
    """AUTO decodes a batch with fewer than 2048 (block, 2 KB tile) pairs and
    e <= 8 in ONE launch (k_rs_tc_fused: decode rows built in the kernel,
    threaded code; C2, one full-row block) and larger batches through
    generated code; both with the erased rows poisoned, recovered bytes
    intact."""
    k, e, L = 16, 4, 1000000
    ctx.set_decode_kernel("auto")
    enc = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=29, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=blocks, seed=29, ctx=ctx)
    ctx.timing_read()
    ctx.timing_enable(True)
    ok = decode_poisoned(ctx, enc, dec)
    names = [n for n, _, _ in ctx.timing_read()]
    ctx.timing_enable(False)
    assert ok
    assert name in names and names[-1] == name, names


@pytest.mark.parametrize("k,e,L,B,name", [(16, 8, 32000, 256, "k_rs_jit(decode)"),
                                          (128, 16, 32000, 256, "k_rs_jit(decode)"),
                                          (64, 32, 32000, 256, "k_rs_jit16(decode)"),
                                          (16, 8, 16000, 512, "k_rs_jit(decode)"),
                                          (16, 8, 8192, 1024, "k_rs_tc(decode)"),
                                          (128, 16, 16000, 512, "k_rs_tc(decode)")])
def test_auto_decode_short_rows_by_code_size(ctx, k, e, L, B, name):
    """Short rows (README.rst:130-133 sweeps symbol_size 32000: 16 column
    tiles per block): AUTO takes generated code from 16 tiles per block, and
    below that where a block's code is at most 2 KB per tile ((16, 8), 10 KB
    per block, at 8 tiles), threaded code above ((16, 8) at 4 tiles, (128,
    16)'s 162 KB at 8); erased rows poisoned."""
    ctx.set_decode_kernel("auto")
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=31, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=31, ctx=ctx)
    ctx.timing_read()
    ctx.timing_enable(True)
    ok = decode_poisoned(ctx, enc, dec)
    names = [n for n, _, _ in ctx.timing_read()]
    ctx.timing_enable(False)
    assert ok and dec.verify_data(enc)
    assert names[-1] == name, names


def test_generated_apply_checks_its_prepare(ctx):
    """The generated decode keeps ONE prepare's code per context: prepare(A),
    prepare(B), apply(A) must fail (RSGPU_ERR_ARG, nothing launched) instead
    of running B's code over A's rows; apply(B) then works, and A works again
    after its own prepare.  Both recoveries are checked with the erased rows
    poisoned."""
    k, e, L = 64, 32, 1 << 17
    ctx.set_decode_kernel("generated")
    try:
        encs = [rsgpu.GpuEncoder(k, L, e, blocks=B, seed=s, ctx=ctx) for B, s in ((3, 41), (2, 43))]
        decs = [rsgpu.GpuDecoder(k, L, e, blocks=B, seed=s, ctx=ctx) for B, s in ((3, 41), (2, 43))]
        for enc in encs:
            enc.encode_all()
        torch.cuda.synchronize()

        def prep(i):
            enc, dec = encs[i], decs[i]
            ctx.decode_prepare(k, e, L, enc.pitch, enc.B, enc.src, enc.par, dec.err, dec.out,
                               dec.ws, dec.status)

        def apply(i):
            enc, dec = encs[i], decs[i]
            ctx.decode_apply(k, e, L, enc.pitch, enc.B, enc.src, enc.par, dec.out, dec.ws,
                             dec.status)

        saved = [poison_rows(enc.src.view(enc.B, k, enc.pitch), dec.err_host, L)
                 for enc, dec in zip(encs, decs)]
        prep(0)
        prep(1)
        with pytest.raises(rsgpu.RsGpuError, match="another prepare"):
            apply(0)
        apply(1)
        prep(0)
        apply(0)
        torch.cuda.synchronize()
        for enc, dec, sv in zip(encs, decs, saved):
            out = dec.out.view(enc.B, e, enc.pitch)
            for b in range(enc.B):
                for i, j in enumerate(dec.err_host[b]):
                    assert torch.equal(out[b, i, :L], sv[(b, int(j))]), (enc.B, b, i)
    finally:
        ctx.set_decode_kernel("auto")


def test_bench_c4_two_ranks_ragged():
    """`bench.py --gpus 2 --config c4` (two ranks on device 0, gloo): 2501
    blocks do not divide by two -- rank 0 streams 1251 and rank 1 1250,
    both in ragged batches, every batch verified; the shares are contiguous
    and cover every block once."""
    line = run_bench(["--gpus", "2", "--same-device", "--dist-backend", "gloo", "--config", "c4",
                      "--blocks", "2501", "--batch", "512", "--warmup", "1", "--no-cpu-baseline"])
    assert line["n_gpus"] == 2 and line["verified"]
    assert line["streamed"]["mismatch_bytes"] == 0 and line["streamed"]["blocks_total"] == 2501
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [(r["block0"], r["blocks"], r["batches"]) for r in ranks] == [(0, 1251, 3), (1251, 1250, 3)]


def test_bench_c5_two_ranks():
    """`bench.py --gpus 2 --config c5` (the 8-GPU wide-stripe config, here
    two ranks on device 0 with 3 blocks each): disjoint shards, erasure lists
    by global block index, verified."""
    line = run_bench(["--gpus", "2", "--same-device", "--dist-backend", "gloo", "--config", "c5",
                      "--blocks", "3", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    assert line["n_gpus"] == 2 and line["verified"]
    assert line["config"]["symbols"] == 100 and line["config"]["erased"] == 20
    ranks = sorted(line["ranks"], key=lambda r: r["rank"])
    assert [(r["block0"], r["blocks"]) for r in ranks] == [(0, 3), (3, 3)]
    for r in ranks:
        err = rsgpu.erasure_patterns(1, r["block0"], r["blocks"], 100, 20)
        assert r["err_sha"] == hashlib.sha256(err.tobytes()).hexdigest()


def test_cpp_runner_threads_share_a_gpu(tmp_path):
    """rs_throughput --gpus 2 --same-device: two host threads, each owning
    its own rsgpu_ctx on device 0, run encode and decode at the same time
    (every timed region starts on a barrier) -- the thread-safety promise of
    include/rsgpu.h for distinct contexts.  Every decode is verified (a
    rejected measurement fails the run) and the job row counts both GPUs'
    bytes."""
    runner = os.path.join(BIN, "rs_throughput")
    csv_path = tmp_path / "mt.csv"
    r = subprocess.run([runner, "--gpus", "2", "--same-device", "--symbols", "64", "16",
                        "--symbol_size", "1000000", "--loss_rate", "0.5", "--blocks", "3", "--runs", "2",
                        "--csv_file", str(csv_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = csv_path.read_text().strip().splitlines()
    head = lines[0].split(",")
    assert head[-5:] == ["gpus", "resident", "run", "seconds", "goodput"]
    assert len(lines) == 1 + 2 * 2 * 2
    for ln in lines[1:]:
        f = dict(zip(head, ln.split(",")))
        assert f["gpus"] == "2" and f["resident"] == "device" and float(f["goodput"]) > 0


def test_cpp_runner_printers_agree(tmp_path):
    """gauge's three printers (README.rst:109-113) with the reference's own
    invocation syntax (README.rst:121: --symbols=100 --symbol_size=1000000
    --loss_rate=0.2 --python_file=... --csv_file=...): the Python file is a
    dictionary of columns (ast.literal_eval), and it, the JSON document and
    the CSV table hold the same rows."""
    import ast
    import csv
    import json as js
    runner = os.path.join(BIN, "rs_throughput")
    py, cs, jn = tmp_path / "r.py", tmp_path / "r.csv", tmp_path / "r.json"
    r = subprocess.run([runner, "--symbols=100", "--symbol_size=1000000", "--loss_rate=0.2", "--blocks=2",
                        "--runs=2", f"--python_file={py}", f"--csv_file={cs}", f"--json_file={jn}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    cols = ast.literal_eval(py.read_text())
    rows = list(csv.DictReader(open(cs)))
    docs = js.loads(jn.read_text())
    assert list(cols) == list(rows[0].keys()) == list(docs[0].keys())
    assert len(rows) == len(docs) == 2 * 2  # encoder + decoder, 2 runs
    for i, row in enumerate(rows):
        for c, v in row.items():
            if isinstance(cols[c][i], str):
                assert cols[c][i] == v == docs[i][c], (c, i)
            else:
                assert float(cols[c][i]) == float(v) == float(docs[i][c]), (c, i)
    assert set(cols["type"]) == {"encoder", "decoder"} and all(x == 100 for x in cols["symbols"])
    assert all(x == 20 for x in cols["erased_symbols"]) and all(g > 0 for g in cols["goodput"])


@pytest.mark.parametrize("extra", [[], ["--gpus", "2", "--same-device"]])
def test_cpp_runner_host_resident(extra):
    """rs_throughput --resident host: the blocks live in pinned host memory as
    the reference's do; encode_all / decode_all carry the copies (the
    library's chunked three-stream pipeline), the recovered rows are compared
    on the host.  Short rows (whole-block copies) and long rows (survivor
    runs), one and two threads."""
    runner = os.path.join(BIN, "rs_throughput")
    r = subprocess.run([runner, "--resident", "host", "--symbols", "64", "16", "--symbol_size", "1000000",
                        "32000", "--loss_rate", "0.5", "--blocks", "3"] + extra,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("resident=host") == 2 * 2 * 2, r.stdout


@pytest.mark.parametrize("k,e,L,B", [(64, 32, 1000000, 3), (16, 4, 1000000, 2), (64, 32, 32000, 100),
                                     (20, 7, 4096, 5), (10, 4, 1000, 3)])
def test_host_resident_api_poisoned(ctx, orc, k, e, L, B):
    """rsgpu_encode_blocks_host / rsgpu_decode_blocks_host on pinned host rows
    with a host pitch of exactly L (the reference's rows; device rows are
    re-pitched): parity equals the device path's, and the decode recovers the
    originals while every erased row in HOST memory holds 0xA5 (only
    survivors and parity may cross the link and be read).  A small block is
    compared with the oracle too."""
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=53, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=53, ctx=ctx)
    torch.cuda.synchronize()
    src_d = enc.src.view(B, k, enc.pitch)[:, :, :L]
    h_src = torch.empty((B, k, L), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(src_d)
    h_par = torch.empty((B, e, L), dtype=torch.uint8, pin_memory=True)
    ctx.encode_blocks_host(k, e, L, L, B, h_src, h_par)
    par_d = enc.par.view(B, e, enc.pitch)[:, :, :L].cpu()
    assert torch.equal(h_par, par_d)
    keep = h_src.clone()
    for b in range(B):
        for j in dec.err_host[b]:
            h_src[b, int(j)] = 0xA5
    h_out = torch.empty((B, e, L), dtype=torch.uint8, pin_memory=True)
    h_st = np.full(B, -7, np.int32)
    err = np.ascontiguousarray(dec.err_host)
    ctx.decode_blocks_host(k, e, L, L, B, h_src, h_par, err, h_out, h_st)
    assert (h_st == 0).all()
    for b in range(B):
        for i, j in enumerate(dec.err_host[b]):
            assert torch.equal(h_out[b, i], keep[b, int(j)]), (b, i)
    data = [keep[0, j].numpy() for j in range(k)]
    rc, rec = orc.decode_block(data, [h_par[0, i].numpy() for i in range(e)], dec.err_host[0])
    assert rc == 0 and all((h_out[0, i].numpy() == rec[i]).all() for i in range(e))


SPLIT_CODES = {(16, 4), (16, 8), (5, 4), (20, 7)}  # rs_bitsliced_split_available


@pytest.mark.parametrize("kernel", ["auto", "one_matrix"])
@pytest.mark.parametrize("k,e,L,B", [(16, 4, 1000000, 1), (16, 8, 64000, 3), (64, 8, 100000, 2), (3, 1, 4096, 4),
                                     (5, 4, 2080, 7), (40, 7, 6144, 5), (8, 8, 2048, 1), (2, 2, 2048, 3),
                                     (64, 1, 32768, 2), (33, 5, 4096, 3), (20, 7, 4096, 3), (16, 4, 96, 2),
                                     (16, 8, 1000000, 1)])
def test_fused_small_decode(ctx, orc, kernel, k, e, L, B):
    """The one-launch small-batch decodes: for the codes with a compiled
    single-chunk program, AUTO runs k_rs_syn_split (syndromes through the
    encode's compile-time programs, erased sources skipped, then the e x e
    solve with runtime coefficients); every other code, and ONE_MATRIX, runs
    k_rs_tc_fused (decode rows in closed form inside the kernel, threaded
    code).  Sources split over four waves, partials reduced in LDS; erased
    rows poisoned; ragged tiles (L % 2048), k below the wave count, e == k;
    block 0 also against the oracle, and a malformed list in the last block
    fails that block only (status -2)."""
    ctx.set_decode_kernel(kernel)
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=61, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=61, ctx=ctx)
    ctx.timing_read()
    ctx.timing_enable(True)
    try:
        ok = decode_poisoned(ctx, enc, dec)
        names = [n for n, _, _ in ctx.timing_read()]
    finally:
        ctx.timing_enable(False)
    want = ("k_rs_syn_split(decode)" if kernel == "auto" and (k, e) in SPLIT_CODES
            else "k_rs_tc_fused(decode)")
    assert ok and names == [want], names
    data = [enc.src.view(B, k, enc.pitch)[0, j, :L].cpu().numpy() for j in range(k)]
    rc, rec = orc.decode_block(data, list(enc.parity_rows(0)), dec.err_host[0])
    got = dec.recovered_rows(0)
    assert rc == 0 and all((got[i] == rec[i]).all() for i in range(e))
    if B > 1 and e > 1:
        bad = dec.err_host.copy()
        bad[B - 1, :2] = bad[B - 1, 1::-1]  # not ascending
        dec.err.copy_(torch.from_numpy(bad).view(dec.err.shape))
        dec.decode_all(enc)
        torch.cuda.synchronize()
        st = dec.status.cpu().numpy()
        assert st[B - 1] == -2 and (st[:B - 1] == 0).all(), st
    ctx.set_decode_kernel("auto")


@pytest.mark.parametrize("off", [1, 2, 3])
@pytest.mark.parametrize("k,e", [(16, 4), (20, 7), (5, 4), (16, 8)])
def test_small_decode_unaligned_erasure_list(ctx, off, k, e):
    """k_rs_syn_split reads a block's list through the scalar cache by the
    aligned words that hold it: lists at any byte offset (a slice of a larger
    batch starts at d_err + b0 * e) decode the same, erased rows poisoned."""
    L, B = 4096, 3
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=89, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=89, ctx=ctx)
    buf = torch.zeros(B * e + 8, dtype=torch.uint8, device="cuda")
    view = buf[off:off + B * e]
    view.copy_(dec.err.view(-1))
    dec.err = view
    ctx.timing_read()
    ctx.timing_enable(True)
    try:
        assert decode_poisoned(ctx, enc, dec)
        names = [n for n, _, _ in ctx.timing_read()]
    finally:
        ctx.timing_enable(False)
    assert names == ["k_rs_syn_split(decode)"], names


@pytest.mark.parametrize("tpw", [2, 3])
@pytest.mark.parametrize("k,e,L,B", [(64, 32, 1000000, 2), (64, 32, 32000, 9), (100, 20, 6144, 3),
                                     (48, 24, 14336, 2)])
def test_jitw_tiles_per_workgroup(ctx, tpw, k, e, L, B):
    """k_rs_jitw with 2 or 3 column tiles per workgroup (the A/B hook
    rsgpu_internal_set_jitw_tiles): the same recovered bytes with the erased
    rows poisoned, including tile counts that do not divide by the group
    (489, 16, 3, 7 tiles per block)."""
    import ctypes
    f = rsgpu.testhooks().rsgpu_internal_set_jitw_tiles
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx.set_decode_kernel("generated")
    assert f(ctx._h, tpw) == 0
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=71, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=71, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
    finally:
        f(ctx._h, 0)
        ctx.set_decode_kernel("auto")


@pytest.mark.gpu
@pytest.mark.parametrize("k,e,L,B", [(64, 32, 1000000, 2), (64, 32, 32000, 9), (100, 20, 6144, 3),
                                     (48, 24, 14336, 2), (64, 17, 2048, 5)])
def test_jitw_code_prefetch(ctx, k, e, L, B):
    """k_rs_jitw with its workgroups pulling the block's code into L2 first
    (the A/B hook rsgpu_internal_set_jitw_prefetch): the same recovered bytes
    with the erased rows poisoned, for block-code sizes that leave some
    workgroups no line to fetch (one tile per block)."""
    import ctypes
    f = rsgpu.testhooks().rsgpu_internal_set_jitw_prefetch
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx.set_decode_kernel("generated")
    assert f(ctx._h, 1) == 0
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=73, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=73, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
    finally:
        f(ctx._h, -1)
        ctx.set_decode_kernel("auto")


@pytest.mark.gpu
@pytest.mark.parametrize("prio", [0, 2])
@pytest.mark.parametrize("k,e,L,B,enc_kernel", [(64, 32, 65536, 3, "compiled"), (64, 32, 32000, 9, "compiled"),
                                                (100, 20, 6144, 3, "generated"), (32, 8, 65536, 3, "generated"),
                                                (16, 4, 65536, 3, "compiled"), (64, 16, 32768, 2, "compiled")])
def test_wave_priority_either_way(ctx, orc, prio, k, e, L, B, enc_kernel):
    """The wave priority over the transposes (round 6; k_rs_bs has a second
    instantiation without it, the generated-code kernels a runtime flag) only
    reorders issue: with it on (2, the default) and off (0) the parity is the
    oracle's and the recovered bytes are the originals, erased rows
    poisoned -- compiled and generated encodes, the 16-, 10- and 8-row
    decodes, long and short rows."""
    import ctypes
    h = rsgpu.testhooks()
    f_bs, f_jw = h.rsgpu_internal_set_bs_prio, h.rsgpu_internal_set_jitw_prio
    for f in (f_bs, f_jw):
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        assert f(ctx._h, prio) == 0
    ctx.set_encode_kernel(enc_kernel)
    ctx.set_decode_kernel("generated")
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=91, ctx=ctx)
        enc.encode_all()
        torch.cuda.synchronize()
        g = orc.init_tables(k, e, orc.gen_rs_matrix(k + e, k)[k:])
        for b in (0, B - 1):
            data = list(enc.source_rows(b))
            ref = [np.zeros(L, np.uint8) for _ in range(e)]
            orc.encode_data(L, k, e, g, data, ref)
            got = enc.par.view(B, e, enc.pitch)[b, :, :L].cpu().numpy()
            assert all((got[r] == ref[r]).all() for r in range(e)), (b, prio)
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=91, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
    finally:
        f_bs(ctx._h, 2)
        f_jw(ctx._h, 2)
        ctx.set_encode_kernel("auto")
        ctx.set_decode_kernel("auto")


def set_pipeline(ctx, n):
    import ctypes
    f = rsgpu.testhooks().rsgpu_internal_set_decode_pipeline
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert f(ctx._h, n) == 0


@pytest.mark.parametrize("parts", [2, 3, 4])
@pytest.mark.parametrize("k,e,L,B", [(64, 32, 32000, 9), (100, 20, 6144, 5), (48, 24, 14336, 4),
                                     (100, 50, 32000, 6), (150, 100, 6144, 6), (64, 32, 1000000, 4)])
def test_pipelined_decode_slices(ctx, parts, k, e, L, B):
    """rsgpu_decode_blocks' short-row path (the A/B hook
    rsgpu_internal_set_decode_pipeline): prepare + emission of each slice of
    blocks on a second stream beside the decode of the slice before; the same
    recovered bytes with the erased rows poisoned (odd block counts, slices of
    unequal size, passes above 64 rows), one decode launch per slice and
    pass, and a malformed list in the last slice fails that block only."""
    ctx.set_decode_kernel("generated")
    set_pipeline(ctx, parts)
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=79, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=79, ctx=ctx)
        ctx.timing_read()
        ctx.timing_enable(True)
        try:
            assert decode_poisoned(ctx, enc, dec)
            recs = ctx.timing_read()
        finally:
            ctx.timing_enable(False)
        n = min(parts, B // 2)  # at most one slice per two blocks
        per = ((B + n - 1) // n + 1) // 2 * 2
        slices = (B + per - 1) // per
        passes = 2 if e > 64 else 1
        dec_recs = [r for r in recs if "(decode)" in r[0]]
        assert len(dec_recs) == slices * passes, recs
        assert sum(r[2] for r in dec_recs) == B * passes
        assert sum(r[2] for r in recs if r[0] == "k_decode_prepare_syn") == B
        bad = dec.err_host.copy()
        bad[B - 1, :2] = bad[B - 1, 1::-1]  # not ascending
        dec.err.copy_(torch.from_numpy(bad).view(dec.err.shape))
        dec.decode_all(enc)
        torch.cuda.synchronize()
        st = dec.status.cpu().numpy()
        assert st[B - 1] == -2 and (st[:B - 1] == 0).all(), st
    finally:
        set_pipeline(ctx, -1)
        ctx.set_decode_kernel("auto")


def test_pipelined_decode_by_default_at_c4_shape(ctx):
    """AUTO at C4's shape (64, 32, 32000) from 2048 blocks: four slices, every
    erased original of every block overwritten before the decode (vectorised
    poison), all recovered; then a plain prepare + apply over the same
    workspace agrees (the code and key left behind are the batch's)."""
    k, e, L, B = 64, 32, 32000, 2048
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=83, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=83, ctx=ctx)
    src = enc.src.view(B, k, enc.pitch)
    bi = torch.arange(B, device="cuda").repeat_interleave(e)
    ji = torch.from_numpy(dec.err_host.astype(np.int64).reshape(-1)).cuda()
    saved = src[bi, ji, :L].clone()
    src[bi, ji, :L] = 0xA5
    ctx.timing_read()
    ctx.timing_enable(True)
    try:
        dec.decode_all(enc)
        torch.cuda.synchronize()
        recs = ctx.timing_read()
    finally:
        ctx.timing_enable(False)
    assert [r[2] for r in recs if r[0] == "k_rs_jit16(decode)"] == [512] * 4, recs
    out = dec.out.view(B, e, dec.pitch)[:, :, :L].reshape(-1, L)
    assert dec.is_complete() and torch.equal(out, saved)
    dec.out.fill_(0)
    ctx.decode_apply(k, e, L, dec.pitch, B, enc.src, enc.par, dec.out, dec.ws, dec.status)
    torch.cuda.synchronize()
    assert torch.equal(dec.out.view(B, e, dec.pitch)[:, :, :L].reshape(-1, L), saved)
    src[bi, ji, :L] = saved


@pytest.mark.parametrize("k,e", [(64, 32), (25, 25), (218, 32), (48, 24), (21, 21), (100, 20), (17, 17),
                                 (230, 20), (100, 50), (128, 64), (70, 45), (40, 33),
                                 (150, 100), (125, 125), (160, 65)])
def test_device_emitter_writes_the_host_emitters_code(ctx, k, e):
    """k_jitw_emit (table-driven, on the device) writes, block for block and
    word for word, the code of the host emitter Wide::code_word, which the
    CPU suite disassembles and interprets (tests/test_jit.py)."""
    import ctypes as C
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_jit import emitw
    rng = np.random.default_rng(k * 1000 + e)
    blocks = 3
    coef = rng.integers(0, 256, (blocks, e, k), dtype=np.uint8)
    coef[0, 1, :5] = 0          # zero coefficients: s_nop pairs
    coef[1, 0, :] = 1
    coef[2, :, 0] = 0x80
    f = rsgpu.testhooks().rsgpu_internal_jitw_emit_device
    f.restype = C.c_longlong
    f.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t]
    need = f(ctx._h, k, e, blocks, coef.ctypes.data, None, 0)
    assert need > 0
    out = np.zeros(need, np.uint8)
    assert f(ctx._h, k, e, blocks, coef.ctypes.data, out.ctypes.data, need) == need
    per = need // blocks
    for b in range(blocks):
        host = emitw(k, e, coef[b])
        assert host.size == per
        assert np.array_equal(out[b * per:(b + 1) * per], host), b


@pytest.mark.parametrize("k,e,L", [(150, 100, 1000000), (125, 125, 1000000), (186, 64, 1000000),
                                   (160, 65, 65536)])
def test_wide_rows_decode_in_at_most_two_launches(ctx, k, e, L):
    """e > 64 (isa.cpp:25-27 allows k + e <= 250): the decode rows come in
    closed form (no k x k inversion) and the generated code runs in passes of
    <= 64 rows, four waves per tile, each source read and transposed once per
    pass: at most two decode launches; the erased rows are poisoned."""
    B = 2
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=5, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=5, ctx=ctx)
    torch.cuda.synchronize()
    ctx.timing_read()
    ctx.timing_enable(True)
    try:
        assert decode_poisoned(ctx, enc, dec)
        names = [r[0] for r in ctx.timing_read()]
    finally:
        ctx.timing_enable(False)
    assert "k_decode_prepare" not in names, names
    assert "k_decode_prepare_syn" in names
    apply = [n for n in names if n.startswith("k_rs_jit")]
    assert 1 <= len(apply) <= 2, names
    assert all(n == ("k_rs_jitw_passes(decode)" if e > 64 else "k_rs_jit16x4(decode)") for n in apply), names


@pytest.mark.gpu
@pytest.mark.parametrize("prefetch", [-1, 1])
@pytest.mark.parametrize("period", [600, 1, 37, 0])
@pytest.mark.parametrize("k,e,L,B", [(64, 32, 1000000, 2), (64, 32, 32000, 9), (100, 20, 6144, 3),
                                     (64, 40, 65536, 3), (150, 100, 16384, 2), (18, 17, 4096, 3)])
def test_jitw_chunk_rotation(ctx, period, prefetch, k, e, L, B):
    """k_rs_jitw's chunk order rotated by the workgroup's start time, for
    periods that put neighbouring workgroups in different phases (1 tick) and
    for none (0):
    every chunk applied exactly once, so the same recovered bytes with the
    erased rows poisoned -- two- and four-wave layouts, passes above 64 rows,
    and a four-chunk block whose last chunk is partial (k 18, CS 5: 5 + 5 +
    5 + 3).  Both users of the kernel rotate: the per-block decode and the
    GENERATED encode's shared program (its parity feeds the decode, so a
    wrong parity shows as wrong recovered bytes).  prefetch 1 turns the
    short-row code prefetch on beside the rotation (the rotation's broadcast
    word lives in chunk buffer 1, which no LDS-DMA may write before the first
    chunk barrier)."""
    import ctypes
    f_rot = rsgpu.testhooks().rsgpu_internal_set_jitw_rot
    f_rot.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f_pf = rsgpu.testhooks().rsgpu_internal_set_jitw_prefetch
    f_pf.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx.set_decode_kernel("generated")
    ctx.set_encode_kernel("generated")
    assert f_rot(ctx._h, period) == 0
    assert f_pf(ctx._h, prefetch) == 0
    try:
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=79, ctx=ctx)
        enc.encode_all()
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=79, ctx=ctx)
        assert decode_poisoned(ctx, enc, dec)
    finally:
        f_rot(ctx._h, -1)
        f_pf(ctx._h, -1)
        ctx.set_encode_kernel("auto")
        ctx.set_decode_kernel("auto")
