#!/usr/bin/env python3
"""bench.py -- device-resident encode+decode goodput of the MI355X RS engine.

Metric (BASELINE.json): "encode+decode goodput GiB/s (device-resident) at
symbols x symbol_size; %HBM roofline".  Workload at N=1: BASELINE.json
configs[2] -- symbols=64, symbol_size=1000000, loss_rate=0.5 (32 erased /
32 parity symbols), 1024 blocks batched on one MI355X.

One step = the timed regions of benchmark/isa_throughput over the whole batch:
  encode_all  -- parity of every block (isa.cpp:69-79), and
  decode_all  -- decode matrix + inversion + reconstruction of the erased
                 originals of every block (isa.cpp:169-213),
with sources, parity and outputs resident in HBM when the timed region starts.
Goodput = (parity bytes + recovered bytes) / time, as the reference's
measurement() counts output bytes (throughput_benchmark.hpp:37-67).

--config c4 streams 2^20 blocks of (64, 32, 32000) (BASELINE.json configs[3])
through two resident batches: sources of batch i+1 are generated on the
device while batch i is encoded and decoded, every batch is verified.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
each process is one rank; `python bench.py --gpus N` without a launcher
spawns the N rank processes itself (the parent never touches the GPU).  Each
rank owns its own shard of blocks (weak scaling, no collective on the data
path); torch.distributed only carries the barrier and the
max-over-ranks time, over gloo by default (host TCP, initialised before the
GPU is touched; RCCL only with --dist-backend nccl).  A rank that fails
leaves its error in the process group's store, and rank 0 prints one JSON
line naming every failed rank.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
import os
import shutil
import signal
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))

CONFIGS = {
    # name: (symbols, symbol_size, loss_rate, blocks per GPU)
    "c1": (16, 64000, 0.5, 1),          # the reference's CPU plumbing case: host only, no GPU
    "c2": (16, 1000000, 0.25, 1),
    "c3": (64, 1000000, 0.5, 1024),
    "c4": (64, 32000, 0.5, 1 << 20),    # 2^20 blocks in total, streamed, split over the GPUs
    "c5": (100, 1000000, 0.2, 512),     # 4096 blocks over 8 GPUs = 512 per GPU
}
C4_BATCH = 16384                        # resident blocks per streamed batch (x2 buffers)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table, spec


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--blocks", type=int, default=None,
                   help="blocks per GPU (c4: blocks in total) override")
    p.add_argument("--batch", type=int, default=C4_BATCH, help="c4: resident blocks per batch")
    p.add_argument("--symbols", type=int, default=None, help="override the config's symbols (k)")
    p.add_argument("--symbol-size", type=int, default=None, help="override the config's symbol_size (L)")
    p.add_argument("--loss-rate", type=float, default=None, help="override the config's loss_rate")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--decode-kernel", default="auto",
                   choices=["auto", "generated", "one_matrix", "general"])
    p.add_argument("--encode-kernel", default="auto",
                   choices=["auto", "compiled", "generated", "threaded"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--c1-seconds", type=float, default=4.0,
                   help="c1: timed CPU seconds per leg (the sample size is calibrated to it)")
    p.add_argument("--cpu-threads", type=int, default=None)
    p.add_argument("--no-ref-base", action="store_true",
                   help="skip the (slow, ~10 s) reference scalar-C CPU sample")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--host-io", type=int, default=0, metavar="BLOCKS",
                   help="also time the host-resident path (H2D + kernel + D2H) on BLOCKS blocks")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06_head", "traffic.json"),
                   help="JSON with PMC-derived HBM bytes per launch of the same workload "
                        "(tools/profile_round.sh)")
    p.add_argument("--sq-counters", default=os.path.join(ROOT, "profiles", "r06_head", "sq_summary.txt"),
                   help="SQ counter summary of the same workload (tools/pmc_sq.sh + "
                        "tools/pmc_summary.py): VALU-issue roofline of each kernel")
    p.add_argument("--valu-ceiling", default=os.path.join(ROOT, "profiles", "r03_valu_ceiling.json"),
                   help="measured VALU issue ceiling (tools/ubench_issue + tools/valu_ceiling.py)")
    # testing the N-rank path on a one-GPU box: every rank on device 0
    p.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    # the collectives (barrier, max time, shard info, verification) lie
    # outside the timed data path: gloo over host TCP by default, so the
    # 8-rank start-up never depends on a multi-rank RCCL init
    p.add_argument("--dist-backend", default="gloo", choices=["gloo", "nccl"])
    p.add_argument("--dist-timeout", type=float, default=900.0,
                   help="seconds a collective waits for the other ranks")
    # tests only: this rank fails right after the process group is up, the
    # others wait in a barrier (the failure path of a multi-rank run)
    p.add_argument("--fail-rank", type=int, default=None, help=argparse.SUPPRESS)
    return p.parse_args(argv)


def shard(rank: int, blocks_per_rank: int):
    """Blocks owned by `rank`: [rank*B, (rank+1)*B) -- independent blocks, no
    exchange between ranks; weak scaling."""
    return rank * blocks_per_rank, blocks_per_rank


def split(total: int, rank: int, world: int):
    """A total of `total` blocks over `world` ranks (C4's 2^20): contiguous
    shares, the first total % world ranks one block more, so every block is
    owned by exactly one rank.  Returns (first block, blocks) of `rank`."""
    base, rem = divmod(total, world)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)


def reduce_max_time(elapsed: float, world: int, device) -> float:
    """Max over ranks of the timed region (the slowest rank bounds the job)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_goodput(out_bytes_per_rank_step: float, steps: int, world: int, elapsed: float) -> float:
    """Whole-job goodput in GiB/s: all ranks' output bytes / max-rank time."""
    return out_bytes_per_rank_step * steps * world / elapsed / 2 ** 30


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv, grace: float = 60.0) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (this parent has not touched the GPU), wait for all, return the
    worst exit status.  After a rank fails the others get `grace` seconds to
    notice (rank 0 then prints the line naming it) before they are stopped."""
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    alive = list(procs)
    stop_at = None
    while alive:
        for p in list(alive):
            r = p.poll()
            if r is None:
                continue
            alive.remove(p)
            rc = max(rc, abs(r))
            if r != 0 and stop_at is None:
                stop_at = time.time() + grace
        if stop_at is not None and time.time() >= stop_at:
            for q in alive:
                q.terminate()
            stop_at = float("inf")
        time.sleep(0.05)
    return rc


def survivor_runs(err, k, pitch, chunk):
    """Byte ranges (offset, length) of the surviving source rows of every
    block in a [blocks][k][pitch] row array, merged into runs of consecutive
    rows and grouped by chunk of `chunk` blocks.  err: [blocks][e] erased
    source indices (isa_decoder's erasure list)."""
    import numpy as np
    blocks = len(err)
    runs = [[] for _ in range((blocks + chunk - 1) // chunk)]
    for blk in range(blocks):
        live = np.ones(k, bool)
        live[np.asarray(err[blk], dtype=np.int64)] = False
        j = 0
        while j < k:
            if live[j]:
                j0 = j
                while j < k and live[j]:
                    j += 1
                runs[blk // chunk].append(((blk * k + j0) * pitch, (j - j0) * pitch))
            else:
                j += 1
    return runs


def poison_erased(enc, dec):
    """Overwrite every erased source row on the device with 0xA5: the
    decode must not read them (isa.cpp:193-197 builds data[] from the
    survivors only).  The host copy restores them for verify_data."""
    src = enc.src.view(enc.B, enc.k, enc.pitch)
    for b in range(enc.B):
        for j in dec.err_host[b]:
            src[b, int(j), :enc.L] = 0xA5


def host_io_rate(rsgpu, ctx, k, e, L, blocks, seed, reps=3):
    """Goodput when the blocks start and end in (pinned) host memory, as the
    reference's buffers do, with the stages in series: encode = H2D(sources)
    + encode + D2H(parity); decode = H2D(surviving sources + parity) +
    decode + D2H(recovered).  The decoder side ships what isa_decoder reads
    (the same bytes as host_io_pipelined; the erased rows stay poisoned on
    the device).  GiB/s of output bytes over the summed wall time (median of
    reps)."""
    import torch
    enc = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    h_src = torch.empty(enc.src.numel(), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty(enc.par.numel(), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(dec.out.numel(), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(enc.src)
    h_par.copy_(enc.par)
    runs = survivor_runs(dec.err_host, k, enc.pitch, blocks)[0]
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc.src.copy_(h_src, non_blocking=True)
        enc.encode_all()
        h_par.copy_(enc.par, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        poison_erased(enc, dec)  # untimed: what the decoder may not read
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for off, n in runs:
            enc.src[off:off + n].copy_(h_src[off:off + n], non_blocking=True)
        enc.par.copy_(h_par, non_blocking=True)
        dec.decode_all(enc)
        h_out.copy_(dec.out, non_blocking=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        times.append((t1 - t0, t3 - t2))
    times.sort(key=lambda x: x[0] + x[1])
    te, td = times[len(times) // 2]
    enc.src.copy_(h_src)  # the originals back for verify_data
    ok = dec.is_complete() and dec.verify_data(enc)
    out_b = e * L * blocks
    return {"blocks": blocks, "encode_s": te, "decode_s": td,
            "goodput_GiBps": 2 * out_b / (te + td) / 2 ** 30,
            "encode_GiBps": out_b / te / 2 ** 30, "decode_GiBps": out_b / td / 2 ** 30,
            "verified": ok, "poisoned": True}


def host_io_pipelined(rsgpu, ctx, k, e, L, blocks, seed, reps=3):
    """The host_io_rate workload through the library's host-resident calls
    (rsgpu_encode_blocks_host / rsgpu_decode_blocks_host, the gpu_plugin's
    --resident host path): blocks in pinned host memory at the reference's
    pitch of exactly L bytes, streamed through device staging in chunks with
    copy-in, kernel and copy-out of consecutive chunks overlapped on three
    streams (both link directions at once).  The decoder ships only what
    isa_decoder reads (survivor runs + parity); the erased rows hold 0xA5 in
    host memory during the decode.  Median of reps."""
    import numpy as np
    import torch
    enc = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    h_src = torch.empty((blocks, k, L), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty((blocks, e, L), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty((blocks, e, L), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(enc.src.view(blocks, k, enc.pitch)[:, :, :L])
    keep = h_src.clone()
    err = np.ascontiguousarray(dec.err_host)
    st = np.full(blocks, -1, np.int32)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        h_src.copy_(keep)
        t0 = time.perf_counter()
        ctx.encode_blocks_host(k, e, L, L, blocks, h_src, h_par)
        t1 = time.perf_counter()
        for b in range(blocks):  # untimed: what the decoder may not read
            h_src[b, torch.from_numpy(err[b].astype(np.int64))] = 0xA5
        t2 = time.perf_counter()
        ctx.decode_blocks_host(k, e, L, L, blocks, h_src, h_par, err, h_out, st)
        t3 = time.perf_counter()
        times.append((t1 - t0, t3 - t2))
    times.sort(key=lambda x: x[0] + x[1])
    te, td = times[len(times) // 2]
    ok = bool((st == 0).all())
    for b in range(blocks):
        idx = torch.from_numpy(err[b].astype(np.int64))
        ok = ok and bool(torch.equal(h_out[b], keep[b, idx]))
    # the parity that came back is the device path's
    enc.encode_all()
    torch.cuda.synchronize()
    ok = ok and bool(torch.equal(h_par, enc.par.view(blocks, e, enc.pitch)[:, :, :L].cpu()))
    out_b = e * L * blocks
    return {"blocks": blocks, "path": "rsgpu_encode_blocks_host / rsgpu_decode_blocks_host",
            "encode_s": te, "decode_s": td,
            "goodput_GiBps": 2 * out_b / (te + td) / 2 ** 30,
            "encode_GiBps": out_b / te / 2 ** 30, "decode_GiBps": out_b / td / 2 ** 30,
            "verified": ok, "poisoned": True}


def host_io_session(rsgpu, ctx, k, e, L, blocks, seed, chunk=4, reps=3):
    """Goodput when the data block starts and ends in host memory and crosses
    the link once each way: per chunk of blocks, H2D of the k source rows,
    encode and decode on the device (the decoder reads the encoder's
    device copy of the survivors, as isa_decoder reads the encoder's buffers,
    isa.cpp:88, :193-197), D2H of the parity and of the recovered rows.
    Three streams (copy-in, kernels, copy-out) over three device slots, so
    both link directions and the kernels of consecutive chunks overlap.  Rows
    at a pitch of exactly L.  The erased originals of each chunk are
    overwritten with 0xA5 on the device between its encode and its decode
    (timed; ~0.5 % of a chunk's time), so a decode that read them would fail
    the verification.  Median of reps; bytes and verification below."""
    import numpy as np
    import torch
    dev = torch.device("cuda", ctx.device)
    pitch = L
    h_src = torch.empty((blocks, k, L), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty((blocks, e, L), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty((blocks, e, L), dtype=torch.uint8, pin_memory=True)
    probe = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    h_src.copy_(probe.src.view(blocks, k, probe.pitch)[:, :, :L])
    probe.encode_all()
    want_par = probe.par.view(blocks, e, probe.pitch)[:, :, :L].cpu()
    del probe
    err_host = rsgpu.erasure_patterns(seed, 0, blocks, k, e)
    d_err = torch.from_numpy(np.ascontiguousarray(err_host)).to(dev)
    # per chunk, the slot rows of its erased originals (poisoned between the
    # encode and the decode, as host_io_rate / host_io_pipelined do)
    erased_rows = []
    for i in range((blocks + chunk - 1) // chunk):
        b0, nb = i * chunk, min(chunk, blocks - i * chunk)
        rows = np.arange(nb)[:, None] * k + err_host[b0:b0 + nb].astype(np.int64)
        erased_rows.append(torch.from_numpy(rows.reshape(-1)).to(dev))
    ws_b = rsgpu.decode_workspace_bytes(k, e, chunk)
    slots = []
    for _ in range(3):
        slots.append({"src": torch.empty(chunk * k * pitch, dtype=torch.uint8, device=dev),
                      "par": torch.empty(chunk * e * pitch, dtype=torch.uint8, device=dev),
                      "out": torch.empty(chunk * e * pitch, dtype=torch.uint8, device=dev),
                      "ws": torch.empty(ws_b, dtype=torch.uint8, device=dev),
                      "st": torch.full((chunk,), -1, dtype=torch.int32, device=dev)})
    s_in, s_cmp, s_out = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    nch = (blocks + chunk - 1) // chunk
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    times = []
    torch.cuda.synchronize()
    ctx.set_stream(s_cmp.cuda_stream)
    try:
        for _ in range(reps):
            ev_in = [torch.cuda.Event() for _ in range(nch)]
            ev_cmp = [torch.cuda.Event() for _ in range(nch)]
            ev_free = [torch.cuda.Event() for _ in range(nch)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(nch):
                b0, nb = i * chunk, min(chunk, blocks - i * chunk)
                sl = slots[i % 3]
                with torch.cuda.stream(s_in):
                    if i >= 3:
                        s_in.wait_event(ev_free[i - 3])
                    sl["src"][:nb * k * L].copy_(h_src[b0:b0 + nb].view(-1), non_blocking=True)
                    ev_in[i].record(s_in)
                s_cmp.wait_event(ev_in[i])
                ctx.encode_blocks(k, e, L, pitch, nb, sl["src"], sl["par"])
                with torch.cuda.stream(s_cmp):  # what the decoder may not read
                    sl["src"][:nb * k * pitch].view(nb * k, pitch).index_fill_(0, erased_rows[i], 0xA5)
                ctx.decode_blocks(k, e, L, pitch, nb, sl["src"], sl["par"], d_err[b0:b0 + nb],
                                  sl["out"], sl["ws"], sl["st"])
                with torch.cuda.stream(s_cmp):
                    bad.add_((sl["st"][:nb] != 0).sum())
                    ev_cmp[i].record(s_cmp)
                with torch.cuda.stream(s_out):
                    s_out.wait_event(ev_cmp[i])
                    h_par[b0:b0 + nb].view(-1).copy_(sl["par"][:nb * e * L], non_blocking=True)
                    h_out[b0:b0 + nb].view(-1).copy_(sl["out"][:nb * e * L], non_blocking=True)
                    ev_free[i].record(s_out)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
    finally:
        ctx.set_torch_stream()
    t = sorted(times)[len(times) // 2]
    ok = int(bad.item()) == 0 and bool(torch.equal(h_par, want_par))
    for b in range(blocks):
        ok = ok and bool(torch.equal(h_out[b], h_src[b, torch.from_numpy(err_host[b].astype(np.int64))]))
    out_b = e * L * blocks
    return {"blocks": blocks, "chunk_blocks": chunk, "wall_s": t,
            "goodput_GiBps": 2 * out_b / t / 2 ** 30,
            "link_bytes": {"h2d": k * L * blocks, "d2h": 2 * e * L * blocks},
            "verified": ok, "poisoned": True}


def host_cpus():
    """CPUs this process may actually use on the box: the affinity mask,
    capped by a cgroup v2 CPU quota when one is set."""
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = allowed if quota is None else max(1, min(allowed, int(quota)))
    return {"nproc_machine": os.cpu_count(), "cpus_allowed": allowed, "cpu_quota": quota,
            "usable": usable}


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(k, e, L, threads, kernel=1, blocks_per_thread=None, one_thread_blocks=2):
    """CPU baseline on the GPU box's host cores, isa.cpp's timed regions
    (encode = matrix + tables + data kernel; decode = k x k inversion + tables
    + data kernel) over a bounded sample.  Matrices, tables and inversion are
    the reference's ISA-L 2.13 C compiled from /root/reference (oracle/_ref).
    The data kernel is
      kernel 1: our AVX2 restatement of ISA-L's asm path (oracle/
                isal_avx2_port.c; the yasm sources cannot be assembled in this
                image) -> kind "port";
      kernel 0: the reference's scalar ec_encode_data_base -> kind "reference".
    Two samples: 1 thread (the reference's single-threaded semantics,
    isa.cpp:69-79, 169-213) and `threads` threads on independent blocks
    (aggregate); `value` is the latter.
    """
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    if not oracle_lib.have_reference():
        return None
    ref = oracle_lib.Reference()
    if kernel == 1 and not ref.have_avx2:
        return {"error": "host CPU has no AVX2"}
    bpt = blocks_per_thread or (4 if kernel == 1 else 1)

    def sample(nt, nb):
        r = ref.cpu_bench(k, e, L, nt, nb, 7, kernel)
        t = r["max_thread_s"]
        return {"threads": nt, "blocks_per_thread": nb,
                "value": 2.0 * e * L * nt * nb / t / 2 ** 30,
                "encode_s_per_block": r["enc_s"] / (nt * nb),
                "decode_s_per_block": r["dec_s"] / (nt * nb),
                "max_thread_s": t, "failures": r["failures"]}

    one = sample(1, one_thread_blocks if kernel == 1 else 1)
    many = sample(threads, bpt)
    what = ("AVX2 restatement of ISA-L 2.13 gf_vect_dot_prod_avx2/ec_encode_data_avx2"
            if kernel == 1 else "ISA-L 2.13 ec_encode_data_base (reference scalar C)")
    return {"value": many["value"], "unit": "GiB/s", "cores": threads,
            "kind": "port" if kernel == 1 else "reference",
            "sample": f"{threads} threads x {bpt} block(s) (k={k}, e={e}, L={L}) encode+decode, "
                      f"{what}, reference matrices/inversion; {many['max_thread_s']:.1f} s per "
                      f"thread, failures={many['failures']}",
            "encode_s_per_block": many["encode_s_per_block"],
            "decode_s_per_block": many["decode_s_per_block"],
            "threads_1": one, "threads_nproc": many}


def c1_line(args) -> dict:
    """BASELINE.json configs[0]: benchmark/isa_throughput on the CPU at
    --symbols=16 --symbol_size=64000 --loss_rate=0.5, plumbing only: the
    engine and the GPU are never touched.  The reference's path as compiled
    from /root/reference (oracle/_ref: gf_gen_rs_matrix, ec_init_tables,
    gf_invert_matrix, ec_encode_data_base) and our AVX2 restatement of its
    asm kernel, each on 1 thread (isa.cpp's single-threaded semantics) and on
    every usable host thread (independent blocks).  Accounting as the
    reference harness (throughput_benchmark.hpp:37-67, 179-196): encoder
    goodput = payload_count x symbol_size / encode time (isa.cpp:38, the e
    parity symbols), decoder goodput = erased x symbol_size / decode time;
    `value` = both outputs over both times, as bench.py's other configs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    k, L, loss, _ = CONFIGS["c1"]
    e = int(math.ceil(k * loss))
    if not oracle_lib.have_reference():
        raise SystemExit("bench.py --config c1 needs oracle/_ref (python __graft_entry__.py build)")
    ref = oracle_lib.Reference()
    cpus = host_cpus()
    nthreads = args.cpu_threads or cpus["usable"]

    def leg(kernel, threads):
        # calibrate on a few blocks, then size the sample to --c1-seconds
        r = ref.cpu_bench(k, e, L, threads, 4, args.seed, kernel)
        per_block = max(r["max_thread_s"] / 4, 1e-6)
        nb = int(min(200000, max(4, args.c1_seconds / per_block)))
        r = ref.cpu_bench(k, e, L, threads, nb, args.seed, kernel)
        blocks = threads * nb
        enc, dec = r["enc_s"] / blocks, r["dec_s"] / blocks  # per block, summed over threads
        out = e * L
        return {"kernel": "ISA-L 2.13 ec_encode_data_base, compiled from the reference (oracle/_ref)"
                          if kernel == 0 else "AVX2 restatement of gf_vect_dot_prod_avx2 (oracle/isal_avx2_port.c)",
                "kind": "reference" if kernel == 0 else "port", "threads": threads,
                "blocks_per_thread": nb, "max_thread_s": round(r["max_thread_s"], 3),
                "failures": r["failures"],
                "encoder_goodput_MBps": round(out / enc / 1e6, 1),
                "decoder_goodput_MBps": round(out / dec / 1e6, 1),
                "encode_us_per_block": round(enc * 1e6, 2), "decode_us_per_block": round(dec * 1e6, 2),
                "goodput_GiBps": 2.0 * out * threads * nb / r["max_thread_s"] / 2 ** 30}

    legs = [leg(0, 1), leg(1, 1), leg(0, nthreads), leg(1, nthreads)]
    head = legs[0]
    ok = all(lg["failures"] == 0 for lg in legs)
    return {
        # not the GPU metric: the same accounting on the host CPU
        "metric": "encode+decode goodput GiB/s on the host CPU (reference accounting)",
        "value": round(head["goodput_GiBps"], 4), "unit": "GiB/s", "n_gpus": 0,
        "steps": head["blocks_per_thread"], "warmup": 0,
        "ms_per_step": round((head["encode_us_per_block"] + head["decode_us_per_block"]) / 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"isa_throughput c1 on the host CPU (plumbing, no GPU): symbols={k} "
                               f"symbol_size={L} loss_rate={loss} erased={e}; value = the reference's "
                               f"compiled C on 1 thread",
                   "symbols": k, "symbol_size": L, "loss_rate": loss, "erased": e,
                   "parallelism": "1 thread (value); all usable threads in legs"},
        "device": "cpu", "verified": ok, "roofline": None,
        "cpu_baseline": {"value": round(head["goodput_GiBps"], 4), "unit": "GiB/s", "cores": 1,
                         "kind": "reference",
                         "sample": f"{head['blocks_per_thread']} blocks (k={k}, e={e}, L={L}) encode+decode "
                                   f"on 1 thread, {head['max_thread_s']} s"},
        "legs": legs, "cpu_model": cpu_model(), **cpus,
    }


def launch_cost(torch, n=400):
    """Per-launch overhead on the engine's stream: n back-to-back launches
    of a near-empty kernel (torch.cuda._sleep of one cycle), timed on the
    device (HIP events: the gap between consecutive dispatches) and on the
    host (enqueue + drain)."""
    torch.cuda._sleep(1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(n):
        torch.cuda._sleep(1)
    e1.record()
    torch.cuda.synchronize()
    host = time.perf_counter() - t0
    return {"empty_kernel_us_device": round(e0.elapsed_time(e1) * 1e3 / n, 3),
            "empty_kernel_us_host": round(host * 1e6 / n, 3)}


def kernel_stats(recs, steps, alg, blocks_step):
    """Per kernel: launches, durations and the algorithmic rate.  A kernel
    that covers a block's rows in passes (e > 32: one launch per 32 rows)
    sees each block once per pass; its algorithmic bytes ((k + e) L per
    block) count once per step, so a launch carries 1 / passes of them."""
    per, each = {}, {}
    for name, ms, nb in recs:
        d = per.setdefault(name, [0.0, 0, 0])
        d[0] += ms
        d[1] += 1
        d[2] += nb
        each.setdefault(name, []).append(ms)
    kernels = {}
    for name, (tot, n, nb) in per.items():
        passes = max(1, round(nb / (blocks_step * steps)))
        per[name].append(passes)
        kernels[name] = {"avg_ms": round(tot / n, 3), "median_ms": round(statistics.median(each[name]), 3),
                         "launches": n,
                         "blocks_per_launch": nb / n,
                         "passes": passes,
                         "alg_GBps": round(alg.get(name, 0.0) * nb / passes / (tot * 1e-3) / 1e9, 1),
                         "ms_per_step": round(tot / steps, 3)}
    return per, kernels


# The VALU issue ceiling, in SIMD cycles per wave64 instruction: the chip
# guide's 2 (SIMD-32: a wave64 VALU issues over 2 cycles, MI355X_MICROARCH.md)
# and the ceiling measured for v_bitop3 on random data with tools/ubench_issue
# (GRBM_GUI_ACTIVE and SQ_INSTS_VALU from ONE counter pass, no wall clock)
GUIDE_CYCLES_PER_VALU = 2.0
SIMDS = 1024  # 256 CUs x 4
XCDS = 8


def sq_counters(path):
    """{kernel: {counter: value per dispatch}} from tools/pmc_summary.py output."""
    out, cur = {}, None
    for ln in open(path):
        if not ln.startswith(" "):
            cur = ln.strip()
            out[cur] = {}
        elif cur is not None:
            name, val = ln.split()
            out[cur][name] = float(val)
    return out


def valu_roofline(counters, kernel, ceiling):
    """How close one kernel's VALU stream runs to the issue ceiling, from
    counters of ONE pass only (time-independent): SIMD-cycles per wave64
    VALU = (GRBM_GUI_ACTIVE / 8 XCDs) * 1024 SIMDs / SQ_INSTS_VALU, against
    the guide's 2 cycles and against the measured ceiling `ceiling`."""
    c = counters.get(kernel) or counters.get(kernel.split("(")[0])
    if not c or "SQ_INSTS_VALU" not in c or "GRBM_GUI_ACTIVE" not in c:
        return None
    cpi = c["GRBM_GUI_ACTIVE"] / XCDS * SIMDS / c["SQ_INSTS_VALU"]
    out = {"valu_insts_per_launch": c["SQ_INSTS_VALU"],
           "valu_insts_per_wave": round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1) if c.get("SQ_WAVES") else None,
           "simd_cycles_per_valu": round(cpi, 3),
           "frac_of_guide_2cycle": round(GUIDE_CYCLES_PER_VALU / cpi, 4)}
    if ceiling:
        out["measured_ceiling_cycles_per_valu"] = ceiling
        out["frac_of_measured_ceiling"] = round(ceiling / cpi, 4)
    return out


def valu_ceiling(path):
    """Best measured issue rate (SIMD cycles per VALU, any occupancy), or None."""
    try:
        return json.load(open(path))["best"]["simd_cycles_per_valu"]
    except (OSError, KeyError, ValueError):
        return None


def hbm_probe(dev, mib=2048, reps=5):
    """Streaming rates torch's own elementwise kernels reach on this GPU
    (confirm the 8 TB/s spec with a copy kernel): int32
    c = a + b (2 reads : 1 write, the (k+e)L mix of an encode/decode with
    e = k/2) and a plain copy.  Best of `reps` after two warm-up passes,
    HIP events on torch's stream; GB/s of bytes moved."""
    import torch
    n = mib * 2 ** 20 // 4
    a = torch.ones(n, dtype=torch.int32, device=dev)
    b = torch.ones(n, dtype=torch.int32, device=dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)

    def best(fn, nbytes):
        for _ in range(2):
            fn()
        ms = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        return round(nbytes / (min(ms) * 1e-3) / 1e9, 1)

    out = {"read2_write1_GBps": best(lambda: torch.add(a, b, out=c), 12.0 * n),
           "copy_GBps": best(lambda: c.copy_(a), 8.0 * n),
           "source": f"torch int32 add / copy, {mib} MiB per tensor, best of {reps}"}
    del a, b, c
    torch.cuda.empty_cache()
    return out


def alg_bytes(k, e, L):
    """Algorithmic HBM bytes per BLOCK of each kernel:
    (k + e) L for an encode or a decode (read k rows, write e)."""
    blk_op = float((k + e) * L)
    return {"k_rs_bs(encode)": blk_op, "k_rs_bs_split(encode)": blk_op, "k_rs_tc_fused(decode)": blk_op,
            "k_rs_syn_split(decode)": blk_op,
            "k_rs_encode_lh": blk_op, "k_dot_generic": blk_op,
            "k_dot_generic(decode)": blk_op,
            "k_rs_tc(encode)": blk_op, "k_rs_tc(decode)": blk_op, "k_rs_jit(decode)": blk_op,
            "k_rs_jit16(decode)": blk_op, "k_rs_jit10(decode)": blk_op, "k_rs_jit12(decode)": blk_op, "k_rs_jit(encode)": blk_op,
            "k_rs_jit16x4(decode)": blk_op, "k_rs_jit12x4(decode)": blk_op, "k_rs_jit10x4(decode)": blk_op,
            "k_rs_jitw_passes(decode)": blk_op,
            "k_decode_prepare": 0.0, "k_decode_prepare_syn": 0.0}


def run_streamed(args, rsgpu, ctx, dev, rank, world, k, e, L, total_blocks):
    """C4: this rank's share of `total_blocks` blocks streamed through two
    resident batches.  Per batch: sources generated on the device and the
    erasure lists (global block index) uploaded on the `gen` stream; encode +
    decode (the timed regions, HIP events) and the device verify on the
    compute stream.
    Each batch runs in the reference's order (isa.cpp / throughput_benchmark:
    setup() fills the blocks, encode_all, decode_all, verify_data): batch
    i+1's generation waits for batch i's verification, and the timed kernels
    run alone.  (Generating batch i+1 beside batch i's verification, the
    round-3 order, shortens the wall time but left the encode that follows a
    verification 1.0-1.4 ms slower per batch, profiles/r03_ab/verify/.)
    Returns (timed seconds, wall seconds,
    mismatching bytes, batches, kernel records)."""
    import numpy as np
    import torch
    blk_base, share = split(total_blocks, rank, world)
    batch = max(1, min(args.batch, share))
    nb_total = (share + batch - 1) // batch
    gen_ctx = rsgpu.Context(dev.index)
    s_cmp, s_gen = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ctx.set_stream(s_cmp.cuda_stream)
    gen_ctx.set_stream(s_gen.cuda_stream)
    sets = []
    for _ in range(2):
        enc = rsgpu.GpuEncoder(k, L, e, blocks=batch, seed=args.seed, ctx=ctx, block0=blk_base)
        dec = rsgpu.GpuDecoder(k, L, e, blocks=batch, seed=args.seed, ctx=ctx, block0=blk_base)
        sets.append((enc, dec))
    torch.cuda.synchronize()
    mism = torch.zeros(nb_total, dtype=torch.int64, device=dev)
    ev_gen = [torch.cuda.Event() for _ in range(nb_total)]
    ev_done = [torch.cuda.Event() for _ in range(nb_total)]
    ev_t = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(nb_total)]
    h_err = [torch.empty((batch, e), dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def generate(i):
        enc, dec = sets[i & 1]
        b0 = blk_base + i * batch
        nb = min(batch, share - i * batch)
        if i >= 2:
            ev_gen[i - 2].synchronize()  # its upload from this pinned buffer is done
        h_err[i & 1][:nb] = torch.from_numpy(rsgpu.erasure_patterns(args.seed, b0, nb, k, e))
        with torch.cuda.stream(s_gen):
            if i >= 1:
                # after batch i-1's verification: never beside the timed
                # encode / decode kernels
                s_gen.wait_event(ev_done[i - 1])
            if i >= 2:
                s_gen.wait_event(ev_done[i - 2])  # batch i-2 (same buffers) verified
            gen_ctx.fill_synthetic(enc.src, nb * k, L, enc.pitch, args.seed, b0 * k)
            dec.err.view(-1)[:nb * e].copy_(h_err[i & 1][:nb].reshape(-1), non_blocking=True)
            ev_gen[i].record(s_gen)

    if args.warmup > 0:
        # one full batch untimed: the generated-code memory, the decode's
        # second stream and the tables reach their timed size here, not in
        # the first timed batch (a 2.46 GB executable allocation and its fill
        # once took 2 s there, profiles/r04_lds/new_c4_2.log)
        generate(0)
        enc, dec = sets[0]
        nb = min(batch, share)
        s_cmp.wait_event(ev_gen[0])
        ctx.encode_blocks(k, e, L, enc.pitch, nb, enc.src, enc.par)
        ctx.decode_blocks(k, e, L, enc.pitch, nb, enc.src, enc.par, dec.err, dec.out, dec.ws, dec.status)
        torch.cuda.synchronize()
    ctx.timing_read()
    ctx.timing_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    generate(0)
    for i in range(nb_total):
        enc, dec = sets[i & 1]
        nb = min(batch, share - i * batch)
        s_cmp.wait_event(ev_gen[i])
        ev_t[i][0].record(s_cmp)
        ctx.encode_blocks(k, e, L, enc.pitch, nb, enc.src, enc.par)
        ctx.decode_blocks(k, e, L, enc.pitch, nb, enc.src, enc.par, dec.err, dec.out, dec.ws,
                          dec.status)
        ev_t[i][1].record(s_cmp)
        if not args.no_verify:
            ctx.verify_blocks(k, e, L, enc.pitch, nb, enc.src, dec.out, dec.err, dec.mism)
            # fold this batch's mismatches (and failed blocks) into its slot
            with torch.cuda.stream(s_cmp):
                bad = dec.mism[:nb].sum() + (dec.status[:nb] != 0).sum() * L
                mism[i:i + 1].copy_(bad.view(1))
                dec.mism.zero_()
        ev_done[i].record(s_cmp)
        if i + 1 < nb_total:
            generate(i + 1)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    per_batch = [a.elapsed_time(b) for a, b in ev_t]
    timed = sum(per_batch) * 1e-3
    recs = ctx.timing_read()
    ctx.timing_enable(False)
    ctx.set_torch_stream()
    gen_ctx.close()
    q = sorted(per_batch)
    batch_ms = {"min": round(q[0], 3), "median": round(statistics.median(q), 3), "max": round(q[-1], 3)}
    return timed, wall, int(mism.sum().item()), nb_total, batch, recs, batch_ms


METRIC = ("encode+decode goodput GiB/s (device-resident) at symbols x symbol_size; "
          "%HBM roofline")
FAIL_KEY = "bench_py/failed/{}"


def init_dist(args, world, device_index):
    """The process group of a multi-rank run.  Returns (store, device of the
    reductions).  gloo (the default) is set up over host TCP before this
    process makes any GPU call; nccl (RCCL, --dist-backend nccl) after the
    rank's device is selected.  One rank: no process group, (None, cpu)."""
    import datetime

    import torch
    import torch.distributed as dist
    if world <= 1:
        return None, torch.device("cpu")
    if args.dist_backend == "nccl":
        torch.cuda.set_device(device_index)
    dist.init_process_group(args.dist_backend, init_method="env://",
                            timeout=datetime.timedelta(seconds=args.dist_timeout))
    try:  # the group's own TCP store (a private accessor: failures then go unnamed)
        store = dist.distributed_c10d._get_default_store()
    except Exception:
        store = None
    red = torch.device("cuda", device_index) if args.dist_backend == "nccl" else torch.device("cpu")
    return store, red


def failure_record(rank, ex) -> dict:
    """What a failed rank leaves for rank 0: its error and the innermost frames."""
    import traceback
    tb = "".join(traceback.format_exception(type(ex), ex, ex.__traceback__)[-3:])
    return {"rank": rank, "error": f"{type(ex).__name__}: {ex}"[:1000], "where": tb[-1500:],
            "t": time.time()}


def collect_failures(store, world, own, wait_s):
    """Rank 0: the records every failed rank left in the store, polled for up
    to wait_s (a peer's failure usually reaches rank 0 as a closed connection
    before its record is read), earliest first -- the first is the cause."""
    found = {own["rank"]: own}
    deadline = time.time() + wait_s
    while True:
        for r in range(world):
            key = FAIL_KEY.format(r)
            if r not in found:
                try:
                    if store.check([key]):
                        found[r] = json.loads(store.get(key).decode())
                except Exception:  # the store is rank 0's own: only a torn read
                    pass
        if len(found) == world or time.time() >= deadline:
            break
        time.sleep(0.2)
    return sorted(found.values(), key=lambda f: f.get("t", 0.0))


def failure_line(args, world, failed) -> dict:
    """The one JSON line of a failed run: no value, every failed rank named."""
    return {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"isa_throughput {args.config}", "dist_backend": args.dist_backend},
            "verified": False, "roofline": None, "cpu_baseline": None,
            "error": {"failed_ranks": [f["rank"] for f in failed], "first": failed[0],
                      "all": failed}}


def report_failure(args, rank, world, store, ex, wait_s=10.0):
    """A rank's exception: its record goes to the process group's store; rank
    0 gathers every rank's record and prints the run's one JSON line.
    Returns (exit status, the line or None)."""
    if world > 1:  # the launcher's stop signal must not cut the report short
        signal.signal(signal.SIGTERM, signal.SIG_IGN)
    rec = failure_record(rank, ex)
    print(f"bench.py rank {rank}: {rec['error']}\n{rec['where']}", file=sys.stderr, flush=True)
    if store is not None:
        try:
            store.set(FAIL_KEY.format(rank), json.dumps(rec))
        except Exception:  # rank 0 (the store's host) is gone: it reports nothing then
            pass
    if rank != 0:
        return 1, None
    failed = collect_failures(store, world, rec, wait_s) if store is not None and world > 1 else [rec]
    line = failure_line(args, world, failed)
    print(json.dumps(line), flush=True)
    return 1, line


class RankStopped(Exception):
    """The launcher stopped this rank (SIGTERM), normally after another rank failed."""


def _stopped(signum, frame):
    raise RankStopped(f"signal {signum}: stopped by the launcher (another rank failed?)")


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        if args.config == "c1":
            print("bench.py: --config c1 is one host-CPU line; run it without --gpus", file=sys.stderr)
            return 2
        # no launcher: this process only spawns the ranks (never touches the GPU)
        return spawn_ranks(args.gpus, argv)
    if args.config == "c1":  # host only: neither torch's GPU side nor the engine
        if args.symbols is not None or args.symbol_size is not None or args.loss_rate is not None \
                or args.blocks is not None:
            print("bench.py: --config c1 is the reference's fixed CPU case (16, 64000, 0.5); "
                  "geometry flags are not taken", file=sys.stderr)
            return 2
        print(json.dumps(c1_line(args)), flush=True)
        return 0
    rank, world, local = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2

    import torch.distributed as dist

    device_index = 0 if args.same_device else local
    store = None
    if world > 1:
        # torch.distributed.run stops every rank (SIGTERM) once one has
        # failed: rank 0 turns that into an exception and still prints the
        # line naming the failed rank (the launcher waits before it kills)
        signal.signal(signal.SIGTERM, _stopped)
    try:
        store, red_dev = init_dist(args, world, device_index)
        if args.fail_rank is not None:
            if rank == args.fail_rank:
                raise RuntimeError(f"injected failure on rank {rank} (--fail-rank)")
            dist.barrier()
        rc = run_rank(args, rank, world, device_index, red_dev)
    except Exception as ex:
        rc, _ = report_failure(args, rank, world, store, ex)
        # no destroy_process_group: the peers may be gone
        return rc
    if world > 1:
        dist.destroy_process_group()
    return rc


def run_rank(args, rank, world, device_index, red_dev):
    """One rank's run (the process group, if any, is up): build the batch,
    warm up, time, verify; rank 0 prints the JSON line.  Returns the exit
    status."""
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(device_index)
    dev = torch.device("cuda", device_index)

    import rsgpu

    k, L, loss, B = CONFIGS[args.config]
    custom = args.symbols is not None or args.symbol_size is not None or args.loss_rate is not None
    k = args.symbols if args.symbols is not None else k
    L = args.symbol_size if args.symbol_size is not None else L
    loss = args.loss_rate if args.loss_rate is not None else loss
    if args.blocks:
        B = args.blocks
    e = int(math.ceil(k * loss))
    ctx = rsgpu.Context(dev.index)
    ctx.set_torch_stream()
    ctx.set_decode_kernel(args.decode_kernel)
    ctx.set_encode_kernel(args.encode_kernel)
    alg = alg_bytes(k, e, L)
    rank_info = None

    if args.config == "c4":
        timed, wall, bad, nbatches, batch, recs, batch_ms = run_streamed(args, rsgpu, ctx, dev, rank, world,
                                                               k, e, L, B)
        blk0, share = split(B, rank, world)
        if world > 1:
            rank_info = [None] * world
            dist.all_gather_object(rank_info, {"rank": rank, "device": device_index, "block0": blk0,
                                               "blocks": share, "batches": nbatches})
        elapsed = reduce_max_time(timed, world, red_dev)
        wall = reduce_max_time(wall, world, red_dev)
        bad_t = torch.tensor([float(bad)], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(bad_t)
        ok = args.no_verify or bad_t.item() == 0
        steps = 1
        # every rank's share counts (shares differ by at most one block)
        out_bytes_step = 2.0 * e * L * B / world
        value = job_goodput(out_bytes_step, 1, world, elapsed)
        ms_step = elapsed * 1e3
        workload = (f"isa_throughput c4: symbols={k} symbol_size={L} loss_rate={loss} erased={e} "
                    f"blocks={B} streamed over {world} GPU(s): {share} on rank {rank} in {nbatches} "
                    f"batches of {batch} (2 resident)")
        extra = {"streamed": {"blocks_total": B, "blocks_per_gpu": B / world, "blocks_rank0": share,
                              "batches": nbatches,
                              "batch_blocks": batch, "timed_s": elapsed, "wall_s": wall,
                              "batch_ms_rank0": batch_ms,
                              "wall_GiBps": 2.0 * e * L * B / wall / 2 ** 30,
                              "mismatch_bytes": bad_t.item(),
                              "note": "value: encode+decode regions (HIP events) summed over "
                                      "the batches; wall: the whole stream incl. on-device "
                                      "source generation and verification"}}
    else:
        # rank r owns global blocks [r*B, (r+1)*B): independent shard, no exchange
        blk0, B = shard(rank, B)
        enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=args.seed, ctx=ctx, block0=blk0)
        dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=args.seed, ctx=ctx, block0=blk0)
        torch.cuda.synchronize()
        if world > 1:
            info = {"rank": rank, "device": device_index, "block0": blk0, "blocks": B,
                    "err_sha": hashlib.sha256(dec.err_host.tobytes()).hexdigest()}
            rank_info = [None] * world
            dist.all_gather_object(rank_info, info)

        def step():
            enc.encode_all()
            dec.decode_all(enc)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if not args.no_verify and args.warmup > 0:
            assert dec.is_complete(), "decode matrix singular"
            assert dec.verify_data(enc), "recovered symbols differ from the originals"
        torch.cuda.synchronize()

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        # per-kernel HIP events in a second pass of the same steps: the two
        # event records per launch cost host time that a short step (C2,
        # ~60 us) would otherwise count
        ctx.timing_read()  # drop anything recorded so far
        ctx.timing_enable(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        recs = ctx.timing_read()
        ctx.timing_enable(False)
        elapsed = reduce_max_time(elapsed, world, red_dev)
        ok = True
        if not args.no_verify:
            ok = dec.is_complete() and dec.verify_data(enc)
        if world > 1:  # the line rank 0 prints speaks for every rank's shard
            ok_t = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=red_dev)
            dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
            ok = ok_t.item() == 1.0
        steps = args.steps
        out_bytes_step = 2.0 * e * L * B            # parity + recovered, per rank
        value = job_goodput(out_bytes_step, steps, world, elapsed)
        ms_step = elapsed / steps * 1e3
        workload = (f"isa_throughput {args.config}{' (custom geometry)' if custom else ''}: symbols={k} symbol_size={L} loss_rate={loss} "
                    f"erased={e} blocks_per_gpu={B}")
        # launches per step and what one launch costs on this stream (short
        # steps: C2's two launches)
        extra = {"launch": dict(launch_cost(torch), launches_per_step=round(len(recs) / steps, 2),
                                step_us=round(ms_step * 1e3, 2))}

    # this rank's blocks per step (C4: its share of the stream)
    per, kernels = kernel_stats(recs, steps, alg, out_bytes_step / (2.0 * e * L) if args.config != "c4" else share)
    # dominant kernel = the most device time per step
    dom = max(per, key=lambda n: per[n][0])
    tot, n, nb, passes = per[dom]
    dom_ms = tot / n
    dom_bytes = alg.get(dom, 0.0) * nb / n / passes  # algorithmic bytes per launch
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    read_bytes = float(k * L) * nb / n / passes if alg.get(dom, 0.0) else 0.0
    # PMC bytes per launch come from a separate rocprofv3 --pmc pass of the
    # same command (counters cannot be read inside this timed run); only
    # valid for the C3 workload they were measured on
    traffic, traffic_src = None, None
    if (args.traffic and os.path.exists(args.traffic) and args.config == "c3" and not args.blocks
            and not custom):
        traffic = json.load(open(args.traffic)).get(dom)
        traffic_src = os.path.relpath(args.traffic, ROOT) if traffic is not None else None
    valu = None
    if (args.sq_counters and os.path.exists(args.sq_counters) and args.config == "c3"
            and not args.blocks and not custom):
        sq = sq_counters(args.sq_counters)
        ceil = valu_ceiling(args.valu_ceiling)
        valu = {kn: r for kn in per if (r := valu_roofline(sq, kn, ceil))}
    op_bytes = float((k + e) * L) * (out_bytes_step / (2.0 * e * L))
    step_frac = (2 * op_bytes) / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS

    line = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": workload, "symbols": k, "symbol_size": L, "loss_rate": loss,
                   "erased": e, "blocks_per_gpu": out_bytes_step / (2.0 * e * L),
                   "parallelism": f"blocks sharded x{world}, no collective",
                   "decode_kernel": args.decode_kernel, "encode_kernel": args.encode_kernel},
        "hbm_roofline_frac_step": round(step_frac, 4),
        "kernels": kernels,
        "verified": ok,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "alg_bytes_per_launch": dom_bytes, "avg_ms": round(dom_ms, 3),
                     # north_star's HBM-read variant: only the k source rows read
                     # per block count
                     "frac_read": round(read_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     # how close each kernel's VALU stream runs to issue
                     # (SQ counters of the same workload, one pass)
                     "valu": valu,
                     "valu_source": (os.path.relpath(args.sq_counters, ROOT) if valu else None),
                     "valu_ceiling_source": (os.path.relpath(args.valu_ceiling, ROOT)
                                             if valu and valu_ceiling(args.valu_ceiling) else None)},
        "cpu_baseline": None,
    }
    line.update(extra)
    if rank == 0:  # after the timed region: what streaming reaches on this GPU
        probe = hbm_probe(dev)
        probe["frac_of_read2_write1"] = round(achieved / probe["read2_write1_GBps"], 4)
        line["roofline"]["measured_peak"] = probe
    if rank_info is not None:
        line["ranks"] = rank_info
    if args.host_io and rank == 0:
        line["host_io"] = host_io_rate(rsgpu, ctx, k, e, L, args.host_io, args.seed)
        line["host_io"]["pipelined"] = host_io_pipelined(rsgpu, ctx, k, e, L, args.host_io,
                                                         args.seed)
        line["host_io"]["session"] = host_io_session(rsgpu, ctx, k, e, L, args.host_io, args.seed)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpus = host_cpus()
        threads = args.cpu_threads or cpus["usable"]
        host = {"cpu_model": cpu_model(), **cpus,
                "asm_available": {"yasm": shutil.which("yasm"), "nasm": shutil.which("nasm")}}
        try:
            line["cpu_baseline"] = cpu_baseline(k, e, L, threads, kernel=1)
            if line["cpu_baseline"]:
                line["cpu_baseline"].update(host)
            if not args.no_ref_base:
                line["cpu_baseline_reference"] = cpu_baseline(k, e, L, threads, kernel=0)
        except Exception as ex:  # reported, never fatal for the GPU number
            line["cpu_baseline"] = {"error": str(ex), **host}
    line["config"]["dist_backend"] = args.dist_backend if world > 1 else None
    if rank == 0:
        print(json.dumps(line), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
