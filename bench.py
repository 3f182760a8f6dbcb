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

Multi-GPU: one process per GPU (torch.distributed, RCCL backend only for the
barrier and the max-over-ranks timing); each rank owns its own 1024 blocks
(weak scaling, no collective on the data path).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))

CONFIGS = {
    # name: (symbols, symbol_size, loss_rate, blocks per GPU)
    "c2": (16, 1000000, 0.25, 1),
    "c3": (64, 1000000, 0.5, 1024),
    "c4": (64, 32000, 0.5, 32768),      # 1M blocks streamed: 32768 resident per pass
    "c5": (100, 1000000, 0.2, 512),     # 4096 blocks over 8 GPUs = 512 per GPU
}
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md chip table, spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    p.add_argument("--blocks", type=int, default=None, help="blocks per GPU (override)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=None)
    p.add_argument("--no-ref-base", action="store_true",
                   help="skip the (slow, ~10 s) reference scalar-C CPU sample")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--host-io", type=int, default=0, metavar="BLOCKS",
                   help="also time the host-resident path (H2D + kernel + D2H) on BLOCKS blocks")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r01_traffic.json"),
                   help="JSON with PMC-derived HBM bytes per launch of the same workload "
                        "(tools/profile_round.sh; default: the committed profiles/r01_traffic.json)")
    return p.parse_args()


def shard(rank: int, blocks_per_rank: int):
    """Blocks owned by `rank`: [rank*B, (rank+1)*B) -- independent blocks, no
    exchange between ranks; weak scaling."""
    return rank * blocks_per_rank, blocks_per_rank


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


def host_io_rate(rsgpu, ctx, k, e, L, blocks, seed, reps=3):
    """Goodput when the blocks start and end in (pinned) host memory, as the
    reference's buffers do: encode = H2D(sources) + encode + D2H(parity);
    decode = H2D(survivors + parity) + decode + D2H(recovered).  Returns
    GiB/s of output bytes over the summed wall time (median of reps)."""
    import torch
    enc = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    h_src = torch.empty(enc.src.numel(), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty(enc.par.numel(), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(dec.out.numel(), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(enc.src)
    h_par.copy_(enc.par)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        enc.src.copy_(h_src, non_blocking=True)
        enc.encode_all()
        h_par.copy_(enc.par, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        # decoder side: survivors (all source rows are shipped; the erased ones
        # are simply not read) + parity in, recovered rows out
        enc.src.copy_(h_src, non_blocking=True)
        enc.par.copy_(h_par, non_blocking=True)
        dec.decode_all(enc)
        h_out.copy_(dec.out, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        times.append((t1 - t0, t2 - t1))
    times.sort(key=lambda x: x[0] + x[1])
    te, td = times[len(times) // 2]
    ok = dec.is_complete() and dec.verify_data(enc)
    out_b = e * L * blocks
    return {"blocks": blocks, "encode_s": te, "decode_s": td,
            "goodput_GiBps": 2 * out_b / (te + td) / 2 ** 30,
            "encode_GiBps": out_b / te / 2 ** 30, "decode_GiBps": out_b / td / 2 ** 30,
            "verified": ok}


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


def host_io_pipelined(rsgpu, ctx, k, e, L, blocks, seed, chunk=4, reps=3):
    """The host_io_rate workload with the copies overlapped: the blocks go in
    chunks of `chunk` blocks through three streams (H2D, compute, D2H) joined
    by events, so chunk i+1 crosses PCIe while chunk i is encoded or decoded
    and chunk i-1 comes back.  H2D and D2H use the two directions of the link
    at once.  The decoder side ships only what isa_decoder reads: the k - e
    surviving source rows (as runs of consecutive rows) and the parity rows.
    Median of reps."""
    import torch
    enc = rsgpu.GpuEncoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=blocks, seed=seed, ctx=ctx)
    nch = (blocks + chunk - 1) // chunk
    rk, re_ = k * enc.pitch, e * enc.pitch
    h_src = torch.empty(enc.src.numel(), dtype=torch.uint8, pin_memory=True)
    h_par = torch.empty(enc.par.numel(), dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(dec.out.numel(), dtype=torch.uint8, pin_memory=True)
    h_src.copy_(enc.src)
    torch.cuda.synchronize()
    # one decode workspace per chunk: the chunks' decodes may overlap their copies
    wss = [torch.empty(rsgpu.decode_workspace_bytes(k, e, chunk), dtype=torch.uint8,
                       device=enc.src.device) for _ in range(nch)]
    # decoder side ships only the survivors (found untimed)
    runs = survivor_runs(dec.err_host, k, enc.pitch, chunk)
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    prev_stream = torch.cuda.current_stream()
    ctx.set_stream(s_cmp.cuda_stream)

    def run(decode):
        for i in range(nch):
            b0, nb = i * chunk, min(chunk, blocks - i * chunk)
            src = enc.src[b0 * rk:(b0 + nb) * rk]
            par = enc.par[b0 * re_:(b0 + nb) * re_]
            out = dec.out[b0 * re_:(b0 + nb) * re_]
            e_in, e_cmp = torch.cuda.Event(), torch.cuda.Event()
            with torch.cuda.stream(s_in):
                if decode:
                    for off, n in runs[i]:
                        enc.src[off:off + n].copy_(h_src[off:off + n], non_blocking=True)
                    par.copy_(h_par[b0 * re_:(b0 + nb) * re_], non_blocking=True)
                else:
                    src.copy_(h_src[b0 * rk:(b0 + nb) * rk], non_blocking=True)
                e_in.record(s_in)
            s_cmp.wait_event(e_in)
            if decode:
                ctx.decode_blocks(k, e, L, enc.pitch, nb, src, par, dec.err[b0:b0 + nb], out,
                                  wss[i], dec.status[b0:b0 + nb])
            else:
                ctx.encode_blocks(k, e, L, enc.pitch, nb, src, par)
            e_cmp.record(s_cmp)
            s_out.wait_event(e_cmp)
            with torch.cuda.stream(s_out):
                if decode:
                    h_out[b0 * re_:(b0 + nb) * re_].copy_(out, non_blocking=True)
                else:
                    h_par[b0 * re_:(b0 + nb) * re_].copy_(par, non_blocking=True)
        torch.cuda.synchronize()

    times = []
    try:
        for _ in range(reps):
            t0 = time.perf_counter()
            run(False)
            t1 = time.perf_counter()
            run(True)
            t2 = time.perf_counter()
            times.append((t1 - t0, t2 - t1))
    finally:
        ctx.set_stream(prev_stream.cuda_stream)
    dec._decoded = True
    times.sort(key=lambda x: x[0] + x[1])
    te, td = times[len(times) // 2]
    ok = dec.is_complete() and dec.verify_data(enc)
    # what came back to the host is what the device holds
    ok = ok and bool(torch.equal(h_out, dec.out.cpu())) and bool(torch.equal(h_par, enc.par.cpu()))
    out_b = e * L * blocks
    return {"blocks": blocks, "chunk_blocks": chunk, "encode_s": te, "decode_s": td,
            "goodput_GiBps": 2 * out_b / (te + td) / 2 ** 30,
            "encode_GiBps": out_b / te / 2 ** 30, "decode_GiBps": out_b / td / 2 ** 30,
            "verified": ok}


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def cpu_baseline(k, e, L, threads, kernel=1, blocks_per_thread=None):
    """CPU baseline on the GPU box's host cores, isa.cpp's timed regions
    (encode = matrix + tables + data kernel; decode = k x k inversion + tables
    + data kernel) over a bounded sample: `threads` workers x
    `blocks_per_thread` blocks of the same geometry.  Matrices, tables and
    inversion are the reference's ISA-L 2.13 C compiled from /root/reference
    (oracle/_ref).  The data kernel is
      kernel 1: our AVX2 restatement of ISA-L's asm path (oracle/
                isal_avx2_port.c; the yasm sources cannot be assembled in this
                image) -> kind "port";
      kernel 0: the reference's scalar ec_encode_data_base -> kind "reference".
    """
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    if not oracle_lib.have_reference():
        return None
    ref = oracle_lib.Reference()
    if kernel == 1 and not ref.have_avx2:
        return {"error": "host CPU has no AVX2"}
    bpt = blocks_per_thread or (8 if kernel == 1 else 1)
    r = ref.cpu_bench(k, e, L, threads, bpt, 7, kernel)
    out_bytes = 2.0 * e * L * threads * bpt
    t = r["max_thread_s"]
    what = ("AVX2 restatement of ISA-L 2.13 gf_vect_dot_prod_avx2/ec_encode_data_avx2"
            if kernel == 1 else "ISA-L 2.13 ec_encode_data_base (reference scalar C)")
    return {"value": out_bytes / t / 2 ** 30, "unit": "GiB/s", "cores": threads,
            "kind": "port" if kernel == 1 else "reference",
            "sample": f"{threads} threads x {bpt} block(s) (k={k}, e={e}, L={L}) encode+decode, "
                      f"{what}, reference matrices/inversion; {t:.1f} s per thread, "
                      f"failures={r['failures']}",
            "encode_s_per_block": r["enc_s"] / (threads * bpt),
            "decode_s_per_block": r["dec_s"] / (threads * bpt)}


def main():
    args = parse()
    rank, world, local = dist_env()
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import rsgpu

    k, L, loss, B = CONFIGS[args.config]
    if args.blocks:
        B = args.blocks
    e = int(math.ceil(k * loss))
    ctx = rsgpu.Context(dev.index)
    ctx.set_torch_stream()

    # rank r owns global blocks [r*B, (r+1)*B): independent shard, no exchange
    blk0, B = shard(rank, B)
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=args.seed, ctx=ctx, block0=blk0)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=args.seed, ctx=ctx, block0=blk0)
    torch.cuda.synchronize()

    # Per-kernel HIP events: the engine brackets every launch on its stream
    # (torch's current stream, handed over by set_torch_stream) when timing is
    # enabled; read back after the timed region.
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
    ctx.timing_read()  # drop anything recorded so far
    ctx.timing_enable(True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    recs = ctx.timing_read()
    ctx.timing_enable(False)
    if world > 1:
        dist.barrier()
    elapsed = reduce_max_time(elapsed, world, dev)

    ok = True
    if not args.no_verify:
        ok = dec.is_complete() and dec.verify_data(enc)

    out_bytes_step = 2.0 * e * L * B            # parity + recovered, per rank
    value = job_goodput(out_bytes_step, args.steps, world, elapsed)
    ms_step = elapsed / args.steps * 1e3
    op_bytes = float((k + e) * L * B)           # one encode or one decode: read k, write e rows
    # algorithmic HBM bytes per BLOCK of each kernel; a
    # launch covers the number of blocks the engine recorded for it (the
    # decode runs in block chunks on two streams)
    blk_op = float((k + e) * L)
    alg = {"k_rs_bs(encode)": blk_op, "k_rs_encode_lh": blk_op, "k_dot_generic": blk_op,
           "k_rs_bs(syndrome)": blk_op, "k_dot_generic(decode)": blk_op,
           "k_dot_generic(solve)": 2.0 * e * L, "k_rs_tc(solve)": 2.0 * e * L,
           "k_rs_decode_fused": blk_op, "k_rs_tc(encode)": blk_op, "k_rs_tc(decode)": blk_op,
           "k_decode_prepare": 0.0, "k_decode_prepare_syn": 0.0}
    per = {}
    for name, ms, nb in recs:
        d = per.setdefault(name, [0.0, 0, 0])
        d[0] += ms
        d[1] += 1
        d[2] += nb
    kernels = {}
    for name, (tot, n, nb) in per.items():
        kernels[name] = {"avg_ms": round(tot / n, 3), "launches": n,
                         "blocks_per_launch": nb / n,
                         "alg_GBps": round(alg.get(name, 0.0) * nb / (tot * 1e-3) / 1e9, 1),
                         "ms_per_step": round(tot / args.steps, 3)}
    # dominant kernel = the most device time per step
    dom = max(per, key=lambda n: per[n][0])
    tot, n, nb = per[dom]
    dom_ms = tot / n
    dom_bytes = alg.get(dom, 0.0) * nb / n      # algorithmic bytes per launch
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    read_bytes = float(k * L) * nb / n if alg.get(dom, 0.0) else 0.0
    # PMC bytes per launch come from a separate rocprofv3 --pmc pass of the
    # same command (counters cannot be read inside this timed run); only
    # valid for the C3 workload they were measured on
    traffic, traffic_src = None, None
    if args.traffic and os.path.exists(args.traffic) and args.config == "c3" and not args.blocks:
        traffic = json.load(open(args.traffic)).get(dom)
        traffic_src = os.path.relpath(args.traffic, ROOT) if traffic is not None else None
    step_frac = (2 * op_bytes) / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBPS

    line = {
        "metric": "encode+decode goodput GiB/s (device-resident) at symbols x symbol_size; "
                  "%HBM roofline",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"isa_throughput {args.config}: symbols={k} symbol_size={L} "
                               f"loss_rate={loss} erased={e} blocks_per_gpu={B}",
                   "symbols": k, "symbol_size": L, "loss_rate": loss, "erased": e,
                   "blocks_per_gpu": B, "parallelism": f"blocks sharded x{world}, no collective"},
        "hbm_roofline_frac_step": round(step_frac, 4),
        "kernels": kernels,
        "verified": ok,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "alg_bytes_per_launch": dom_bytes, "avg_ms": round(dom_ms, 3),
                     # north_star's HBM-read variant: only the k source rows read
                     # per block count
                     "frac_read": round(read_bytes / (dom_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
        "cpu_baseline": None,
    }
    if args.host_io and rank == 0:
        line["host_io"] = host_io_rate(rsgpu, ctx, k, e, L, args.host_io, args.seed)
        line["host_io"]["pipelined"] = host_io_pipelined(rsgpu, ctx, k, e, L, args.host_io,
                                                         args.seed)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        try:
            line["cpu_baseline"] = cpu_baseline(k, e, L, threads, kernel=1)
            if not args.no_ref_base:
                line["cpu_baseline_reference"] = cpu_baseline(k, e, L, threads, kernel=0)
        except Exception as ex:  # reported, never fatal for the GPU number
            line["cpu_baseline"] = {"error": str(ex)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
