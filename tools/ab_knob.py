#!/usr/bin/env python3
"""ab_knob.py -- same-process A/B of a layout knob at the STEP level (tool,
not the product; round 5).

The C3 step (encode_all + decode_all over 1024 blocks, bench.py's step) is
bound by the average power over both kernels: a change that makes one
kernel faster can leave the other slower, and process-to-process drift on a
box (~1 %) is as large as the effects being decided.  So one process builds
the workload once and alternates the configurations in ABBA order, each
block of `--steps` timed steps after `--warmup` untimed ones, and reports
per configuration the median step and kernel times and the paired
differences.

    python3 tools/ab_knob.py --knob rsgpu_internal_set_jitw_rot --values 0,-1 [--reps 8]

`--knob` names a librsgpu_testhooks.so setter (ctx, int); `--encode-kernel`
/ `--decode-kernel` values switch the public kernel choice instead
(--knob encode_kernel --values compiled,generated).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--symbols", type=int, default=64)
    ap.add_argument("--symbol-size", type=int, default=1000000)
    ap.add_argument("--erased", type=int, default=32)
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--encode-kernel", default=None, help="fixed encode kernel for every configuration")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import rsgpu

    k, L, e, B = args.symbols, args.symbol_size, args.erased, args.blocks
    ctx = rsgpu.Context(0)
    ctx.set_torch_stream()
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    vals = args.values.split(",")
    if args.encode_kernel:
        ctx.set_encode_kernel(args.encode_kernel)

    def apply(v):
        if args.knob == "encode_kernel":
            ctx.set_encode_kernel(v)
        elif args.knob == "decode_kernel":
            ctx.set_decode_kernel(v)
        else:
            # several knobs at once: --knob a+b --values 0+0,2+2
            for kn, kv in zip(args.knob.split("+"), v.split("+")):
                f = getattr(rsgpu.testhooks(), kn)
                f.argtypes = [ctypes.c_void_p, ctypes.c_int]
                assert f(ctx._h, int(kv)) == 0, (kn, kv)

    def step():
        enc.encode_all()
        dec.decode_all(enc)

    res = {v: {"step_ms": [], "kernels": {}} for v in vals}
    order = []
    for r in range(args.reps):
        order += vals if r % 2 == 0 else vals[::-1]
    for v in order:
        apply(v)
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        res[v]["step_ms"].append((time.perf_counter() - t0) / args.steps * 1e3)
        ctx.timing_read()
        ctx.timing_enable(True)
        step()
        torch.cuda.synchronize()
        for name, ms, _ in ctx.timing_read():
            res[v]["kernels"].setdefault(name, []).append(ms)
        ctx.timing_enable(False)
    ok = dec.is_complete() and dec.verify_data(enc)
    out = {"tool": "tools/ab_knob.py", "knob": args.knob, "order": order, "verified": ok,
           "workload": f"k={k} L={L} e={e} blocks={B}", "steps_per_block": args.steps}
    for v in vals:
        s = res[v]["step_ms"]
        out[v] = {"step_ms_median": round(statistics.median(s), 3), "step_ms": [round(x, 3) for x in s],
                  "goodput_GiBps": round(2 * e * L * B / (statistics.median(s) * 1e-3) / 2 ** 30, 1),
                  "kernels_ms_median": {n: round(statistics.median(m), 3) for n, m in res[v]["kernels"].items()}}
    base = res[vals[0]]["step_ms"]
    for v in vals[1:]:
        d = [b - a for a, b in zip(base, res[v]["step_ms"])]
        out[v]["paired_delta_ms_vs_" + vals[0]] = {"median": round(statistics.median(d), 3),
                                                   "min": round(min(d), 3), "max": round(max(d), 3)}
    print(json.dumps(out, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
