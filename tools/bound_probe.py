#!/usr/bin/env python3
"""bound_probe.py -- what bounds the C3 kernels: all-zero vs random inputs,
and the in-kernel clock (MI355X_MICROARCH.md "DVFS give-back" items 1 and 6).

One process, C3 (k 64, e 32, L 1e6, 1024 blocks): the compiled encode
(k_rs_bs) and the generated decode (k_rs_jit16, decode_apply after ONE
prepare) each launched back to back for >= --seconds per phase, on the
seeded random sources and on all-zero sources (parity zero too), phases in
the order --order gives (default alternates, so drift shows).  Per phase:
the median launch time from HIP events on the engine's stream, and -- with
the diagnostic library (RSGPU_LIB=tools/diag/librsgpu_diag.so, built by
`make -C storage-benchmarks_amd diag`) -- the in-kernel clock of the last
launch, delta s_memtime / delta s_memrealtime x 100 MHz per stamped
workgroup, median over workgroups (diag_clock.h).  The product library has
no stamps; run the timing arm with it and the clock arm with the diagnostic
build (never quote the diagnostic build's times).

Under `rocprofv3 --pmc ...` the same command gives per-dispatch counters;
--launches fixes the count per phase and the JSON's "dispatches" list names
every dispatch of each kernel in order (tools/bound_summary.py groups them).

Prints one JSON object (also written to --out).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))

ENC, DEC = "k_rs_bs(encode)", "k_rs_jit16(decode)"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--symbol-size", type=int, default=1000000, help="L (32000: C4's rows)")
    ap.add_argument("--seconds", type=float, default=2.5, help="per phase (ignored with --launches)")
    ap.add_argument("--launches", type=int, default=0, help="fixed launches per phase")
    ap.add_argument("--order", default="enc:rand,enc:zero,dec:zero,dec:rand,enc:rand,enc:zero,dec:zero,dec:rand")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    import rsgpu

    lib = rsgpu.lib()
    diag = hasattr(lib, "rsgpu_diag_clock_read")
    if diag:
        import ctypes as C
        lib.rsgpu_diag_clock_read.argtypes = [C.c_int, C.c_void_p, C.c_size_t]
        lib.rsgpu_diag_clock_read.restype = C.c_int
        lib.rsgpu_diag_clock_clear.restype = C.c_int
        lib.rsgpu_diag_clock_slots.restype = C.c_int
    k, e, L, B = 64, 32, args.symbol_size, args.blocks
    ctx = rsgpu.Context(0)
    ctx.set_torch_stream()
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    alg = float((k + e) * L * B)
    dispatches = []  # (kernel, label, count) in issue order

    def note(kernel, label, n):
        if dispatches and dispatches[-1][0] == kernel and dispatches[-1][1] == label:
            dispatches[-1][2] += n
        else:
            dispatches.append([kernel, label, n])

    def make_random():
        ctx.fill_synthetic(enc.src, B * k, L, enc.pitch, 1)
        enc.encode_all()
        note(ENC, "setup", 1)

    def make_zero():
        enc.src.zero_()
        enc.par.zero_()

    make_random()
    ctx.decode_prepare(k, e, L, enc.pitch, B, enc.src, enc.par, dec.err, dec.out, dec.ws, dec.status)
    torch.cuda.synchronize()
    assert (dec.status[:B] == 0).all().item()

    def launch(kind):
        if kind == "enc":
            enc.encode_all()
        else:
            ctx.decode_apply(k, e, L, enc.pitch, B, enc.src, enc.par, dec.out, dec.ws, dec.status)

    state = "rand"
    phases = []
    for item in args.order.split(","):
        kind, data = item.split(":")
        if data != state:
            make_zero() if data == "zero" else make_random()
            state = data
        torch.cuda.synchronize()
        if diag:
            assert lib.rsgpu_diag_clock_clear() == 0
        kname = ENC if kind == "enc" else DEC
        ctx.timing_read()
        ctx.timing_enable(True)
        n = 0
        t0 = time.perf_counter()
        while True:
            launch(kind)
            n += 1
            if args.launches:
                if n >= args.launches:
                    break
            elif n % 8 == 0:
                torch.cuda.synchronize()
                if time.perf_counter() - t0 >= args.seconds:
                    break
            if n % 64 == 0:  # keep the event records bounded
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        recs = [r for r in ctx.timing_read() if r[0] == kname]
        ctx.timing_enable(False)
        note(kname, item, n)
        ms = [r[1] for r in recs]
        tail = ms[len(ms) // 3:] or ms
        ph = {"phase": item, "kernel": kname, "launches": n, "wall_s": round(wall, 3),
              "median_ms": round(statistics.median(tail), 4), "min_ms": round(min(tail), 4),
              "max_ms": round(max(tail), 4),
              "TBps_alg": round(alg / (statistics.median(tail) * 1e-3) / 1e12, 3)}
        if diag:
            import numpy as np
            slots = lib.rsgpu_diag_clock_slots()
            buf = np.zeros((slots, 4), np.uint64)
            assert lib.rsgpu_diag_clock_read(0 if kind == "enc" else 1, buf.ctypes.data, buf.nbytes) == 0
            t = buf.astype(np.float64)
            ok = (t[:, 3] > t[:, 1]) & (t[:, 2] > t[:, 0])
            clk = (t[ok, 2] - t[ok, 0]) / (t[ok, 3] - t[ok, 1]) * 100.0  # MHz
            life = (t[ok, 3] - t[ok, 1]) / 100.0  # us of wave 0 lifetime
            if ok.any():
                ph["clock_MHz_median"] = round(float(np.median(clk)), 1)
                ph["clock_MHz_p10_p90"] = [round(float(np.percentile(clk, 10)), 1),
                                           round(float(np.percentile(clk, 90)), 1)]
                ph["wg_life_us_median"] = round(float(np.median(life)), 2)
                ph["stamped_wgs"] = int(ok.sum())
            if kind == "dec" and hasattr(lib, "rsgpu_diag_phase_read"):
                # variant 6 builds: k_rs_jitw's per-wave cycles per phase
                lib.rsgpu_diag_phase_read.argtypes = [C.c_void_p, C.c_size_t]
                pt = np.zeros((slots, 4, 8), np.uint64)
                assert lib.rsgpu_diag_phase_read(pt.ctypes.data, pt.nbytes) == 0
                pt = pt.astype(np.float64)
                live = pt[:, :, 7] > 0
                if live.any():
                    names = ["loop", "wait_dma", "transpose", "barrier", "issue_ptrs", "code", "store", "life"]
                    mean = pt[live].mean(axis=0)
                    ph["phase_cycles_per_wave"] = {n: round(float(v), 0) for n, v in zip(names, mean)}
                    ph["phase_frac"] = {n: round(float(v / mean[7]), 4) for n, v in zip(names[:7], mean[:7])}
        phases.append(ph)
        print(json.dumps(ph), flush=True)

    out = {"tool": "tools/bound_probe.py", "library": rsgpu.LIB_PATH, "diagnostic_build": diag,
           "workload": f"k={k} e={e} L={L} blocks={B}", "alg_bytes_per_launch": alg,
           "phases": phases, "dispatches": dispatches}
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({"dispatches": dispatches}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
