#!/usr/bin/env python3
"""power_split.py -- package power and clock of each C3 kernel run alone,
beside a pure streaming kernel (tool, not product).

Each phase loops one kind of work for ~4 s while a thread samples
`rocm-smi --showpower --showclocks`; printed per phase: median package power,
median sclk, and the phase's rate.  It shows how the 1400 W cap is spent:
HBM streaming at the encode/decode's byte rate versus their VALU work.

  python3 tools/power_split.py [--blocks 1024]
"""
import argparse
import os
import re
import statistics
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))


class Sampler(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.samples, self.stop, self.tag = [], False, None

    def run(self):
        while not self.stop:
            out = subprocess.run(["rocm-smi", "--showpower", "--showclocks"], capture_output=True,
                                 text=True).stdout
            p = re.search(r"Package Power \(W\): ([0-9.]+)", out)
            c = re.search(r"sclk clock level: \S+: \((\d+)Mhz\)", out)
            if p and c and self.tag:
                self.samples.append((self.tag, float(p.group(1)), int(c.group(1))))
            time.sleep(0.2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=4.0)
    args = ap.parse_args()
    import torch
    import rsgpu

    dev = torch.device("cuda", 0)
    k, L, e, B = 64, 1000000, 32, args.blocks
    ctx = rsgpu.Context(0)
    ctx.set_torch_stream()
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=1, ctx=ctx)
    enc.encode_all()
    dec.decode_all(enc)
    torch.cuda.synchronize()
    n = 512 * 2 ** 20  # int32 elements: 2 GiB per tensor
    a = torch.ones(n, dtype=torch.int32, device=dev)
    b = torch.ones(n, dtype=torch.int32, device=dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)

    phases = [
        ("stream add (2R:1W)", lambda: torch.add(a, b, out=c), 12.0 * n),
        ("encode k_rs_bs", enc.encode_all, (k + e) * L * B),
        ("decode k_rs_jit", lambda: dec.decode_all(enc), (k + e) * L * B),
    ]
    s = Sampler()
    s.start()
    for tag, fn, nbytes in phases:
        fn()
        torch.cuda.synchronize()
        s.tag = tag
        t0, reps = time.perf_counter(), 0
        while time.perf_counter() - t0 < args.seconds:
            fn()
            reps += 1
            if reps % 4 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s.tag = None
        time.sleep(0.5)
        got = [x for x in s.samples if x[0] == tag][2:]  # skip the ramp
        pw = statistics.median(x[1] for x in got) if got else float("nan")
        ck = statistics.median(x[2] for x in got) if got else float("nan")
        rate = nbytes * reps / dt / 1e12
        print(f"{tag:20s} {rate:6.2f} TB/s   package {pw:6.0f} W   sclk {ck:5.0f} MHz   "
              f"({len(got)} samples, {reps} reps)", flush=True)
    s.stop = True


if __name__ == "__main__":
    main()
