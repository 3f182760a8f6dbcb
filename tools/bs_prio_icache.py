#!/usr/bin/env python3
"""bs_prio_icache.py -- round 6 (a tool): run the C3 encode a few times with
each k_rs_bs priority instantiation (rsgpu_internal_set_bs_prio 0, 1, 3) so a
`rocprofv3 --pmc SQC_ICACHE_MISSES ...` pass over this process gives each
instantiation's instruction-cache counters (the kernel names differ by the
template argument)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))
import torch  # noqa: E402
import rsgpu  # noqa: E402

ctx = rsgpu.Context(0)
ctx.set_torch_stream()
enc = rsgpu.GpuEncoder(64, 1000000, 32, blocks=1024, seed=1, ctx=ctx)
f = rsgpu.testhooks().rsgpu_internal_set_bs_prio
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
for v in (0, 1, 3):
    assert f(ctx._h, v) == 0
    for _ in range(3):
        enc.encode_all()
    torch.cuda.synchronize()
print("ok")
