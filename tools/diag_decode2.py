"""Syndrome-path decode: pattern-dependence vs block-index dependence (debug)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rsgpu  # noqa: E402

ctx = rsgpu.Context(0)
ctx.set_torch_stream()
k, e, L = 64, 32, 4096
for B, blk0 in [(1, 0), (1, 1), (2, 0), (2, 1), (4, 0)]:
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=3, ctx=ctx, block0=blk0)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=3, ctx=ctx, block0=blk0)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    res = []
    for b in range(B):
        want = enc.source_rows(b)
        got = dec.recovered_rows(b)
        ok = all((got[i] == want[j]).all() for i, j in enumerate(dec.err_host[b]))
        res.append((b, ok, list(dec.err_host[b][:6])))
    print("B", B, "block0", blk0, res, flush=True)
