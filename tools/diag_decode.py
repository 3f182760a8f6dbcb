"""Decode round trips for a list of shapes, printing verify per shape (debug
tool).  usage: python tools/diag_decode.py  [RSGPU_NO_TC=1 to use k_dot_generic]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "storage-benchmarks_amd"))
import torch  # noqa: E402
import rsgpu  # noqa: E402

ctx = rsgpu.Context(0)
ctx.set_torch_stream()
for k, e, L, B in [(64, 32, 4096, 2), (64, 32, 1000000, 2), (64, 32, 32000, 8), (100, 20, 4096, 2),
                   (64, 16, 4096, 2), (16, 8, 4096, 2), (64, 32, 2048, 1), (64, 32, 6144, 1)]:
    enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=3, ctx=ctx)
    enc.encode_all()
    dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=3, ctx=ctx)
    dec.decode_all(enc)
    torch.cuda.synchronize()
    bad = []
    for b in range(B):
        want = enc.source_rows(b)
        got = dec.recovered_rows(b)
        if got is not None:
            errs = dec.err_host[b]
            for i, j in enumerate(errs):
                if not (got[i] == want[j]).all():
                    nz = (got[i] != want[j]).nonzero()[0]
                    bad.append((b, i, int(j), len(nz), int(nz[0])))
    print(k, e, L, B, "complete", dec.is_complete(), "verify", dec.verify_data(enc), bad[:6],
          flush=True)
