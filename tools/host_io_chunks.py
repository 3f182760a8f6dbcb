"""Pipelined PCIe-inclusive rate (bench.host_io_pipelined) per chunk size,
C3 geometry, 64 blocks:  python3 tools/host_io_chunks.py [chunk ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402
import rsgpu  # noqa: E402


def main():
    chunks = [int(x) for x in sys.argv[1:]] or [2, 4, 8, 16]
    torch.cuda.set_device(0)
    ctx = rsgpu.Context(0)
    ctx.set_torch_stream()
    for c in chunks:
        r = bench.host_io_pipelined(rsgpu, ctx, 64, 32, 1000000, 64, seed=1, chunk=c)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
