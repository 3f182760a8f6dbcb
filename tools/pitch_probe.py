"""C3 encode / decode kernel times for several row pitches (a tool, not the
product): does the distance between rows in HBM matter?  Run on the GPU box
from the repo root:  python3 tools/pitch_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "storage-benchmarks_amd")]
import torch  # noqa: E402
import rsgpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    k, e, L, B = 64, 32, 1000000, 1024
    ctx = rsgpu.Context(0)
    ctx.set_torch_stream()
    pitches = [rsgpu.row_pitch(L), 1000448, 1001472, 1003520, 1 << 20, (1 << 20) + 256, (1 << 20) + 4096]
    for rep in range(reps):
        for p in pitches:
            enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=1, ctx=ctx, pitch=p)
            dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=1, ctx=ctx, pitch=p)
            for _ in range(2):
                enc.encode_all()
                dec.decode_all(enc)
            torch.cuda.synchronize()
            ctx.timing_read()
            ctx.timing_enable(True)
            for _ in range(5):
                enc.encode_all()
                dec.decode_all(enc)
            torch.cuda.synchronize()
            recs = ctx.timing_read()
            ctx.timing_enable(False)
            ok = dec.is_complete() and dec.verify_data(enc)
            t = {}
            for n, ms, _ in recs:
                t.setdefault(n, []).append(ms)
            print(rep, p, ok, {n: round(sorted(v)[len(v) // 2], 3) for n, v in t.items()}, flush=True)
            del enc, dec
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
