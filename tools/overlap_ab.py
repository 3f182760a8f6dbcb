"""tools/overlap_ab.py [groups] -- pipelining experiment (tool, not product): decode of block group i beside encode of group i+1
(two contexts, two streams) vs the plain step, C3."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "storage-benchmarks_amd"))
import torch, rsgpu
dev = torch.device("cuda", 0)
k, e, L, B = 64, 32, 1000000, 1024
G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ce, cd = rsgpu.Context(0), rsgpu.Context(0)
se, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ce.set_stream(se.cuda_stream); cd.set_stream(sd.cuda_stream)
enc = rsgpu.GpuEncoder(k, L, e, blocks=B, seed=1, ctx=ce)
dec = rsgpu.GpuDecoder(k, L, e, blocks=B, seed=1, ctx=cd)
torch.cuda.synchronize()
P = enc.pitch
nb = B // G
wsz = rsgpu.decode_workspace_bytes(k, e, nb)
ws = [torch.empty(wsz, dtype=torch.uint8, device=dev) for _ in range(G)]

def plain():
    enc.encode_all()
    torch.cuda.synchronize()
    dec.decode_all(enc)
    torch.cuda.synchronize()

def piped():
    evs = [torch.cuda.Event() for _ in range(G)]
    for g in range(G):
        s0 = g * nb
        ce.encode_blocks(k, e, L, P, nb, enc.src.view(-1)[s0 * k * P:], enc.par.view(-1)[s0 * e * P:])
        evs[g].record(se)
    for g in range(G):
        s0 = g * nb
        sd.wait_event(evs[g])
        cd.decode_blocks(k, e, L, P, nb, enc.src.view(-1)[s0 * k * P:], enc.par.view(-1)[s0 * e * P:],
                         dec.err.view(-1)[s0 * e:], dec.out.view(-1)[s0 * e * P:], ws[g], dec.status.view(-1)[s0:])
    torch.cuda.synchronize()

for f in (plain, piped, plain, piped):
    f()
    t = time.perf_counter()
    for _ in range(5):
        f()
    dt = (time.perf_counter() - t) / 5
    print(f.__name__, G, f"{dt*1e3:.2f} ms/step", f"{2*e*L*B/dt/2**30:.1f} GiB/s", flush=True)
print("verified", dec.is_complete() and dec.verify_data(enc))
