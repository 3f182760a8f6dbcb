"""Multi-rank path of bench.py on CPU (gloo, world_size 2).

Each rank owns an independent shard of blocks (no data-path collective); the
only collectives are the barrier and the max-over-ranks time reduction.  The
per-block work here is done by the CPU oracle (test infrastructure) so the
sharding, the reduction and the goodput arithmetic can be checked without a
GPU: every block's parity/recovery must be identical whichever rank owns it.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from golden.synth import erasure_pattern, synth_block
from oracle_lib import Oracle

K, E, L, BPR = 8, 4, 256, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = Oracle()
    blk0, nb = bench.shard(rank, BPR)
    res = {}
    for b in range(blk0, blk0 + nb):
        data = list(synth_block(11, b, K, L))
        par = orc.encode_block(data, E)
        err = erasure_pattern(11, b, K, E)
        rc, rec = orc.decode_block(data, par, err)
        assert rc == 0 and all((rec[i] == data[err[i]]).all() for i in range(E))
        res[b] = np.stack(par)
    elapsed = 0.5 + rank  # rank 1 is the slow one
    dist.barrier()
    t = bench.reduce_max_time(elapsed, world, torch.device("cpu"))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), t=t, blocks=np.array(sorted(res)),
             **{f"b{b}": v for b, v in res.items()})
    dist.destroy_process_group()


def test_two_rank_shards_and_max_time(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = np.load(tmp_path / "r0.npz")
    r1 = np.load(tmp_path / "r1.npz")
    # shards are disjoint and cover [0, world*BPR)
    assert sorted(list(r0["blocks"]) + list(r1["blocks"])) == list(range(world * BPR))
    # both ranks agree on the job time = slowest rank
    assert float(r0["t"]) == float(r1["t"]) == 1.5
    # a block's parity does not depend on which rank computed it
    orc = Oracle()
    for r in (r0, r1):
        for b in r["blocks"]:
            ref = np.stack(orc.encode_block(list(synth_block(11, int(b), K, L)), E))
            assert (r[f"b{b}"] == ref).all()
    # goodput arithmetic: all ranks' bytes / max time
    g = bench.job_goodput(2.0 * E * L * BPR, 1, world, 1.5)
    assert abs(g - 2 * 2.0 * E * L * BPR / 1.5 / 2 ** 30) < 1e-12


def test_single_rank_reduce_is_identity():
    assert bench.reduce_max_time(0.25, 1, torch.device("cpu")) == 0.25
    assert bench.shard(3, 1024) == (3072, 1024)


@pytest.mark.parametrize("total,world", [(2500, 2), (2500, 3), (7, 8), (1 << 20, 8), (5, 1)])
def test_split_covers_every_block_once(total, world):
    """C4's 2^20 blocks (or any --blocks) over the ranks: contiguous, disjoint
    shares that cover every block; sizes differ by at most one (no remainder
    is dropped)."""
    shares = [bench.split(total, r, world) for r in range(world)]
    owned = [b for b0, n in shares for b in range(b0, b0 + n)]
    assert owned == list(range(total))
    sizes = [n for _, n in shares]
    assert max(sizes) - min(sizes) <= 1
