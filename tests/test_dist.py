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


def _default_backend_worker(rank, world, port, outdir):
    """bench.init_dist with bench.py's default arguments: a gloo group, no
    GPU call before it (RCCL never initialised)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    args = bench.parse(["--gpus", str(world)])
    store, red = bench.init_dist(args, world, rank)
    info = {"backend": dist.get_backend(), "red": str(red), "cuda_init": torch.cuda.is_initialized(),
            "nccl_avail_used": dist.is_nccl_available() and dist.get_backend() == "nccl",
            "store": store is not None}
    t = bench.reduce_max_time(0.5 + rank, world, red)
    info["t"] = t
    dist.destroy_process_group()
    np.save(os.path.join(outdir, f"d{rank}.npy"), np.array([repr(info)]))


def test_default_backend_is_gloo_and_touches_no_gpu(tmp_path):
    """the barrier / max-time / verification reductions
    run over gloo unless --dist-backend nccl is given, set up before any GPU
    call, so the driver's 8-rank start-up never depends on a multi-rank RCCL
    init."""
    assert bench.parse([]).dist_backend == "gloo"
    world = 2
    mp.spawn(_default_backend_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        info = eval(str(np.load(tmp_path / f"d{r}.npy")[0]))
        assert info["backend"] == "gloo" and info["red"] == "cpu" and info["store"]
        assert not info["cuda_init"] and not info["nccl_avail_used"]
        assert info["t"] == 1.5


def _failing_rank_worker(rank, world, port, outdir):
    """Rank 1 fails on its own; rank 0, waiting in a barrier, sees the
    closed connection and reports -- naming rank 1 first."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    args = bench.parse(["--gpus", str(world)])
    store, red = bench.init_dist(args, world, rank)
    try:
        if rank == 1:
            raise RuntimeError("simulated HIP error on rank 1")
        dist.barrier()
        raise AssertionError("barrier passed with rank 1 gone")
    except Exception as ex:
        rc, line = bench.report_failure(args, rank, world, store, ex, wait_s=20.0)
    if rank == 0:
        with open(os.path.join(outdir, "line.json"), "w") as f:
            f.write(__import__("json").dumps(line))
    os._exit(rc)  # no destroy: the peer is gone


def test_failed_rank_is_named_by_rank0(tmp_path):
    import json
    world = 2
    ctx = mp.start_processes(_failing_rank_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                             join=False, start_method="spawn")
    for p in ctx.processes:
        p.join(120)
    assert all(p.exitcode == 1 for p in ctx.processes), [p.exitcode for p in ctx.processes]
    line = json.loads((tmp_path / "line.json").read_text())
    assert line["value"] is None and line["verified"] is False and line["n_gpus"] == 2
    assert line["error"]["first"]["rank"] == 1
    assert "simulated HIP error on rank 1" in line["error"]["first"]["error"]
    assert sorted(line["error"]["failed_ranks"]) == [0, 1]


def test_bench_ranks_on_cpu_report_their_failure():
    """`bench.py --gpus 2` end to end on this GPU-less host: the spawned ranks
    set up gloo, then fail at their first GPU call; rank 0 prints ONE JSON
    line naming both ranks (the line the driver keeps instead of nothing)."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    line = json.loads(lines[0])
    assert line["value"] is None and sorted(line["error"]["failed_ranks"]) == [0, 1]
    assert line["config"]["dist_backend"] == "gloo"
    assert "nccl" not in r.stderr.lower()


def test_failed_rank_named_under_torch_distributed_run():
    """The driver's launcher: `torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2`.  Rank 1 fails right after the process group is up
    (--fail-rank 1) while rank 0 waits in a barrier; the launcher then stops
    the survivors.  Rank 0 still prints ONE JSON line naming rank 1 first."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2", "--fail-rank", "1",
           "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout + r.stderr[-3000:]
    line = json.loads(lines[0])
    assert line["value"] is None and line["error"]["first"]["rank"] == 1
    assert "injected failure on rank 1" in line["error"]["first"]["error"]
    assert 1 in line["error"]["failed_ranks"]
