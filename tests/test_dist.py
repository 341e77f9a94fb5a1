"""Multi-process path of bench.py on CPU: gloo, world_size 2.

The decode path shards by image (no data-path collective); the only collective is one all-gather
of per-rank counters, after which rank 0 reports max-over-ranks time and summed work.  Here the
same functions bench.py uses run under gloo with two ranks.
"""
import hashlib
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import jd_synth

    seed0 = bench.rank_seed(rank, batch)
    datas = jd_synth.make_batch(batch, 64, 48, 90, "4:2:0", 1, 0, seed0, workers=1)
    digests = [hashlib.sha1(d).hexdigest() for d in datas]
    elapsed = 1.0 + rank  # rank 1 is the slow one
    local = torch.tensor([elapsed, 64 * 48 * batch, batch, 100.0 * (rank + 1), 7.0], dtype=torch.float64)
    t_max, sums = bench.gather_counters(local, world)
    q.put((rank, digests, t_max, sums))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_sharding_and_counter_gather_gloo():
    world, batch = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out.sort()
    d0, d1 = set(out[0][1]), set(out[1][1])
    assert len(d0) == batch and len(d1) == batch and not (d0 & d1), "ranks must decode disjoint images"
    for _, _, t_max, sums in out:
        assert t_max == 2.0                      # max over ranks, not rank 0's own clock
        assert sums[0] == 2 * 64 * 48 * batch    # pixels summed over ranks
        assert sums[1] == 2 * batch
        assert sums[2] == 300.0
        assert sums[3] == 14.0
