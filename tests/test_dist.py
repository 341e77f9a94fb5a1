"""Multi-process path of bench.py on CPU: gloo, world_size 2.

The decode path shards by image (no data-path collective); the only collective is one all-gather
of per-rank counters, after which rank 0 reports max-over-ranks time and summed work.  Here
bench.py's own rank/device selection (dist_setup), shard assignment (shard_seeds), host-thread
split (host_threads) and counter all-gather run under gloo with two ranks.
"""
import hashlib
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "gpu-jpeg-decoder_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, q):
    for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "gpu-jpeg-decoder_amd")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), JD_DIST_BACKEND="gloo")
    import bench
    import jd_synth

    d = bench.dist_setup()
    threads, info = bench.host_threads(d)
    seeds_c2 = bench.shard_seeds("c2", batch, d["rank"], d["world"])
    seeds_c5 = bench.shard_seeds("c5", batch, d["rank"], d["world"])
    jobs = jd_synth.make_jobs(seeds_c2, 64, 48, 90, "4:2:0", 1, 0)
    digests = [hashlib.sha1(x).hexdigest() for x in jd_synth.make_images(jobs, workers=1)]
    elapsed = 1.0 + rank  # rank 1 is the slow one
    local = torch.tensor([elapsed, 64 * 48 * batch, batch, 100.0 * (rank + 1), 7.0], dtype=torch.float64)
    t_max, sums = bench.gather_counters(local, world)
    mat = bench.gather_matrix(torch.tensor([float(rank), float(len(seeds_c5))], dtype=torch.float64), world)
    # the bench's real per-rank vector: rank 1 is host-bound (slow parse + plan, slow e2e leg)
    host = {"parse": 0.5 + 2.0 * rank, "plan": 0.25 + rank, "stage_inputs": 1.0, "wait": 0.1}
    vec = bench.rank_vector(2.0 + rank, 64 * 48, batch, 1000.0, 1500.0, 10, host, 20.0 + 5 * rank, 50.0 - rank,
                            12.0 + rank, 11.5 + rank)
    full = bench.gather_matrix(torch.tensor(vec, dtype=torch.float64), world)
    table = bench.per_rank_table(full, 10)
    # rank 0's single-host measurements after the gather, the other rank waiting at the barrier
    # (an N > 1 line carries the CPU baseline and the copy peak)
    calls = []
    extra = bench.rank0_measurements(d["rank"], d["world"], copy_fn=lambda: calls.append("copy") or 5650.0,
                                     cpu_fn=lambda: calls.append("cpu") or {"value": 1750.0, "cores": 16})
    kern = {"k_piece": {"launches": 3, "total_ms": 8.4, "bytes": 3 * 2.3e9},
            "k_idct_color": {"launches": 3, "total_ms": 8.45, "bytes": 3 * 8.1e9},
            "k_scan": {"launches": 3, "total_ms": 0.6, "bytes": 3 * 0.65e9}}
    roof = bench.roofline_block(kern, "c2", extra["copy_peak"], 3) if d["rank"] == 0 else None
    # within 1 % by hipEvents: the committed rocprof averages decide
    roof_rp = bench.roofline_block(kern, "c2", extra["copy_peak"], 3, {"k_piece": 2.95, "k_idct_color": 2.90})
    line = {"cpu_baseline": extra["cpu_baseline"], "roofline": roof} if d["rank"] == 0 else None
    q.put((rank, d, threads, info, seeds_c2, seeds_c5, digests, t_max, sums, mat.tolist(), table, full.tolist(),
           calls, line, roof_rp["kernel"]))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_rank_setup_sharding_and_counter_gather_gloo():
    world, batch = 2, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    for rank, d, threads, info, _, _, _, t_max, sums, mat, table, full, calls, line, picked in out:
        assert d["world_seen"] == world and d["rank"] == rank and d["backend"] == "gloo"
        assert d["device_index"] == rank  # one device per local rank (no GPU here: index only)
        assert 1 <= threads <= bench_share() and info["rank_cpus"] >= 1
        assert t_max == 2.0                      # max over ranks, not rank 0's own clock
        assert sums[0] == 2 * 64 * 48 * batch    # pixels summed over ranks
        assert sums[1] == 2 * batch
        assert sums[2] == 300.0
        assert sums[3] == 14.0
        assert [r[0] for r in mat] == [0.0, 1.0] and sum(r[1] for r in mat) == world * batch
        # per-rank diagnostics: every rank's row, in rank order
        assert table["ms_per_step"] == [200.0, 300.0]
        assert table["parse_ms"] == [0.5, 2.5] and table["plan_ms"] == [0.25, 1.25]
        assert table["stage_ms"] == [1.0, 1.0] and table["wait_ms"] == [0.1, 0.1]
        assert table["e2e_ms"] == [20.0, 25.0] and table["h2d_GB_s"] == [50.0, 49.0]
        assert table["e2e_registered_ms"] == [12.0, 13.0]  # each H2D leg on its own, no best-of
        assert table["e2e_pinned_arena_ms"] == [11.5, 12.5]
        if rank == 0:  # the 2-rank line carries the CPU baseline and the in-run copy peak
            assert calls == ["copy", "cpu"]
            assert line["cpu_baseline"]["value"] == 1750.0
            assert line["roofline"]["measured_copy_peak"] == 5650.0
            assert line["roofline"]["kernel"] == "k_idct_color" and line["roofline"]["co_dominant"]["kernel"] == "k_piece"
            assert line["roofline"]["frac_of_measured_peak"] > 0
        else:
            assert calls == [] and line is None
        assert picked == "k_piece"
        assert table["host_parse_plan_over_step"] == [round(0.75 / 200.0, 4), round(3.75 / 300.0, 4)]
        assert max(r[0] for r in full) == 3.0 and sum(r[1] for r in full) == 2 * 64 * 48 * 10
    d0, d1 = set(out[0][6]), set(out[1][6])
    assert len(d0) == batch and len(d1) == batch and not (d0 & d1), "ranks must decode disjoint images"
    c2 = [set(o[4]) for o in out]
    assert not (c2[0] & c2[1]) and c2[0] | c2[1] == set(range(world * batch))
    c5 = [set(o[5]) for o in out]
    assert not (c5[0] & c5[1]) and c5[0] | c5[1] == set(range(world * batch))
    assert all(len(s) == batch for s in c5)


def bench_share():
    import bench

    return bench.BOX_CPU_SHARE


def test_mixed_shards_balance_entropy_bytes():
    """C5-style mixed batch at 1080p (sizes vary 5x by subsampling and quality): the greedy
    assignment by estimated ECS bytes balances the ranks' real encoded bytes better than
    contiguous seed ranges."""
    import bench
    import jd_synth

    world, batch = 4, 6
    seeds = range(world * batch)
    sizes = {s: len(b) for s, b in zip(seeds, jd_synth.make_images(jd_synth.make_jobs(seeds, 1920, 1080, mixed=True)))}
    greedy = [sum(sizes[s] for s in bench.shard_seeds("c5", batch, r, world)) for r in range(world)]
    contiguous = [sum(sizes[s] for s in range(r * batch, (r + 1) * batch)) for r in range(world)]
    assert sorted(s for r in range(world) for s in bench.shard_seeds("c5", batch, r, world)) == list(seeds)
    imb = lambda v: max(v) / np.mean(v)  # noqa: E731
    assert imb(greedy) <= 1.08, greedy
    assert imb(greedy) <= imb(contiguous), (greedy, contiguous)
