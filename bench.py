#!/usr/bin/env python3
"""Batched JPEG decode benchmark (BASELINE.json metric: MPixels/s decoded, images/s, % HBM roofline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5|c1] [--batch B]

One step = one pass of the decode path (host header parse + plan, RST scan, Huffman, IDCT/colour)
over one batch of synthetic JPEGs whose bytes are already resident in HBM; RGB stays in HBM.
N>1: one process per GPU (torch.distributed.run), images sharded by rank (weak scaling: each rank
decodes its own batch of B images, BASELINE config 4 = 8 x config 2), no collective on the data
path; one all-gather of per-rank counters at the end (RCCL over xGMI).

Rank 0 prints one JSON line (contract in the task statement); "roofline" reports the dominant
kernel's algorithmic bytes / its hipEvent-measured average launch time against the 8 TB/s HBM
peak, and "cpu_baseline" the oracle (CPU restatement of the reference decoder) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "gpu-jpeg-decoder_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

CONFIGS = {
    # name: (width, height, subsampling, restart_rows, batch, description)
    "c1": (512, 512, "4:4:4", 0, 1, "512x512 4:4:4 q90, no RST (BASELINE config 1)"),
    "c2": (1920, 1080, "4:2:0", 1, 1024, "1024 x 1920x1080 4:2:0 q90, DRI = 1 MCU row (BASELINE config 2)"),
    "c3": (3840, 2160, "4:2:0", 1, 256, "256 x 3840x2160 4:2:0 q90, DRI = 1 MCU row (BASELINE config 3)"),
    "c5": (1920, 1080, "mixed", 0, 1024, "1024 x 1080p mixed 4:4:4/4:2:2/4:2:0, q in {50,75,90,95}, no RST "
                                         "(BASELINE config 5)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def measured_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC profile of this config
    (profiles/<round>_traffic.json, written by tools/profile_summary.py), or None."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        with open(f) as fh:
            t = json.load(fh)
        if t.get("config") == config and kernel in t.get("kernels", {}):
            return t["kernels"][kernel]["hbm_bytes"], os.path.relpath(f, ROOT)
    return None


def rank_seed(rank: int, batch: int) -> int:
    """First synthetic-image seed of a rank: ranks decode disjoint images (weak scaling)."""
    return rank * batch


def gather_counters(local, world: int):
    """One all-gather of the per-rank [elapsed, pixels, images, ecs bytes, file bytes] counters
    (RCCL over xGMI on the GPU box, gloo in tests/test_dist.py).  Returns (max elapsed, sums)."""
    import torch
    import torch.distributed as dist

    if world > 1:
        allc = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(allc, local)
        allc = torch.stack(allc).cpu().numpy()
    else:
        allc = local.cpu().numpy()[None]
    return float(allc[:, 0].max()), tuple(float(allc[:, k].sum()) for k in range(1, allc.shape[1]))


def cpu_baseline(hosts, hdrs, n_req: int, target_s: float = 12.0):
    """The oracle (CPU restatement of the reference decoder, full decode to RGB) on one core over a
    bounded sample of the same workload: n_req images, or (n_req < 0) as many as take ~target_s."""
    import jdoracle

    n = len(hosts)
    if n_req < 0:
        probe = min(n, 4)
        secs, _, _ = jdoracle.decode_many(hosts[:probe], threads=1, want_rgb=True)
        n_req = int(max(probe, min(n, target_s / max(secs / probe, 1e-6))))
    n_req = min(n_req, n)
    secs, st, _ = jdoracle.decode_many(hosts[:n_req], threads=1, want_rgb=True)
    if any(st):
        raise SystemExit(f"oracle failed on the CPU sample: {sorted(set(st))}")
    cpx = float(sum(h.width * h.height for h in hdrs[:n_req]))
    return {"value": cpx / secs / 1e6, "unit": "MPixels/s", "cores": 1, "kind": "port",
            "sample": f"first {n_req} of the workload's images decoded to RGB by oracle/liboracle.so "
                      f"(bit-serial Huffman, reference IDCT + colour), 1 thread, {secs:.2f} s",
            "images_per_s": n_req / secs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override images per rank")
    ap.add_argument("--quality", type=int, default=90)
    ap.add_argument("--cpu-sample", type=int, default=-1, help="images for the CPU baseline (-1 auto, 0 off)")
    ap.add_argument("--verify", type=int, default=2, help="images checked bit-exact vs the oracle")
    ap.add_argument("--path", default="auto", choices=["auto", "sync", "lanes", "full"],
                    help="entropy-decode path (auto: lanes for images with restart intervals)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one blocking jd_decode_batch per step instead of jd_decode_batch_async (which "
                         "parses and plans step k+1 on the host while the GPU decodes step k)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import numpy as np
    import torch
    import torch.distributed as dist

    # one process per GPU; JD_DIST_BACKEND=gloo with more ranks than GPUs rehearses the
    # multi-rank path on a one-GPU box (ranks then share devices round-robin)
    backend = os.environ.get("JD_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" or ndev == 0:
        device_index = local_rank
    else:
        device_index = local_rank % ndev
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(device_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", device_index)
    local_rank = device_index

    import jd_synth
    import jdamd

    W, H, ss, rrows, batch, desc = CONFIGS[args.config]
    if args.batch:
        batch = args.batch
    seed0 = rank_seed(rank, batch)  # disjoint images per rank: shard by image
    t_gen = time.time()
    datas = jd_synth.make_batch(batch, W, H, args.quality, "4:2:0" if ss == "mixed" else ss, rrows, 0, seed0,
                                mixed=(ss == "mixed"))
    t_gen = time.time() - t_gen
    hosts = [np.frombuffer(d, np.uint8).copy() for d in datas]
    hdrs = [jdamd.parse(d) for d in datas]
    in_offs, tot = [], 0
    for h in hosts:
        in_offs.append(tot)
        tot += (h.nbytes + 64 + 255) // 256 * 256
    out_offs, otot = [], 0
    for h in hdrs:
        out_offs.append(otot)
        otot += (h.width * h.height * 3 + 255) // 256 * 256
    # device memory through torch (plumbing); the decoder gets raw pointers over the C ABI
    jpeg_dev = torch.empty(tot, dtype=torch.uint8, device=dev)
    rgb_dev = torch.empty(otot, dtype=torch.uint8, device=dev)
    flat = np.zeros(tot, np.uint8)
    for h, o in zip(hosts, in_offs):
        flat[o:o + h.nbytes] = h
    jpeg_dev.copy_(torch.from_numpy(flat))
    torch.cuda.synchronize(dev)

    dec = jdamd.Decoder(local_rank, timing=True, path=args.path)
    prepared = dec.make_batch(hosts, [jpeg_dev.data_ptr() + o for o in in_offs],
                              [rgb_dev.data_ptr() + o for o in out_offs])
    pixels = float(sum(h.width * h.height for h in hdrs))
    ecs = float(sum(len(d) - h.ecs_offset for d, h in zip(datas, hdrs)))
    jpeg_bytes = float(sum(len(d) for d in datas))

    pipelined = not args.no_pipeline
    for _ in range(args.warmup):
        dec.decode_prepared(prepared, pipelined=pipelined)
    dec.wait()
    status = [r.status for r in prepared[1]]
    if any(status):
        raise SystemExit(f"decode failed: statuses {sorted(set(status))}")

    # correctness spot check against the oracle (outside the timed region)
    verified = 0
    if args.verify:
        import jdoracle

        for i in range(min(args.verify, batch)):
            h = hdrs[i]
            got = rgb_dev[out_offs[i]:out_offs[i] + h.width * h.height * 3].cpu().numpy().reshape(h.height, h.width, 3)
            st, ref = jdoracle.decode(datas[i])
            if st != 0 or not np.array_equal(got, ref):
                raise SystemExit(f"bit-exactness check failed on image {i}")
            verified += 1

    dec.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dec.decode_prepared(prepared, pipelined=pipelined)
    dec.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if any(r.status for r in prepared[1]):  # the last timed batch's per-image statuses
        raise SystemExit("decode failed inside the timed region")
    st = dec.stats()

    # one all-gather of per-rank counters (RCCL over xGMI when N > 1)
    local = torch.tensor([elapsed, pixels * args.steps, batch * args.steps, ecs * args.steps,
                          jpeg_bytes * args.steps], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
    t_max, (tot_px, tot_img, tot_ecs, tot_bytes) = gather_counters(local, world)

    if rank == 0:
        kern = st["kernels"]
        dom = max(kern, key=lambda k: kern[k]["total_ms"])
        traffic = measured_traffic(args.config, dom)
        kd = kern[dom]
        avg_ms = kd["total_ms"] / max(1, kd["launches"])
        per_launch_bytes = kd["bytes"] / max(1, kd["launches"])
        achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        cpu = None
        if args.cpu_sample and world == 1:  # the CPU baseline is an N=1 figure
            cpu = cpu_baseline(hosts, hdrs, args.cpu_sample)
        res = {
            "metric": "MPixels/s decoded (and images/s) at 1/2/4/8 MI355X; % HBM roofline",
            "value": tot_px / t_max / 1e6,
            "unit": "MPixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic (seeded sinusoid + noise, baseline encode q{args.quality} by "
                    f"{'tools/jdenc.c' if jd_synth.default_encoder() == 'jdenc' else 'Pillow'}, std Huffman tables)",
            "config": {"workload": desc, "config": args.config, "images_per_rank": batch,
                       "global_batch": batch * world, "width": W, "height": H, "subsampling": ss,
                       "restart_rows": rrows, "parallelism": f"dp{world} (image sharding)",
                       "entropy_path": args.path, "host_pipelined": pipelined},
            "images_per_s": tot_img / t_max,
            "jpeg_MB_per_s": tot_bytes / t_max / 1e6,
            "ecs_MB_per_s": tot_ecs / t_max / 1e6,
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic[0] if traffic else None,
                         "traffic_source": traffic[1] if traffic else None,
                         "avg_launch_ms": avg_ms, "algorithmic_bytes_per_launch": per_launch_bytes},
            "kernels_ms_per_step": {k: v["total_ms"] / max(1, v["launches"]) for k, v in kern.items()},
            "path_roofline_frac": ((ecs + 3 * pixels) / (t_max / args.steps) / 1e9) / HBM_PEAK_GBS,
            "cpu_baseline": cpu,
            "verified_bit_exact": verified,
            "gen_s": t_gen,
        }
        print(json.dumps(res))
    dec.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
