#!/usr/bin/env python3
"""Batched JPEG decode benchmark (BASELINE.json metric: MPixels/s decoded, images/s, % HBM roofline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c5|c1] [--batch B]

One step = one pass of the decode path (host header parse + plan, RST scan, Huffman, IDCT/colour)
over one batch of synthetic JPEGs whose bytes are already resident in HBM; RGB stays in HBM.
N>1: one process per GPU (torch.distributed.run; `--gpus N` without a launcher starts one itself),
images sharded by rank (weak scaling: each rank decodes its own batch of B images, BASELINE
config 4 = 8 x config 2; mixed batches are balanced by estimated entropy-coded bytes), no
collective on the data path; one all-gather of per-rank counters at the end (RCCL over xGMI).

Rank 0 prints one JSON line (contract in the task statement) with, besides the contract keys:
  roofline      the dominant kernel's algorithmic bytes / its hipEvent-measured average launch time
                against the 8 TB/s HBM peak, the same against an in-run copy-kernel peak (the
                library's 16-byte-per-lane copy, jd_test_copy_peak), its HBM traffic and VALU issue
                fraction from the committed PMC profiles (profiles/); `bound` names the roof that
                binds it: "valu" when the committed SQ profile's VALU issue model (instructions x 4
                cycles, below) exceeds 0.7, "hbm" when the kernel streams above half the HBM peak,
                else "latency" (neither roof: a dependency- or parallelism-bound launch).  When the
                two largest kernels are within 5 % of each other, `roofline.co_dominant` gives the
                second one's figures too
  e2e_h2d       the same batch with the JPEG bytes handed over in host memory (PCIe-inclusive,
                pipelined: host staging of batch k+1 overlaps the GPU's batch k), next to an in-run
                pinned H2D rate of the same byte count
  per_rank      every rank's step time, host phase times (parse, plan, input staging, wait) and its
                concurrent e2e_h2d leg, from the one all-gather (shows whether the host feed binds)
  cpu_baseline  the reference's own CPU decoder (oracle/_ref/ref_bench, built from its sources) on
                the BASELINE config-1 image, and the oracle (the CPU restatement, which also decodes
                4:2:0 / RST) on a bounded sample of this workload, 1 core and all cores, with the
                port/reference calibration ratio (reference time: cpp-decoder/benchmark/benchmark.cc:29-35)
"""
import argparse
import glob
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
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
    # the reference's own benchmark format (4:4:4 q95: data_preprocessing/image_converter.py:6,18) at
    # its latency-benchmark sizes 200^2 .. 2000^2 (cuda-decoder/benchmark/benchmark.cu:87), image i
    # of size REF_SIZES[i % 10], in its throughput benchmark's batch of 3000
    # (cuda-decoder/benchmark_thoughput/benchmark.cu:30); --sweep adds its two published curves
    "ref444": (0, 0, "ref", 0, 3000, "3000 x 4:4:4 q95, sizes 200^2..2000^2 cycling, no RST (the reference's "
                                     "benchmark format)"),
    # config 2 with libjpeg's fancy upsampling (JD_FLAG_FANCY_UPSAMPLING; --fancy on any config)
    "c2f": (1920, 1080, "4:2:0", 1, 1024, "1024 x 1920x1080 4:2:0 q90, DRI = 1 MCU row, fancy upsampling "
                                          "(BASELINE config 2 shape, an option beyond the reference)"),
}
REF_SIZES = (200, 400, 600, 800, 1000, 1200, 1400, 1600, 1800, 2000)  # cuda-decoder/benchmark/benchmark.cu:87
REF_QUALITY = 95                                                      # data_preprocessing/image_converter.py:6
REF_BATCHES = (1, 10, 50, 100, 250, 500, 1000, 3000)                  # figures/batchsize.pdf's range
REF_PUBLISHED_MB_S = 552.0  # CUDA decoder, batch 3000, RTX 2080 Ti, kernel time only
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SIMDS = 1024               # 256 CUs x 4 SIMD-32
# SQ_ACTIVE_INST_VALU counts quad-cycles (MI355X_MICROARCH.md); on gfx950 most 32-bit integer VALU
# instructions (shifts, bfe, mad24, cndmask, perm, packed 16-bit, med3) issue at one wave64 per 4
# cycles, v_add/v_and/v_add_f32 at ~2 (tools/micro/valurate.hip)
VALU_CYCLES_PER_QUAD = 4
BOX_CPU_SHARE = 16         # CPUs a one-GPU share of the box gets (task environment)


# ---------------------------------------------------------------------------------------------
# launch, ranks, shards
# ---------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def maybe_launch(args):
    """`--gpus N` without a launcher: start torch.distributed.run with N ranks as a child process
    (nothing has touched the GPU yet) and return its exit code; None when this process is a rank."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)]
        cmd += sys.argv[1:]
        return subprocess.call(cmd)
    if int(world_env) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")
    return None


def dist_setup():
    """Rank / device selection and process-group init (one process per GPU).  JD_DIST_BACKEND=gloo
    with more ranks than GPUs rehearses the multi-rank path on a one-GPU box (ranks then share
    devices round-robin).  Returns a dict; 'world_seen' is the process group's own size."""
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    backend = os.environ.get("JD_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    device_index = local_rank if (backend == "nccl" or ndev == 0) else local_rank % ndev
    world_seen = 1
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if ndev:
            torch.cuda.set_device(device_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device_index))
        else:
            dist.init_process_group(backend)
        world_seen = dist.get_world_size()
        if world_seen != world:
            raise SystemExit(f"process group has {world_seen} ranks, WORLD_SIZE={world}")
    return {"rank": rank, "world": world, "local_rank": local_rank, "local_world": local_world,
            "backend": backend if world > 1 else "none", "device_index": device_index, "world_seen": world_seen}


def rank_seed(rank: int, batch: int) -> int:
    """First synthetic-image seed of a rank: ranks decode disjoint images (weak scaling)."""
    return rank * batch


def shard_seeds(config: str, batch: int, rank: int, world: int):
    """The global image seeds rank `rank` decodes.  Uniform configs: a contiguous range of `batch`
    seeds per rank.  Mixed batches (C5) vary 5x in size per image, so the world * batch images are
    assigned greedily, largest estimated entropy-coded size first, to the least-loaded rank
    (SURVEY.md §8e); sizes come from jd_synth's per-(subsampling, quality) model, so every rank
    computes the same assignment without encoding the others' images."""
    import jd_synth

    W, H, ss, _, _, _ = CONFIGS[config]
    if ss != "mixed" or world == 1:
        s0 = rank_seed(rank, batch)
        return list(range(s0, s0 + batch))
    est = [(jd_synth.estimated_bytes(W, H, *jd_synth.mixed_params(g)), g) for g in range(world * batch)]
    est.sort(key=lambda t: (-t[0], t[1]))
    load = [0.0] * world
    count = [0] * world
    mine = []
    for b, g in est:
        r = min((k for k in range(world) if count[k] < batch), key=lambda k: (load[k], k))
        load[r] += b
        count[r] += 1
        if r == rank:
            mine.append(g)
    return sorted(mine)


def ref444_jobs(seeds, quality: int = REF_QUALITY):
    """jd_synth jobs of the ref444 workload: image `seed` is REF_SIZES[seed % 10] square, 4:4:4, no DRI."""
    return [(REF_SIZES[s % len(REF_SIZES)], REF_SIZES[s % len(REF_SIZES)], int(s), quality, "4:4:4", 0, 0, None)
            for s in seeds]


def numa_cpus(device_index: int):
    """Host CPUs of the GPU's NUMA node that this process may run on (None if unknown)."""
    try:
        import torch

        pr = torch.cuda.get_device_properties(device_index)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        node = int(open(f"/sys/bus/pci/devices/{bdf}/numa_node").read())
        if node < 0:
            return None
        cpus = set()
        for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        mine = cpus & os.sched_getaffinity(0)
        return sorted(mine) or None
    except Exception:
        return None


def host_threads(d):
    """Parse/plan workers for this rank: a slice of the CPUs of its GPU's NUMA node (or of all it
    may use), one slice per local rank on that node, at most the box's one-GPU share; with several
    ranks the process is pinned to its slice so the ranks' workers do not compete."""
    allowed = sorted(os.sched_getaffinity(0))
    lw = max(1, d["local_world"])
    node = numa_cpus(d["device_index"]) if d["world"] > 1 else None
    if node:  # the local ranks whose GPUs sit on this node share its CPUs (GPUs spread evenly)
        share = max(1, min(lw, round(lw * len(node) / len(allowed))))
        per = max(1, len(node) // share)
        k = d["local_rank"] % share
        mine = node[k * per:(k + 1) * per]
    else:
        per = max(1, len(allowed) // lw)
        k = d["local_rank"] % lw
        mine = allowed[k * per:(k + 1) * per] or allowed
    threads = max(1, min(BOX_CPU_SHARE, len(mine)))
    if d["world"] > 1:
        try:
            os.sched_setaffinity(0, mine)
        except OSError:
            pass
    return threads, {"cpus_allowed": len(allowed), "numa_node_cpus": len(node) if node else None,
                     "rank_cpus": len(mine), "parse_threads": threads}


def gather_matrix(local, world: int):
    """One all-gather of the per-rank counter vector (RCCL over xGMI on the GPU box, gloo in
    tests/test_dist.py); returns a [world, k] numpy array."""
    import torch
    import torch.distributed as dist

    if world > 1:
        allc = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(allc, local)
        return torch.stack(allc).cpu().numpy()
    return local.cpu().numpy()[None]


RANK_FIELDS = ["elapsed_s", "pixels", "images", "ecs_bytes", "jpeg_bytes", "ecs_bytes_per_step",
               "images_per_step", "ms_per_step", "parse_ms", "plan_ms", "stage_ms", "wait_ms", "e2e_ms",
               "h2d_GB_s", "e2e_registered_ms", "e2e_pinned_arena_ms"]


def rank_vector(elapsed, pixels, n, ecs, jpeg_bytes, steps, host_ms_step, e2e_ms, h2d_gbs, reg_ms=0.0,
                arena_ms=0.0):
    """This rank's counter vector for the one all-gather (order: RANK_FIELDS; column 0 = elapsed
    is max-reduced, 1-4 summed).  The three H2D-inclusive legs (staged, registered arena, pinned
    arena) are reported separately, each from its own timed run."""
    return [elapsed, pixels * steps, n * steps, ecs * steps, jpeg_bytes * steps, ecs, n,
            elapsed / max(1, steps) * 1e3, host_ms_step.get("parse", 0.0), host_ms_step.get("plan", 0.0),
            host_ms_step.get("stage_inputs", 0.0), host_ms_step.get("wait", 0.0), e2e_ms, h2d_gbs, reg_ms,
            arena_ms]


def per_rank_table(allc, steps):
    """Per-rank diagnostics from the gathered matrix: step time, host phases per step (parse, plan,
    input staging, time blocked waiting for the GPU), the concurrent e2e_h2d leg and pinned H2D rate."""
    keys = RANK_FIELDS[7:]
    out = {k: [round(float(x), 4) for x in allc[:, RANK_FIELDS.index(k)]] for k in keys}
    host = allc[:, 8] + allc[:, 9]
    out["host_parse_plan_over_step"] = [round(float(h / m), 4) if m > 0 else None for h, m in zip(host, allc[:, 7])]
    return out


def rank0_measurements(rank: int, world: int, copy_fn=None, cpu_fn=None):
    """The line's single-host measurements, run by rank 0 only and after the counter all-gather (so
    they never overlap any rank's timed region): the in-run HBM copy peak on rank 0's GPU and the
    CPU baseline on rank 0's host cores (north_star: the reference's CPU decoder "in the same run",
    at any world size).  The other ranks wait at a barrier meanwhile, so no rank's GPU or host work
    competes with them.  Returns {"copy_peak": GB/s or None, "cpu_baseline": dict or None}."""
    import torch.distributed as dist

    out = {"copy_peak": None, "cpu_baseline": None}
    if rank == 0:
        if copy_fn is not None:
            out["copy_peak"] = copy_fn()
        if cpu_fn is not None:
            out["cpu_baseline"] = cpu_fn()
    if world > 1:
        dist.barrier()
    return out


def roofline_block(kern: dict, config: str, copy_gbs, kernel_steps: int, rocprof_ms=None):
    """The line's `roofline` object for the dominant kernel slot: algorithmic bytes per launch over
    its average hipEvent launch time against the 8 TB/s HBM peak and the in-run copy peak, its PMC
    traffic and VALU issue model.  When the two largest slots are within 1 % by hipEvents, the
    committed rocprofv3 averages (`rocprof_ms`, profiles/*_kernel_stats.csv) pick the dominant one;
    within 5 %, `co_dominant` gives the runner-up's figures too."""
    by_time = sorted((k for k in kern if kern[k]["launches"]), key=lambda k: kern[k]["total_ms"] / kern[k]["launches"],
                     reverse=True)
    avg = {k: kern[k]["total_ms"] / max(1, kern[k]["launches"]) for k in by_time}
    if (len(by_time) > 1 and rocprof_ms and by_time[0] in rocprof_ms and by_time[1] in rocprof_ms
            and avg[by_time[1]] >= 0.99 * avg[by_time[0]] and rocprof_ms[by_time[1]] > rocprof_ms[by_time[0]]):
        by_time[0], by_time[1] = by_time[1], by_time[0]
        picked = "rocprofv3 averages (hipEvent times within 1 %)"
    else:
        picked = "hipEvent averages"

    def figures(name):
        k = kern[name]
        ms = avg[name]
        b = k["bytes"] / max(1, k["launches"])
        a = b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        vb = valu_issue(config, name, ms)
        tr = measured_traffic(config, name)
        bound = "valu" if vb and vb["busy_frac"] > 0.7 else "hbm" if a / HBM_PEAK_GBS > 0.5 else "latency"
        return ms, b, a, vb, tr, bound

    dom = by_time[0]
    ms, b, a, vb, tr, bound = figures(dom)
    co_dom = None
    if len(by_time) > 1 and avg[by_time[1]] >= 0.95 * ms:
        ms2, b2, a2, vb2, tr2, bound2 = figures(by_time[1])
        co_dom = {"kernel": by_time[1], "avg_launch_ms": ms2, "algorithmic_bytes_per_launch": b2, "achieved": a2,
                  "frac": a2 / HBM_PEAK_GBS, "traffic": tr2[0] if tr2 else None, "valu": vb2, "bound": bound2}
    # the roof that binds: VALU issue when the committed SQ profile shows the SIMDs busy, HBM when the
    # byte stream is near its peak, else neither (a latency- / parallelism-bound launch, e.g. C1's
    # one image on a few CUs)
    return {"bound": bound, "kernel": dom, "kernel_picked_by": picked, "achieved": a, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": a / HBM_PEAK_GBS, "traffic": tr[0] if tr else None,
            "traffic_source": tr[1] if tr else None, "measured_copy_peak": copy_gbs,
            "frac_of_measured_peak": a / copy_gbs if copy_gbs else None, "valu": vb, "avg_launch_ms": ms,
            "algorithmic_bytes_per_launch": b,
            "timing": f"hipEvents on the decode stream, {max(1, kernel_steps)} serialized batches",
            "co_dominant": co_dom}


def rocprof_averages(config: str):
    """Per kernel slot: the average duration (ms) in the newest committed rocprofv3 --stats summary
    of this config (profiles/<tag>_<config>_kernel_stats.csv), or None."""
    import csv

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_kernel_stats.csv")), key=_profile_order,
                   reverse=True)
    if not files:
        return None
    out = {}
    for r in csv.DictReader(open(files[0])):
        name = r["Name"].split("(")[0].replace("void ", "").replace("jd::", "").split("<")[0]
        slot = {"k_dc_sum": "k_dc_pred", "k_dc_scan": "k_dc_pred", "k_pieceplan": "k_subplan",
                "k_chain_fix": "k_chain", "k_idct_color_exact": "k_idct_color"}.get(name, name)
        out[slot] = out.get(slot, 0.0) + float(r["AverageNs"]) / 1e6  # instances of a slot: one each per batch
    return out


def gather_counters(local, world: int):
    """(max over ranks of counter 0 = elapsed, sums of the other counters)."""
    allc = gather_matrix(local, world)
    return float(allc[:, 0].max()), tuple(float(allc[:, k].sum()) for k in range(1, allc.shape[1]))


# ---------------------------------------------------------------------------------------------
# measurement helpers
# ---------------------------------------------------------------------------------------------
def _profile_order(path: str):
    """Run tags go r03a .. r03z, r03aa .. : newer = longer, then later in the alphabet."""
    tag = os.path.basename(path).split("_")[0]
    return tag[:3], len(tag), tag


def newest_profile(pattern: str, config: str, kernel: str):
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=_profile_order, reverse=True):
        with open(f) as fh:
            t = json.load(fh)
        if t.get("config") == config and kernel in t.get("kernels", {}):
            return t["kernels"][kernel], os.path.relpath(f, ROOT)
    return None, None


def measured_traffic(config: str, kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC traffic profile of this
    config (profiles/<round>_traffic.json, tools/profile_summary.py), or None."""
    k, src = newest_profile("*_traffic.json", config, kernel)
    # per timing slot: a slot may dispatch several instances per batch (one per sampling layout)
    return (k.get("hbm_bytes_per_batch", k["hbm_bytes"]), src) if k else None


def valu_issue(config: str, kernel: str, avg_ms: float):
    """VALU issue model of `kernel` from the newest committed SQ profile of this config
    (profiles/<round>_sq_<config>.json): SQ_ACTIVE_INST_VALU per launch x 4 cycles
    (VALU_CYCLES_PER_QUAD) over the SIMD-cycles of the launch at the clock the profiled run held
    (GRBM_GUI_ACTIVE / 8 XCDs / time).  On gfx950 SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU within
    0.3 % for these kernels, so the figure is an instruction count priced at 4 cycles each, not a
    measured utilisation: tools/micro/valurate.hip measures ~2.8 cycles for v_add / v_and and ~4.6
    for shifts, v_bfe, v_mad_*24, v_perm and packed 16-bit ops."""
    k, src = newest_profile("*_sq_*.json", config, kernel)
    if not k or avg_ms <= 0:
        return None
    clk = k.get("clock_ghz") or 2.4
    n = k.get("dispatches_per_batch", 1.0)  # instances per timing slot (one per sampling layout)
    busy = (k.get("counters", {}).get("SQ_ACTIVE_INST_VALU") or k["valu_insts"]) * n
    cyc, wsrc = valu_weight(kernel)
    frac = busy * cyc / (SIMDS * clk * 1e9 * avg_ms * 1e-3)
    return {"valu_insts_per_launch": k["valu_insts"] * n, "dispatches_per_batch": n, "clock_ghz": clk, "busy_frac": frac,
            "busy_frac_x4": busy * VALU_CYCLES_PER_QUAD / (SIMDS * clk * 1e9 * avg_ms * 1e-3),
            "cycles_per_valu": cyc,
            "note": "issue model, not a measured utilisation: VALU instructions (SQ_ACTIVE_INST_VALU, equal to "
                    "SQ_INSTS_VALU on gfx950) x the kernel's static-mix issue cycles per instruction (" + wsrc +
                    ") over the launch's SIMD cycles; busy_frac_x4 prices every instruction at 4 cycles",
            "source": src}


def valu_weight(kernel: str):
    """Wave64 issue cycles per VALU instruction of `kernel` (the mean over its instances, e.g. one
    k_idct_color per sampling layout) from the committed static-mix table (tools/valu_weights.py:
    the ISA's opcode mix priced by tools/micro/valurate.hip's measured rates), else 4."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_valu_weights.json")), key=_profile_order, reverse=True)
    if files:
        ks = json.load(open(files[0]))["kernels"]
        w = [v["cycles_per_valu"] for v in ks.values() if re.match(rf"{kernel}(E|I)", v["name"])]
        if w:
            return sum(w) / len(w), os.path.relpath(files[0], ROOT)
    return float(VALU_CYCLES_PER_QUAD), "flat 4 cycles"


def kernel_rooflines(kern: dict, config: str) -> dict:
    """Per kernel slot: average launch time, algorithmic GB/s and its fraction of the 8 TB/s HBM
    peak, HBM traffic per launch (committed PMC profile) and the VALU-busy fraction (committed SQ
    profile).  The two big kernels are VALU-bound, so the last figure is the roof that applies."""
    out = {}
    for k, v in kern.items():
        if not v["launches"] or v["total_ms"] <= 0:
            continue
        ms = v["total_ms"] / v["launches"]
        gbs = v["bytes"] / v["launches"] / (ms * 1e-3) / 1e9
        names = {"k_dc_pred": "k_dc_sum"}.get(k, k)
        tr = measured_traffic(config, names)
        vb = valu_issue(config, names, ms)
        out[k] = {"avg_ms": round(ms, 4), "GB_s": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4),
                  "traffic_bytes": tr[0] if tr else None, "valu_busy": round(vb["busy_frac"], 3) if vb else None}
    return out


def copy_peak_gbs(dec, dev, gib: float = 4.0, reps: int = 10):
    """In-run HBM peak: the library's 16-byte-per-lane copy kernel (jd_test_copy_peak, the guide's
    "float4 copy" of MI355X_MICROARCH.md) over `gib` GiB, read + write bytes / time (hipEvents on the
    decoder's stream)."""
    import torch

    n = int(gib * (1 << 30)) // 16 * 16
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    torch.cuda.synchronize(dev)
    gbs = dec.copy_peak(a.data_ptr(), b.data_ptr(), n, reps)
    del a, b
    torch.cuda.empty_cache()
    return gbs


def pinned_h2d_gbs(nbytes: int, dev, reps: int = 3):
    """In-run pinned host -> device copy rate for `nbytes` (the PCIe leg of e2e_h2d)."""
    import torch

    src = torch.empty(int(nbytes), dtype=torch.uint8).pin_memory()
    dst = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize(dev)
    t = time.perf_counter() - t
    del src, dst
    return nbytes * reps / t / 1e9


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def ref_bench(paths, procs: int, reps: int):
    """The reference decoder (oracle/_ref/ref_bench: cpp-decoder's JPEGParser compiled from its own
    sources; extract()+decode() timed like cpp-decoder/benchmark/benchmark.cc:29-35) in `procs`
    parallel processes.  Returns (aggregate images/s, per-process seconds)."""
    import jdoracle

    if not os.path.exists(jdoracle.REF_BENCH):
        return None
    ps = [subprocess.Popen([jdoracle.REF_BENCH, str(reps)] + list(paths), stdout=subprocess.PIPE, text=True)
          for _ in range(procs)]
    rate, secs = 0.0, []
    for p in ps:
        out, _ = p.communicate(timeout=300)
        if p.returncode != 0:
            return None
        r = json.loads(out.strip().splitlines()[-1])
        rate += r["images"] / r["seconds"]
        secs.append(r["seconds"])
    return rate, secs


def cpu_baseline(hosts, hdrs, target_s: float = 5.0):
    """CPU decoders on this host, 1 core and all cores (the box's one-GPU CPU share):
      reference : the reference's JPEGParser (oracle/_ref/ref_bench) on the BASELINE config-1 image
                  (512x512 4:4:4 q90, no RST) — the only shape it decodes correctly
      port      : the oracle (CPU restatement; bit-serial Huffman, reference IDCT + colour) on the
                  first images of this workload, and on the config-1 image for the calibration
      port_fast : the oracle's "fast" mode (9-bit LUT Huffman, 64-bit bit buffer,
                  integer colour terms; same pixels and status, tests/test_oracle.py) on the same sample
    value = the fast port on this workload at all cores (kind "port"); `reference_equivalent` scales
    the faithful port by the calibration ratio."""
    import numpy as np

    import jd_synth
    import jdoracle

    cores = max(1, min(BOX_CPU_SHARE, len(os.sched_getaffinity(0))))
    res = {"unit": "MPixels/s", "kind": "port", "cores": cores, "nproc": os.cpu_count(),
           "cpus_allowed": len(os.sched_getaffinity(0)), "cpu_model": cpu_model()}

    def port(sample, threads, fast=False):
        secs, st, _ = jdoracle.decode_many(sample, threads=threads, want_rgb=True, fast=fast)
        if any(st):
            raise SystemExit(f"oracle failed on the CPU sample: {sorted(set(st))}")
        return secs

    n = len(hosts)
    probe = min(n, 2)
    per = port(hosts[:probe], 1) / probe
    n1 = int(max(1, min(n, target_s / max(per, 1e-6))))
    s1 = port(hosts[:n1], 1)
    px1 = float(sum(h.width * h.height for h in hdrs[:n1]))
    nall = int(max(cores, min(n, cores * target_s / max(per, 1e-6))))
    sample = [hosts[i % n] for i in range(nall)]
    sall = port(sample, cores)
    pxall = float(sum(hdrs[i % n].width * hdrs[i % n].height for i in range(nall)))
    res["port_1core"] = {"MPix_s": px1 / s1 / 1e6, "images": n1, "seconds": s1, "mode": "faithful"}
    res["port_all_cores"] = {"MPix_s": pxall / sall / 1e6, "images": nall, "seconds": sall, "threads": cores,
                             "mode": "faithful"}
    # the fast mode on its own bounded sample (about target_s of CPU time each)
    fper = port(hosts[:probe], 1, fast=True) / probe
    f1n = int(max(1, min(n, target_s / max(fper, 1e-6))))
    f1 = port(hosts[:f1n], 1, fast=True)
    fpx1 = float(sum(h.width * h.height for h in hdrs[:f1n]))
    fan = int(max(cores, min(4 * n, cores * target_s / max(fper, 1e-6))))
    fsample = [hosts[i % n] for i in range(fan)]
    fall = port(fsample, cores, fast=True)
    fpxall = float(sum(hdrs[i % n].width * hdrs[i % n].height for i in range(fan)))
    res["port_fast_1core"] = {"MPix_s": fpx1 / f1 / 1e6, "images": f1n, "seconds": f1}
    res["port_fast_all_cores"] = {"MPix_s": fpxall / fall / 1e6, "images": fan, "seconds": fall, "threads": cores}
    res["value"] = res["port_fast_all_cores"]["MPix_s"]
    res["value_mode"] = "fast (jdo_decode_fast: LUT Huffman; BASELINE.md §3)"
    # every CPU this process may use: the box's rules cap one GPU's job at BOX_CPU_SHARE threads, so
    # this is the measured per-thread rate at `cores` threads scaled linearly (an upper bound: no
    # memory-bandwidth or SMT saturation is modelled), not a measurement
    allowed = len(os.sched_getaffinity(0))
    res["port_all_allowed_projected"] = {"MPix_s": res["value"] / cores * allowed, "cpus": allowed,
                                         "note": f"linear extrapolation of the {cores}-thread rate"}

    c1 = jd_synth.encode(jd_synth.synth_pixels(512, 512, 0), 90, "4:4:4", 0, 0)
    c1a = np.frombuffer(c1, np.uint8).copy()
    pc1 = port([c1a] * 20, 1) / 20
    res["port_c1_1core_MPix_s"] = 512 * 512 / pc1 / 1e6
    sample_desc = (f"port: first {n1} workload images on 1 thread ({s1:.1f} s), {nall} on {cores} threads "
                   f"({sall:.1f} s); fast port: {f1n} on 1 thread ({f1:.1f} s), {fan} on {cores} threads ({fall:.1f} s)")
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "c1_512x512_444_q90.jpg")
        with open(path, "wb") as f:
            f.write(c1)
        one = ref_bench([path], 1, 4)
        if one:
            per_ref = one[1][0] / 4
            reps = int(max(4, target_s / max(per_ref, 1e-6)))
            r1 = ref_bench([path], 1, reps)
            rall = ref_bench([path], cores, max(2, reps // 2))
            res["reference_c1"] = {"MPix_s_1core": r1[0] * 512 * 512 / 1e6,
                                   "MPix_s_all_cores": rall[0] * 512 * 512 / 1e6, "processes": cores,
                                   "binary": "oracle/_ref/ref_bench (cpp-decoder sources, g++ -O2)",
                                   "decodes_1core": reps}
            cal = res["port_c1_1core_MPix_s"] / res["reference_c1"]["MPix_s_1core"]
            res["calibration_port_over_reference"] = cal
            res["reference_equivalent"] = {"MPix_s_1core": px1 / s1 / 1e6 / cal,
                                           "MPix_s_all_cores": res["value"] / cal,
                                           "MPix_s_all_allowed_projected": res["value"] / cal / cores * allowed}
            sample_desc += f"; reference: config-1 image x{reps} on 1 process, x{max(2, reps // 2)} on {cores}"
        else:
            res["reference_c1"] = None
            sample_desc += "; reference binary oracle/_ref/ref_bench not built on this box"
    res["sample"] = sample_desc
    return res


def ref_sweep(dec, datas, hosts, hdrs, in_ptrs, rgb_bufs, out_offs, dev, reps: int = 5, part: str = "all"):
    """The reference's two published curves on its own format (ref444), GPU beside its CPU decoder:
      batch   throughput vs batch size B in REF_BATCHES (figures/batchsize.pdf; method
              cuda-decoder/benchmark_thoughput/benchmark.cu:43-106: batches decoded one after another,
              JPEG file bytes / time): `serial` = one blocking jd_decode_batch per batch (host parse +
              plan + kernels + status readback, the reference's loop without its per-image
              cudaMalloc), `kernel_ms` = the sum of the batch's kernel hipEvents (the reference's
              cudaEvent pair around batchDecodeKernel), `pipelined` = jd_decode_batch_async steady state
      latency single-image decode per size (figures/runtime.png; cuda-decoder/benchmark/benchmark.cu:
              29-100: 10 iterations per image, cudaEvent around decodeKernel): median wall time of a
              blocking one-image jd_decode_batch and its kernel hipEvent sum, next to the reference's
              C++ decoder (oracle/_ref/ref_bench: extract + decode, cpp-decoder/benchmark/
              benchmark.cc:29-35) on the same files, 1 thread"""
    import numpy as np
    import torch

    import jdoracle

    n = len(datas)
    jbytes = [len(d) for d in datas]
    out = {"published_MB_s_batch3000": REF_PUBLISHED_MB_S, "published_hw": "RTX 2080 Ti (BASELINE.md §1)",
           "format": f"4:4:4 q{REF_QUALITY}, no RST, sizes {REF_SIZES[0]}^2..{REF_SIZES[-1]}^2 cycling by image",
           "batch": [], "latency": []}

    def kernel_ms(st):
        return sum(v["total_ms"] for v in st["kernels"].values())

    for B in (REF_BATCHES if part in ("all", "batch") else ()):
        B = min(B, n)
        sets = [dec.make_batch(hosts[:B], in_ptrs[:B], [rb.data_ptr() + o for o in out_offs[:B]]) for rb in rgb_bufs]
        mb = sum(jbytes[:B]) / 1e6
        px = float(sum(h.width * h.height for h in hdrs[:B]))
        r = max(2, min(reps * 4, int(20000 // B)))  # ~20 K images per point, at least 2 batches
        dec.decode_prepared(sets[0], pipelined=False)
        dec.reset_stats()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for k in range(r):
            dec.decode_prepared(sets[k % len(sets)], pipelined=False)
        torch.cuda.synchronize(dev)
        ser = (time.perf_counter() - t) / r
        kms = kernel_ms(dec.stats()) / r
        for k in range(len(sets)):
            dec.decode_prepared(sets[k], pipelined=True)
        dec.wait()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for k in range(r):
            dec.decode_prepared(sets[k % len(sets)], pipelined=True)
        dec.wait()
        torch.cuda.synchronize(dev)
        pip = (time.perf_counter() - t) / r
        if any(x.status for st in sets for x in st[1]):
            raise SystemExit(f"ref444 sweep: decode failed at batch {B}")
        out["batch"].append({"images": B, "jpeg_MB": mb, "serial_ms": ser * 1e3, "kernel_ms": kms,
                             "pipelined_ms": pip * 1e3, "serial_MB_s": mb / ser, "kernel_MB_s": mb / (kms * 1e-3),
                             "pipelined_MB_s": mb / pip, "pipelined_MPix_s": px / pip / 1e6,
                             "vs_published_batch3000_kernel": mb / (kms * 1e-3) / REF_PUBLISHED_MB_S,
                             "batches_timed": r})
    per_size = 5  # images of each size (the reference: every file of its size folder)
    with tempfile.TemporaryDirectory() as td:
        for si, size in enumerate(REF_SIZES if part in ("all", "latency") else ()):
            idx = [i for i in range(n) if i % len(REF_SIZES) == si][:per_size]
            walls, kerns, paths, per_k = [], [], [], {}
            for i in idx:
                one = dec.make_batch([hosts[i]], [in_ptrs[i]], [rgb_bufs[0].data_ptr() + out_offs[i]])
                dec.decode_prepared(one, pipelined=False)
                ws = []
                dec.reset_stats()
                for _ in range(10):
                    t = time.perf_counter()
                    dec.decode_prepared(one, pipelined=False)
                    ws.append(time.perf_counter() - t)
                stt = dec.stats()
                kerns.append(kernel_ms(stt) / 10)
                for kn, kv in stt["kernels"].items():
                    if kv["launches"]:
                        per_k[kn] = per_k.get(kn, 0.0) + kv["total_ms"] / kv["launches"] / len(idx)
                walls.append(float(np.median(ws)) * 1e3)
                path = os.path.join(td, f"{size}_{i}.jpeg")
                with open(path, "wb") as f:
                    f.write(datas[i])
                paths.append(path)
            ref = None
            if os.path.exists(jdoracle.REF_BENCH):
                rr = ref_bench(paths, 1, 2 if size >= 1400 else 5)
                ref = 1e3 / rr[0] if rr else None  # ms per image, 1 process
            out["latency"].append({"size": size, "images": len(idx), "gpu_wall_ms_median": float(np.median(walls)),
                                   "gpu_kernel_ms": float(np.median(kerns)), "ref_cpu_ms": ref,
                                   "kernels_ms": {k: round(v, 4) for k, v in per_k.items()},
                                   "gpu_MPix_s": size * size / float(np.median(walls)) / 1e3,
                                   "ref_cpu_MPix_s": size * size / ref / 1e3 if ref else None})
    return out


# ---------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the driver's own command (--steps 20 --warmup 5): a bare `python bench.py` measures what it measures
    # (the pipeline's fill and drain, ~1 % of 20 C2 steps, are inside the timed region: profiles/r06_ramp.json)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override images per rank")
    ap.add_argument("--quality", type=int, default=0, help="JPEG quality (default: 90; ref444: 95)")
    ap.add_argument("--sweep", nargs="?", const="all", default=None, choices=["all", "batch", "latency"],
                    help="ref444: print the reference's two published curves instead of the bench line: "
                         "throughput vs batch size (JPEG MB/s) and single-image latency per size, next to the "
                         "reference's own CPU decoder (oracle/_ref/ref_bench) on the same files")
    ap.add_argument("--cpu-sample", type=int, default=1, help="1: time the CPU baselines, 0: skip")
    ap.add_argument("--verify", type=int, default=1, help="check images {0, n/2, n-1} bit-exact vs the oracle")
    ap.add_argument("--e2e-steps", type=int, default=24, help="steps of each H2D-inclusive leg (0: skip; the last batch's kernels after its DMA are ~6 ms of pipeline drain, so few steps understate the rate)")
    ap.add_argument("--copy-peak", type=int, default=1, help="measure an in-run HBM copy peak")
    ap.add_argument("--kernel-steps", type=int, default=3,
                    help="serialized (non-overlapped) steps after the timed region for per-kernel times")
    ap.add_argument("--path", default="auto", choices=["auto", "sync", "lanes", "full"],
                    help="entropy-decode path (auto: lanes for images with restart intervals)")
    ap.add_argument("--fancy", action="store_true",
                    help="libjpeg's triangular chroma upsampling (JD_FLAG_FANCY_UPSAMPLING; an option beyond the "
                         "reference, parity unpinned) instead of replication")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one blocking jd_decode_batch per step instead of jd_decode_batch_async (which "
                         "parses and plans step k+1 on the host while the GPU decodes step k)")
    args = ap.parse_args()
    if args.config == "c2f":
        args.fancy = True
    rc = maybe_launch(args)
    if rc is not None:
        sys.exit(rc)

    import numpy as np
    import torch
    import torch.distributed as dist

    d = dist_setup()
    rank, world = d["rank"], d["world"]
    dev = torch.device("cuda", d["device_index"])

    import jd_synth
    import jdamd

    W, H, ss, rrows, batch, desc = CONFIGS[args.config]
    if args.batch:
        batch = args.batch
    seeds = shard_seeds(args.config, batch, rank, world)  # disjoint images per rank: shard by image
    t_gen = time.time()
    quality = args.quality or (REF_QUALITY if ss == "ref" else 90)
    if ss == "ref":
        jobs = ref444_jobs(seeds, quality)
    else:
        jobs = jd_synth.make_jobs(seeds, W, H, quality, "4:2:0" if ss == "mixed" else ss, rrows, 0,
                                  mixed=(ss == "mixed"))
    datas = jd_synth.make_images(jobs)
    t_gen = time.time() - t_gen
    n = len(datas)
    hosts = [np.frombuffer(x, np.uint8).copy() for x in datas]
    hdrs = [jdamd.parse(x) for x in datas]
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
    # three output buffers: consecutive pipelined batches write different memory, as distinct
    # batches of a real stream would; jd_decode_batch_async keeps two batches in flight and a
    # batch's buffers are free again once it is collected, two calls later (include/jd.h)
    rgb_bufs = [torch.empty(otot, dtype=torch.uint8, device=dev) for _ in range(3 if not args.no_pipeline else 1)]
    nb = len(rgb_bufs)
    flat = np.zeros(tot, np.uint8)
    for h, o in zip(hosts, in_offs):
        flat[o:o + h.nbytes] = h
    jpeg_dev.copy_(torch.from_numpy(flat))
    torch.cuda.synchronize(dev)

    threads, thread_info = host_threads(d)
    dec = jdamd.Decoder(d["device_index"], timing=True, path=args.path, parse_threads=threads, fancy=args.fancy)
    batches = [dec.make_batch(hosts, [jpeg_dev.data_ptr() + o for o in in_offs],
                              [rb.data_ptr() + o for o in out_offs]) for rb in rgb_bufs]
    pixels = float(sum(h.width * h.height for h in hdrs))
    ecs = float(sum(len(x) - h.ecs_offset for x, h in zip(datas, hdrs)))
    jpeg_bytes = float(sum(len(x) for x in datas))

    pipelined = not args.no_pipeline
    for w in range(max(nb, args.warmup)):
        dec.decode_prepared(batches[w % nb], pipelined=pipelined)
    dec.wait()
    status = [r.status for b in batches for r in b[1]]
    if any(status) and args.verify:  # --verify 0: ablation builds decode wrong on purpose
        raise SystemExit(f"decode failed: statuses {sorted(set(status))}")

    # correctness spot check against the oracle (outside the timed region): head, middle, tail
    verified = []
    if args.verify:
        import jdoracle

        for i in sorted({0, n // 2, n - 1}):
            h = hdrs[i]
            st, ref = jdoracle.decode(datas[i], fancy=args.fancy)
            for rb in rgb_bufs:
                got = rb[out_offs[i]:out_offs[i] + h.width * h.height * 3].cpu().numpy().reshape(h.height, h.width, 3)
                if st != 0 or not np.array_equal(got, ref):
                    raise SystemExit(f"bit-exactness check failed on image {i}")
            verified.append(i)

    if args.sweep:
        if ss != "ref" or world > 1:
            raise SystemExit("--sweep: --config ref444 on one GPU")
        res = ref_sweep(dec, datas, hosts, hdrs, [jpeg_dev.data_ptr() + o for o in in_offs], rgb_bufs, out_offs, dev,
                        part=args.sweep)
        res.update({"metric": "ref444 sweep (throughput vs batch, latency vs size)", "verified_bit_exact": verified,
                    "cpu_model": cpu_model(), "gen_s": t_gen})
        print(json.dumps(res))
        dec.close()
        return

    dec.reset_stats()
    torch.cuda.reset_peak_memory_stats(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        dec.decode_prepared(batches[k % nb], pipelined=pipelined)
    dec.wait()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if args.verify and any(r.status for b in batches for r in b[1]):  # the last timed batches' statuses
        raise SystemExit("decode failed inside the timed region")
    st_overlap = dec.stats()
    host_ms_step = {k: v / args.steps for k, v in st_overlap["host_ms"].items()}
    # per-kernel times for the roofline from serialized batches (outside the timed region): in the
    # timed loop consecutive batches overlap on the slot streams, so a kernel's hipEvent span there
    # includes the other batch's kernels
    dec.reset_stats()
    for k in range(max(1, args.kernel_steps)):
        dec.decode_prepared(batches[k % nb], pipelined=False)
    st = dec.stats()

    # PCIe-inclusive rate (not `value`): the JPEG bytes handed over in host memory, RGB to HBM;
    # pipelined like the timed loop (the host stages batch k+1 while the GPU decodes batch k), run
    # by every rank at once so a multi-GPU run shows the shared host's feed rate
    e2e = None
    e2e_ms = h2d_gbs = reg_ms = arena_ms = 0.0
    if args.e2e_steps:
        def e2e_leg(batches):
            """The pipelined timed loop over host-input batches: (seconds, library stats)."""
            for k in range(len(batches)):
                dec.decode_prepared(batches[k], pipelined=True)
            dec.wait()
            dec.reset_stats()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for k in range(args.e2e_steps):
                dec.decode_prepared(batches[k % len(batches)], pipelined=True)
            dec.wait()
            torch.cuda.synchronize(dev)
            t = time.perf_counter() - t
            if any(r.status for b in batches for r in b[1]):
                raise SystemExit("decode failed in the H2D-inclusive run")
            return t, dec.stats()

        def leg_dict(t, st, dram, note):
            ms = t / args.e2e_steps * 1e3
            return {"MPix_s": pixels * args.e2e_steps / t / 1e6, "ms_per_step": ms,
                    "frac_of_h2d_bound": bound_ms / ms,
                    "host_ms_per_step": {k: v / args.e2e_steps for k, v in st["host_ms"].items()},
                    "h2d_registered_bytes_per_step": st["h2d_registered_bytes"] / args.e2e_steps,
                    "host_dram_bytes_per_step": dram, "note": note}

        def packed(arena):
            views, o = [], 0
            for h in hosts:
                arena[o:o + h.nbytes] = h
                views.append(arena[o:o + h.nbytes])
                o += (h.nbytes + 63) // 64 * 64
            return views

        arena_bytes = sum((h.nbytes + 63) // 64 * 64 for h in hosts)
        # 1. staged: files in pageable memory, copied by the library's workers into pinned staging
        te, se = e2e_leg([dec.make_batch(hosts, [None] * n, [rb.data_ptr() + o for o in out_offs]) for rb in rgb_bufs])
        # 2. registered: the files packed in one caller-owned arena registered with jd_host_register
        arena = np.empty(arena_bytes, np.uint8)
        views = packed(arena)
        t_reg = time.perf_counter()
        dec.register_host(arena)
        t_reg = time.perf_counter() - t_reg
        tr, sr = e2e_leg([dec.make_batch(views, [None] * n, [rb.data_ptr() + o for o in out_offs]) for rb in rgb_bufs])
        dec.unregister_host(arena)
        del arena, views
        # 3. pinned arena: the files read into a jd_host_alloc arena (hipHostMalloc)
        parena = dec.host_alloc(arena_bytes)
        pviews = packed(parena)
        tp, sp = e2e_leg([dec.make_batch(pviews, [None] * n, [rb.data_ptr() + o for o in out_offs]) for rb in rgb_bufs])
        dec.host_free(parena)
        del parena, pviews
        e2e_ms = te / args.e2e_steps * 1e3
        reg_ms = tr / args.e2e_steps * 1e3
        arena_ms = tp / args.e2e_steps * 1e3
        h2d_gbs = pinned_h2d_gbs(int(jpeg_bytes), dev)
        bound_ms = jpeg_bytes / (h2d_gbs * 1e9) * 1e3
        e2e = leg_dict(te, se, 3 * jpeg_bytes,
                       "per rank; JPEG bytes from pageable host memory, copied by the library's host workers into "
                       "per-slot pinned staging and uploaded on the slot's stream while the other slot decodes "
                       "(jd_decode_batch_async); RGB left in HBM; host DRAM traffic = the staging copy's read + "
                       "write and the DMA's read")
        e2e.update({"steps": args.e2e_steps, "pinned_h2d_GB_s": h2d_gbs, "h2d_bound_ms_per_step": bound_ms})
        e2e["registered"] = dict(leg_dict(tr, sr, jpeg_bytes,
                                          "the same files packed in one caller-owned arena registered once with "
                                          "jd_host_register (hipHostRegister): uploaded straight from it by DMA, no "
                                          "staging copy; host DRAM traffic = the DMA's read"),
                                 register_ms=t_reg * 1e3)
        e2e["pinned_arena"] = leg_dict(tp, sp, jpeg_bytes,
                                       "the same files read into an arena from jd_host_alloc (hipHostMalloc): "
                                       "uploaded straight from it by DMA, no staging copy")

    # one all-gather of per-rank counters (RCCL over xGMI when N > 1): totals for the line, and
    # every rank's step time and host feed (so an 8-GPU run shows whether the host binds)
    local = torch.tensor(rank_vector(elapsed, pixels, n, ecs, jpeg_bytes, args.steps, host_ms_step, e2e_ms, h2d_gbs, reg_ms,
                                     arena_ms),
                         dtype=torch.float64, device=dev if d["backend"] == "nccl" else "cpu")
    allc = gather_matrix(local, world)
    t_max = float(allc[:, 0].max())
    tot_px, tot_img, tot_ecs, tot_bytes = (float(allc[:, k].sum()) for k in range(1, 5))

    # rank 0's single-host measurements after the gather, at every world size (the others wait)
    extra = rank0_measurements(rank, world,
                               copy_fn=(lambda: copy_peak_gbs(dec, dev)) if args.copy_peak else None,
                               cpu_fn=(lambda: cpu_baseline(hosts, hdrs)) if args.cpu_sample else None)
    if rank == 0:
        kern = st["kernels"]
        copy_gbs = extra["copy_peak"]
        cpu = extra["cpu_baseline"]
        px_rank = float(sum(h.width * h.height for h in hdrs))
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
            "data": f"synthetic (seeded sinusoid + noise, baseline encode "
                    f"{'q in {50,75,90,95}' if ss == 'mixed' else f'q{quality}'} by "
                    f"{'tools/jdenc.c' if jd_synth.default_encoder() == 'jdenc' else 'Pillow'}, std Huffman tables)",
            "config": {"workload": desc, "config": args.config, "images_per_rank": n,
                       "global_batch": int(allc[:, 6].sum()), "width": W or list(REF_SIZES), "height": H or list(REF_SIZES),
                       "subsampling": "4:4:4" if ss == "ref" else ss,
                       "restart_rows": rrows, "parallelism": f"dp{world} (image sharding)",
                       "entropy_path": args.path, "host_pipelined": pipelined,
                       "upsampling": "fancy (libjpeg triangular)" if args.fancy else "replicate",
                       "bpp_file": 8 * jpeg_bytes / px_rank, "bpp_ecs": 8 * ecs / px_rank},
            "world_size_seen": d["world_seen"],
            "dist_backend": d["backend"],
            "shards": {"images": [int(x) for x in allc[:, 6]], "ecs_MB": [round(x / 1e6, 3) for x in allc[:, 5]],
                       "ecs_max_over_mean": float(allc[:, 5].max() / allc[:, 5].mean()),
                       "balance": "greedy by estimated ECS bytes" if ss == "mixed" and world > 1 else "contiguous"},
            "host": thread_info,
            "images_per_s": tot_img / t_max,
            "jpeg_MB_per_s": tot_bytes / t_max / 1e6,
            "ecs_MB_per_s": tot_ecs / t_max / 1e6,
            "roofline": roofline_block(kern, args.config, copy_gbs, args.kernel_steps, rocprof_averages(args.config)),
            "kernel_rooflines": kernel_rooflines(kern, args.config),
            "kernels_ms_per_step": {k: v["total_ms"] / max(1, v["launches"]) for k, v in kern.items()},
            "kernels_ms_per_step_overlapped": {k: v["total_ms"] / max(1, v["launches"])
                                               for k, v in st_overlap["kernels"].items()},
            "path_roofline_frac": ((ecs + 3 * pixels) / (t_max / args.steps) / 1e9) / HBM_PEAK_GBS,
            "e2e_h2d": e2e,
            "per_rank": per_rank_table(allc, args.steps),
            "device_memory": {"decoder_pools_peak_GB": dec.device_bytes()[1] / 1e9,
                              "torch_peak_GB": torch.cuda.max_memory_allocated(dev) / 1e9,
                              "pools": "optimistic (default; an image that overflows one is decoded again "
                                       "with worst-case pools: include/jd.h JD_FLAG_WORST_CASE_POOLS)",
                              "retried_images_timed": st_overlap["retried_images"],
                              "note": "rank 0: the library's grow-only pools (two in-flight slots) and the "
                                      "bench's own input/output buffers"},
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
