"""Reduces a tools/round_profile.sh run to the committed profile artifacts.

    python tools/round_summary.py TAG gpurun_out/TAG [configs...]

Per config:
  profiles/TAG_<cfg>_bench.json        the bench line
  profiles/TAG_<cfg>_kernel_stats.csv  rocprofv3 --kernel-trace --stats (serialized steps)
  profiles/TAG_<cfg>_traffic.json      HBM bytes per launch per kernel, from separate FETCH_SIZE /
                                       WRITE_SIZE passes, corrected as MI355X_MICROARCH.md's HBM
                                       section prescribes (KiB units; gfx950 FETCH_SIZE counts half
                                       of a 16 B/lane streaming read, so reads are doubled)
  profiles/TAG_sq_<cfg>.json           SQ counters per kernel (every config): instruction counts, wave-cycle
                                       split, clock held (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time)
Kernel names drop their template arguments (k_idct_color<1> -> k_idct_color; per-launch averages
over the instances that ran, with the dispatches per batch beside them).  bench.py reads traffic and valu_insts/clock_ghz from these files.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

tag, run = sys.argv[1], sys.argv[2]
cfgs = sys.argv[3:] or ["c1", "c2", "c3", "c5"]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")


def kname(k):
    return k.split("(")[0].replace("void ", "").replace("jd::", "").split("<")[0]


def counters(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] in ("GRBM_GUI_ACTIVE",):
                vals[k]["_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    out = {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in vals.items()}
    # dispatches of each kernel name per batch (k_scan runs once per batch): a timing slot such as
    # k_idct_color launches one instance per sampling layout present, so per-slot figures are the
    # per-dispatch averages times this
    nb = max(len(v) for v in vals.get("k_scan", {"": [1]}).values()) if vals else 1
    for k, c in vals.items():
        out[k]["_per_batch"] = max(len(v) for n, v in c.items() if not n.startswith("_")) / nb
    return out


for c in cfgs:
    b = os.path.join(run, f"{c}.json")
    if os.path.exists(b):
        lines = [l for l in open(b) if l.startswith("{")]
        if lines:
            open(os.path.join(prof, f"{tag}_{c}_bench.json"), "w").write(lines[-1])
    st = glob.glob(os.path.join(run, f"{c}_stats", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        shutil.copy(st[0], os.path.join(prof, f"{tag}_{c}_kernel_stats.csv"))
    fe, wr = counters(os.path.join(run, f"{c}_fetch")), counters(os.path.join(run, f"{c}_write"))
    if fe or wr:
        out = {"config": c, "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE, separate passes "
               "over serialized steps; bytes = 2 * FETCH_SIZE + WRITE_SIZE per launch (KiB -> B; gfx950 FETCH_SIZE "
               "halves 16 B/lane streaming reads)", "kernels": {}}
        for k in sorted(set(fe) | set(wr)):
            f = fe.get(k, {}).get("FETCH_SIZE", 0.0) * 1024.0
            w = wr.get(k, {}).get("WRITE_SIZE", 0.0) * 1024.0
            n = (fe.get(k) or wr.get(k))["_per_batch"]
            out["kernels"][k] = {"fetch_size_bytes": f, "write_size_bytes": w, "hbm_bytes": 2 * f + w,
                                 "dispatches_per_batch": n, "hbm_bytes_per_batch": (2 * f + w) * n}
        json.dump(out, open(os.path.join(prof, f"{tag}_{c}_traffic.json"), "w"), indent=1)
    sq = counters(os.path.join(run, f"{c}_sq"))
    if sq:
        out = {"config": c, "method": "rocprofv3 --kernel-trace --pmc, SQ groups in separate passes over serialized "
               "steps; per-launch averages", "kernels": {}}
        for k, m in sorted(sq.items()):
            e = {"valu_insts": m.get("SQ_INSTS_VALU"), "salu_insts": m.get("SQ_INSTS_SALU"),
                 "lds_insts": m.get("SQ_INSTS_LDS"), "vmem_rd_insts": m.get("SQ_INSTS_VMEM_RD"),
                 "vmem_wr_insts": m.get("SQ_INSTS_VMEM_WR"), "waves": m.get("SQ_WAVES"),
                 "lds_bank_conflict_frac": (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"])
                 if m.get("SQ_LDS_IDX_ACTIVE") else None, "dispatches_per_batch": m["_per_batch"]}
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                e["wave_cycles_split"] = {"active": m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                                          "issue_stalled": m.get("SQ_WAIT_INST_ANY", 0) / wc,
                                          "waiting": m.get("SQ_WAIT_ANY", 0) / wc}
            if m.get("GRBM_GUI_ACTIVE") and m.get("_ns"):
                e["clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8.0 / m["_ns"]
                e["dispatch_ms"] = m["_ns"] * 1e-6
            e["counters"] = {n: v for n, v in m.items() if not n.startswith("_")}
            out["kernels"][k] = e
        json.dump(out, open(os.path.join(prof, f"{tag}_sq_{c}.json"), "w"), indent=1)
    print(c, "done")
