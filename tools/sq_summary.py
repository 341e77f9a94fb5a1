"""Per-kernel SQ / GRBM counter summary of a tools/prof_pmc.sh run -> profiles/<tag>_sq_<config>.json.

    python tools/sq_summary.py TAG RUN_DIR --config c2

Per kernel (averages over its launches): VALU / SALU / LDS / VMEM instruction counts per launch,
the wave-cycle split (active / issue-stalled / waiting; SQ_WAVE_CYCLES and the SQ_WAIT_* /
SQ_ACTIVE_* counters are in quad-cycles, MI355X_MICROARCH.md) and the clock the profiled run held
(GRBM_GUI_ACTIVE / 8 XCDs / dispatch time).  bench.py reads valu_insts and clock_ghz for the
roofline's VALU issue fraction.
"""
import argparse
import collections
import csv
import glob
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("run_dir")
ap.add_argument("--config", default="c2")
a = ap.parse_args()
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(a.run_dir, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("jd::", "")
        k = k
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            vals[k]["_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
out = {"config": a.config, "method": "rocprofv3 --kernel-trace --pmc, SQ groups in separate passes "
       "(tools/prof_pmc.sh); per-launch averages", "kernels": {}}
for k, c in sorted(vals.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    e = {"valu_insts": m.get("SQ_INSTS_VALU"), "salu_insts": m.get("SQ_INSTS_SALU"),
         "lds_insts": m.get("SQ_INSTS_LDS"), "vmem_rd_insts": m.get("SQ_INSTS_VMEM_RD"),
         "vmem_wr_insts": m.get("SQ_INSTS_VMEM_WR"), "waves": m.get("SQ_WAVES"),
         "lds_bank_conflict_frac": (m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"])
         if m.get("SQ_LDS_IDX_ACTIVE") else None}
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
dst = os.path.join(root, "profiles", f"{a.tag}_sq_{a.config}.json")
with open(dst, "w") as fh:
    json.dump(out, fh, indent=1)
for k, e in out["kernels"].items():
    print(k, {x: (round(y, 3) if isinstance(y, float) else y) for x, y in e.items() if x != "counters"})
