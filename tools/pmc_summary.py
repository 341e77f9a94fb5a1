"""Per-kernel averages of every PMC counter in a tools/prof_pmc.sh run directory.

    python tools/pmc_summary.py gpurun_out/<dir> [kernel-substring]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("jd::", "")
        if sub in k:
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(vals.items()):
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {sum(v) / len(v):16.1f}")
