"""Per-kernel average of rocprofv3 counter_collection.csv files: python tools/pmc_summary.py DIR..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f)
        for k, v in agg.items():
            print(f"  {k:28s}", "  ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
