"""Collects the bench lines of a tools/ab.sh output directory into one JSON summary for profiles/.

    python tools/ab_summary.py gpurun_out/TAG/ab profiles/TAG_ab.json "what was compared"
"""
import glob
import json
import os
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    note = sys.argv[3] if len(sys.argv) > 3 else ""
    runs = []
    for f in sorted(glob.glob(os.path.join(src, "*.json")), key=os.path.getmtime):
        lines = [l for l in open(f) if l.startswith('{"metric"')]
        if not lines:
            continue
        d = json.loads(lines[-1])
        runs.append({"run": os.path.basename(f)[:-5], "ms_per_step": round(d["ms_per_step"], 4),
                     "MPix_s": round(d["value"]), "config": d["config"]["config"],
                     "kernels_ms": {k: round(v, 4) for k, v in d.get("kernels_ms_per_step", {}).items() if v}})
    json.dump({"note": note, "runs_in_order": runs}, open(dst, "w"), indent=1)
    print(f"{len(runs)} runs -> {dst}")


if __name__ == "__main__":
    main()
