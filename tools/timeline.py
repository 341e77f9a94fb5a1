"""Kernel timeline of a pipelined bench run from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace -d trace -o run -f csv -- python3 bench.py --steps 12 --warmup 3 \\
        --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0
    python tools/timeline.py trace/run_kernel_trace.csv [batches]

Prints, for the last `batches` batches (default 4), every k_* dispatch with its hardware queue
(one per slot stream), start and end in microseconds from the first k_scan shown, and duration,
so that a kernel waiting for resources under the other batch's kernels stands out.
"""
import csv
import sys


def name(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("jd::", "")


def main():
    path = sys.argv[1]
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = [r for r in csv.DictReader(open(path)) if name(r).startswith("k_")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    scans = [i for i, r in enumerate(rows) if name(r) == "k_scan"]
    if len(scans) < nb + 1:
        nb = max(1, len(scans) - 1)
    i0, i1 = scans[-nb - 1], scans[-1]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{name(r)[:28]:28s} q{r.get('Queue_Id', '?'):>3s} {s:9.1f} {e:9.1f} {e - s:8.1f}")
    per = (int(rows[i1]["Start_Timestamp"]) - t0) / 1e3 / nb
    print(f"period: {per:.1f} us per batch over {nb} batches")


if __name__ == "__main__":
    main()
