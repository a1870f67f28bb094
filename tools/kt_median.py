"""Median kernel duration per (kernel, grid) from a rocprofv3 --kernel-trace CSV directory.
usage: kt_median.py <dir> [name-substring]; clusters of one grid are split at the largest gap."""
import csv, glob, os, sys
from collections import defaultdict
f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
d = defaultdict(list)
for r in csv.DictReader(open(f)):
    if sub in r["Kernel_Name"]:
        d[(r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items()):
    v.sort()
    gaps = [(v[i + 1] / v[i], i) for i in range(len(v) - 1)]
    cut = max(gaps)[1] + 1 if gaps and max(gaps)[0] > 1.5 else len(v)
    parts = [v[:cut], v[cut:]] if cut < len(v) else [v]
    print(k, " | ".join(f"n={len(p)} median {p[len(p) // 2]:.2f} us" for p in parts if p))
