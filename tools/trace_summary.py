"""Per-(kernel, grid) duration summary of a rocprofv3 kernel_trace.csv."""
import collections, csv, statistics, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    g = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
    d[(k, g)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (k, g), v in sorted(d.items()):
    print(f"{k:40s} grid={'x'.join(g[:2])} wg={g[2]:5s} n={len(v):5d} mean={statistics.mean(v)/1e3:8.2f}us "
          f"med={statistics.median(v)/1e3:8.2f} min={min(v)/1e3:8.2f} max={max(v)/1e3:8.2f}")
