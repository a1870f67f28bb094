"""Per-step device spans of the decode GEMVs in a rocprofv3 kernel trace (tools/run.sh PARTS=prof).

The roofline's rocprof_check compares the GEMVs' traced busy time per step with a step time.  The untraced
headline step is the wrong yardstick for that: the tracer stamps every dispatch and its durations run longer than
the same kernels untraced.  This tool prices the check inside the traced run itself:
  - every 128 consecutive GEMV launches (one decode step: 32 layers x 4 sibling launches) form a window;
  - span = last end - first start of the window (device clock), sum = the window's summed kernel durations;
  - gap_free windows are those without an idle gap > 20 us (host-bound stalls), i.e. device-bound steps;
  - traced_ms_per_step = the bench line the traced run printed (prof.log).

usage: python tools/trace_steps.py <prof dir with run_kernel_trace.csv> <prof.log> > profiles/rNN_bench_rocprofv3_step_spans.json
"""
import csv
import json
import os
import statistics
import sys

LAUNCHES = 128
GAP_NS = 20000


def windows(trace_csv, launches=LAUNCHES):
    rows = [r for r in csv.DictReader(open(trace_csv)) if "k_gemv_q4_0<1," in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    S = [int(r["Start_Timestamp"]) for r in rows]
    E = [int(r["End_Timestamp"]) for r in rows]
    out = []
    for w in range(len(rows) // launches):
        a, b = w * launches, (w + 1) * launches
        gaps = [S[i] - E[i - 1] for i in range(a + 1, b)]
        out.append({"span_us": (max(E[a:b]) - S[a]) / 1e3,
                    "sum_us": sum(E[i] - S[i] for i in range(a, b)) / 1e3,
                    "gap_free": max(gaps) <= GAP_NS})
    return len(rows), out


def summarize(trace_csv, prof_log=None):
    n, ws = windows(trace_csv)
    free = [w for w in ws if w["gap_free"]]
    res = {"source": trace_csv, "gemv_launches": n, "windows": len(ws), "gap_free_windows": len(free),
           "launches_per_window": LAUNCHES}
    for name, sel in (("all", ws), ("gap_free", free)):
        if sel:
            res[name] = {"span_us_median": round(statistics.median(w["span_us"] for w in sel), 1),
                         "sum_us_median": round(statistics.median(w["sum_us"] for w in sel), 1),
                         "sum_le_span": sum(1 for w in sel if w["sum_us"] <= w["span_us"])}
    if prof_log and os.path.exists(prof_log):
        for line in open(prof_log):
            if line.startswith("{"):
                try:
                    r = json.loads(line)
                except ValueError:
                    continue
                res["traced_ms_per_step"] = r.get("ms_per_step")
                res["traced_decode_path"] = r.get("config", {}).get("decode_path", "")[:60]
    return res


if __name__ == "__main__":
    d = sys.argv[1]
    print(json.dumps(summarize(os.path.join(d, "run_kernel_trace.csv"), sys.argv[2] if len(sys.argv) > 2 else None),
                     indent=1))
