"""tools/trace_steps.py: per-step windows of a synthetic rocprofv3 kernel trace (CPU)."""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import trace_steps  # noqa: E402


def _trace(path, starts_durs, name="void ghip::k_gemv_q4_0<1, 16, 1, 3, 1, 0, 0, 0>(float const*)"):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerow(["ghip::k_engine_q4_0(ghip::EngArgs)", 0, 5])        # other kernels are ignored
        for s, d in starts_durs:
            w.writerow([name, s, s + d])


def test_windows_spans_and_gaps(tmp_path):
    L = trace_steps.LAUNCHES
    ev, t = [], 1000
    for _ in range(L):                 # window 0: back to back, 7 us each
        ev.append((t, 7000)); t += 7000
    for i in range(L):                 # window 1: one 50 us host stall inside
        ev.append((t, 7000)); t += 7000 + (50000 if i == 10 else 0)
    for _ in range(5):                 # a partial window is dropped
        ev.append((t, 7000)); t += 7000
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, ev)
    log = tmp_path / "prof.log"
    log.write_text("noise\n" + json.dumps({"ms_per_step": 1.05, "config": {"decode_path": "eager"}}) + "\n")
    r = trace_steps.summarize(str(p), str(log))
    assert r["gemv_launches"] == 2 * L + 5 and r["windows"] == 2 and r["gap_free_windows"] == 1
    assert r["gap_free"]["span_us_median"] == r["gap_free"]["sum_us_median"] == L * 7.0
    assert r["all"]["sum_le_span"] == 2
    assert r["traced_ms_per_step"] == 1.05
