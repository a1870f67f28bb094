"""The committed bench line's decode roofline closes against the committed profiles (verdict r5 item 5), on CPU:
achieved = the step's algorithmic bytes / ms_per_step, frac = achieved / 8 TB/s, and the rocprof_check figures are
what bench.py derives from profiles/r06_bench_rocprofv3_kernel_stats.csv and ..._step_spans.json: the GEMVs' traced
busy time per step is at most the traced run's own step, and the device-bound windows' summed kernel time is at
most their device span."""
import json
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = os.path.join(ROOT, "profiles", "r06_bench_line.json")


@pytest.fixture(scope="module")
def line():
    if not os.path.exists(LINE):
        pytest.skip("no committed r06 bench line")
    return json.load(open(LINE))


def test_decode_frac_from_step(line):
    rf = line["roofline"]
    achieved = rf["algorithmic_bytes_per_step"] / (line["ms_per_step"] * 1e-3) / 1e9
    assert abs(achieved - rf["achieved"]) <= 0.1 + 1e-3 * achieved
    assert abs(rf["frac"] - achieved / rf["peak"]) < 1e-3
    assert rf["peak"] == bench.HBM_PEAK_GBPS
    assert abs(rf["avg_launch_us"] - line["ms_per_step"] * 1e3 / rf["launches_per_step"]) < 0.01


def test_rocprof_check_matches_committed_profiles(line):
    rc = line["roofline"]["rocprof_check"]
    st = bench.rocprof_stats(os.path.join(ROOT, rc["source"]))
    calls = sum(c for k, (c, _) in st.items() if "k_gemv_q4_0<1," in k)
    ns = sum(t for k, (c, t) in st.items() if "k_gemv_q4_0<1," in k)
    busy = ns / (calls / line["roofline"]["launches_per_step"]) / 1e3
    assert calls == rc["gemv_calls"]
    assert abs(busy - rc["gemv_busy_us_per_step"]) < 0.1
    sp = json.load(open(os.path.join(ROOT, rc["spans_source"])))
    assert abs(sp["traced_ms_per_step"] * 1e3 - rc["traced_step_us"]) < 0.1
    # like for like inside the traced run: busy <= its own step, summed durations <= device span
    assert rc["busy_le_traced_step"] and busy <= rc["traced_step_us"]
    assert rc["window_sum_le_span"] and rc["window_sum_us_median"] <= rc["window_span_us_median"]
    assert sp["gap_free_windows"] == rc["device_bound_windows"] > 0


def test_prefill_roofline_names_the_instruction(line):
    rf = line["prefill"]["roofline"]
    assert "v_mfma_scale_f32_32x32x64_f8f6f4" in json.dumps(rf)
    assert 0 < rf["frac"] < 1
