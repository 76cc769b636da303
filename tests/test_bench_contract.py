"""The committed bench line (profiles/r01/bench.json, written by bench.py on an
MI355X) keeps the driver's contract: the BASELINE metric and unit, whole-job
throughput consistent with ms_per_step, the roofline object (bound, achieved,
peak, unit, frac = achieved / peak, traffic from the PMC passes) with the
VALU-issue evidence of profiles/r01/valu_issue.json, and a bounded
cpu_baseline.  CPU-only: it reads files, it runs nothing."""
import json
import os

from conftest import REPO

BENCH = os.path.join(REPO, "profiles", "r01", "bench.json")


def load(name):
    with open(os.path.join(REPO, "profiles", "r01", name)) as f:
        return json.load(f)


def test_bench_line_contract():
    b = load("bench.json")
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert b["metric"].startswith("Msamples/sec")
    assert "Msamples/sec" in base["metric"]
    assert b["unit"] == "Msamples/s" and b["higher_is_better"] is True and b["scaling"] == "weak"
    assert b["n_gpus"] == 1 and b["dtype"] == "f64" and b["vs_baseline"] is None
    c = b["config"]
    assert (c["width"], c["height"], c["spp_frame"], c["max_depth"], c["seed"]) == (1200, 675, 500, 50, 42)
    samples = c["width"] * c["height"] * c["spp_frame"]
    # value = samples / wall time of one step (ms_per_step), within rounding
    assert abs(b["value"] - samples / (b["ms_per_step"] * 1e-3) / 1e6) / b["value"] < 0.01


def test_roofline_fields_are_consistent():
    r = load("bench.json")["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["unit"] == "TFLOP/s" and r["peak"] == 78.6
    # achieved = algorithmic flops per launch / the launch's average duration
    assert abs(r["achieved"] - r["flop_per_launch"] / (r["trace_ms_per_launch"] * 1e-3) / 1e12) < 0.01 * r["achieved"]
    t = load("traffic.json")
    assert r["traffic"] == round(t["traffic_bytes_per_launch"])
    v = load("valu_issue.json")
    assert r["valu_issue"]["busy_frac"] == v["valu_busy_frac"]
    assert r["valu_issue"]["valu_per_wave_iteration"] == v["valu_per_wave_iteration"]
    assert 0.5 < v["valu_busy_frac"] <= 1.0
    h = r["hbm"]
    assert h["unit"] == "GB/s" and h["peak"] == 8000.0 and h["frac"] < 0.01


def test_rocprof_summary_agrees_with_the_event_timing():
    import csv
    r = load("bench.json")["roofline"]
    rows = list(csv.DictReader(open(os.path.join(REPO, "profiles", "r01", "bench_kernel_stats.csv"))))
    trace = [x for x in rows if x["Name"].startswith("void rtwk::trace_kernel<double, false, 0,")]
    assert trace, "no f64 trace_kernel row in the rocprofv3 summary"
    avg_ms = float(trace[0]["AverageNs"]) / 1e6
    assert abs(avg_ms - r["trace_ms_per_launch"]) / avg_ms < 0.05


def test_cpu_baseline_is_bounded_and_stated():
    cb = load("bench.json")["cpu_baseline"]
    assert cb["unit"] == "Msamples/s" and cb["cores"] == 1 and cb["kind"] in ("port", "reference")
    assert cb["value"] > 0 and "spp" in cb["sample"]


def test_wavefront_traffic_is_the_pmc_measurement():
    wf = load("bench.json")["wavefront_variant"]["roofline"]
    t = load("wf_traffic.json")
    assert wf["traffic"] == round(t["traffic_bytes_per_frame"])
    # the queues move close to their algorithmic bytes (no wasted re-reads)
    assert 0.8 < wf["traffic"] / wf["algorithmic_bytes_per_frame"] < 1.5
    assert abs(wf["frac"] - wf["achieved"] / wf["peak"]) < 1e-3
