"""VALU-issue accounting of one f64 trace launch (configs[1]) from the PMC
passes of tools/gpu_pmc_valu.sh -> profiles/<tag>/valu_issue.json, read by
bench.py for roofline.valu_issue.  Usage: valu_json.py <dir_a> <dir_b> <dir_c> <out>

busy_frac = SQ_ACTIVE_INST_VALU (quad-cycles, ~one per VALU instruction) x 4 /
(SIMDs x GRBM_GUI_ACTIVE / 8): the share of SIMD cycles in which the VALU
issues.  f64 add/mul/fma, f32 fma, v_pk_fma_f32 and 32-bit integer multiplies
take one wave64 instruction per ~4 cycles on a SIMD (tools/ubench_valu.hip)."""
import csv
import glob
import json
import re
import sys

SIMDS = 256 * 4
SEGMENTS = 922534227  # segments of one configs[1] launch (bench.py counts pass; seed 42)
# Phase costs from the phase-duplication builds (RTW_MEASURE, tools/gpu_measure.sh,
# variant 516): delta SQ_INSTS_VALU per wave-iteration when the phase runs twice.
PHASES = {"narrow_sphere_pretest": 371, "unit_ball_sampler_coop_reject": 347,
          "sample_start_uv_disk_camera_ray": 336, "hit_record_and_scatter": 236}


def counters(d):
    vals, var, ms = {}, None, None
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            m = re.search(r"trace_kernel<double, false, 0, (\d+)>", r["Kernel_Name"])
            if m:
                var = int(m.group(1))
                vals[r["Counter_Name"]] = vals.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for f in glob.glob(f"{d}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if re.search(r"trace_kernel<double, false, 0, ", r["Kernel_Name"]):
                ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return vals, var, ms


def main():
    a, b, c, out = sys.argv[1:5]
    res = {"what": "VALU issue accounting of ONE f64 trace_kernel launch, BASELINE configs[1] (1200x675x500), "
                   "rocprofv3 --kernel-trace --pmc, one pass per counter set (tools/gpu_pmc_valu.sh)",
           "config": {"width": 1200, "height": 675, "spp": 500, "precision": "f64"}}
    for d in (a, b, c):
        v, var, ms = counters(d)
        res.update({k: float(f"{x:.4g}") for k, x in v.items()})
        res.setdefault("dispatch_ms", ms)
        res["variant"] = var
    cyc = res["GRBM_GUI_ACTIVE"] / 8
    res["clock_ghz"] = round(cyc / (res["dispatch_ms"] * 1e-3) / 1e9, 3)
    res["segments_per_launch"] = SEGMENTS
    res["valu_per_wave_iteration"] = round(res["SQ_INSTS_VALU"] / (SEGMENTS / 64))
    res["valu_busy_frac"] = round(res["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * cyc), 3)
    # instruction mix per wave-iteration; "other" = moves, selects, compares,
    # bit operations and lane ops (the VALU classes the SQ does not count apart)
    wi = SEGMENTS / 64
    cls = {"f64": ["ADD_F64", "MUL_F64", "FMA_F64", "TRANS_F64"], "f32": ["ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32"],
           "int": ["INT32", "INT64"], "cvt": ["CVT"]}
    mix = {k: sum(res.get("SQ_INSTS_VALU_" + c, 0.0) for c in v) / wi for k, v in cls.items()}
    mix["other"] = res["SQ_INSTS_VALU"] / wi - sum(mix.values())
    res["valu_mix_per_wave_iteration"] = {k: round(x) for k, x in mix.items()}
    res["valu_mix_share"] = {k: round(x / (res["SQ_INSTS_VALU"] / wi), 3) for k, x in mix.items()}
    res["salu_per_wave_iteration"] = round(res["SQ_INSTS_SALU"] / wi)
    res["phase_valu_per_wave_iteration"] = dict(PHASES, variant_measured=516,
                                                method="phase executed twice on laundered inputs (same image)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
