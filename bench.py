#!/usr/bin/env python3
"""bench.py — Msamples/s of the RTIOW cover-scene render on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--precision f64|f32] [--config 1|2]
  (N > 1: one rank per GPU, RCCL backend.  Either launched by
  torch.distributed.run, or — plain `python bench.py --gpus N` — this script
  starts torch.distributed.run itself as a child process before touching the
  GPU; rank 0 prints the one JSON line, with "dist": backend, world size,
  samples per rank and the time of one gather.)

Workload (BASELINE.json configs[1]): cover scene (generateRandomScene,
DefaultPrng.init(42), main.zig:157-221), 1200x675 (16:9), 500 spp per GPU,
depth 50, scene resident in HBM before the timed region.  A step is one whole
frame: the trace megakernel + the chunk-combine/quantise kernel (+ at N > 1
the RCCL gather of every rank's interleaved rows to rank 0).

Weak scaling: at N GPUs the job is the same 1200x675 frame at N*500 spp,
image rows interleaved across ranks (rank r: rows r, r+N, ...), so every rank
traces 1200 x 675/N x 500N ~= 405 M samples, bit-identical to the same rows of
a 1-GPU render of the N*500-spp frame.  value = samples of all ranks / max
rank time.

Extra fields: roofline (dominant kernel = trace; HIP events on the render
stream), cpu_baseline (oracle Tier A = the reference's algorithm, sequential
RNG, one core, on a bounded sample of the same frame), f32_hybrid_variant,
wavefront_variant (BASELINE configs[3]: the same frame on the wavefront
engine, bit-identical image, with its HBM roofline), globe_10k_variant
(configs[4]: globe + 10k spheres through the BVH world kernel) and
cornell_variant (scene 6, the reference's default scene) at N = 1.
--engine wavefront makes the wavefront engine the headline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))

W_IMG, ASPECT, SPP, DEPTH, SEED = 1200, 16 / 9, 500, 50, 42
# Algorithmic flops per sphere test, counted from hittable.zig:96-101 with the
# per-segment invariants hoisted: static 17, moving 23.
FLOP_STATIC, FLOP_MOVING = 17, 23
PEAK_FP64_VALU_TF = 78.6   # MI355X FP64 vector (MI355X_MICROARCH.md: FP32 157.3 = 2x)
PEAK_FP32_VALU_TF = 157.3
PEAK_HBM_GBS = 8000.0


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--engine", default="megakernel", choices=["megakernel", "wavefront"],
                    help="headline engine (the other one is reported as a variant)")
    ap.add_argument("--wf-paths", type=int, default=0, help="wavefront in-flight paths (0 = library default)")
    ap.add_argument("--wf-sets", type=int, default=0, help="wavefront queue sets, params.wf_sets (0 = library default)")
    ap.add_argument("--wf-drain", default="samples", choices=["samples", "slots", "none"], help="params.wf_drain")
    ap.add_argument("--wf-form", default="fused", choices=["fused", "split"], help="params.wf_form")
    ap.add_argument("--wf-bounces", type=int, default=0, help="params.wf_bounces: bounce segments per wf_step launch")
    ap.add_argument("--wf-passes", type=int, default=0, help="params.wf_passes: queue passes per wf_step launch")
    ap.add_argument("--no-wavefront-variant", action="store_true")
    ap.add_argument("--no-world-variants", action="store_true", help="skip the configs[4] globe and Cornell lines")
    ap.add_argument("--config", type=int, default=1, choices=[1, 2],
                    help="BASELINE config: 1 = 1200x675, 500 spp per GPU (weak scaling, default); "
                         "2 = 3840x2160 at 2000 spp for the whole job (strong scaling)")
    ap.add_argument("--spp", type=int, default=SPP, help="spp per GPU (default 500 = configs[1])")
    ap.add_argument("--width", type=int, default=W_IMG)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-f32-variant", action="store_true")
    ap.add_argument("--cpu-spp", type=int, default=64, help="spp of the bounded CPU sample (~15-25 s on one core)")
    return ap.parse_args(argv)


def parse():
    return parse_args()


EVIDENCE_ROUNDS = ("r06", "r05", "r04", "r03", "r02", "r01")  # newest first


def evidence(name):
    """Path of a committed PMC evidence file: the newest round's copy
    (profiles/r06, else r05, r04, ...)."""
    for rnd in EVIDENCE_ROUNDS:
        path = os.path.join(REPO, "profiles", rnd, name)
        if os.path.exists(path):
            return path
    return os.path.join(REPO, "profiles", EVIDENCE_ROUNDS[-1], name)


def same_per_rank_work(c, args, W, rc, spp):
    """Does a committed PMC evidence file (measured on ONE launch of the N=1
    frame: c = its width, height, spp, precision) describe this rank's launch?
    At N > 1 a rank renders rows r::N of the frame at N x spp (weak scaling),
    i.e. the N=1 frame's samples within 1 % (the row split's remainder), with
    the same kernel, scene and per-unit work, so the per-launch evidence
    applies to every rank's launch; `evidence_scope` in the line says so."""
    if (c.get("width"), c.get("precision")) != (W, args.precision) or not c.get("height") or not c.get("spp"):
        return False
    ev = c["height"] * c["spp"]
    return abs(rc * spp - ev) <= 0.01 * ev


def evidence_scope(world, W, rc, spp):
    """What the PMC figures of a roofline (traffic, valu_issue) describe: the
    committed passes named by its *_source fields, made in another process
    (usually on another box) on the same workload — not this line's launch."""
    if world == 1:
        return (f"same workload ({W}x{rc} at {spp} spp, N=1): committed PMC passes named in the *_source "
                f"fields, another process; not this launch")
    return (f"per-rank launch: rows r::{world} at {spp} spp = {rc * W * spp / 1e6:.1f} M samples, the N=1 frame's "
            f"workload within 1 %; evidence: committed PMC passes of the N=1 workload named in the *_source fields")


def traffic_per_launch(args, W, rc, spp):
    """HBM bytes per trace launch from the committed PMC passes of the same
    per-rank workload (evidence("traffic.json"), tools/gpu_evidence.sh), else None."""
    path = evidence("traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    if not same_per_rank_work(t.get("config", {}), args, W, rc, spp):
        return None
    return round(t["traffic_bytes_per_launch"])


def valu_issue(args, W, rc, spp):
    """VALU-issue evidence of the same per-rank workload from the committed PMC
    passes (evidence("valu_issue.json"), tools/gpu_pmc_valu.sh + tools/valu_json.py),
    else None: the share of SIMD cycles the VALU issues and the VALU
    instructions per wave-iteration (one bounce segment per lane)."""
    path = evidence("valu_issue.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    if not same_per_rank_work(t.get("config", {}), args, W, rc, spp):
        return None
    return {"busy_frac": t["valu_busy_frac"], "valu_per_wave_iteration": t["valu_per_wave_iteration"],
            "variant": t.get("variant"), "source": os.path.relpath(path, REPO) + " (PMC SQ_ACTIVE_INST_VALU, "
            "SQ_INSTS_VALU of one launch)"}


def wf_traffic(args, W, rc, spp):
    """HBM bytes of one wavefront frame (every bounce launch + the drain) from
    the committed PMC passes of the same per-rank workload and engine form
    (evidence("wf_traffic.json"), tools/gpu_pmc_wf.sh), else None."""
    path = evidence("wf_traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    c = t.get("config", {})
    fused = args.wf_form == "fused"
    if not same_per_rank_work(c, args, W, rc, spp) or args.wf_paths != 0 or c.get("fused", False) != fused \
            or c.get("sets", 1) != wf_sets(args) or args.wf_drain != "samples" \
            or (fused and c.get("passes", 1) != wf_passes(args)) or (args.wf_bounces or 1) != c.get("bounces", 1):
        return None
    return round(t["traffic_bytes_per_frame"])


def wf_sets(args):
    """Queue sets of the wavefront engine (--wf-sets = params.wf_sets, else the library default)."""
    import rtw_amd as R
    return int(args.wf_sets or R.DEFAULT_WF_SETS)


def wf_passes(args):
    """Queue passes per wf_step launch (--wf-passes = params.wf_passes, else the library default)."""
    import rtw_amd as R
    return int(args.wf_passes or R.DEFAULT_WF_PASSES)


def wf_params(args):
    """The wavefront engine's configuration fields of rtw_params (ABI v4)."""
    return dict(wf_paths=args.wf_paths, wf_sets=args.wf_sets, wf_drain=args.wf_drain, wf_form=args.wf_form,
                wf_bounces=args.wf_bounces, wf_passes=args.wf_passes)


def wf_kernels(args):
    """The kernels one wavefront frame runs under this configuration."""
    bounce = "wf_step" if args.wf_form == "fused" else "wf_extend + wf_shade"
    drain = {"samples": " + wf_drain", "slots": " + wf_finish", "none": ""}[args.wf_drain]
    return bounce + " (all bounce launches of one frame, every queue set)" + drain


_CPU_CHILD = r"""
import json, os, sys, tempfile, time
sys.path.insert(0, os.path.join(sys.argv[1], "oracle"))
import rtw_oracle as O
W, H, spp, spp_a, depth, seed, aspect = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), \
    int(sys.argv[6]), int(sys.argv[7]), float(sys.argv[8])
allowed = sorted(os.sched_getaffinity(0))
d = tempfile.mkdtemp()
cmd = O.build_cpu_port(os.path.join(d, "port.so"))  # -O3 -march=native on THIS host
L = O.cpu_port_lib(os.path.join(d, "port.so"))
cam = O.cover_camera(aspect)
# one core at a time, like the single-threaded reference: the first and the
# last core of this process's set (a shared host's core 0 may be busier),
# half the sample each after a short warm-up; the faster core is reported
runs = []
for core in sorted({allowed[0], allowed[-1]}):
    os.sched_setaffinity(0, {core})
    sc, rng = O.cover_scene(seed)
    O.render_cpu_port(L, sc, cam, rng, W, 8, 4, depth)  # warm-up (clock ramp, page faults)
    sc, rng = O.cover_scene(seed)
    t0 = time.perf_counter()
    O.render_cpu_port(L, sc, cam, rng, W, H, spp // 2, depth)
    runs.append((W * H * (spp // 2) / (time.perf_counter() - t0) / 1e6, core, time.perf_counter() - t0))
rate, core, dt = max(runs)
os.sched_setaffinity(0, {core})
sc, rng = O.cover_scene(seed)
t1 = time.perf_counter()
_, _, st = O.render_tier_a(sc, cam, rng, W, H, spp_a, depth)
dta = time.perf_counter() - t1
print(json.dumps({"core": core, "cmd": cmd, "port_s": dt, "port_samples": W * H * (spp // 2), "tier_a_s": dta,
                  "tier_a_samples": st["samples"], "runs": [[round(r, 3), c] for r, c, _ in runs]}))
"""


def cpu_baseline(width, height, spp_sample):
    """The reference's CPU render loop on ONE pinned core of this host: the
    performance port oracle/ro_cpu_port.c (Tier A's algorithm and image, bit
    for bit: one sequential DefaultPrng(42) stream, recursive rayColor, f64;
    tests/test_oracle_tier_a.py), compiled here with -O3 -march=native
    -ffp-contract=off, timed on the same frame at reduced spp in a child
    process pinned with sched_setaffinity.  Beside it: the oracle's Tier A
    (the checker) on a smaller sample, and Tier B on 16 threads.  Test /
    measurement infrastructure used only as the timed CPU baseline."""
    import subprocess
    spp_a = max(1, spp_sample // 8)
    out = subprocess.run([sys.executable, "-c", _CPU_CHILD, REPO, str(width), str(height), str(spp_sample), str(spp_a),
                          str(DEPTH), str(SEED), repr(ASPECT)], check=True, capture_output=True, text=True).stdout
    c = json.loads(out.strip().splitlines()[-1])
    try:
        cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        cpu = "unknown"
    res = {"value": round(c["port_samples"] / c["port_s"] / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
           "kind_detail": "C performance port of the reference's loop (oracle/ro_cpu_port.c: Tier A's algorithm and "
                          "image bit for bit, SIMD discriminants, hoisted invariants; Zig is unbuildable here), built "
                          f"on this host as `{c['cmd']}`, pinned to one core at a time (sched_setaffinity; the "
                          f"first and the last core of the process's set, the faster reported: Msamples/s per core "
                          f"{c['runs']}), timed on {spp_sample // 2} of {SPP} spp and reported as a per-sample rate",
           "sample": f"{width}x{height}x{spp_sample // 2} spp cover frame per core (1/{SPP // (spp_sample // 2)} of "
                     f"the spp), {c['port_samples']} samples in {c['port_s']:.1f} s on core {c['core']}; single "
                     f"thread; host CPU {cpu}",
           "oracle_tier_a": {"value": round(c["tier_a_samples"] / c["tier_a_s"] / 1e6, 3), "unit": "Msamples/s",
                             "cores": 1, "build": "oracle/Makefile (-O2 -ffp-contract=off): the checker, same image",
                             "sample": f"{width}x{height}x{spp_a} spp in {c['tier_a_s']:.1f} s, core {c['core']}"}}
    # Beside it: the GPU's own contract (Tier B, counter RNG, pixels independent)
    # on the box's CPU share (16 threads, OpenMP over rows) — context only.
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import rtw_oracle as O
    sc, _ = O.cover_scene(SEED)
    cam = O.cover_camera(ASPECT)
    threads = 16
    t0 = time.perf_counter()
    _, stb = O.render_tier_b(sc, cam, width, height, 2 * spp_sample, DEPTH, threads=threads)
    dtb = time.perf_counter() - t0
    res["multicore"] = {"value": round(stb["samples"] / dtb / 1e6, 3), "unit": "Msamples/s", "cores": threads,
                        "kind": "port (oracle Tier B, OpenMP over rows)",
                        "sample": f"{width}x{height}x{2 * spp_sample} spp, {stb['samples']} samples in {dtb:.1f} s"}
    return res


def world_roofline(scene, s, kernel_ms, info, lane=False):
    """Roofline of the world kernel: VALU issue.  Its byte stream is tiny
    (records and BVH nodes are L2-resident: nothing to price against HBM), so
    the roof is the SIMDs' instruction issue: 1024 SIMDs x clock / 4 cycles per
    wave64 VALU instruction.  achieved = the VALU instructions of one launch
    (PMC SQ_INSTS_VALU of the same config, profiles/rNN/world_pmc_<scene>.json,
    tools/gpu_world_pmc.sh + tools/world_pmc_json.py) / the launch time
    measured here; traffic = its PMC FETCH_SIZE (x2, gfx950) + WRITE_SIZE.
    With the per-lane BVH walk (lane) the instructions are each lane's own
    path, not the union of the wave's: the line's node visits per segment are
    per lane (the algorithm's work), and the vector memory pipeline's busy
    shares (td_busy_frac_pmc: the per-lane loads' data return) show the other
    bound the walk runs against."""
    path = evidence(f"world_pmc_{scene}.json")
    trav = "per-lane BVH walks (vector node loads)" if lane else "wave-cooperative BVH traversal (scalar node loads)"
    bound = "valu-issue (" + (trav if info["nodes"] else "wave-uniform scalar-loaded records; linear list, no BVH") + ")"
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return {"bound": bound, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    if f"{s.width}x{s.height}x{s.spp}" not in t["what"]:
        return {"bound": bound, "achieved": None, "peak": None, "unit": None, "frac": None, "traffic": None}
    insts = t["counters"]["SQ_INSTS_VALU"]
    achieved = insts / (kernel_ms * 1e-3) / 1e9
    peak = 1024 * t["clock_ghz"] / 4
    valu = {"achieved": round(achieved, 1), "peak": round(peak, 1), "unit": "G wave64 VALU instructions/s",
            "frac": round(achieved / peak, 4)}
    common = {"traffic": round(t["hbm_fetch_bytes"] + t["hbm_write_bytes"]),
              "valu_busy_frac_pmc": t["valu_busy_frac"], "wait_frac_of_wave_cycles": t["wait_frac_of_wave_cycles"],
              "valu_per_wave_iteration": t["valu_per_wave_iteration"], "kernel": "world_kernel",
              "source": os.path.relpath(path, REPO)}
    if lane and "td_busy_frac" in t:
        # The per-lane walk is bound by the vector memory pipeline's per-lane
        # data return: every node visit is three 16-B per-lane
        # loads and every primitive test seven, returned through the CU's TD.
        # achieved = the TD-busy cycles of the PMC launch (TD_TD_BUSY summed
        # over the 256 TDs) / the launch time measured here; peak = every TD
        # busy every cycle (256 x clock).  VALU issue rides along as a side field.
        tdc = t["vmem_counters"]["TD_TD_BUSY_sum"]
        a_td = tdc / (kernel_ms * 1e-3) / 1e9
        p_td = 256 * t["clock_ghz"]
        return {"bound": "vmem-return (TD: " + trav + ")", "achieved": round(a_td, 1), "peak": round(p_td, 1),
                "unit": "G TD-busy cycles/s", "frac": round(a_td / p_td, 4), "valu_issue": valu,
                "td_busy_frac_pmc": t["td_busy_frac"], "ta_busy_frac_pmc": t["ta_busy_frac"], **common}
    return {"bound": bound, **valu, **common,
            **({"td_busy_frac_pmc": t["td_busy_frac"], "ta_busy_frac_pmc": t["ta_busy_frac"]} if "td_busy_frac" in t else {})}


class ClockWindow:
    """The average shader clock over a timed loop (box-to-box
    spreads read beside the clock): rtw_sclk_probe on a side stream, one wave
    spinning for ~90 % of the loop's expected wall time (est_ms, from the LAST
    warm-up step: the first ones carry code-object loads and allocations),
    read after.  window_ms goes into the line beside the loop's wall time."""

    def __init__(self, R, torch, est_ms):
        self.side = torch.cuda.Stream()
        self.window_ms = round(max(1.0, 0.9 * est_ms), 3)
        self.p = R.SclkProbe(self.side.cuda_stream, self.window_ms)

    def mhz(self):
        return round(self.p.read(), 1)


def warm(fn, n, torch):
    """Run fn() n (>= 1) times; the wall time of the last one in ms."""
    for _ in range(max(1, n) - 1):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def world_variant(R, torch, scene, steps, warmup):
    """A general-world scene on the world kernel (csrc/rtw_world.hip) at the
    scene's own main.zig settings: scene 6 (Cornell box, the reference's
    default scene, 600x600x200) or 7 (BASELINE configs[4]: globe + 10k
    spheres, BVH, 1200x675x100, textured with the reference asset sekaichizu.png).
    Timed with HIP events around the world kernel; a counts pass gives the
    BVH statistics (node visits and primitive tests per segment, counted per
    active lane of the wave-cooperative traversal)."""
    from rtw_amd import world as Wd
    earth = Wd.earth_map()  # the reference asset assets/sekaichizu.png (configs[4])
    b = Wd.BuiltScene(scene, SEED, image=earth if scene in (4, 7) else None)
    s = b.settings
    cam = b.camera()
    p = R.make_params(s.width, s.height, s.spp, DEPTH, SEED, background=b.background)
    dw = Wd.DeviceWorld(b.desc)
    need = dw.workspace_bytes(p)  # + the tail dealing's rings (rtw_world_workspace_bytes)
    ws = torch.empty(need + 256, dtype=torch.uint8, device="cuda:0")
    ptr = (ws.data_ptr() + 255) & ~255
    rgb = torch.empty((s.height, s.width, 3), dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    warm_ms = warm(lambda: dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st), warmup, torch)
    timers = [R.Timer() for _ in range(steps)]
    clk = ClockWindow(R, torch, steps * warm_ms)
    a = time.perf_counter()
    for i in range(steps):
        dw.render_async(cam, p, ptr, need, rgb.data_ptr(), None, st, timers[i])
    torch.cuda.synchronize()
    e = time.perf_counter() - a
    sclk = clk.mhz()
    ms = sum(t.elapsed_ms() for t in timers) / steps
    for t in timers:
        t.close()
    c = dw.counts(cam, p, ptr, need)
    info = dw.bvh_info()
    launch = dw.launch_info(p)
    dw.close()
    samples = s.width * s.height * s.spp
    lane = c.get("lane_interior_iters", 0) > 0
    roof = world_roofline(scene, s, ms, info, lane)
    return {"value": round(samples * steps / e / 1e6, 2), "unit": "Msamples/s", "ms_per_step": round(e / steps * 1e3, 3),
            "kernel_ms": round(ms, 3), "sclk_mhz": sclk, "sclk_window_ms": clk.window_ms,
            "tail_dealing": c["tail_dealing"],
            "traversal": ("per-lane walks" if lane else "wave union") if info["nodes"] else "linear",
            "config": {"scene": scene, "name": Wd.SCENES[scene], "width": s.width,
                                                  "height": s.height, "spp": s.spp, "max_depth": DEPTH},
            "bvh": info, "launch": launch, "segments_per_sample": round(c["segments"] / samples, 3),
            "node_visits_per_segment": round(c["node_visits"] / max(1, c["segments"]), 2),
            "prim_tests_per_segment": round(c["prim_tests"] / max(1, c["segments"]), 2),
            "roofline": roof,
            "note": "world kernel, f64, bit-identical to oracle Tier B (tests/test_gpu_world.py)"}


def wavefront_bytes(counts, precision, units, fused=True, bounces=1):
    """Algorithmic HBM bytes of one wavefront frame (rtw_wavefront.hip): per
    bounce segment of the fused engine (default), wf_step reads the path +
    its hit winner and writes the next path + its winner (since round 6 a hit
    path's origin IS its hit point, so the root is not stored: 200 B f64,
    216 B before); of the split
    engine (--wf-form split), extend reads o, d, time (+ the skip word in f32)
    and writes (root, winner), shade reads the path + (root, winner) and
    writes the path.  Per sample: the home slot's unit, sample index and f64x3 sum
    (read + write).  Per unit: the f64x3 chunk sum.  `counts` is the
    wavefront engine's own counts pass: segments traced by the in-register
    drain (wf_finish, counts["drain_segments"]) move no queue bytes (its one
    load of each live path, <= 96 B x slots, is left out: < 0.1 %).  With
    `bounces` segments per wf_step launch (params.wf_bounces) a path crosses
    the queues once per `bounces` segments."""
    r = 8 if precision == "f64" else 4
    path = 10 * r + 8 + 4 + 4
    if fused:  # fused engine: path + hit winner read, path + winner written (o = the hit point: no root)
        seg = 2 * (path + 4)
    else:  # extend reads o, d, time (+ skip), writes the hit; shade reads path + hit, writes the path
        seg = (7 * r + (4 if precision == "f32" else 0)) + (r + 4) + (path + r + 4) + path
    queued = counts["segments"] - counts.get("drain_segments", 0)
    return queued * seg // max(1, bounces) + counts["samples"] * (2 * (24 + 4) + 4) + units * 24


def wf_frame_bytes(args, counts, units):
    """wavefront_bytes of a frame rendered with args' engine configuration: the
    fused form crosses the queues once per args.wf_bounces segments, the split
    form once per segment.  The one call both wavefront rooflines (the headline
    with --engine wavefront and the wavefront_variant line) make, so they agree
    (the headline passed no bounce count)."""
    fused = args.wf_form == "fused"
    return wavefront_bytes(counts, args.precision, units, fused, (args.wf_bounces or 1) if fused else 1)


def wavefront_variant(args, R, rend, cam, out, W, H, spp, rb, rs, rc, counts, samples_all, world, rank, dist,
                      tg, torch):
    """configs[3]: the same frame on the wavefront engine (bit-identical image,
    tests/test_gpu_wavefront.py), timed the same way; roofline = HBM (the
    path queues stream through HBM every bounce)."""
    p = R.make_params(W, H, spp, DEPTH, SEED, row_begin=rb, row_stride=rs, row_count=rc,
                      precision=args.precision, engine="wavefront", **wf_params(args))
    counts = rend.counts(cam, p)  # untimed: the queue / in-register split of the segments
    torch.cuda.synchronize()
    warm_ms = warm(lambda: rend.render(cam, p, out=out), args.warmup, torch)
    timers = [R.Timer() for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    clk = ClockWindow(R, torch, args.steps * warm_ms)
    a = time.perf_counter()
    for i in range(args.steps):
        rend.render(cam, p, out=out, timer=timers[i])
        if world > 1:
            tg.gather(out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    e = time.perf_counter() - a
    if world > 1:
        t = torch.tensor([e], dtype=torch.float64, device=out.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        e = float(t.item())
    ms = sum(t.elapsed_ms() for t in timers) / len(timers)
    for t in timers:
        t.close()
    sclk = clk.mhz()
    chunk = min(R.DEFAULT_CHUNK, spp)
    units = rc * W * ((spp + chunk - 1) // chunk)
    byts = wf_frame_bytes(args, counts, units)
    gbs = byts / (ms * 1e-3) / 1e9
    drain = counts.get("drain_segments", 0) / max(1, counts["segments"])
    # The same frame with 2 and 3 bounce segments per wf_step launch
    # (params.wf_bounces; the path kept in registers between them: fewer,
    # longer launches and 1/K of the queue bytes), timed the same way.
    sweep = {}
    if args.wf_bounces == 0 and args.wf_form == "fused":
        for k in (2, 3):
            pk = R.make_params(W, H, spp, DEPTH, SEED, row_begin=rb, row_stride=rs, row_count=rc,
                               precision=args.precision, engine="wavefront", **{**wf_params(args), "wf_bounces": k})
            warm(lambda: rend.render(cam, pk, out=out), 1, torch)
            tk = [R.Timer() for _ in range(args.steps)]
            if world > 1:
                dist.barrier()
            a = time.perf_counter()
            for i in range(args.steps):
                rend.render(cam, pk, out=out, timer=tk[i])
                if world > 1:
                    tg.gather(out)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            ek = time.perf_counter() - a
            if world > 1:
                t = torch.tensor([ek], dtype=torch.float64, device=out.device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                ek = float(t.item())
            msk = sum(t.elapsed_ms() for t in tk) / len(tk)
            for t in tk:
                t.close()
            bk = wavefront_bytes(counts, args.precision, units, True, k)
            sweep[str(k)] = {"value": round(samples_all * args.steps / ek / 1e6, 2),
                             "ms_per_step": round(ek / args.steps * 1e3, 3), "loop_ms_per_frame": round(msk, 3),
                             "hbm_frac": round(bk / (msk * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
                             "algorithmic_bytes_per_frame": bk}
    return {"value": round(samples_all * args.steps / e / 1e6, 2), "ms_per_step": round(e / args.steps * 1e3, 3),
            "wf_paths": args.wf_paths or R.DEFAULT_WF_PATHS, "wf_sets": wf_sets(args), "wf_drain": args.wf_drain,
            "wf_form": args.wf_form, "wf_bounces": args.wf_bounces or 1,
            "wf_passes": wf_passes(args) if args.wf_form == "fused" else 1, "sclk_mhz": sclk, "sclk_window_ms": clk.window_ms,
            "bounces_per_launch": sweep,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": wf_traffic(args, W, rc, spp),
                         "traffic_source": os.path.relpath(evidence("wf_traffic.json"), REPO),
                         "evidence_scope": evidence_scope(world, W, rc, spp),
                         "kernel": wf_kernels(args),
                         "loop_ms_per_frame": round(ms, 3), "algorithmic_bytes_per_frame": byts,
                         "drain_segment_frac": round(drain, 4)},
            "note": "engine=wavefront (BASELINE configs[3]): per-bounce kernels over SoA path queues in HBM; "
                    "same Tier-B image as the megakernel, bit for bit"}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, n, port):
    """The torch.distributed.run command that starts one rank per GPU with the
    same bench arguments (rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def maybe_launch(args, argv) -> int | None:
    """`python bench.py --gpus N` with N > 1 and no rank environment: start N
    rank processes (one per GPU) as children and return their exit code.
    Runs before anything touches the GPU (the parent never initialises HIP,
    and starts the ranks as child processes, never by exec)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = launch_command(argv, args.gpus, free_port())
    return subprocess.run(cmd, env=env).returncode


def dry_run(args):
    """RTW_BENCH_DRYRUN=1: the launcher, rendezvous, shard split, gather and
    max-over-ranks path of a multi-rank run without a GPU (gloo, CPU tensors,
    no rendering) — the CPU test of the launcher path (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist

    from rtw_amd.shard import TileGather, shard_rows
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    W, H, spp = workload(args, world)
    rb, rs, rc = shard_rows(H, rank, world)
    out = torch.full((rc, 4, 3), rank, dtype=torch.uint8)
    tg = TileGather(out, H, rank, world)
    t0 = time.perf_counter()
    for _ in range(max(1, args.steps)):
        tg.gather(out)
    step_ms = (time.perf_counter() - t0) / max(1, args.steps) * 1e3
    img = tg.image()
    samples = torch.tensor([float(rc * W * spp)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(samples)
    # the per-rank timing fields of the GPU line (the "trace" here is the dry
    # step, made rank-dependent so the max-over-ranks rule is visible)
    own = step_ms * (1.0 + 0.25 * rank)
    per = rank_times(dist, world, step_ms, own, torch.device("cpu"))
    if rank == 0:
        ok = bool((img[:, 0, 0] == torch.arange(H) % world).all())
        # the PMC evidence the GPU line would carry for this rank's launch
        ev = {"traffic": traffic_per_launch(args, W, rc, spp), "valu_issue": valu_issue(args, W, rc, spp),
              "wf_traffic": wf_traffic(args, W, rc, spp), "evidence_scope": evidence_scope(world, W, rc, spp)}
        print(json.dumps({"dry_run": True, "dist": {"backend": dist.get_backend() if world > 1 else None,
                                                    "world_size": world, **per},
                          "width": W, "height": H, "spp_frame": spp, "samples_all": samples.item(),
                          "rows_interleaved_ok": ok, "evidence": ev,
                          "trace_ms_per_launch": round(roofline_launch_ms(world, own, per), 3)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def rank_times(dist, world, step_ms, trace_ms, dev):
    """Every rank's mean step time and mean trace-kernel time (all_gather) and
    the trace imbalance max/mean: whether the interleaved rows balance."""
    import torch
    mine = torch.tensor([step_ms, trace_ms], dtype=torch.float64, device=dev)
    if world > 1:
        allr = [torch.zeros(2, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(allr, mine)
    else:
        allr = [mine]
    step = [round(float(x[0]), 3) for x in allr]
    trace = [round(float(x[1]), 3) for x in allr]
    return {"rank_step_ms": step, "rank_trace_ms": trace,
            "imbalance": round(max(trace) / (sum(trace) / len(trace)), 4) if sum(trace) > 0 else None}


def roofline_launch_ms(world, own_ms, per_rank):
    """The trace-launch time the roofline divides by: at N > 1 the SLOWEST
    rank's (as `elapsed` is the slowest rank's wall time), so a fast rank 0
    does not flatter the frac (VERDICT r5 ask 6; every rank's launch does the
    same work within 1 %); at N = 1 this rank's own."""
    return max(per_rank["rank_trace_ms"]) if world > 1 else own_ms


def workload(args, world):
    """(W, H, frame spp) of the run.  configs[1] (default): 1200x675, 500 spp per
    GPU (weak scaling: the frame gets N x 500 spp).  configs[2] (--config 2):
    3840x2160 at 2000 spp for the whole job (strong scaling: total work fixed,
    rows split over the ranks)."""
    import rtw_amd as R
    if args.config == 2:
        return 3840, R.image_height(3840, ASPECT), 2000
    return args.width, R.image_height(args.width, ASPECT), args.spp * world


def main():
    args = parse()
    rc = maybe_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("RTW_BENCH_DRYRUN"):
        return dry_run(args)
    import torch
    import torch.distributed as dist

    import rtw_amd as R
    from rtw_amd.device import TorchRenderer
    from rtw_amd.shard import TileGather, shard_rows

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (no CPU fallback)")
    # Rehearsal knobs (N > 1 on a box with fewer GPUs; never used by the
    # driver): RTW_DIST_BACKEND=gloo, RTW_SHARE_GPU=1 (rank r on GPU r mod count).
    backend = os.environ.get("RTW_DIST_BACKEND", "nccl")
    if os.environ.get("RTW_SHARE_GPU"):
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    W, H, spp = workload(args, world)  # configs[1]: the frame gets N x spp (weak); configs[2]: fixed (strong)
    sph, mats, _ = R.cover_scene(SEED)
    cam = R.cover_camera(ASPECT)
    rb, rs, rc = shard_rows(H, rank, world)
    params = R.make_params(W, H, spp, DEPTH, SEED, row_begin=rb, row_stride=rs, row_count=rc,
                           precision=args.precision, engine=args.engine, **wf_params(args))
    rend = TorchRenderer(sph, mats, local)
    out = torch.empty((rc, W, 3), dtype=torch.uint8, device=f"cuda:{local}")
    samples_rank = rc * W * spp
    tg = TileGather(out, H, rank, world)  # send tile + rank 0's receive tiles, allocated once

    # Untimed: counts pass (algorithmic flops of one trace launch) + warmup.
    counts = rend.counts(cam, R.make_params(W, H, spp, DEPTH, SEED, row_begin=rb, row_stride=rs, row_count=rc,
                                            precision=args.precision))
    torch.cuda.synchronize()

    def step_warm():
        rend.render(cam, params, out=out)
        if world > 1:
            tg.gather(out)
    warm_ms = warm(step_warm, args.warmup, torch) if args.warmup > 0 else 0.0

    # One HIP-event pair per step brackets that step's trace-kernel launch on
    # the render stream (torch's current stream), read after the region.
    timers = [R.Timer() for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    clk = ClockWindow(R, torch, args.steps * warm_ms) if args.warmup > 0 else None
    t0 = time.perf_counter()
    for i in range(args.steps):
        rend.render(cam, params, out=out, timer=timers[i])
        if world > 1:
            tg.gather(out)  # RCCL gather of the row tile to rank 0 (no allocation, no assembly)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    per = [t.elapsed_ms() for t in timers]
    trace_ms_avg = sum(per) / len(per)
    for t in timers:
        t.close()
    sclk = clk.mhz() if clk is not None else None

    dist_info = {"backend": None, "world_size": 1, "samples_per_rank": [samples_rank], "gather_ms": None}
    per_rank_t = rank_times(dist, world, elapsed / args.steps * 1e3, trace_ms_avg, torch.device("cuda", local))
    if world > 1:
        frame = tg.image()  # rank 0 interleaves the last gathered tiles once, after the timed region
        if rank == 0:
            assert frame.shape == (H, W, 3)
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [torch.zeros(1, dtype=torch.float64, device=f"cuda:{local}") for _ in range(world)]
        dist.all_gather(per_rank, torch.tensor([float(samples_rank)], dtype=torch.float64, device=f"cuda:{local}"))
        per_rank = [int(x.item()) for x in per_rank]
        samples_all = float(sum(per_rank))
        # One more gather, timed alone (it is also inside every timed step above).
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        tg.gather(out)
        torch.cuda.synchronize()
        gt = torch.tensor([time.perf_counter() - g0], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "samples_per_rank": per_rank, "gather_ms": round(float(gt.item()) * 1e3, 3)}
    dist_info.update(per_rank_t)
    if world == 1:
        samples_all = float(samples_rank)
    trace_ms_avg = roofline_launch_ms(world, trace_ms_avg, per_rank_t)

    ms_per_step = elapsed / args.steps * 1e3
    value = samples_all * args.steps / elapsed / 1e6

    # Roofline of the dominant kernel (trace): algorithmic flops per launch /
    # average launch time.  HBM: algorithmic bytes per launch = one f64x3
    # chunk sum (24 B) per (pixel, chunk) unit written + scene tables read.
    flops = counts["static_tests"] * FLOP_STATIC + counts["moving_tests"] * FLOP_MOVING
    achieved_tf = flops / (trace_ms_avg * 1e-3) / 1e12
    peak = PEAK_FP64_VALU_TF if args.precision == "f64" else PEAK_FP32_VALU_TF
    chunk = min(R.DEFAULT_CHUNK, spp)
    n_chunks = (spp + chunk - 1) // chunk
    hbm_bytes = rc * W * n_chunks * 24
    hbm_gbs = hbm_bytes / (trace_ms_avg * 1e-3) / 1e9
    if args.engine == "megakernel":
        roofline = {
            "bound": "valu-fp64" if args.precision == "f64" else "valu-fp32",
            "achieved": round(achieved_tf, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved_tf / peak, 4),
            "traffic": traffic_per_launch(args, W, rc, spp),
            "traffic_source": os.path.relpath(evidence("traffic.json"), REPO),
            "kernel": "trace_kernel", "trace_ms_per_launch": round(trace_ms_avg, 3), "sclk_mhz": sclk,
            "sclk_window_ms": clk.window_ms if clk is not None else None,
            "flop_per_launch": flops, "segments_per_launch": counts["segments"],
            "hbm": {"achieved": round(hbm_gbs, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(hbm_gbs / PEAK_HBM_GBS, 7), "algorithmic_bytes_per_launch": hbm_bytes},
            "valu_issue": valu_issue(args, W, rc, spp),
            "evidence_scope": evidence_scope(world, W, rc, spp),
            "note": "megakernel is VALU-issue bound (valu_issue.busy_frac: the fraction of SIMD cycles in "
                    "which the VALU issues; f64, f32 and integer-multiply wave64 instructions each take ~4 cycles) plus "
                    "divergence; `achieved` counts only the algorithm's sphere-test flops; MFMA n/a (no "
                    "contraction); HBM traffic is ~24 B per chunk of samples by construction (DESIGN.md §Roofline)",
        }
    else:  # wavefront headline: HBM-bound path queues
        byts = wf_frame_bytes(args, rend.counts(cam, params), rc * W * n_chunks)
        gbs = byts / (trace_ms_avg * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": wf_traffic(args, W, rc, spp),
                    "traffic_source": os.path.relpath(evidence("wf_traffic.json"), REPO),
                    "evidence_scope": evidence_scope(world, W, rc, spp),
                    "kernel": wf_kernels(args), "wf_sets": wf_sets(args), "wf_drain": args.wf_drain,
                    "loop_ms_per_frame": round(trace_ms_avg, 3), "algorithmic_bytes_per_frame": byts,
                    "valu": {"achieved": round(achieved_tf, 3), "peak": peak, "unit": "TFLOP/s",
                             "frac": round(achieved_tf / peak, 4)}}

    extra = {}
    if not args.no_f32_variant and args.precision == "f64":
        p32 = R.make_params(W, H, spp, DEPTH, SEED, row_begin=rb, row_stride=rs, row_count=rc, precision="f32",
                            engine=args.engine, **wf_params(args))
        for _ in range(max(1, args.warmup)):
            rend.render(cam, p32, out=out)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        a = time.perf_counter()
        for _ in range(args.steps):
            rend.render(cam, p32, out=out)
            if world > 1:
                tg.gather(out)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e32 = time.perf_counter() - a
        if world > 1:
            t = torch.tensor([e32], dtype=torch.float64, device=f"cuda:{local}")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e32 = float(t.item())
        extra["f32_hybrid_variant"] = {"value": round(samples_all * args.steps / e32 / 1e6, 2),
                                       "ms_per_step": round(e32 / args.steps * 1e3, 3),
                                       "note": "precision=f32 (f32 + f64 wide spheres + convex self-skip); "
                                               "not the headline: the reference computes in f64"}

    if not args.no_wavefront_variant and args.engine == "megakernel":
        extra["wavefront_variant"] = wavefront_variant(args, R, rend, cam, out, W, H, spp, rb, rs, rc, counts,
                                                       samples_all, world, rank, dist, tg, torch)

    if world == 1 and not args.no_world_variants:
        # (at least 10 renders each: one world render varies +-7 % on one box, profiles/r05/world_spread.txt)
        extra["globe_10k_variant"] = world_variant(R, torch, 7, max(10, args.steps // 2), 2)
        extra["cornell_variant"] = world_variant(R, torch, 6, max(10, args.steps // 2), 2)

    res = {
        "metric": "Msamples/sec (pixels x spp / s), RTIOW cover scene; trace-kernel roofline",
        "value": round(value, 2),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.config == 2 else "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic: the reference's own scene generator (seed 42); no external data",
        "config": {"workload": (f"BASELINE configs[2]: RTIOW cover scene {W}x{H}, {spp} spp frame, depth {DEPTH}, "
                                f"rows interleaved over {world} GPU(s)") if args.config == 2 else
                               (f"BASELINE configs[1]: RTIOW cover scene {W}x{H}, {args.spp} spp per GPU ({spp} spp "
                                f"frame), depth {DEPTH}, rows interleaved over {world} GPU(s)"),
                   "width": W, "height": H, "spp_frame": spp, "max_depth": DEPTH, "seed": SEED,
                   "precision": args.precision, "parallelism": f"rows{world}"},
        "dist": dist_info,
        "roofline": roofline,
    }
    res.update(extra)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(W, H, args.cpu_spp)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
