"""BASELINE configs[0] as named: "RTIOW final cover scene, 400x225, 100 spp,
depth 50 -- Zig CPU reference to PPM (no GPU)".

Zig cannot run here, so the artifact is the oracle's Tier A restatement of the
reference's whole main() for scene 1 (oracle/rtw_oracle.c ro_main_cover:
DefaultPrng.init(42) shared by generateRandomScene and the raster-order render
loop, main.zig:295-402, f64, recursive rayColor, quantise :395-400), one
thread.  Records the sha256 of its PPM (the bytes the reference's PNG would
hold, main.zig:396/405), the per-channel image mean, the oracle's counts and
the single-core wall time of this run.
Writes tests/golden/config0_tier_a_400x225x100.json
(tests/test_oracle_tier_a.py::test_config0_artifact re-renders and compares).
python tests/golden/make_config0.py"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

W, ASPECT, SPP, DEPTH, SEED = 400, 16 / 9, 100, 50, 42


def ppm_bytes(img) -> bytes:
    h, w, _ = img.shape
    return b"P6\n%d %d\n255\n" % (w, h) + img.tobytes()


def render():
    import rtw_oracle as O
    t0 = time.perf_counter()
    img, st = O.main_cover(W, ASPECT, SPP, DEPTH, SEED)
    return img, st, time.perf_counter() - t0


if __name__ == "__main__":
    img, st, dt = render()
    try:
        cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        cpu = "unknown"
    rec = {"config": "BASELINE configs[0]: RTIOW cover scene 400x225, 100 spp, depth 50, seed 42 (oracle Tier A = "
                     "the reference main() restated, sequential DefaultPrng(42) stream)",
           "width": W, "height": int(img.shape[0]), "spp": SPP, "max_depth": DEPTH, "seed": SEED,
           "ppm_sha256": hashlib.sha256(ppm_bytes(img)).hexdigest(),
           "mean_rgb": [round(float(x), 4) for x in img.reshape(-1, 3).mean(0)],
           "samples": st["samples"], "segments": st["segments"],
           "wall_s_one_core": round(dt, 2), "msamples_per_s_one_core": round(st["samples"] / dt / 1e6, 3),
           "host_cpu": cpu}
    with open(os.path.join(HERE, "config0_tier_a_400x225x100.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
