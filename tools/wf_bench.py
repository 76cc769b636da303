"""Wavefront-engine timing of BASELINE configs[1] (1200x675x500, f64): best of
N renders, HIP events around the bounce loop.
  python tools/wf_bench.py [N] [CFG ...]
CFG (in-process A/B, configurations interleaved per round): comma-separated
rtw_params fields "paths=<wf_paths>", "sets=<wf_sets>", "drain=samples|slots|none",
"form=fused|split", "bounces=<wf_bounces>", "passes=<wf_passes>", "chunk=<chunk>", and environment settings that only a -DRTW_MEASURE library
reads (development knobs, e.g. "RTW_WF_GRID=4"); "-" is the default configuration."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfgs = sys.argv[2:] or ["-"]
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
base_env = dict(os.environ)


def apply(cfg):
    """Set the configuration's environment; return its params."""
    os.environ.clear()
    os.environ.update(base_env)
    kw = {}
    for kv in ([] if cfg == "-" else cfg.split(",")):
        k, v = kv.split("=")
        if k == "paths":
            kw["wf_paths"] = int(v)
        elif k == "sets":
            kw["wf_sets"] = int(v)
        elif k in ("drain", "form"):
            kw["wf_" + k] = v
        elif k == "bounces":
            kw["wf_bounces"] = int(v)
        elif k == "passes":
            kw["wf_passes"] = int(v)
        elif k == "chunk":
            kw["chunk"] = int(v)
        else:
            os.environ[k] = v
    return R.make_params(W, H, spp, engine="wavefront", **kw)


best = {c: 1e9 for c in cfgs}
for c in cfgs:  # warm-up (allocations, code objects)
    rend.render(cam, apply(c))
torch.cuda.synchronize()
for _ in range(n):
    for c in cfgs:
        p = apply(c)
        t = R.Timer()
        rend.render(cam, p, timer=t)
        torch.cuda.synchronize()
        best[c] = min(best[c], t.elapsed_ms())
        t.close()
for c in cfgs:
    tag = "" if cfgs == ["-"] else f"[{c}] "
    print(f"wavefront f64 {tag}{best[c]:.3f} ms {W * H * spp / best[c] / 1e3:.0f} Msamples/s", flush=True)
