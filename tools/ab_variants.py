"""In-process A/B of trace-kernel tuning variants (RTW_VARIANT), interleaved
rounds on one device (guide §5.4 rule 24).  Usage: ab_variants.py prec v1,v2,... [rounds]
An item may carry environment settings read by the library at each render:
"0:RTW_UNIT_ORDER=fwd" (several joined by '+')."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "f64"
variants = (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
p = R.make_params(W, H, spp, precision=prec)
ref = None
res = {v: [] for v in variants}
timer = R.Timer()
for r in range(rounds + 1):
    for v in variants:
        var, _, envs = v.partition(":")
        for kv in [e for e in envs.split("+") if e]:
            os.environ[kv.split("=")[0]] = kv.split("=", 1)[1]
        os.environ["RTW_VARIANT"] = var
        img = rend.render(cam, p, timer=timer)
        ms = timer.elapsed_ms()
        if r == 0:  # warmup + equality check
            a = img.cpu()
            if ref is None:
                ref = a
            assert torch.equal(a, ref), f"variant {v} changed the image"
            continue
        res[v].append(ms)
        for kv in [e for e in envs.split("+") if e]:
            os.environ.pop(kv.split("=")[0], None)
for v in variants:
    xs = sorted(res[v])
    print(f"{prec} var {v}: median {xs[len(xs)//2]:.3f} ms  min {xs[0]:.3f}  -> {W*H*spp/xs[len(xs)//2]/1e3:.0f} Msamples/s",
          flush=True)
