"""Wavefront-engine timing of BASELINE configs[1] (1200x675x500, f64): best of
N renders, HIP events around the bounce loop.  python tools/wf_bench.py [N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
p = R.make_params(W, H, spp, engine="wavefront")
rend.render(cam, p)
torch.cuda.synchronize()
best = 1e9
for _ in range(n):
    t = R.Timer()
    rend.render(cam, p, timer=t)
    torch.cuda.synchronize()
    best = min(best, t.elapsed_ms())
    t.close()
print(f"wavefront f64 {best:.3f} ms {W * H * spp / best / 1e3:.0f} Msamples/s", flush=True)
