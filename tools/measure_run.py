"""One configs[1] render per RTW_VARIANT (for rocprofv3 --pmc passes: the
kernel name carries the variant).  Usage: measure_run.py prec v1,v2,..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

prec = sys.argv[1]
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
p = R.make_params(W, H, spp, precision=prec)
for v in sys.argv[2].split(","):
    os.environ["RTW_VARIANT"] = v
    rend.render(cam, p)
    torch.cuda.synchronize()
print("done", flush=True)
