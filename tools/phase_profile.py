"""Diagnostic: per-phase wave-cycle shares of the trace kernel (s_memtime
stamps, RTW_PHASE_PROFILE=1 build variant) at BASELINE configs[1]."""
import os
import sys

os.environ["RTW_PHASE_PROFILE"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

W, spp = 1200, int(sys.argv[1]) if len(sys.argv) > 1 else 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
for prec in ("f64", "f32"):
    print(f"--- {prec}", flush=True)
    c = rend.counts(cam, R.make_params(W, H, spp, precision=prec))
    print(prec, c, flush=True)
