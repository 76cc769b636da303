"""Counts pass of the wavefront engine at BASELINE configs[1] (1200x675x500,
f64): samples, segments, the drain's share; with RTW_COUNTS_VERBOSE=1 the
library also prints the drain's lane utilisation (stderr)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracinginoneweekend.zig_amd"))
import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
print(rend.counts(cam, R.make_params(1200, 675, 500, engine="wavefront")), flush=True)
