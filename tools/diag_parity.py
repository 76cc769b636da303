"""Diagnostic (GPU box): where the f64 megakernel's configs[1] frame differs
from oracle Tier B, down to the sample.  Renders the full 1200x675x500 frame,
compares it with the oracle (16 threads), then re-renders each affected row
with chunk = 1 (the workspace's chunk sums are then the per-sample radiances)
and compares every sample of each differing pixel with the oracle's
(ro_tierb_samples), printing the oracle's segment trace of each differing
sample.  python tools/diag_parity.py [max_rows] > gpurun_out/diag_parity.json"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
import rtw_oracle as O  # noqa: E402
from helpers import to_oracle_camera, to_oracle_scene  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

max_rows = int(sys.argv[1]) if len(sys.argv) > 1 else 20
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
osc, ocam = to_oracle_scene(O, sph, mats), to_oracle_camera(O, cam)
rend = TorchRenderer(sph, mats, 0)
img = rend.render(cam, R.make_params(W, H, spp))
torch.cuda.synchronize()
img = img.cpu().numpy()
ref, _ = O.render_tier_b(osc, ocam, W, H, spp, threads=16)
ys, xs, cs = np.nonzero(img.astype(int) != ref.astype(int))
res = {"n_channels": int(len(ys)), "pixels": []}
for y in sorted(set(ys.tolist()))[:max_rows]:
    p = R.make_params(W, H, spp, row_begin=y, row_stride=1, row_count=1, chunk=1)
    rend.render(cam, p)
    torch.cuda.synchronize()
    ws = rend._ws
    off = ((ws.data_ptr() + 255) & ~255) - ws.data_ptr()
    part = ws[off:off + spp * W * 3 * 8].cpu().numpy().view(np.float64).reshape(spp, W, 3)
    for x in sorted(set(xs[ys == y].tolist())):
        gs = part[:, x, :]
        os_ = O.tierb_samples(osc, ocam, W, H, y, x, 0, spp)
        bad = np.nonzero((gs != os_).any(axis=1))[0]
        ent = {"y": int(y), "x": int(x), "gpu_rgb": img[y, x].tolist(), "oracle_rgb": ref[y, x].tolist(),
               "samples": [{"s": int(s), "gpu": gs[s].tolist(), "oracle": os_[s].tolist()} for s in bad[:8]]}
        res["pixels"].append(ent)
        for s in bad[:2]:
            print(f"--- oracle trace y {y} x {x} s {s}", file=sys.stderr, flush=True)
            O.tierb_samples(osc, ocam, W, H, y, x, int(s), 1, trace=True)
print(json.dumps(res))
