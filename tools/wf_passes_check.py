"""Bit identity of wavefront configurations against the megakernel (same Tier-B
image): python tools/wf_passes_check.py CFG ...  with CFG as tools/wf_bench.py
(rtw_params fields and -DRTW_MEASURE development knobs).  Renders the cover
scene at 1200x675x40 and compares the f32 mean images bit for bit."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

W, spp = 1200, 40
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
base_env = dict(os.environ)


def render(engine, cfg):
    os.environ.clear()
    os.environ.update(base_env)
    kw = {}
    for kv in ([] if cfg == "-" else cfg.split(",")):
        k, v = kv.split("=")
        if k == "bounces":
            kw["wf_bounces"] = int(v)
        elif k == "passes":
            kw["wf_passes"] = int(v)
        elif k == "sets":
            kw["wf_sets"] = int(v)
        elif k in ("drain", "form"):
            kw["wf_" + k] = v
        else:
            os.environ[k] = v
    p = R.make_params(W, H, spp, engine=engine, **kw)
    mean = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    rend.render(cam, p, mean=mean)
    torch.cuda.synchronize()
    return mean


ref = render("megakernel", "-")
ok = True
for c in sys.argv[1:] or ["-"]:
    m = render("wavefront", c)
    same = bool(torch.equal(m.view(torch.int32), ref.view(torch.int32)))
    ok &= same
    print(f"wavefront [{c}] bit-identical to the megakernel: {same}", flush=True)
sys.exit(0 if ok else 1)
