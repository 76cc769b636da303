"""do the wavefront's two queue sets still overlap when the process holds many
other streams (RCCL's, torch's)?  python tools/wf_streams_run.py N_EXTRA
Creates N_EXTRA torch streams and runs a small kernel on each (so each is bound to a hardware
queue) BEFORE the library creates its side stream, then renders the configs[1] wavefront frame
twice (under rocprofv3 --kernel-trace, tools/wf_overlap_summary.py reads the last one) and
prints the frame time."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

n_extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
extra = [torch.cuda.Stream() for _ in range(n_extra)]
bufs = []
for s in extra:
    with torch.cuda.stream(s):
        bufs.append(torch.ones(1 << 20, device="cuda") * 2.0)
torch.cuda.synchronize()
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
p = R.make_params(W, H, spp, engine="wavefront")
for i in range(2):
    t = R.Timer()
    rend.render(cam, p, timer=t)
    torch.cuda.synchronize()
    print(f"extra streams {n_extra}: frame {i} {t.elapsed_ms():.2f} ms", flush=True)
    t.close()
