"""Wavefront engine sweep on the GPU box: ms/frame of configs[1] for several
queue capacities (wf_paths) and both precisions, HIP-event timed."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

W, H, SPP = 1200, 675, int(os.environ.get("SPP", "500"))
precs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["f64"]
paths = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1 << 18, 1 << 19, 1 << 20, 1 << 21]
reps = int(os.environ.get("REPS", "3"))
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
for prec in precs:
    for n in paths:
        p = R.make_params(W, H, SPP, precision=prec, engine="wavefront", wf_paths=n)
        rend.render(cam, p, out=out)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t = R.Timer()
            a = time.perf_counter()
            rend.render(cam, p, out=out, timer=t)
            torch.cuda.synchronize()
            ts.append((t.elapsed_ms(), (time.perf_counter() - a) * 1e3))
            t.close()
        best = min(ts)
        print(f"{prec} wf_paths {n:>9}: loop {best[0]:8.2f} ms  wall {best[1]:8.2f} ms  "
              f"{W * H * SPP / best[1] / 1e3:8.1f} Msamples/s", flush=True)
