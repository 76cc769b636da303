"""Megakernel timing of BASELINE configs[1] (1200x675x500, f64) against the
accumulation chunk (params.chunk: samples per work unit; the Tier-B image's
summation grouping, so each chunk is its own bit-exact image): best of N
HIP-event timed renders per chunk, chunks interleaved in one process.
  python tools/mk_chunk_ab.py [N] [CHUNK ...]   (PREC=f32 for the f32-hybrid kernel)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
chunks = [int(c) for c in sys.argv[2:]] or [32, 16, 64, 100]
W, spp = 1200, 500
H = R.image_height(W, 16 / 9)
sph, mats, _ = R.cover_scene(42)
cam = R.cover_camera(16 / 9)
rend = TorchRenderer(sph, mats, 0)
prec = os.environ.get("PREC", "f64")
best = {c: 1e9 for c in chunks}
for c in chunks:
    rend.render(cam, R.make_params(W, H, spp, chunk=c, precision=prec))
torch.cuda.synchronize()
for _ in range(n):
    for c in chunks:
        t = R.Timer()
        rend.render(cam, R.make_params(W, H, spp, chunk=c, precision=prec), timer=t)
        torch.cuda.synchronize()
        best[c] = min(best[c], t.elapsed_ms())
        t.close()
for c in chunks:
    print(f"megakernel {prec} chunk {c}: {best[c]:.3f} ms {W * H * spp / best[c] / 1e3:.0f} Msamples/s", flush=True)
