"""Oracle fixtures of the world kernel at BASELINE configs[4]'s workload.

The globe + 10k-sphere world (scene 7: main.zig:223-234's earth with the
reference's assets/sekaichizu.png, plus 10k random spheres) at its bench
size 1200x675x100, rendered by oracle world Tier B (oracle/rtw_world.c: a
LINEAR closest-hit loop over all 10,003 primitives, hittable.zig:231-244, no
BVH) on the rows y = 7, 49, ..., 637 (row_begin 7, stride 42: 16 rows spread
over the image, 1.92 M samples).  The linear oracle takes ~15 CPU-minutes
for these rows, too long for a GPU-box test, so they are rendered here once
and committed; tests/test_gpu_world.py compares the GPU's BVH render of the
full frame with them (and renders 2 further rows live on the box).

Writes tests/golden/globe_1200x675x100_rows7s42.npz: rgb (16, 1200, 3) u8,
the row list and the oracle's sample / segment counts.
python tests/golden/make_world_fixtures.py [--threads N]"""
import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.join(HERE, "..", "..")
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

W, H, SPP, ROW_BEGIN, ROW_STRIDE = 1200, 675, 100, 7, 42
NAME = f"globe_{W}x{H}x{SPP}_rows{ROW_BEGIN}s{ROW_STRIDE}.npz"

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    import rtw_oracle as O
    from rtw_amd.world import earth_map
    o = O.OracleWorld(7, 42, image=earth_map())
    t0 = time.time()
    rgb, st = o.render_tier_b(o.camera(), W, H, SPP, row_begin=ROW_BEGIN, row_stride=ROW_STRIDE,
                              threads=args.threads)
    dt = time.time() - t0
    rows = np.arange(ROW_BEGIN, H, ROW_STRIDE)
    assert rgb.shape == (len(rows), W, 3) and st["samples"] == len(rows) * W * SPP
    np.savez_compressed(os.path.join(HERE, NAME), rgb=rgb, rows=rows, samples=st["samples"],
                        segments=st["segments"])
    print(NAME, rgb.shape, f"{dt:.1f} s on {args.threads} threads", st)
