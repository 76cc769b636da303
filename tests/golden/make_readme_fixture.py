"""Fixtures of the reference's README image for tests/test_readme_image.py.

Reads /root/reference/RayTracingInOneWeekend.png (600x400 RGB, a render the
reference's own code produced) and writes its 4x4 block means, rounded to
uint8 (150x100x3), as tests/golden/readme_image_150x100.npy, and its exact
2x2 block sums (uint16, 300x200x3) as tests/golden/readme_image_300x200_sum4.npz
(the matched-filter statistic).  Data only: the reference tree does not exist
on the GPU box, and the tests compare oracle renders with these block values.
python tests/golden/make_readme_fixture.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "raytracinginoneweekend.zig_amd"))
from rtw_amd.world import load_png  # noqa: E402

SRC = "/root/reference/RayTracingInOneWeekend.png"
F = 4

if __name__ == "__main__":
    img = load_png(SRC)[..., :3].astype(np.float64)
    h, w = img.shape[0] // F, img.shape[1] // F
    blocks = img.reshape(h, F, w, F, 3).mean(axis=(1, 3))
    out = np.rint(blocks).astype(np.uint8)
    np.save(os.path.join(HERE, f"readme_image_{w}x{h}.npy"), out)
    print(f"readme_image_{w}x{h}.npy", out.shape, out.reshape(-1, 3).mean(0))
    px = load_png(SRC)[..., :3].astype(np.uint16)
    sums = px.reshape(200, 2, 300, 2, 3).sum(axis=(1, 3)).astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "readme_image_300x200_sum4.npz"), sum4=sums)
    print("readme_image_300x200_sum4.npz", sums.shape, sums.reshape(-1, 3).mean(0) / 4)
