"""One render of BASELINE configs[1] per precision, for rocprofv3 (kernel
trace / PMC passes).  Usage: python tools/prof_run.py [f64|f32|both|wf64] [reps] [field=value ...]
(wf64: the same frame on the wavefront engine, BASELINE configs[3]; field=value: rtw_params
fields of that render, e.g. wf_sets=1 — the library reads no environment for them)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracinginoneweekend.zig_amd"))

import torch  # noqa: E402

import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    kw = {k: int(v) if v.isdigit() else v for k, v in (a.split("=", 1) for a in sys.argv[3:])}
    W, spp = 1200, 500
    H = R.image_height(W, 16 / 9)
    sph, mats, _ = R.cover_scene(42)
    cam = R.cover_camera(16 / 9)
    rend = TorchRenderer(sph, mats, 0)
    for prec in (["f64", "f32"] if which == "both" else [which]):
        if prec == "wf64":
            p = R.make_params(W, H, spp, precision="f64", engine="wavefront", **kw)
        else:
            p = R.make_params(W, H, spp, precision=prec, **kw)
        for _ in range(reps):
            rend.render(cam, p)
        torch.cuda.synchronize()
        print(prec, "done", flush=True)


if __name__ == "__main__":
    main()
