"""One-rank RCCL rehearsal of the multi-GPU exchange (run as a child process by
tests/test_gpu_rccl.py on a one-GPU box).

The N-GPU bench (bench.py, rtw_amd/shard.py) renders interleaved row shards and
assembles them on rank 0 with one `dist.gather` over the "nccl" backend (RCCL
on ROCm) plus one `all_reduce` of the sample counts.  A one-GPU box cannot run
two RCCL ranks on one device, so this runs the same collectives in a
world-size-1 RCCL group on GPU tensors the C ABI rendered: RCCL initialises on
the card, the gather moves the rendered row tile bit-exactly, and the
interleave of two shards rendered here assembles the 1-GPU frame.
Prints one JSON line; exit code 0 = all checks held.
"""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "raytracinginoneweekend.zig_amd"))
import rtw_amd as R  # noqa: E402
from rtw_amd.device import TorchRenderer  # noqa: E402
from rtw_amd.shard import assemble, max_rows, shard_rows  # noqa: E402


def main():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    W, spp, world = 160, 8, 2
    H = R.image_height(W, 16 / 9)
    sph, mats, _ = R.cover_scene(42)
    cam = R.cover_camera(16 / 9)
    rend = TorchRenderer(sph, mats, 0)
    full = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    rend.render(cam, R.make_params(W, H, spp, 50, 42), out=full)
    tiles, gathered = [], []
    for r in range(world):
        rb, rs, rc = shard_rows(H, r, world)
        out = torch.empty((rc, W, 3), dtype=torch.uint8, device="cuda:0")
        rend.render(cam, R.make_params(W, H, spp, 50, 42, row_begin=rb, row_stride=rs, row_count=rc), out=out)
        tile = torch.zeros((max_rows(H, world), W, 3), dtype=torch.uint8, device="cuda:0")
        tile[:rc] = out
        gl = [torch.empty_like(tile)]
        dist.gather(tile, gather_list=gl, dst=0)  # RCCL
        gathered.append(bool(torch.equal(gl[0], tile)))
        tiles.append(gl[0])
    samples = torch.tensor([float(W * H * spp)], dtype=torch.float64, device="cuda:0")
    dist.all_reduce(samples)  # RCCL
    img = assemble(tiles, H, world)
    res = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
           "gather_bit_exact": all(gathered), "assembled_equals_full": bool(torch.equal(img, full)),
           "all_reduce": samples.item(), "device": torch.cuda.get_device_name(0)}
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)
    ok = (res["backend"] == "nccl" and res["gather_bit_exact"] and res["assembled_equals_full"]
          and res["all_reduce"] == W * H * spp)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
