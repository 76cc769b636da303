"""Row sharding of one image across ranks (one process per GPU).

Rank r renders the image rows y = r, r + N, r + 2N, ... (interleaved, so
cheap sky rows and expensive ground rows spread evenly), with the RNG keyed
by the GLOBAL pixel index, so every rank's rows are bit-identical to the same
rows of a 1-GPU render.  The only exchange step is assembling the image on
rank 0: one gather of equal-size row tiles (RCCL over xGMI on the GPU box,
gloo in the CPU tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_rows(height: int, rank: int, world: int):
    """(row_begin, row_stride, row_count) of `rank` in image-row space."""
    if not (0 <= rank < world) or world < 1:
        raise ValueError(f"rank {rank} / world {world}")
    count = len(range(rank, height, world))
    return rank, world, count


def max_rows(height: int, world: int) -> int:
    return (height + world - 1) // world


def assemble(tiles, height: int, world: int) -> torch.Tensor:
    """tiles[r]: (max_rows, W, C) padded row tile of rank r -> (height, W, C)."""
    W = tiles[0].shape[1]
    out = torch.empty((height,) + tuple(tiles[0].shape[1:]), dtype=tiles[0].dtype, device=tiles[0].device)
    for r in range(world):
        _, _, cnt = shard_rows(height, r, world)
        if cnt:
            out[r::world] = tiles[r][:cnt]
    assert out.shape[1] == W
    return out


class TileGather:
    """The gather of one rank's row tile to rank 0 with its buffers allocated
    once (the padded send tile, rank 0's receive tiles): `gather(local)` is
    just the copy into the tile + one collective, so a timed loop that
    gathers every frame allocates nothing; `image()` interleaves the last
    gathered tiles into the frame on rank 0 (once, outside a timed loop)."""

    def __init__(self, like: torch.Tensor, height: int, rank: int, world: int, group=None):
        self.height, self.rank, self.world, self.group = height, rank, world, group
        self.dev = like.device
        host = like.is_cuda and world > 1 and dist.get_backend(group) == "gloo"  # gloo gathers host tensors only
        tdev = torch.device("cpu") if host else like.device
        self.tile = torch.zeros((max_rows(height, world),) + tuple(like.shape[1:]), dtype=like.dtype, device=tdev)
        self.recv = ([torch.empty_like(self.tile) for _ in range(world)] if rank == 0 else None) if world > 1 \
            else [self.tile]

    def gather(self, local: torch.Tensor) -> None:
        self.tile[: local.shape[0]].copy_(local, non_blocking=self.tile.device == local.device)
        if self.world > 1:
            dist.gather(self.tile, gather_list=self.recv, dst=0, group=self.group)

    def image(self):
        """The assembled (height, W, C) frame on rank 0, None elsewhere."""
        if self.rank != 0:
            return None
        return assemble(self.recv, self.height, self.world).to(self.dev)


def gather_image(local: torch.Tensor, height: int, rank: int, world: int, group=None):
    """Gather every rank's rows to rank 0 and interleave them; None on other ranks."""
    mr = max_rows(height, world)
    tile = torch.zeros((mr,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    tile[: local.shape[0]] = local
    if world == 1:
        return assemble([tile], height, 1)
    dev = tile.device
    if tile.is_cuda and dist.get_backend(group) == "gloo":  # gloo gathers host tensors only
        tile = tile.cpu()
    gl = [torch.empty_like(tile) for _ in range(world)] if rank == 0 else None
    dist.gather(tile, gather_list=gl, dst=0, group=group)
    if rank != 0:
        return None
    return assemble(gl, height, world).to(dev)
