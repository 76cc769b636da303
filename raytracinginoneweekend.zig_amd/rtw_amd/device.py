"""Torch-side plumbing for the device-resident API: HBM buffers from torch's
caching allocator, the render launched on torch's current HIP stream.
Torch is plumbing here (device memory, streams, torch.distributed); the
rendering is the HIP kernels of lib/librtw_hip.so."""
from __future__ import annotations

import torch

from . import Camera, DeviceScene, Params, Timer, workspace_bytes


class TorchRenderer:
    def __init__(self, spheres, mats, device: int | torch.device = 0):
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the rtw render path has no CPU fallback")
        torch.cuda.set_device(self.device)
        self.scene = DeviceScene(spheres, mats)  # uploads to the current device
        self._ws = None

    def workspace(self, params: Params) -> torch.Tensor:
        need = workspace_bytes(params)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need + 256, dtype=torch.uint8, device=self.device)
        return self._ws

    def _ws_ptr(self, params: Params):
        ws = self.workspace(params)
        base = ws.data_ptr()
        ptr = (base + 255) & ~255
        return ptr, ws.numel() - (ptr - base)

    def render(self, cam: Camera, params: Params, out: torch.Tensor | None = None,
               mean: torch.Tensor | None = None, timer: Timer | None = None) -> torch.Tensor:
        """Asynchronous on torch.cuda.current_stream(); returns the rgb tensor (rows, W, 3) uint8."""
        if out is None:
            out = torch.empty((params.row_count, params.width, 3), dtype=torch.uint8, device=self.device)
        assert out.is_contiguous() and out.dtype == torch.uint8 and out.numel() == params.row_count * params.width * 3
        if mean is not None:
            assert mean.is_contiguous() and mean.dtype == torch.float32 and mean.numel() == out.numel()
        ptr, nbytes = self._ws_ptr(params)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.scene.render_async(cam, params, ptr, nbytes, out.data_ptr(),
                                mean.data_ptr() if mean is not None else None, stream, timer)
        return out

    def counts(self, cam: Camera, params: Params) -> dict:
        ptr, nbytes = self._ws_ptr(params)
        torch.cuda.synchronize(self.device)
        return self.scene.counts(cam, params, ptr, nbytes)

    def stats(self, cam: Camera, params: Params) -> dict:
        ptr, nbytes = self._ws_ptr(params)
        torch.cuda.synchronize(self.device)
        return self.scene.stats(cam, params, ptr, nbytes)
