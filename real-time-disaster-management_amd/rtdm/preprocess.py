"""The classifier CLI transform on device (rtdm_preprocess_frames).

get_val_torchvision_transforms (disaster_detection/dataloaders/aider.py:412-426):
Resize(int(1.14*S)) with Pillow's 8-bit antialiased BILINEAR -> CenterCrop(S) ->
ToTensor -> Normalize(ImageNet), for a batch of uint8 RGB frames.
"""
from __future__ import annotations

import torch

from . import _lib as L


def preprocess_frames(frames: torch.Tensor, size: int) -> torch.Tensor:
    """frames: [N,H,W,3] uint8 CUDA -> [N,3,size,size] fp32 (what the reference feeds model())."""
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
        raise ValueError("frames must be uint8 [N,H,W,3]")
    frames = frames.contiguous()
    n, h, w, _ = frames.shape
    out = torch.empty((n, 3, size, size), device=frames.device, dtype=torch.float32)
    with torch.cuda.device(frames.device):
        L.check(L.lib().rtdm_preprocess_frames(L.ptr(frames), n, h, w, size, L.ptr(out), L.stream_ptr()))
    return out


def aider_transforms_gpu(frames: torch.Tensor) -> torch.Tensor:  # aider.py:430
    return preprocess_frames(frames, 240)


def squeeze_transforms_gpu(frames: torch.Tensor) -> torch.Tensor:  # aider.py:431
    return preprocess_frames(frames, 140)
