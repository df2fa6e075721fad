"""Detector frame ingest: letterbox + box rescaling on the HIP runtime
(victim_localization/yolov3/utils/datasets.py:508-522 load_image, :599-631 letterbox;
utils/utils.py:123-142 scale_coords / clip_coords).

The resize runs on the device (``rtdm_letterbox``): cv2.INTER_AREA semantics — area
averaging when shrinking, INTER_AREA's linear coefficients when growing — restated from
OpenCV's published algorithm because cv2 is not part of this stack (pixel parity with
cv2 is unpinned; the kernel is bit-exact against oracle/letterbox.py).  JPEG decoding
stays on the host (Pillow): there is no rocJPEG in this ROCm image.  The geometry —
scale ratio, unpadded size, padding split, label transforms — follows the reference
exactly, so boxes map back to the same source coordinates.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L


def geometry(in_h: int, in_w: int, new_shape=416, auto: bool = True, scale_fill: bool = False,
             scaleup: bool = True):
    """letterbox() shape arithmetic (datasets.py:603-627) ->
    (new_h, new_w, out_h, out_w, top, left), computed by rtdm_letterbox_geometry."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    g = (ctypes.c_int * 6)()
    L.check(L.lib().rtdm_letterbox_geometry(int(in_h), int(in_w), int(new_shape[0]), int(new_shape[1]), int(auto),
                                            int(scale_fill), int(scaleup), g))
    return tuple(g)


def ratio_pad(in_h: int, in_w: int, new_shape=416, auto: bool = True, scaleup: bool = True):
    """The (ratio, (dw, dh)) pair letterbox() returns (datasets.py:631)."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = max(new_shape) / max(in_h, in_w)
    if not scaleup:
        r = min(r, 1.0)
    nw, nh = int(round(in_w * r)), int(round(in_h * r))
    dw, dh = new_shape[1] - nw, new_shape[0] - nh
    if auto:
        dw, dh = dw % 32, dh % 32
    return (r, r), (dw / 2, dh / 2)


def dataset_geometry(h0: int, w0: int, img_size: int):
    """LoadImagesAndLabels evaluation path: load_image shrinks to (int(w0*r), int(h0*r))
    (datasets.py:515-520, never grows), then letterbox(auto=False, scaleup=False) pads to
    img_size² without a second resize.  Returns (geom, (h, w), ratio, pad)."""
    r = img_size / max(h0, w0)
    h, w = (int(h0 * r), int(w0 * r)) if r < 1 else (h0, w0)
    g = geometry(h, w, img_size, auto=False, scaleup=False)
    ratio, pad = ratio_pad(h, w, img_size, auto=False, scaleup=False)
    # the second letterbox never resizes (ratio 1): the device resize goes h0 x w0 -> g's new size
    return g, (h, w), ratio, pad


def letterbox_frames(frames: torch.Tensor, geom, color=(128, 128, 128), bgr: bool = False,
                     out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """frames: uint8 [N, H, W, 3] on the GPU (rows may be pitched: stride(1) >= 3*W, unit
    channel/pixel strides) -> [N, out_h, out_w, 3] uint8 RGB letterboxed frames, the
    detector's RTDM_INPUT_FRAME_U8 input.  bgr=True reads cv2-order frames."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
        raise ValueError("letterbox_frames: frames must be uint8 [N,H,W,3] on the GPU")
    if frames.stride(3) != 1 or frames.stride(2) != 3 or frames.stride(0) != frames.stride(1) * frames.shape[1]:
        frames = frames.contiguous()
    n, h, w, _ = frames.shape
    new_h, new_w, out_h, out_w, top, left = geom
    if out is None:
        out = torch.empty((n, out_h, out_w, 3), dtype=torch.uint8, device=frames.device)
    if tuple(out.shape) != (n, out_h, out_w, 3) or not out.is_contiguous():
        raise ValueError("letterbox_frames: out must be a contiguous [N, out_h, out_w, 3] uint8 tensor")
    pad = int(color[0]) | (int(color[1]) << 8) | (int(color[2]) << 16)
    with torch.cuda.device(frames.device):
        L.check(L.lib().rtdm_letterbox(L.ptr(frames), n, h, w, frames.stride(1), new_h, new_w, out_h, out_w, top,
                                       left, pad, int(bgr), L.ptr(out), L.stream_ptr(stream)))
    return out


def letterbox(img: np.ndarray, new_shape=416, color=(128, 128, 128), auto: bool = True, scaleFill: bool = False,
              scaleup: bool = True, device=None):
    """datasets.py:599-631 for one host image, resized on the GPU.  Returns
    (img [h, w, 3] uint8 numpy, (ratio_w, ratio_h), (dw, dh)) like the reference."""
    g = geometry(img.shape[0], img.shape[1], new_shape, auto, scaleFill, scaleup)
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    x = torch.from_numpy(np.ascontiguousarray(img))[None].to(dev)
    out = letterbox_frames(x, g, color)
    ratio, pad = ratio_pad(img.shape[0], img.shape[1], new_shape, auto, scaleup)
    if scaleFill:
        ratio, pad = (g[1] / img.shape[1], g[0] / img.shape[0]), (0.0, 0.0)
    return out[0].cpu().numpy(), ratio, pad


def scale_coords(img1_shape, coords, img0_shape, ratio_pad=None):
    """utils.py:123-136: corner boxes from the letterboxed frame back to the source image.
    The reference then calls clip_coords (:139-142), which clamps a copy made by advanced
    indexing and so leaves the boxes as they are; that behaviour is kept (no clamp)."""
    if ratio_pad is None:
        gain = max(img1_shape) / max(img0_shape)
        pad = (img1_shape[1] - img0_shape[1] * gain) / 2, (img1_shape[0] - img0_shape[0] * gain) / 2
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    coords[:, [0, 2]] -= pad[0]
    coords[:, [1, 3]] -= pad[1]
    coords[:, :4] /= gain
    return coords


def labels_to_letterbox(x: np.ndarray, ratio, pad, h: int, w: int, out_h: int, out_w: int) -> np.ndarray:
    """datasets.py:441-458 + 475-482: label rows (cls, x, y, w, h normalised to the source)
    -> (cls, x, y, w, h normalised to the letterboxed frame), in float32 like the reference."""
    if not x.size:
        return np.zeros((0, 5), np.float32)
    lab = x.astype(np.float32).copy()
    x1 = ratio[0] * w * (x[:, 1] - x[:, 3] / 2) + pad[0]
    y1 = ratio[1] * h * (x[:, 2] - x[:, 4] / 2) + pad[1]
    x2 = ratio[0] * w * (x[:, 1] + x[:, 3] / 2) + pad[0]
    y2 = ratio[1] * h * (x[:, 2] + x[:, 4] / 2) + pad[1]
    lab[:, 1], lab[:, 2], lab[:, 3], lab[:, 4] = x1, y1, x2, y2
    xyxy = lab[:, 1:5].copy()
    lab[:, 1] = (xyxy[:, 0] + xyxy[:, 2]) / 2
    lab[:, 2] = (xyxy[:, 1] + xyxy[:, 3]) / 2
    lab[:, 3] = xyxy[:, 2] - xyxy[:, 0]
    lab[:, 4] = xyxy[:, 3] - xyxy[:, 1]
    lab[:, [2, 4]] /= out_h
    lab[:, [1, 3]] /= out_w
    return lab


def resize_linear(frames: torch.Tensor, out_h: int, out_w: int, swap_rb: bool = False, stream=None) -> torch.Tensor:
    """cv2.resize(frame, (out_w, out_h)) with the default INTER_LINEAR, on the device
    (rtdm_resize_linear; real-time-inference.py:185).  frames: uint8 [N,H,W,3] (or [H,W,3])
    CUDA; swap_rb=True also turns BGR into RGB.  Returns uint8 [N,out_h,out_w,3]."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.shape[-1] != 3:
        raise ValueError("frames must be uint8 [N,H,W,3] on the GPU")
    one = frames.dim() == 3
    x = (frames[None] if one else frames).contiguous()
    n, h, w, _ = x.shape
    out = torch.empty((n, out_h, out_w, 3), dtype=torch.uint8, device=x.device)
    with torch.cuda.device(x.device):
        L.check(L.lib().rtdm_resize_linear(L.ptr(x), n, h, w, w * 3, out_h, out_w, 1 if swap_rb else 0, L.ptr(out),
                                           L.stream_ptr(stream)))
    return out[0] if one else out
