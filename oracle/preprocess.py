"""Classifier CLI transform restated in numpy (TEST INFRASTRUCTURE ONLY).

dataloaders/aider.py:412-426: transforms.Resize(int(S*1.14)) -> CenterCrop(S) ->
ToTensor -> Normalize(mean=[0.485,0.456,0.406], std=[0.229,0.224,0.225]).
Resize on a PIL image is Pillow's 8-bit antialiased BILINEAR resample
(Resample.c: precompute_coeffs, normalize_coeffs_8bpc with PRECISION_BITS=22,
horizontal pass then vertical pass, each rounding + clip8 to uint8);
torchvision 0.8.2 size rule: shorter side -> size, longer int(size*long/short);
CenterCrop offset int(round((dim - S) / 2.)).
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2
MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def _coeffs(in_size: int, out_size: int):
    scale = float(in_size) / out_size
    filterscale = max(1.0, scale)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.float64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        ws = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(ws)
        for x in range(xmax):
            kk[xx, x] = ws[x] / ww if ww != 0.0 else ws[x]
        bounds[xx] = (xmin, xmax)
    ik = np.where(kk < 0, np.trunc(-0.5 + kk * (1 << PRECISION_BITS)),
                  np.trunc(0.5 + kk * (1 << PRECISION_BITS))).astype(np.int64)
    return bounds, ik


def _pass(img: np.ndarray, axis: int, out_size: int) -> np.ndarray:
    """One Pillow resample pass along `axis` (1 = horizontal, 0 = vertical) of HxWx3 uint8.
    The integer multiply-accumulate is evaluated as a dense float64 matmul: every
    partial sum is an integer below 2^31, so float64 is exact."""
    in_size = img.shape[axis]
    if in_size == out_size:
        return img
    bounds, k = _coeffs(in_size, out_size)
    dense = np.zeros((out_size, in_size), np.float64)
    for o in range(out_size):
        xmin, xmax = bounds[o]
        dense[o, xmin:xmin + xmax] = k[o, :xmax]
    src = np.moveaxis(img, axis, 0).astype(np.float64)  # [in, other, 3]
    acc = (dense @ src.reshape(in_size, -1)).astype(np.int64) + (1 << (PRECISION_BITS - 1))
    out = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8).reshape((out_size,) + src.shape[1:])
    return np.moveaxis(out, 0, axis)


def resize_shorter(img: np.ndarray, size: int) -> np.ndarray:
    h, w = img.shape[:2]
    if (w <= h and w == size) or (h <= w and h == size):
        return img
    if w < h:
        ow, oh = size, int(size * h / w)
    else:
        oh, ow = size, int(size * w / h)
    return _pass(_pass(img, 1, ow), 0, oh)


def center_crop(img: np.ndarray, s: int) -> np.ndarray:
    h, w = img.shape[:2]
    top = int(round((h - s) / 2.0))
    left = int(round((w - s) / 2.0))
    return img[top:top + s, left:left + s]


def to_tensor_normalize(img: np.ndarray) -> np.ndarray:
    """HWC uint8 -> CHW fp32, ((u8 / 255) - mean) / std in fp32."""
    x = img.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    return np.ascontiguousarray(((x - MEAN[:, None, None]) / STD[:, None, None]).astype(np.float32))


def cli_transform(img: np.ndarray, s: int) -> np.ndarray:
    return to_tensor_normalize(center_crop(resize_shorter(img, int(s * 1.14)), s))


def pil_resize_shorter(img: np.ndarray, size: int) -> np.ndarray:
    """The same resize through Pillow itself (the pinning reference for _pass)."""
    from PIL import Image
    h, w = img.shape[:2]
    if w < h:
        ow, oh = size, int(size * h / w)
    else:
        oh, ow = size, int(size * w / h)
    return np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
