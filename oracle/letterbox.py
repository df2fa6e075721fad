"""Letterbox restatement in numpy (TEST INFRASTRUCTURE ONLY).

Follows yolov3/utils/datasets.py:599-631 (letterbox) and :508-522 (load_image), whose
resize is cv2.resize(..., interpolation=cv2.INTER_AREA).  cv2 (opencv-python, unpinned
in requirements-fyp.txt) is absent from this image, so its published INTER_AREA
algorithm (imgproc/src/resize.cpp, the scalar code paths) is restated here:
  * both scale factors >= 1 and integral: resizeAreaFast — integer box sum times
    (float)(1/area), cvRound (nearest, ties to even);
  * both >= 1: resizeArea — per-axis tables from computeResizeAreaTab (alpha =
    overlap / cellWidth, float), horizontal row sums h = h + S*alpha, then
    v = beta0*h0 + beta1*h1 + ... in float32, cvRound;
  * otherwise: the INTER_AREA coefficients of the linear resizer (fx = (d+1) -
    (sx+1)/scale wrapped to [0,1), 11-bit fixed point, HResizeLinear int sums,
    FixedPtCast >> 22 with rounding).
Parity with cv2 itself is UNPINNED (no cv2 here and the reference ships no letterboxed
fixtures); the HIP kernel is held bit-exact to this restatement.
"""
from __future__ import annotations

import math

import numpy as np


def geometry(in_h, in_w, new_shape=416, auto=True, scale_fill=False, scaleup=True):
    """datasets.py:603-627 -> (new_h, new_w, out_h, out_w, top, left)."""
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = max(new_shape) / max(in_h, in_w)
    if not scaleup:
        r = min(r, 1.0)
    new_unpad = int(round(in_w * r)), int(round(in_h * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, 32), np.mod(dh, 32)
    elif scale_fill:
        dw, dh = 0.0, 0.0
        new_unpad = new_shape
    dw /= 2
    dh /= 2
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    return new_unpad[1], new_unpad[0], new_unpad[1] + top + bottom, new_unpad[0] + left + right, top, left


def _area_tab(ssize, dsize):
    scale = 1.0 / (dsize / ssize)
    tab = []
    for d in range(dsize):
        f1 = d * scale
        f2 = f1 + scale
        cell = min(scale, ssize - f1)
        s1, s2 = math.ceil(f1), math.floor(f2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        t = []
        if s1 - f1 > 1e-3:
            t.append((s1 - 1, np.float32((s1 - f1) / cell)))
        for s in range(s1, s2):
            t.append((s, np.float32(1.0 / cell)))
        if f2 - s2 > 1e-3:
            t.append((s2, np.float32(min(min(f2 - s2, 1.0), cell) / cell)))
        tab.append(t)
    return tab


def _linear_tab(ssize, dsize):
    inv = dsize / ssize
    scale = 1.0 / inv
    out = []
    for d in range(dsize):
        s = math.floor(d * scale)
        f = np.float32((d + 1) - (s + 1) * inv)
        f = np.float32(0) if f <= 0 else np.float32(f - np.floor(f))
        if s < 0:
            s, f = 0, np.float32(0)
        if s >= ssize - 1:
            s, f = ssize - 1, np.float32(0)
        c0 = int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048)))
        c1 = int(np.rint(f * np.float32(2048)))
        out.append((s, min(s + 1, ssize - 1), c0, c1))
    return out


def resize_area(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h), interpolation=cv2.INTER_AREA) as restated above."""
    in_h, in_w = img.shape[:2]
    scx, scy = 1.0 / (new_w / in_w), 1.0 / (new_h / in_h)
    src = img.astype(np.int64)
    if scx >= 1 and scy >= 1:
        isx, isy = int(round(scx)), int(round(scy))
        if abs(scx - isx) < 2.220446049250313e-16 and abs(scy - isy) < 2.220446049250313e-16:
            s = src[:new_h * isy, :new_w * isx].reshape(new_h, isy, new_w, isx, 3).sum(axis=(1, 3))
            v = s.astype(np.float32) * (np.float32(1) / np.float32(isx * isy))
            return np.clip(np.rint(v), 0, 255).astype(np.uint8)
        xt, yt = _area_tab(in_w, new_w), _area_tab(in_h, new_h)
        f = img.astype(np.float32)
        # horizontal: h[y, dx] = sum_k S[y, xs_k] * a_k, in table order
        tx = max(len(t) for t in xt)
        xs = np.array([[t[min(k, len(t) - 1)][0] for k in range(tx)] for t in xt])
        xw = np.array([[t[k][1] if k < len(t) else 0.0 for k in range(tx)] for t in xt], np.float32)
        h = np.zeros((in_h, new_w, 3), np.float32)
        for k in range(tx):
            h = h + f[:, xs[:, k], :] * xw[:, k][None, :, None]
        out = np.empty((new_h, new_w, 3), np.float32)
        for dy, t in enumerate(yt):
            v = t[0][1] * h[t[0][0]]
            for (sy, b) in t[1:]:
                v = v + b * h[sy]
            out[dy] = v
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    xt, yt = _linear_tab(in_w, new_w), _linear_tab(in_h, new_h)
    x0 = np.array([t[0] for t in xt])
    x1 = np.array([t[1] for t in xt])
    c0 = np.array([t[2] for t in xt], np.int64)[None, :, None]
    c1 = np.array([t[3] for t in xt], np.int64)[None, :, None]
    hrow = src[:, x0, :] * c0 + src[:, x1, :] * c1
    out = np.empty((new_h, new_w, 3), np.int64)
    for dy, (y0, y1, b0, b1) in enumerate(yt):
        out[dy] = (b0 * hrow[y0] + b1 * hrow[y1] + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.uint8)


def _inter_linear_tab(ssize, dsize):
    """cv2.INTER_LINEAR coefficients (resize.cpp): fx = (float)((d + 0.5) * scale - 0.5),
    s = floor(fx), f = fx - s; clamped to the border pixel (f = 0) outside; 11-bit weights
    by cvRound (nearest, ties to even)."""
    scale = 1.0 / (dsize / ssize)
    out = []
    for d in range(dsize):
        fx = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(fx))
        f = np.float32(fx - np.float32(s))
        if s < 0:
            s, f = 0, np.float32(0)
        if s >= ssize - 1:
            s, f = ssize - 1, np.float32(0)
        c0 = int(np.rint(np.float32(np.float32(1) - f) * np.float32(2048)))
        c1 = int(np.rint(f * np.float32(2048)))
        out.append((s, min(s + 1, ssize - 1), c0, c1))
    return out


def resize_linear(img: np.ndarray, new_w: int, new_h: int) -> np.ndarray:
    """cv2.resize(img, (new_w, new_h)) -- INTER_LINEAR, the default interpolation used by
    real-time-inference.py:185 -- as restated above (same fixed-point sums as the
    INTER_AREA growing path: int horizontal taps, (b0*h0 + b1*h1 + 2^21) >> 22).  That is
    OpenCV's scalar vertical rounding; its SIMD 8-bit path (>> 4, mulhi, (x + 2) >> 2) can
    differ by 1 LSB, and with cv2 absent neither is pinned against cv2 itself."""
    src = img.astype(np.int64)
    xt, yt = _inter_linear_tab(img.shape[1], new_w), _inter_linear_tab(img.shape[0], new_h)
    x0 = np.array([t[0] for t in xt])
    x1 = np.array([t[1] for t in xt])
    c0 = np.array([t[2] for t in xt], np.int64)[None, :, None]
    c1 = np.array([t[3] for t in xt], np.int64)[None, :, None]
    hrow = src[:, x0, :] * c0 + src[:, x1, :] * c1
    out = np.empty((new_h, new_w, 3), np.int64)
    for dy, (y0, y1, b0, b1) in enumerate(yt):
        out[dy] = (b0 * hrow[y0] + b1 * hrow[y1] + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.uint8)


def letterbox(img: np.ndarray, geom, color=(128, 128, 128)) -> np.ndarray:
    """Resize to (new_w, new_h) and pad into the (out_h, out_w) canvas (datasets.py:626-630)."""
    new_h, new_w, out_h, out_w, top, left = geom
    out = np.empty((out_h, out_w, 3), np.uint8)
    out[...] = np.asarray(color, np.uint8)
    res = img if img.shape[:2] == (new_h, new_w) else resize_area(img, new_w, new_h)
    out[top:top + new_h, left:left + new_w] = res
    return out
