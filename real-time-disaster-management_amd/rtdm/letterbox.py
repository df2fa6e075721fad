"""Host-side frame ingest for the detector CLIs: letterbox + box rescaling
(victim_localization/yolov3/utils/datasets.py:508-522, 599-631; utils/utils.py:123-142).

The reference decodes with cv2 and resizes with cv2.INTER_AREA; cv2 is not part of
this stack, so shrinking uses Pillow's BOX filter and growing BILINEAR (pixel parity
with cv2 is unpinned: cv2 is absent here).  Geometry — the scale ratio, the unpadded
size, the split of the padding, the label/box transforms — follows the reference
exactly, so boxes map back to the same source coordinates.
"""
from __future__ import annotations

import numpy as np


def resize(img: np.ndarray, size_wh) -> np.ndarray:
    from PIL import Image
    w, h = int(size_wh[0]), int(size_wh[1])
    if (img.shape[1], img.shape[0]) == (w, h):
        return img
    shrink = w < img.shape[1] or h < img.shape[0]
    return np.asarray(Image.fromarray(img).resize((w, h), Image.BOX if shrink else Image.BILINEAR), np.uint8)


def load_image(img: np.ndarray, img_size: int, augment: bool = False):
    """datasets.py:508-522: shrink so the longer side is img_size (never grow at test time).
    Returns (img, (h0, w0), (h, w))."""
    h0, w0 = img.shape[:2]
    r = img_size / max(h0, w0)
    if r < 1 or (augment and r != 1):
        img = resize(img, (int(w0 * r), int(h0 * r)))
    return img, (h0, w0), img.shape[:2]


def letterbox(img: np.ndarray, new_shape=416, color=(128, 128, 128), auto: bool = True, scaleFill: bool = False,
              scaleup: bool = True):
    """datasets.py:599-631.  Returns (img, (ratio_w, ratio_h), (dw, dh)) with dw/dh the
    per-side padding before rounding (float, as the reference returns it)."""
    shape = img.shape[:2]
    if isinstance(new_shape, int):
        new_shape = (new_shape, new_shape)
    r = max(new_shape) / max(shape)
    if not scaleup:
        r = min(r, 1.0)
    ratio = r, r
    new_unpad = int(round(shape[1] * r)), int(round(shape[0] * r))
    dw, dh = new_shape[1] - new_unpad[0], new_shape[0] - new_unpad[1]
    if auto:
        dw, dh = np.mod(dw, 32), np.mod(dh, 32)
    elif scaleFill:
        dw, dh = 0.0, 0.0
        new_unpad = new_shape
        ratio = new_shape[0] / shape[1], new_shape[1] / shape[0]
    dw /= 2
    dh /= 2
    if shape[::-1] != tuple(new_unpad):
        img = resize(img, new_unpad)
    top, bottom = int(round(dh - 0.1)), int(round(dh + 0.1))
    left, right = int(round(dw - 0.1)), int(round(dw + 0.1))
    out = np.empty((img.shape[0] + top + bottom, img.shape[1] + left + right, 3), np.uint8)
    out[...] = np.asarray(color, np.uint8)
    out[top:top + img.shape[0], left:left + img.shape[1]] = img
    return out, ratio, (dw, dh)


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
