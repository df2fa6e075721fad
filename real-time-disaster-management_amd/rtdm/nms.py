"""non_max_suppression on the HIP runtime (rtdm_nms).

Same signature and output as victim_localization/yolov3/utils/utils.py:488-557
(method 'vision_batch', the reference's hard-coded path): a list with one
[k, 6] tensor (x1, y1, x2, y2, conf, cls) per image in descending score order,
or None for an image without detections.  ``nms_batched`` is the fixed-shape,
sync-free form the pipeline uses (padded rows + counts + survivor indices).
"""
from __future__ import annotations

import torch

from . import _lib as L

_ws_cache = {}


def _workspace(device, n, n_anchors, nc):
    need = int(L.lib().rtdm_nms_workspace_size(n, n_anchors, nc))
    key = (str(device),)
    buf = _ws_cache.get(key)
    if buf is None or buf.numel() < need:
        buf = torch.empty(need, dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    return buf, need


def class_mask(classes) -> int:
    if not classes:
        return (1 << 64) - 1
    m = 0
    for c in classes:
        if not 0 <= int(c) < 64:
            raise ValueError(f"classes filter: class {c} outside the 64-bit mask (nc > 64 needs classes=None)")
        m |= 1 << int(c)
    return m


def workspace_bytes(n, n_anchors, nc) -> int:
    return int(L.lib().rtdm_nms_workspace_size(n, n_anchors, nc))


def nms_batched(prediction: torch.Tensor, conf_thres: float = 0.1, iou_thres: float = 0.6, multi_label: bool = True,
                classes=None, agnostic: bool = False, max_det: int = 300, out=None, stream=None, workspace=None):
    """prediction: io [N, A, 5+nc] fp32 CUDA.  Returns (det [N,max_det,6], idx [N,max_det,2] int32
    (anchor row, class), count [N] int32 = survivors per image; rows >= min(count, max_det) are
    undefined).  No host synchronisation.  workspace: a caller-owned uint8 device buffer of
    workspace_bytes(...) (callers with work in flight on several streams need their own);
    default: one shared per device."""
    if prediction.dtype != torch.float32:
        prediction = prediction.float()
    prediction = prediction.contiguous()
    n, a, no = prediction.shape
    dev = prediction.device
    if out is None:
        det = torch.empty((n, max_det, 6), device=dev, dtype=torch.float32)
        idx = torch.empty((n, max_det, 2), device=dev, dtype=torch.int32)
        count = torch.empty((n,), device=dev, dtype=torch.int32)
    else:
        det, idx, count = out
    with torch.cuda.device(dev):
        if workspace is not None:
            ws, need = workspace, workspace_bytes(n, a, no - 5)
            if ws.numel() < need:
                raise ValueError(f"nms workspace has {ws.numel()} bytes, needs {need}")
        else:
            ws, need = _workspace(dev, n, a, no - 5)
        L.check(L.lib().rtdm_nms(L.ptr(prediction), n, a, no, float(conf_thres), float(iou_thres),
                                 1 if multi_label else 0, 1 if agnostic else 0, class_mask(classes), int(max_det),
                                 L.ptr(ws), need, L.ptr(det), L.ptr(idx), L.ptr(count), L.stream_ptr(stream)))
    return det, idx, count


def non_max_suppression(prediction, conf_thres=0.1, iou_thres=0.6, multi_label=True, classes=None, agnostic=False):
    """utils.py:488 drop-in (returns every survivor, like the reference)."""
    n, a, no = prediction.shape
    max_det = a * max(1, no - 5)
    det, _, count = nms_batched(prediction, conf_thres, iou_thres, multi_label, classes, agnostic, max_det)
    counts = count.cpu().tolist()
    return [det[i, :c].clone() if c > 0 else None for i, c in enumerate(counts)]
