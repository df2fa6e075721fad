"""TensorRT YOLO plugin decode + host post-processing, numpy restatement (TEST INFRASTRUCTURE ONLY).

Restates tensorrt_inference/plugins/yolo_layer.cu:203-306 (CalDetection,
CalDetection_NewCoords) record by record in fp32, and
tensorrt_inference/utils/yolo_with_plugins.py:59-162 (_nms_boxes,
_postprocess_yolo) with explicit Python loops.

Pinning: the plugin is CUDA (not buildable here) and the reference ships no TRT
outputs, so CalDetection is pinned through an identity with the reference's
own PyTorch YOLOLayer golden io (tests/golden/det_golden.npz): with
scale_x_y = 1, det_conf = io[4], class_conf = max(io[5:]), w = io[2] / input_w,
x = io[0] / input_w - w / 2 (tests/test_oracle_golden.py).  The post-processing
restatement is unpinned (cv2/tensorrt/pycuda absent): parity unpinned there.
"""
from __future__ import annotations

import numpy as np

F = np.float32


def _sig(v):
    return F(1.0) / (F(1.0) + np.exp(F(-v), dtype=F))


def cal_detection_rows(raw: np.ndarray, heads, in_w: int, in_h: int) -> np.ndarray:
    """raw: [n, rows, 5+nc] head predictions in io row order; heads: list of dicts
    {na, ny, nx, anchors [(w,h)...] pixels, scale_x_y, new_coords} in cfg order.
    -> Detection records [n, rows, 7] (yolo_layer.h:26-31)."""
    raw = np.asarray(raw, F)
    n, rows, no = raw.shape
    nc = no - 5
    out = np.zeros((n, rows, 7), F)
    for b in range(n):
        r0 = 0
        for hd in heads:
            na, ny, nx = hd["na"], hd["ny"], hd["nx"]
            s = F(hd.get("scale_x_y", 1.0))
            newc = hd.get("new_coords", 0)
            iw = F(nx * (in_w // nx))
            ih = F(ny * (in_h // ny))
            for a in range(na):
                aw, ah = F(hd["anchors"][a][0]), F(hd["anchors"][a][1])
                for gy in range(ny):
                    for gx in range(nx):
                        r = r0 + (a * ny + gy) * nx + gx
                        v = raw[b, r]
                        cls, best = 0, F(-np.inf)
                        for c in range(nc):
                            if v[5 + c] > best:
                                best, cls = v[5 + c], c
                        if not newc:
                            bx = (F(gx) + (s * _sig(v[0]) - (s - F(1)) * F(0.5))) / F(nx)
                            by = (F(gy) + (s * _sig(v[1]) - (s - F(1)) * F(0.5))) / F(ny)
                            bw = np.exp(v[2], dtype=F) * aw / iw
                            bh = np.exp(v[3], dtype=F) * ah / ih
                            dc, cc = _sig(v[4]), _sig(best)
                        else:
                            bx = (F(gx) + (s * v[0] - (s - F(1)) * F(0.5))) / F(nx)
                            by = (F(gy) + (s * v[1] - (s - F(1)) * F(0.5))) / F(ny)
                            bw = v[2] * v[2] * F(4) * aw / iw
                            bh = v[3] * v[3] * F(4) * ah / ih
                            dc, cc = v[4], best
                        out[b, r] = (bx - bw / F(2), by - bh / F(2), bw, bh, dc, F(cls), cc)
            r0 += na * ny * nx
    return out


def nchw_to_rows(p: np.ndarray, na: int) -> np.ndarray:
    """Plugin input binding [n, na*no, ny, nx] -> rows [n, na*ny*nx, no]."""
    n, c, ny, nx = p.shape
    no = c // na
    return p.reshape(n, na, no, ny, nx).transpose(0, 1, 3, 4, 2).reshape(n, na * ny * nx, no)


def nms_boxes(dets: np.ndarray, thr: float):
    """_nms_boxes (yolo_with_plugins.py:59-97) as a loop; fixtures assert no score ties."""
    score = [float(F(d[4]) * F(d[6])) for d in dets]
    order = sorted(range(len(dets)), key=lambda i: -score[i])
    keep = []
    while order:
        i = order.pop(0)
        keep.append(i)
        xi, yi, wi, hi = (F(v) for v in dets[i, :4])
        rest = []
        for j in order:
            xj, yj, wj, hj = (F(v) for v in dets[j, :4])
            iw = max(F(0), min(xi + wi, xj + wj) - max(xi, xj) + F(1))
            ih = max(F(0), min(yi + hi, yj + hj) - max(yi, yj) + F(1))
            inter = F(iw * ih)
            iou = inter / (wi * hi + wj * hj - inter)
            if iou <= thr:
                rest.append(j)
        order = rest
    return keep


def postprocess_yolo(trt_outputs, img_w, img_h, conf_th, nms_threshold, input_shape, letter_box=False):
    """_postprocess_yolo (yolo_with_plugins.py:100-162)."""
    dets = [r for o in trt_outputs for r in np.asarray(o, F).reshape(-1, 7) if F(r[4]) * F(r[6]) >= conf_th]
    if not dets:
        return np.zeros((0, 4), np.int64), np.zeros((0,), F), np.zeros((0,), F)
    dets = np.array(dets, F)
    old_h, old_w, off_h, off_w = img_h, img_w, 0, 0
    if letter_box:
        if img_w / input_shape[1] >= img_h / input_shape[0]:
            old_h = int(input_shape[0] * img_w / input_shape[1])
            off_h = (old_h - img_h) // 2
        else:
            old_w = int(input_shape[1] * img_h / input_shape[0])
            off_w = (old_w - img_w) // 2
    dets[:, 0:4] *= np.array([old_w, old_h, old_w, old_h], F)
    out = []
    for c in set(dets[:, 5]):
        cd = dets[dets[:, 5] == c]
        out += [cd[k] for k in nms_boxes(cd, nms_threshold)]
    nd = np.array(out, F).reshape(-1, 7)
    boxes = np.zeros((len(nd), 4), np.int64)
    for i, d in enumerate(nd):
        x, y = d[0] - F(off_w), d[1] - F(off_h)
        boxes[i] = [int(v + F(0.5)) for v in (x, y, x + d[2], y + d[3])]
    return boxes, nd[:, 4] * nd[:, 6], nd[:, 5]
