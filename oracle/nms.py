"""non_max_suppression restatement in numpy (TEST INFRASTRUCTURE ONLY).

Follows yolov3/utils/utils.py:488-557 (method 'vision_batch') step by step in
fp32, and restates the third-party kernel it calls at utils.py:552,
torchvision.ops.boxes.nms — torchvision 0.8.2 (requirements-fyp.txt:198), CPU
nms_kernel: order = scores sorted descending; areas = (x2-x1)*(y2-y1);
for each i in order not yet suppressed: keep i; for each later j not
suppressed: inter = max(0, min(x2)-max(x1)) * max(0, min(y2)-max(y1)),
ovr = inter / (area_i + area_j - inter) (fp32), suppressed if
(double)ovr > iou_threshold.  Ties in score are broken by candidate index
(stable sort) — torchvision 0.8.2's sort is not specified as stable, so the
fixtures assert no exact score ties.  Parity of this kernel is UNPINNED
(torchvision is absent here and the reference ships no NMS test vectors).
"""
from __future__ import annotations

import numpy as np


def nms_kernel(boxes: np.ndarray, scores: np.ndarray, iou_thres: float) -> np.ndarray:
    boxes = boxes.astype(np.float32)
    scores = scores.astype(np.float32)
    n = boxes.shape[0]
    if n == 0:
        return np.zeros(0, np.int64)
    x1, y1, x2, y2 = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    areas = ((x2 - x1) * (y2 - y1)).astype(np.float32)
    order = np.argsort(-scores, kind="stable")
    suppressed = np.zeros(n, bool)
    keep = []
    for _i in range(n):
        i = order[_i]
        if suppressed[i]:
            continue
        keep.append(i)
        rest = order[_i + 1:]
        rest = rest[~suppressed[rest]]
        if rest.size == 0:
            continue
        xx1 = np.maximum(x1[i], x1[rest])
        yy1 = np.maximum(y1[i], y1[rest])
        xx2 = np.minimum(x2[i], x2[rest])
        yy2 = np.minimum(y2[i], y2[rest])
        w = np.maximum(np.float32(0), (xx2 - xx1).astype(np.float32))
        h = np.maximum(np.float32(0), (yy2 - yy1).astype(np.float32))
        inter = (w * h).astype(np.float32)
        denom = ((areas[i] + areas[rest]).astype(np.float32) - inter).astype(np.float32)
        ovr = (inter / denom).astype(np.float32)
        suppressed[rest[ovr.astype(np.float64) > iou_thres]] = True
    return np.asarray(keep, np.int64)


def non_max_suppression(prediction: np.ndarray, conf_thres=0.1, iou_thres=0.6, multi_label=True, classes=None,
                        agnostic=False, return_index=False):
    """prediction: [N, A, 5+nc] float32 -> list of [k, 6] float32 arrays or None
    (and, with return_index, [k, 2] int arrays of (anchor row, class))."""
    min_wh, max_wh = 2, 4096
    prediction = np.asarray(prediction, np.float32)
    nc = prediction.shape[2] - 5
    multi_label = multi_label and nc > 1
    conf = np.float32(conf_thres)
    output, index = [None] * len(prediction), [None] * len(prediction)
    for image_i, pred in enumerate(prediction):
        rows = np.arange(pred.shape[0])
        sel = pred[:, 4] > conf
        pred, rows = pred[sel], rows[sel]
        sel = ((pred[:, 2:4] > min_wh) & (pred[:, 2:4] < max_wh)).all(1)
        pred, rows = pred[sel], rows[sel]
        if not pred.shape[0]:
            continue
        pred = pred.copy()
        pred[:, 5:] *= pred[:, 4:5]
        box = np.empty((pred.shape[0], 4), np.float32)
        box[:, 0] = pred[:, 0] - pred[:, 2] / np.float32(2)
        box[:, 1] = pred[:, 1] - pred[:, 3] / np.float32(2)
        box[:, 2] = pred[:, 0] + pred[:, 2] / np.float32(2)
        box[:, 3] = pred[:, 1] + pred[:, 3] / np.float32(2)
        if multi_label:
            i, j = np.nonzero(pred[:, 5:] > conf)
            det = np.concatenate((box[i], pred[i, j + 5][:, None], j.astype(np.float32)[:, None]), 1)
            src = np.stack((rows[i], j), 1)
        else:
            j = pred[:, 5:].argmax(1)
            cf = pred[np.arange(len(j)), j + 5]
            det = np.concatenate((box, cf[:, None], j.astype(np.float32)[:, None]), 1)
            src = np.stack((rows, j), 1)
        if classes:
            sel = np.isin(j, np.asarray(classes))
            det, src, j = det[sel], src[sel], j[sel]
        fin = np.isfinite(det).all(1)
        det, src = det[fin], src[fin]
        if not det.shape[0]:
            continue
        c = det[:, 5] * 0 if agnostic else det[:, 5]
        boxes = (det[:, :4] + (c[:, None] * np.float32(max_wh))).astype(np.float32)
        keep = nms_kernel(boxes, det[:, 4], iou_thres)
        output[image_i] = det[keep].astype(np.float32)
        index[image_i] = src[keep].astype(np.int64)
    return (output, index) if return_index else output


def score_ties(prediction: np.ndarray, conf_thres: float, iou_thres: float):
    """(tied candidate scores, harmful ties): a tie is harmful when two equal-score
    candidates of the same class overlap with IoU > iou_thres, i.e. when the
    unspecified tie order of the sort could change which survives."""
    p = np.asarray(prediction, np.float32)
    ties = harmful = 0
    for pred in p:
        pred = pred[pred[:, 4] > np.float32(conf_thres)]
        s = pred[:, 5:] * pred[:, 4:5]
        i, j = np.nonzero(s > np.float32(conf_thres))
        sc = s[i, j]
        vals, inv, cnt = np.unique(sc, return_inverse=True, return_counts=True)
        ties += int((cnt - 1).sum())
        for g in np.nonzero(cnt > 1)[0]:
            members = np.nonzero(inv == g)[0]
            for a in range(len(members)):
                for b in range(a + 1, len(members)):
                    ma, mb = members[a], members[b]
                    if j[ma] != j[mb]:
                        continue
                    ba = pred[i[ma], :4]
                    bb = pred[i[mb], :4]
                    box = lambda r: (r[0] - r[2] / 2, r[1] - r[3] / 2, r[0] + r[2] / 2, r[1] + r[3] / 2)
                    xa, xb = box(ba), box(bb)
                    iw = max(0.0, min(xa[2], xb[2]) - max(xa[0], xb[0]))
                    ih = max(0.0, min(xa[3], xb[3]) - max(xa[1], xb[1]))
                    inter = iw * ih
                    ua = (xa[2] - xa[0]) * (xa[3] - xa[1]) + (xb[2] - xb[0]) * (xb[3] - xb[1]) - inter
                    if ua > 0 and inter / ua > iou_thres:
                        harmful += 1
    return ties, harmful


def _cands(pred: np.ndarray, conf: float):
    """(keys [(row, class)], xyxy boxes, scores, obj) of one image's multi-label candidates
    (utils.py:507-524 filters)."""
    pred = np.asarray(pred, np.float32)
    rows = np.nonzero((pred[:, 4] > np.float32(conf)) & ((pred[:, 2:4] > 2) & (pred[:, 2:4] < 4096)).all(1))[0]
    p = pred[rows]
    s = p[:, 5:] * p[:, 4:5]
    i, j = np.nonzero(s > np.float32(conf))
    b = p[i, :4]
    box = np.stack([b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2, b[:, 0] + b[:, 2] / 2, b[:, 1] + b[:, 3] / 2], 1)
    return [(int(rows[a]), int(c)) for a, c in zip(i, j)], box.astype(np.float64), s[i, j].astype(np.float64), \
        p[i, 4].astype(np.float64)


def _iou_matrix(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    iw = np.clip(np.minimum(a[:, None, 2], b[None, :, 2]) - np.maximum(a[:, None, 0], b[None, :, 0]), 0, None)
    ih = np.clip(np.minimum(a[:, None, 3], b[None, :, 3]) - np.maximum(a[:, None, 1], b[None, :, 1]), 0, None)
    inter = iw * ih
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / np.maximum(area_a[:, None] + area_b[None, :] - inter, 1e-30)


def survivors_equal_outside_band(io_ref: np.ndarray, io_got: np.ndarray, conf_thres: float, iou_thres: float,
                                 band: float = 1e-3):
    """SURVEY §8d's end-to-end fp16 rule: the NMS survivor sets of two io tensors are equal
    after excluding the candidates within `band` of the thresholds.  A candidate (row,
    class) is near a threshold when, in either io, its objectness or its score is within
    `band` of conf_thres, or when it overlaps a same-class candidate with IoU within `band`
    of iou_thres, or with IoU > iou_thres - band and a score within `band` of its own (the
    greedy order between them is then undecided); a candidate that overlaps (IoU >
    iou_thres - band) a higher-scored excluded candidate of its class is excluded too (its
    fate follows that one's).  Returns (n_ref survivors, n_got survivors, excluded
    differences, unexplained differences [(image, row, class)])."""
    ref_s, ref_i = non_max_suppression(io_ref, conf_thres, iou_thres, return_index=True)
    got_s, got_i = non_max_suppression(io_got, conf_thres, iou_thres, return_index=True)
    n_ref = n_got = n_exc = 0
    bad = []
    for b in range(len(io_ref)):
        R = set() if ref_i[b] is None else {tuple(map(int, r)) for r in ref_i[b]}
        G = set() if got_i[b] is None else {tuple(map(int, r)) for r in got_i[b]}
        n_ref += len(R)
        n_got += len(G)
        D = R ^ G
        if not D:
            continue
        # candidates of both io at a slightly lower threshold, so a near-threshold one is seen
        keys, box, sc, obj = _cands(io_ref[b], conf_thres - band)
        keys_g, _, sc_g, obj_g = _cands(io_got[b], conf_thres - band)
        idx = {k: n for n, k in enumerate(keys)}
        near = np.zeros(len(keys), bool)
        near |= (np.abs(obj - conf_thres) <= band) | (np.abs(sc - conf_thres) <= band)
        near_g = set()
        for n, k in enumerate(keys_g):
            if abs(obj_g[n] - conf_thres) <= band or abs(sc_g[n] - conf_thres) <= band:
                near_g.add(k)
                if k in idx:
                    near[idx[k]] = True
        cls = np.array([k[1] for k in keys])
        iou = _iou_matrix(box, box)
        same = cls[:, None] == cls[None, :]
        np.fill_diagonal(same, False)
        ov = same & (iou > iou_thres - band)
        near |= (same & (np.abs(iou - iou_thres) <= band)).any(1)
        near |= (ov & (np.abs(sc[:, None] - sc[None, :]) <= band)).any(1)
        order = np.argsort(-sc, kind="stable")
        for n in order:  # cascade downward in score
            if not near[n]:
                higher = ov[n] & (sc > sc[n])
                if (higher & near).any():
                    near[n] = True
        for k in D:
            if (near[idx[k]] if k in idx else k in near_g):
                n_exc += 1
            else:
                bad.append((b,) + k)
    return n_ref, n_got, n_exc, bad
