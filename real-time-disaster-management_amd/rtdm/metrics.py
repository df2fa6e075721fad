"""Detection metrics of the mAP harness (victim_localization/yolov3/test.py:11-197,
utils/utils.py:145-234, 283-307), restated for the rtdm detector.

Host-side bookkeeping that sits after ``rtdm_nms``: per-image true-positive
matching at IoU 0.5 (test.py:115-164), the per-class precision/recall curve and
101-point interpolated AP (``ap_per_class`` / ``compute_ap``), and the
(P, R, mAP@0.5, F1) summary test.py prints and returns.  These are float64 numpy
reductions over at most a few thousand survivors per image; nothing here is on
the frame path, so they run on the host on purpose.  The reference's result for
the same survivors and labels is reproduced exactly (tests/test_metrics.py pins it
against fixtures produced by the reference's own ``test.test``).

Two reference behaviours kept on purpose for metric parity:
  * ``clip_coords`` (utils.py:139-142) clamps a copy made by advanced indexing, so
    test.py:130 leaves predicted boxes unclipped; ``DetectionStats(clip=False)``
    (the default) does the same, ``clip=True`` really clamps.
  * only mAP@0.5 is evaluated (test.py:52 keeps ``iouv[0]``), P and R are read
    off the curves at score 0.1 (``pr_score``, utils.py:164).
"""
from __future__ import annotations

import numpy as np
import torch

PR_SCORE = 0.1   # utils.py:164
IOU_V = np.array([0.5], np.float32)   # test.py:51-53: linspace(0.5, 0.95, 10)[0]


def xywh2xyxy(x):
    """utils.py:93-101: centre/size to corner boxes (numpy or torch)."""
    y = torch.zeros_like(x) if isinstance(x, torch.Tensor) else np.zeros_like(x)
    half_w, half_h = x[:, 2] / 2, x[:, 3] / 2
    y[:, 0] = x[:, 0] - half_w
    y[:, 1] = x[:, 1] - half_h
    y[:, 2] = x[:, 0] + half_w
    y[:, 3] = x[:, 1] + half_h
    return y


def box_iou(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """utils.py:283-307: pairwise IoU of corner boxes [N,4] x [M,4] -> [N,M], in the
    boxes' own dtype (float32 for detector output), same operation order."""
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lo = np.maximum(a[:, None, :2], b[None, :, :2])
    hi = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(hi - lo, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter)


def clip_coords(boxes, img_shape):
    """Clamp corner boxes to (height, width) in place (the intent of utils.py:139-142;
    see the module docstring for why the evaluator does not call it by default)."""
    h, w = img_shape
    if isinstance(boxes, torch.Tensor):
        boxes[:, 0].clamp_(0, w)
        boxes[:, 2].clamp_(0, w)
        boxes[:, 1].clamp_(0, h)
        boxes[:, 3].clamp_(0, h)
    else:
        boxes[:, 0] = np.clip(boxes[:, 0], 0, w)
        boxes[:, 2] = np.clip(boxes[:, 2], 0, w)
        boxes[:, 1] = np.clip(boxes[:, 1], 0, h)
        boxes[:, 3] = np.clip(boxes[:, 3], 0, h)
    return boxes


def compute_ap(recall: np.ndarray, precision: np.ndarray) -> float:
    """utils.py:208-234: area under the precision envelope, 101-point interpolated
    (COCO) and integrated with the trapezoid rule."""
    r = np.concatenate(([0.0], recall, [min(recall[-1] + 1e-3, 1.0)]))
    p = np.concatenate(([0.0], precision, [0.0]))
    p = np.maximum.accumulate(p[::-1])[::-1]   # monotone envelope from the right
    x = np.linspace(0, 1, 101)
    y = np.interp(x, r, p)
    return float(np.add.reduce(np.diff(x) * (y[1:] + y[:-1]) / 2.0))


def ap_per_class(tp, conf, pred_cls, target_cls):
    """utils.py:145-205.  tp [n, niou] bool, conf/pred_cls [n], target_cls [m] ->
    (p, r, ap, f1) each [n_target_classes, niou] and the target classes (int32).
    Classes are those with ground truth; a class with no predictions scores 0."""
    tp = np.asarray(tp)
    conf = np.asarray(conf)
    pred_cls = np.asarray(pred_cls)
    target_cls = np.asarray(target_cls)
    order = np.argsort(-conf)   # same sort (numpy default kind) => same tie order
    tp, conf, pred_cls = tp[order], conf[order], pred_cls[order]
    classes = np.unique(target_cls)
    shape = (len(classes), tp.shape[1])
    ap, p, r = np.zeros(shape), np.zeros(shape), np.zeros(shape)
    for ci, c in enumerate(classes):
        sel = pred_cls == c
        n_gt = (target_cls == c).sum()
        n_p = sel.sum()
        if n_p == 0 or n_gt == 0:
            continue
        tp_c = tp[sel]
        tpc = tp_c.cumsum(0)
        fpc = (1 - tp_c).cumsum(0)
        recall = tpc / (n_gt + 1e-16)
        precision = tpc / (tpc + fpc)
        # P and R at score PR_SCORE: conf decreases along the curve, so interpolate on -conf
        r[ci] = np.interp(-PR_SCORE, -conf[sel], recall[:, 0])
        p[ci] = np.interp(-PR_SCORE, -conf[sel], precision[:, 0])
        for j in range(tp.shape[1]):
            ap[ci, j] = compute_ap(recall[:, j], precision[:, j])
    f1 = 2 * p * r / (p + r + 1e-16)
    return p, r, ap, f1, classes.astype("int32")


def match_image(pred: np.ndarray, labels: np.ndarray, width: float, height: float,
                iouv: np.ndarray = IOU_V) -> np.ndarray:
    """test.py:133-160 for one image.  pred [k,6] (x1,y1,x2,y2,score,cls) in NMS order,
    labels [nl,5] (cls, x, y, w, h normalised).  Returns correct [k, niou] bool.

    Per target class (ascending), each prediction of that class in order takes its
    best-IoU target of the class if IoU > iouv[0] and that target is still free; a
    prediction whose best target is taken is not re-assigned (reference greedy)."""
    correct = np.zeros((pred.shape[0], iouv.size), bool)
    nl = labels.shape[0]
    if not nl or not pred.shape[0]:
        return correct
    whwh = np.array([width, height, width, height], np.float32)
    tcls = labels[:, 0]
    tbox = xywh2xyxy(labels[:, 1:5].astype(np.float32)) * whwh
    detected = set()
    for c in np.unique(tcls):
        ti = np.nonzero(tcls == c)[0]
        pi = np.nonzero(pred[:, 5] == c)[0]
        if not pi.size:
            continue
        iou = box_iou(pred[pi, :4], tbox[ti])
        best = iou.argmax(1)
        best_iou = iou[np.arange(pi.size), best]
        for j in np.nonzero(best_iou > iouv[0])[0]:
            d = int(ti[best[j]])
            if d in detected:
                continue
            detected.add(d)
            correct[pi[j]] = best_iou[j] > iouv
            if len(detected) == nl:
                break
    return correct


class DetectionStats:
    """Accumulates test.py's per-image ``stats`` (correct, conf, pcls, tcls) and
    reduces them like test.py:166-197.  Feed it NMS output (list of [k,6] tensors or
    None per image, rtdm.nms.non_max_suppression's format) and the collated targets
    [nt,6] (image, cls, x, y, w, h normalised; datasets.py:501-505)."""

    def __init__(self, nc: int, clip: bool = False):
        self.nc = nc
        self.clip = clip
        self.seen = 0
        self.stats = []

    def update(self, output, targets, height: int, width: int) -> None:
        t = targets.detach().cpu().numpy() if isinstance(targets, torch.Tensor) else np.asarray(targets)
        for si, pred in enumerate(output):
            labels = t[t[:, 0] == si, 1:]
            tcls = labels[:, 0].tolist()
            self.seen += 1
            if pred is None:
                if len(labels):
                    self.stats.append((np.zeros((0, IOU_V.size), bool), np.zeros(0, np.float32),
                                       np.zeros(0, np.float32), tcls))
                continue
            pr = pred.detach().cpu().numpy() if isinstance(pred, torch.Tensor) else np.asarray(pred)
            if self.clip:
                pr = clip_coords(pr.copy(), (height, width))
            correct = match_image(pr, labels, width, height)
            self.stats.append((correct, pr[:, 4], pr[:, 5], tcls))

    def compute(self):
        """-> dict(mp, mr, map, mf1, maps[nc], per-class p/r/ap/f1, ap_class, nt, seen)."""
        nc = self.nc
        out = {"seen": self.seen}
        cols = [np.concatenate([np.asarray(s[k]) for s in self.stats], 0) for k in range(4)] if self.stats else []
        if cols:
            p, r, ap, f1, ap_class = ap_per_class(*cols)
            with np.errstate(invalid="ignore", divide="ignore"):
                mp, mr, map_, mf1 = (float(np.mean(v)) for v in (p, r, ap, f1))
            nt = np.bincount(cols[3].astype(np.int64), minlength=nc)
        else:
            p = r = ap = f1 = np.zeros((0, 1))
            ap_class = np.zeros(0, np.int32)
            mp = mr = map_ = mf1 = 0.0
            nt = np.zeros(1, np.int64)
        maps = np.zeros(nc) + map_
        for i, c in enumerate(ap_class):
            maps[c] = ap[i, 0]
        out.update(mp=mp, mr=mr, map=map_, mf1=mf1, maps=maps, p=p[:, 0], r=r[:, 0], ap=ap[:, 0], f1=f1[:, 0],
                   ap_class=ap_class, nt=nt)
        return out
