"""TensorRT-YOLO drop-in on the HIP runtime.

Counterpart of victim_localization/tensorrt_inference/utils/yolo_with_plugins.py
(``TrtYOLO``, ``_postprocess_yolo``, ``_nms_boxes``) and of the YoloLayer_TRT
plugin (plugins/yolo_layer.cu).  The engine is replaced by the cfg-driven
Darknet runtime; its output bindings by ``rtdm_detect_trt``, which writes the
plugin's Detection records {x, y, w, h, det_conf, class_id, class_conf}
(yolo_layer.h:26-31) for every head straight from the head convs.  The host
post-processing keeps the reference's semantics: score = det_conf * class_conf
>= conf_th (yolo_with_plugins.py:115-118), per-class greedy NMS with the +1 px
IoU (:59-97), ``+ 0.5`` and integer truncation of the boxes (:158-159), clip to
the image (:331-332).
"""
from __future__ import annotations

import os
import re

import numpy as np
import torch

from . import _lib as L
from .darknet import Darknet, load_darknet_weights

_CFG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cfg")
# trt_yolo.py --model families (trt_yolo.py:33-37) -> the repo's Darknet cfgs
MODEL_CFGS = {
    "yolov3": "yolov3-aider-416",
    "yolov3-spp": "yolov3-spp-aider",
    "yolov3-tiny": "yolov3-tiny-aider-416",
    "yolov4-tiny": "yolov4-tiny-aider-416",
}


def parse_model_name(model: str):
    """'[family]-[dim]' with dim 'S' or 'WxH' (trt_yolo.py:33-37) -> (family, (h, w))."""
    m = re.fullmatch(r"(.+?)-(\d+)(?:x(\d+))?", model)
    if not m or m.group(1) not in MODEL_CFGS:
        raise SystemExit(f"ERROR: bad model ({model})!")
    w = int(m.group(2))
    h = int(m.group(3)) if m.group(3) else w
    if w % 32 or h % 32:
        raise SystemExit(f"ERROR: bad model ({model})!")
    return m.group(1), (h, w)


def nms_boxes(detections: np.ndarray, nms_threshold: float) -> np.ndarray:
    """_nms_boxes (yolo_with_plugins.py:59-97): rows [x, y, w, h, det_conf, cls, cls_conf]
    of one class -> kept row indices, greedy in descending det_conf*cls_conf; a box is
    dropped when its IoU with the kept one (areas w*h, intersection with the +1 px
    convention) exceeds the threshold.  Equal scores: the reference's
    ``argsort()[::-1]`` leaves their order to numpy's quicksort; here the later row
    goes first (a stable ascending sort, reversed)."""
    x, y, w, h = (detections[:, i] for i in range(4))
    score = detections[:, 4] * detections[:, 6]
    area = w * h
    order = np.argsort(score, kind="stable")[::-1]
    keep = []
    while order.size:
        i, rest = order[0], order[1:]
        keep.append(i)
        iw = np.maximum(0.0, np.minimum(x[i] + w[i], x[rest] + w[rest]) - np.maximum(x[i], x[rest]) + 1)
        ih = np.maximum(0.0, np.minimum(y[i] + h[i], y[rest] + h[rest]) - np.maximum(y[i], y[rest]) + 1)
        inter = iw * ih
        iou = inter / (area[i] + area[rest] - inter)
        order = rest[iou <= nms_threshold]
    return np.array(keep, dtype=np.int64)


def postprocess_yolo(trt_outputs, img_w, img_h, conf_th, nms_threshold, input_shape, letter_box=False):
    """_postprocess_yolo (yolo_with_plugins.py:100-162): Detection records of all heads ->
    (boxes int [k,4] x1y1x2y2, scores [k], classes [k]) in image pixels."""
    dets = np.concatenate([np.asarray(o, np.float32).reshape(-1, 7) for o in trt_outputs], axis=0)
    dets = dets[dets[:, 4] * dets[:, 6] >= conf_th]
    if len(dets) == 0:
        return np.zeros((0, 4), np.int64), np.zeros((0,), np.float32), np.zeros((0,), np.float32)
    old_h, old_w, off_h, off_w = img_h, img_w, 0, 0
    if letter_box:
        if img_w / input_shape[1] >= img_h / input_shape[0]:
            old_h = int(input_shape[0] * img_w / input_shape[1])
            off_h = (old_h - img_h) // 2
        else:
            old_w = int(input_shape[1] * img_h / input_shape[0])
            off_w = (old_w - img_w) // 2
    dets[:, 0:4] *= np.array([old_w, old_h, old_w, old_h], dtype=np.float32)
    kept = [np.zeros((0, 7), dets.dtype)]
    for c in set(dets[:, 5]):  # per-class NMS, classes in the reference's set() order
        cd = dets[dets[:, 5] == c]
        kept.append(cd[nms_boxes(cd, nms_threshold)])
    nd = np.concatenate(kept, axis=0)
    xx, yy = nd[:, 0:1], nd[:, 1:2]
    if letter_box:
        xx, yy = xx - off_w, yy - off_h
    boxes = (np.concatenate([xx, yy, xx + nd[:, 2:3], yy + nd[:, 3:4]], axis=1) + 0.5).astype(np.int64)
    return boxes, nd[:, 4] * nd[:, 6], nd[:, 5]


class TrtYOLO:
    """TrtYOLO (yolo_with_plugins.py:232-333) on librtdm.so.

    model: '[yolov3|yolov3-spp|yolov3-tiny|yolov4-tiny]-[dim]'; weights: the darknet
    .weights file the reference engine was built from (yolo_to_onnx.py); half: fp16
    compute (the TRT engines' default precision)."""

    def __init__(self, model, category_num=80, letter_box=False, cuda_ctx=None, weights=None, cfg=None,
                 half=True, device=0):
        self.model = model
        self.category_num = category_num
        self.letter_box = letter_box
        family, self.input_shape = parse_model_name(model)
        cfg = cfg or os.path.join(_CFG_DIR, MODEL_CFGS[family] + ".cfg")
        if weights is None or not os.path.exists(weights):
            raise FileNotFoundError(f"darknet weights for {model} not found: {weights}")
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.net = Darknet(cfg, self.input_shape)
        if self.net.info.nc != category_num:
            raise ValueError(f"cfg has {self.net.info.nc} classes, category_num={category_num}")
        load_darknet_weights(self.net, weights)
        if half:
            self.net.half()

    def infer(self, frames: torch.Tensor) -> torch.Tensor:
        """frames: uint8 RGB [n, H, W, 3] on the device -> Detection records [n, rows, 7]."""
        n = frames.shape[0]
        out = torch.empty((n, self.net.n_anchors, 7), device=frames.device, dtype=torch.float32)
        with torch.cuda.device(frames.device):
            h = self.net.handle(n)
            L.check(L.lib().rtdm_detect_trt(h, L.ptr(frames.contiguous()), L.RTDM_INPUT_FRAME_U8, n, L.ptr(out),
                                            L.stream_ptr()))
        return out

    def detect(self, img: np.ndarray, conf_th=0.3, letter_box=None):
        """img: BGR uint8 [H, W, 3] at the engine input size (cv2.resize of other sizes is
        not available in this image).  Returns (boxes, scores, classes)."""
        letter_box = self.letter_box if letter_box is None else letter_box
        if img.shape[:2] != tuple(self.input_shape):
            raise ValueError(f"image {img.shape[:2]} must match the model input {self.input_shape}")
        rgb = torch.from_numpy(np.ascontiguousarray(img[..., ::-1])).to(self.device)[None]
        dets = self.infer(rgb)[0].cpu().numpy()
        boxes, scores, classes = postprocess_yolo([dets], img.shape[1], img.shape[0], conf_th, nms_threshold=0.5,
                                                  input_shape=self.input_shape, letter_box=letter_box)
        boxes[:, [0, 2]] = np.clip(boxes[:, [0, 2]], 0, img.shape[1] - 1)
        boxes[:, [1, 3]] = np.clip(boxes[:, [1, 3]], 0, img.shape[0] - 1)
        return boxes, scores, classes
