"""Two-stage classify -> detect pipeline over a batch of uint8 frames.

Per batch, all on one stream, no host synchronisation:
  classifier: CLI transform (resize/crop/normalize) + ACFF model -> logits, probs
  detector:   Darknet forward with the /255 fused into the stem, YOLO decode fused
              into the head convs -> io
  NMS:        per-image greedy NMS -> det [B,max_det,6], idx, count
The reference has no code joining the two stages; this composes
aider-predict.py's predict() and detect.py's forward + non_max_suppression.
"""
from __future__ import annotations

import torch

from . import _lib as L
from .nms import nms_batched


class TwoStagePipeline:
    def __init__(self, classifier, detector, conf_thres: float = 0.3, iou_thres: float = 0.4, max_det: int = 300,
                 multi_label: bool = True, agnostic: bool = False):
        self.classifier = classifier
        self.detector = detector
        self.conf_thres = conf_thres
        self.iou_thres = iou_thres
        self.max_det = max_det
        self.multi_label = multi_label
        self.agnostic = agnostic
        self._bufs = {}

    def _buffers(self, n, device):
        key = (n, str(device))
        b = self._bufs.get(key)
        if b is None:
            f32 = dict(device=device, dtype=torch.float32)
            b = dict(logits=torch.empty((n, 5), **f32), probs=torch.empty((n, 5), **f32),
                     io=torch.empty((n, self.detector.n_anchors, self.detector.no), **f32),
                     det=torch.empty((n, self.max_det, 6), **f32),
                     idx=torch.empty((n, self.max_det, 2), device=device, dtype=torch.int32),
                     count=torch.empty((n,), device=device, dtype=torch.int32))
            self._bufs[key] = b
        return b

    def __call__(self, frames: torch.Tensor, stream=None) -> dict:
        """frames: [B,H,W,3] uint8 CUDA (H,W = detector img_size)."""
        n = frames.shape[0]
        b = self._buffers(n, frames.device)
        sp = L.stream_ptr(stream)
        with torch.cuda.device(frames.device):
            hc = self.classifier._get_handle(n)
            L.check(L.lib().rtdm_classify(hc, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, frames.shape[1],
                                          frames.shape[2], L.ptr(b["logits"]), L.ptr(b["probs"]), sp))
            hd = self.detector.handle(n)
            L.check(L.lib().rtdm_detect(hd, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, L.ptr(b["io"]), sp))
        nms_batched(b["io"], self.conf_thres, self.iou_thres, self.multi_label, None, self.agnostic, self.max_det,
                    out=(b["det"], b["idx"], b["count"]), stream=stream)
        return b
