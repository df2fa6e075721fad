"""Two-stage classify -> detect pipeline over a batch of uint8 frames.

Per batch, no host synchronisation:
  classifier: CLI transform (resize/crop/normalize) + ACFF model -> logits, probs
              (on a side stream forked from the caller's stream: the two stages are
              independent, so the classifier's small, latency-bound kernels fill the
              CUs the detector's GEMM tails and launch gaps leave idle)
  detector:   Darknet forward with the /255 fused into the stem, YOLO decode fused
              into the head convs -> io (caller's stream)
  NMS:        per-image greedy NMS -> det [B,max_det,6], idx, count (caller's stream,
              which then waits for the classifier's event: every output is ready on it)
The reference has no code joining the two stages; this composes
aider-predict.py's predict() and detect.py's forward + non_max_suppression.
"""
from __future__ import annotations

import torch

from . import _lib as L
from .nms import nms_batched


class TwoStagePipeline:
    def __init__(self, classifier, detector, conf_thres: float = 0.3, iou_thres: float = 0.4, max_det: int = 300,
                 multi_label: bool = True, agnostic: bool = False, overlap: bool = True, priority: bool = False):
        self.classifier = classifier
        self.detector = detector
        self.conf_thres = conf_thres
        self.iou_thres = iou_thres
        self.max_det = max_det
        self.multi_label = multi_label
        self.agnostic = agnostic
        # overlap=True: the classifier runs on a forked side stream beside the detector;
        # False: both stages on the caller's stream, one after the other
        self.overlap = overlap
        # priority=True: detector + NMS on a high-priority stream, classifier on a low one
        # (measured: no gain over one priority, 34.4k vs 34.7k frames/s)
        self.priority = priority
        self._bufs = {}
        self._side = {}

    def _side_stream(self, device):
        key = str(device)
        if key not in self._side:
            lo, hi = torch.cuda.Stream.priority_range()
            # classifier: lowest priority; detector + NMS: highest (the critical path),
            # so the dispatcher hands free CUs to the detector's workgroups first
            self._side[key] = (torch.cuda.Stream(device=device, priority=lo), torch.cuda.Event(), torch.cuda.Event(),
                               torch.cuda.Stream(device=device, priority=hi), torch.cuda.Event())
        return self._side[key]

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
        with torch.cuda.device(frames.device):
            main = stream if stream is not None else torch.cuda.current_stream()
            side, forked, joined, crit, crit_done = self._side_stream(frames.device)
            if not self.overlap:
                side = crit = main
            elif not self.priority:
                crit = main
            forked.record(main)
            side.wait_event(forked)
            crit.wait_event(forked)
            hc = self.classifier._get_handle(n)
            L.check(L.lib().rtdm_classify(hc, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, frames.shape[1],
                                          frames.shape[2], L.ptr(b["logits"]), L.ptr(b["probs"]),
                                          L.stream_ptr(side)))
            joined.record(side)
            hd = self.detector.handle(n)
            L.check(L.lib().rtdm_detect(hd, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, L.ptr(b["io"]),
                                        L.stream_ptr(crit)))
            nms_batched(b["io"], self.conf_thres, self.iou_thres, self.multi_label, None, self.agnostic,
                        self.max_det, out=(b["det"], b["idx"], b["count"]), stream=crit)
            crit_done.record(crit)
            main.wait_event(joined)
            main.wait_event(crit_done)
        return b
