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
from .nms import nms_batched, workspace_bytes


def unpack_record(flat: torch.Tensor, pipe, n: int) -> dict:
    """Views of one flat output record (TwoStagePipeline.record_layout) as named tensors."""
    lay, total = pipe.record_layout(n)
    if flat.numel() != total:
        raise ValueError(f"record has {flat.numel()} floats, layout needs {total}")
    out = {"record": flat}
    for k, (o, s) in lay.items():
        c = 1
        for d in s:
            c *= d
        v = flat[o:o + c]
        if k in ("idx", "count"):
            v = v.view(torch.int32)
        out[k] = v.view(s)
    return out


class TwoStagePipeline:
    def __init__(self, classifier, detector, conf_thres: float = 0.3, iou_thres: float = 0.4, max_det: int = 300,
                 multi_label: bool = True, agnostic: bool = False, overlap: bool = True, priority: bool = False,
                 graphs: bool = False):
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
        # graphs=True: the whole batch (both stages, NMS, every cross-stream fork/join) is
        # captured once per (batch size, input buffer, handles) into a hipGraph and replayed:
        # one host call per batch instead of ~35 launches + stream/event operations, so the
        # small per-rank batches of frame-sharded multi-GPU runs are not host-bound
        self.graphs = graphs
        self._bufs = {}
        self._side = {}
        self._graphs = {}

    def _side_stream(self, device):
        key = str(device)
        if key not in self._side:
            lo, hi = torch.cuda.Stream.priority_range()
            # classifier: lowest priority; detector + NMS: highest (the critical path),
            # so the dispatcher hands free CUs to the detector's workgroups first
            self._side[key] = (torch.cuda.Stream(device=device, priority=lo), torch.cuda.Event(), torch.cuda.Event(),
                               torch.cuda.Stream(device=device, priority=hi), torch.cuda.Event())
        return self._side[key]

    def record_layout(self, n):
        """Field -> (offset, shape) in the flat per-batch output record: every per-frame
        output (logits, probs, det, idx, count) is a contiguous slice of ONE float32 buffer,
        so a rank ships its whole result to rank 0 with a single gather;
        idx and count are int32 bit patterns in that buffer."""
        shapes = (("logits", (n, 5)), ("probs", (n, 5)))
        if self.detector is not None:  # None: classification only (BASELINE config 2)
            shapes += (("det", (n, self.max_det, 6)), ("idx", (n, self.max_det, 2)), ("count", (n,)))
        out, o = {}, 0
        for k, s in shapes:
            out[k] = (o, s)
            c = 1
            for d in s:
                c *= d
            o += c
        return out, o

    def _buffers(self, n, device):
        key = (n, str(device))
        b = self._bufs.get(key)
        if b is None:
            b = unpack_record(torch.empty(self.record_layout(n)[1], device=device, dtype=torch.float32), self, n)
            if self.detector is not None:
                b["io"] = torch.empty((n, self.detector.n_anchors, self.detector.no), device=device,
                                      dtype=torch.float32)
                # NMS scratch of this pipeline alone: pipelines may run on several streams at once
                b["ws"] = torch.empty(workspace_bytes(n, self.detector.n_anchors, self.detector.no - 5),
                                      device=device, dtype=torch.uint8)
            self._bufs[key] = b
        return b

    def record(self, n, device):
        """The flat output record of batch size n (valid after a call with that n)."""
        return self._buffers(n, device)["record"]

    def __call__(self, frames: torch.Tensor, stream=None) -> dict:
        """frames: [B,H,W,3] uint8 CUDA (H,W = detector img_size; any size without a
        detector).  Returns the output views
        (logits, probs, det, idx, count, io, record), valid once `stream` reaches this point."""
        if not self.graphs:
            return self._launch(frames, stream)
        n = frames.shape[0]
        with torch.cuda.device(frames.device):
            key = self._graph_key(frames)
            g = self._graphs.pop(key, None)
            if g is None:
                self._launch(frames)  # first call: handles, plans, workspaces, resize tables
                torch.cuda.synchronize()
                key = self._graph_key(frames)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._launch(frames)
            self._graphs[key] = g  # (re)inserted last: most recently used
            self._drop_stale_graphs(key)
            if stream is None:
                g.replay()
            else:
                with torch.cuda.stream(stream):
                    g.replay()
        return self._buffers(n, frames.device)

    # at most this many captured graphs per pipeline (least recently used dropped first)
    max_graphs = 8

    def _graph_key(self, frames):
        """Handles are created on demand (and recreated for a larger batch, a dtype change or
        new weights), so a graph is keyed on the handles' GENERATION counters: a destroyed
        handle's successor may reuse its heap address, and a graph replaying the old
        handle's arena and weights would read freed memory."""
        n = frames.shape[0]
        gc = -1
        if self.classifier is not None:
            self.classifier._get_handle(n)
            gc = self.classifier.handle_generation
        gd = -1
        if self.detector is not None:
            self.detector.handle(n)
            gd = self.detector.handle_generation
        return (n, frames.data_ptr(), tuple(frames.shape), str(frames.device), gc, gd)

    def _drop_stale_graphs(self, key):
        """Forget graphs of older handle generations, then bound the cache (LRU)."""
        gens = key[4:]
        for k in [k for k in self._graphs if k[4:] != gens]:
            del self._graphs[k]
        while len(self._graphs) > self.max_graphs:
            del self._graphs[next(iter(self._graphs))]

    def _launch(self, frames: torch.Tensor, stream=None) -> dict:
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
            if self.classifier is not None:  # None: detection only (BASELINE config 3)
                hc = self.classifier._get_handle(n)
                L.check(L.lib().rtdm_classify(hc, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, frames.shape[1],
                                              frames.shape[2], L.ptr(b["logits"]), L.ptr(b["probs"]),
                                              L.stream_ptr(side)))
            joined.record(side)
            if self.detector is not None:  # None: classification only (BASELINE config 2)
                hd = self.detector.handle(n)
                L.check(L.lib().rtdm_detect(hd, L.ptr(frames), L.RTDM_INPUT_FRAME_U8, n, L.ptr(b["io"]),
                                            L.stream_ptr(crit)))
                nms_batched(b["io"], self.conf_thres, self.iou_thres, self.multi_label, None, self.agnostic,
                            self.max_det, out=(b["det"], b["idx"], b["count"]), stream=crit, workspace=b["ws"])
            crit_done.record(crit)
            main.wait_event(joined)
            main.wait_event(crit_done)
        return b


class FrameUploader:
    """Host -> HBM frame upload overlapped with compute (the reference's per-image
    `torch.from_numpy(img).to(device)`, detect.py:79-83, made asynchronous): pinned host
    batches are copied on a dedicated copy stream into one of two device buffers per
    pipeline while the pipeline's stream still computes on the other; the pipeline's stream
    waits only for its own buffer's copy, and a buffer is not overwritten before the
    pipeline call that read it has finished (events, no host synchronisation).

        up = FrameUploader([pipe0, pipe1], streams)
        out = up.submit(k, host_frames)   # batch k runs on pipes[k % P] / streams[k % P]
    """

    def __init__(self, pipes, streams, device=None):
        self.pipes = list(pipes)
        self.streams = list(streams)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.copy = torch.cuda.Stream(device=self.device)
        self._bufs = {}  # (pipe j, slot, shape) -> device tensor
        self._free = {}  # (pipe j, slot) -> event recorded after the call that read it
        self._count = [0] * len(self.pipes)

    def submit(self, k: int, host: torch.Tensor) -> dict:
        j = k % len(self.pipes)
        slot = self._count[j] % 2
        self._count[j] += 1
        key = (j, slot, tuple(host.shape))
        dst = self._bufs.get(key)
        if dst is None:
            dst = self._bufs[key] = torch.empty(host.shape, dtype=host.dtype, device=self.device)
        ev_free = self._free.get((j, slot))
        with torch.cuda.stream(self.copy):
            if ev_free is not None:
                self.copy.wait_event(ev_free)
            dst.copy_(host, non_blocking=True)
            copied = torch.cuda.Event()
            copied.record(self.copy)
        s = self.streams[j]
        with torch.cuda.stream(s):  # the call's first (eager) run and its graph replays: on s
            s.wait_event(copied)
            out = self.pipes[j](dst)
            done = torch.cuda.Event()
            done.record(s)
        self._free[(j, slot)] = done
        return out
