"""int8 quantisation models of the RTDM_I8 paths (TEST INFRASTRUCTURE ONLY).

Classifier (cls_calibrate / cls_int8_hook, on oracle.classifier.forward's fusion hook):
the ACFF 1x1 fusion GEMM of the blocks the C++ planner marks int8 (classifier.cpp;
rtdm_classifier_describe lists them) takes the depthwise concat quantised per concat
channel, s_k = |x|max_k / 127 over the calibration frames, and the fusion weights times
s_k quantised symmetric per output channel — the detector scheme below on the concat.

Detector:

The reference has no numeric int8 path (opaque TensorRT engines and
entropy-calibration caches, tensorrt_inference/yolo/calibrator.py:87-153), so the int8
check compares the HIP int8 io with the fp32 oracle relative to this model of the same
scheme on the oracle (conv_hook of oracle.darknet.DarknetRef in f16_storage mode):
  * quantised convs: 3x3 [convolutional] layers with cin % 128 == 0 and cout % 128 == 0,
    except a conv whose output only a YOLO head conv reads (the int8-eligible convs of the
    C++ planner, detector.cpp);
  * calibration: per input channel |x|max over the calibration frames' fp16-storage
    forward; s_c = HEADROOM * |x|max_c / 127 (HEADROOM 2: frames beyond the calibration
    set's extremes round instead of clamping);
  * weights: BN-folded fp16 weights times s_c, symmetric int8 per output channel
    (s_w[o] = max|W'[o]| / 127); activations q = clamp(rint(x / s_c), -127, 127).
"""
from __future__ import annotations

import torch


def _consumers(mdefs, i):
    """Layers reading layer i's output (models.py:332-395: the next layer unless it is a
    route, plus routes / shortcuts naming i)."""
    out = []
    if i + 1 < len(mdefs) and mdefs[i + 1]["type"] != "route":
        out.append(i + 1)
    for j in range(i + 1, len(mdefs)):
        t = mdefs[j]["type"]
        refs = mdefs[j].get("layers", []) if t == "route" else mdefs[j].get("from", []) if t == "shortcut" else []
        if any((j + l if l < 0 else l) == i for l in refs) and j not in out:
            out.append(j)
    return out


def pre_head(mdefs, i):
    """Layer i's output is read only by a YOLO head conv (the conv right before [yolo])."""
    c = _consumers(mdefs, i)
    return (len(c) == 1 and mdefs[c[0]]["type"] == "convolutional" and c[0] + 1 < len(mdefs)
            and mdefs[c[0] + 1]["type"] == "yolo")


def eligible(mdefs, i, cin, out_stride):
    """out_stride: the conv's output grid stride in image pixels (tools/int8_scope.py
    experiments with the pre-head rule by stride)."""
    m = mdefs[i]
    return (m["type"] == "convolutional" and cin % 128 == 0 and int(m["filters"]) % 128 == 0
            and int(m["size"]) == 3 and not pre_head(mdefs, i))


def calibrate(ref, x):
    """Per-channel |x|max of every eligible conv input on frames x ([N,3,H,W] in [0,1])."""
    amax = {}
    img_h = x.shape[2]

    def hook(i, xi, w, b):
        out_h = (xi.shape[2] - 1) // int(ref.mdefs[i].get("stride", 1)) + 1
        if eligible(ref.mdefs, i, xi.shape[1], img_h // out_h):
            m = xi.abs().amax(dim=(0, 2, 3))
            amax[i] = torch.maximum(amax[i], m) if i in amax else m
        return xi, w, b

    ref.forward(x, f16_storage=True, conv_hook=hook)
    return amax


HEADROOM = 2.0  # detector.cpp kI8Headroom


def int8_hook(amax, headroom=HEADROOM):
    """conv_hook applying the RTDM_I8 quantisation to the calibrated layers (activation
    scales s_c = headroom * |x|max_c / 127)."""
    def hook(i, x, w, b):
        if i not in amax:
            return x, w, b
        a = amax[i] * headroom
        s = torch.where(a > 0, a / 127.0, torch.ones_like(a)).view(1, -1, 1, 1)
        xq = torch.round(x / s).clamp(-127, 127)
        wp = w * s.view(1, -1, 1, 1)  # fold the activation scales into the input channels
        sw = wp.abs().flatten(1).amax(1).clamp_min(1e-30) / 127.0
        wq = torch.round(wp / sw.view(-1, 1, 1, 1)).clamp(-127, 127)
        return xq, wq * sw.view(-1, 1, 1, 1), b
    return hook


def cls_calibrate(kind, sd, x, blocks):
    """Per-concat-channel |x|max of the int8 blocks' fusion inputs on inputs x ([N,3,S,S])."""
    from oracle import classifier as OC
    amax = {}

    def hook(p, cat, w, b):
        if p in blocks:
            m = cat.abs().amax(dim=(0, 2, 3))
            amax[p] = torch.maximum(amax[p], m) if p in amax else m
        return cat, w, b

    OC.forward(kind, sd, x, hook)
    return amax


def cls_int8_hook(amax):
    """oracle.classifier fusion hook applying the classifier RTDM_I8 quantisation (no
    headroom: classifier.cpp scales by |x|max / 127)."""
    inner = int8_hook(amax, 1.0)

    def hook(p, cat, w, b):
        return inner(p, cat, w, b)
    return hook
