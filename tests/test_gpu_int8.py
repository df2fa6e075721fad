"""GPU: the int8-quantised detector (RTDM_I8, BASELINE config 5) against fp16 and the
fp32 oracle.  The reference has no numeric int8 oracle (its int8 artefacts are opaque
TensorRT engines / calibration caches); SURVEY §8d's task-level bar is a
detection match >= 97 % (oracle survivor at conf 0.3 / IoU 0.4 matched by an int8
survivor of the same class with IoU >= 0.9).  This round's int8 path does not reach it
on the synthetic-weight detectors (measured below); the tests pin the kernel's error at
its first int8 layer and the measured end-to-end level.  Calibration frames are
disjoint from the evaluation frames.
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import cfg_text

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _iou(a, b):
    x1 = np.maximum(a[0], b[:, 0])
    y1 = np.maximum(a[1], b[:, 1])
    x2 = np.minimum(a[2], b[:, 2])
    y2 = np.minimum(a[3], b[:, 3])
    inter = np.clip(x2 - x1, 0, None) * np.clip(y2 - y1, 0, None)
    return inter / ((a[2] - a[0]) * (a[3] - a[1]) + (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]) - inter)


@pytest.mark.parametrize("case,nframes", [("yolov4-tiny-aider-416@608", 3)])
def test_int8_detector_vs_fp32_oracle(dev, case, nframes):
    """Measured, not the §8d bar: per-tensor int8 (MSE-clipped calibration) on these
    synthetic-weight nets compounds ~3-4 % relative error per int8 layer; the first int8
    layer (L6) must stay within 6 % mean relative error of fp16, objectness within 0.15,
    and at least a third of the oracle's survivors must be matched (measured 39 %,
    DESIGN.md §5: below the 97 % bar, so RTDM_I8 stays opt-in)."""
    from oracle import nms as ON
    from oracle.darknet import DarknetRef
    from rtdm.darknet import Darknet
    from rtdm.nms import non_max_suppression
    from rtdm.synth import BASE_SEED, load_calibration, synth_darknet_weights, synth_frames
    cfg, size = case.split("@")
    size = int(size)
    text = cfg_text(cfg)
    stream = synth_darknet_weights(text, calib=load_calibration(cfg))
    m = Darknet(text, (size, size))
    m.load_weight_stream(stream)
    calib = torch.from_numpy(synth_frames(8, size, size, seed=BASE_SEED + 4321)).to(dev)
    m.int8(calib)
    frames = synth_frames(nframes, size, size, seed=BASE_SEED + 700)
    x = torch.from_numpy(frames).to(dev)
    io, _ = m(x)
    assert " dtype i8 " in m.describe()
    l6_i8 = m.layer_output(6, nframes)
    f = Darknet(text, (size, size))
    f.load_weight_stream(stream)
    f.half()
    f(x)
    l6 = f.layer_output(6, nframes)
    assert float((l6 - l6_i8).abs().mean() / l6.abs().mean()) <= 0.06
    got = non_max_suppression(io, 0.3, 0.4)
    ref_io = DarknetRef(text, stream).forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).numpy()
    ref = ON.non_max_suppression(ref_io, 0.3, 0.4)
    matched = total = 0
    for b in range(nframes):
        r = np.zeros((0, 6), np.float32) if ref[b] is None else ref[b]
        g = np.zeros((0, 6), np.float32) if got[b] is None else got[b].cpu().numpy()
        r = r[r[:, 4] > 0.32]
        total += len(r)
        for row in r:
            same = g[g[:, 5] == row[5]]
            if len(same) and _iou(row[:4], same[:, :4]).max() >= 0.9:
                matched += 1
    assert total > 20, total
    print(f"int8 detection match {matched}/{total}")
    assert matched / total >= 0.33, (case, matched, total)
    assert np.abs(io.cpu().numpy()[..., 4] - ref_io[..., 4]).max() <= 0.15


def test_int8_requires_calibration(dev):
    from rtdm import _lib as L
    from rtdm.synth import load_calibration, synth_darknet_weights
    text = cfg_text("yolov4-tiny-aider-416")
    stream = synth_darknet_weights(text, calib=load_calibration("yolov4-tiny-aider-416"))
    h = ctypes.c_void_p()
    L.check(L.lib().rtdm_detector_create(text.encode(), 256, 256, L.RTDM_I8,
                                         stream.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), stream.size, 2,
                                         ctypes.byref(h)))
    try:
        x = torch.zeros((2, 256, 256, 3), dtype=torch.uint8, device=dev)
        info = L.rtdm_detector_info()
        L.check(L.lib().rtdm_detector_get_info(h, ctypes.byref(info)))
        io = torch.empty((2, info.n_anchors_total, info.no), device=dev)
        st = L.lib().rtdm_detect(h, L.ptr(x), L.RTDM_INPUT_FRAME_U8, 2, L.ptr(io), L.stream_ptr())
        assert st == 1 and b"calibrated" in L.lib().rtdm_last_error()
        L.check(L.lib().rtdm_detector_calibrate(h, L.ptr(x), L.RTDM_INPUT_FRAME_U8, 2, 1, L.stream_ptr()))
        L.check(L.lib().rtdm_detect(h, L.ptr(x), L.RTDM_INPUT_FRAME_U8, 2, L.ptr(io), L.stream_ptr()))
        torch.cuda.synchronize()
        assert bool(torch.isfinite(io).all())
    finally:
        L.lib().rtdm_detector_destroy(h)
