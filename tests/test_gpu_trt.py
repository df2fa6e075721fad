"""GPU parity of the TensorRT-YOLO output path:
rtdm_yolo_layer_trt (the YoloLayer_TRT plugin enqueue), rtdm_detect_raw,
rtdm_detect_trt and TrtYOLO.detect, against the oracle restatement
(oracle/trt_yolo.py, pinned to the reference YOLOLayer io in
tests/test_oracle_golden.py).  Tolerances: Detection x/y/w/h (normalised to the
input) <= 2e-6 + 2e-5 relative and confidences <= 1e-6 on identical raw inputs
(the plugin uses __expf; both sides here use an IEEE expf, so only rounding order
differs); class id exact where the top-2 class logits differ by > 1e-6.  Through
the full fp32 detector the raw head rows carry the conv accumulation-order error
(<= 1e-4 absolute at these depths), so those comparisons use 1e-4.
"""
import ctypes
import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import cfg_text

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _cmp_det(got, exp, raw, tol_box=(2e-6, 2e-5), tol_p=1e-6, gap=1e-6):
    assert got.shape == exp.shape
    a, r = tol_box
    # x, y are top-left corners (centre - size/2): their error scale includes w, h
    scale = np.abs(exp[..., :4]) + np.concatenate([np.abs(exp[..., 2:4])] * 2, -1)
    assert np.all(np.abs(got[..., :4] - exp[..., :4]) <= a + r * scale), \
        np.abs(got[..., :4] - exp[..., :4]).max()
    assert np.all(np.abs(got[..., [4, 6]] - exp[..., [4, 6]]) <= tol_p)
    cls = np.sort(raw[..., 5:], -1)
    clear = (cls[..., -1] - cls[..., -2]) > gap if cls.shape[-1] > 1 else np.ones(cls.shape[:-1], bool)
    assert np.array_equal(got[..., 5][clear], exp[..., 5][clear])


@pytest.mark.parametrize("na,nc,ny,nx,mult,sxy,newc", [(3, 2, 19, 19, 32, 1.0, 0), (3, 2, 38, 38, 16, 1.05, 0),
                                                      (4, 80, 13, 20, 32, 1.2, 0), (3, 2, 52, 52, 8, 2.0, 1),
                                                      (6, 1, 7, 9, 16, 1.0, 0)])
def test_yolo_layer_trt_plugin_vs_oracle(dev, na, nc, ny, nx, mult, sxy, newc):
    from oracle import trt_yolo as OT
    from rtdm import _lib as L
    g = torch.Generator().manual_seed(na * 1000 + ny)
    b = 3
    p = torch.randn(b, na * (5 + nc), ny, nx, generator=g) * 3
    if newc:
        p = torch.sigmoid(p)  # scaled-YOLOv4 heads emit logistic outputs
    anchors = (torch.rand(na * 2, generator=g) * 200 + 5).numpy().astype(np.float32)
    out = torch.empty(b, na * ny * nx, 7, device=dev)
    L.check(L.lib().rtdm_yolo_layer_trt(L.ptr(p.to(dev)), b, nx, ny, na,
                                        anchors.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), nc, mult, sxy, newc,
                                        L.ptr(out), L.stream_ptr()))
    torch.cuda.synchronize()
    rows = OT.nchw_to_rows(p.numpy(), na)
    heads = [{"na": na, "ny": ny, "nx": nx, "anchors": anchors.reshape(-1, 2).tolist(), "scale_x_y": sxy,
              "new_coords": newc}]
    exp = OT.cal_detection_rows(rows, heads, nx * mult, ny * mult)
    _cmp_det(out.cpu().numpy(), exp, rows)


def test_yolo_layer_trt_asserts_become_status(dev):
    from rtdm import _lib as L
    lib = L.lib()
    a = np.ones(14, np.float32)
    ap = a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    x = torch.zeros(1, 21, 4, 4, device=dev)
    o = torch.zeros(1, 48, 7, device=dev)
    assert lib.rtdm_yolo_layer_trt(L.ptr(x), 1, 4, 4, 7, ap, 2, 32, 1.0, 0, L.ptr(o), None) == 1  # > MAX_ANCHORS
    assert lib.rtdm_yolo_layer_trt(L.ptr(x), 1, 4, 4, 3, ap, 2, 12, 1.0, 0, L.ptr(o), None) == 1  # multiplier
    assert lib.rtdm_yolo_layer_trt(L.ptr(x), 1, 4, 4, 3, ap, 2, 32, 0.5, 0, L.ptr(o), None) == 1  # scale_x_y < 1
    assert lib.rtdm_yolo_layer_trt(L.ptr(x), 1, 4, 4, 3, ap, 0, 32, 1.0, 0, L.ptr(o), None) == 1  # classes
    a[0] = 0
    assert lib.rtdm_yolo_layer_trt(L.ptr(x), 1, 4, 4, 3, ap, 2, 32, 1.0, 0, L.ptr(o), None) == 1  # anchors


def _net(cfg, size, half):
    from rtdm.darknet import Darknet
    from rtdm.synth import load_calibration, synth_darknet_weights
    text = cfg_text(cfg)
    stream = synth_darknet_weights(text, calib=load_calibration(cfg))
    m = Darknet(text, (size, size))
    m.load_weight_stream(stream)
    if half:
        m.half()
    return m, text, stream


@pytest.mark.parametrize("cfg,size", [("yolov4-tiny-aider-416", 256), ("yolov3-tiny-aider-416", 416),
                                      ("yolov4-tiny-aider-416", 608)])
def test_detect_raw_and_trt_vs_oracle(dev, det_golden, cfg, size):
    from oracle.darknet import DarknetRef
    from oracle import trt_yolo as OT
    from rtdm.synth import BASE_SEED, synth_frames
    m, text, stream = _net(cfg, size, False)
    frames = synth_frames(2, size, size, seed=BASE_SEED + 700)
    x = torch.from_numpy(frames).to(dev)
    ref = DarknetRef(text, stream)
    raw_ref = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0, raw=True).numpy()
    raw = m.forward_raw(x).cpu().numpy()
    assert raw.shape == raw_ref.shape
    assert np.abs(raw - raw_ref).max() <= 1e-4 * max(1.0, np.abs(raw_ref).max())
    # decoded io and raw rows come from the same launch plan: the io is still right afterwards
    io, _ = m(x)
    io_ref = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).numpy()
    assert np.abs(io.cpu().numpy()[..., 4:] - io_ref[..., 4:]).max() <= 1e-5
    det = m.forward_trt(x).cpu().numpy()
    # identical raw input: the decode itself is exact to rounding
    _cmp_det(det, OT.cal_detection_rows(raw, ref.heads, size, size), raw)
    # against the all-oracle chain: raw rows differ by the conv accumulation order
    exp = OT.cal_detection_rows(raw_ref, ref.heads, size, size)
    # (class ids compared where the top-2 gap exceeds twice the observed raw difference)
    _cmp_det(det, exp, raw_ref, tol_box=(2e-6, 2e-4), tol_p=2e-5, gap=2 * float(np.abs(raw - raw_ref).max()) + 1e-6)


def test_detect_trt_fp16(dev):
    from oracle.darknet import DarknetRef
    from oracle import trt_yolo as OT
    from rtdm.synth import BASE_SEED, synth_frames
    m, text, stream = _net("yolov4-tiny-aider-416", 608, True)
    frames = synth_frames(4, 608, 608, seed=BASE_SEED + 3)
    det = m.forward_trt(torch.from_numpy(frames).to(dev)).cpu().numpy()
    ref = DarknetRef(text, stream)
    exp = OT.cal_detection_rows(ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0,
                                            raw=True).numpy(), ref.heads, 608, 608)
    # fp16 tolerance: 0.5 px of 608 on x/y, 3e-2 relative on w/h, 2e-2 on probabilities
    # (x, y are top-left corners: centre error + half the w/h error)
    wh_tol = 0.5 / 608 + 3e-2 * np.abs(exp[..., 2:4])
    assert np.all(np.abs(det[..., 2:4] - exp[..., 2:4]) <= wh_tol)
    assert np.all(np.abs(det[..., :2] - exp[..., :2]) <= 0.5 / 608 + 0.5 * wh_tol)
    assert np.abs(det[..., [4, 6]] - exp[..., [4, 6]]).max() <= 2e-2


def test_trt_yolo_detect_end_to_end(dev):
    from oracle import trt_yolo as OT
    from rtdm.synth import BASE_SEED, synth_frames, write_darknet_weights
    from rtdm.trt_yolo import TrtYOLO
    _, text, stream = _net("yolov4-tiny-aider-416", 416, False)
    with tempfile.TemporaryDirectory() as d:
        w = os.path.join(d, "yolov4-tiny-416.weights")
        write_darknet_weights(w, stream)
        trt = TrtYOLO("yolov4-tiny-416", category_num=2, weights=w, half=False)
        with pytest.raises(SystemExit):
            TrtYOLO("yolov9-416", category_num=2, weights=w)
        with pytest.raises(FileNotFoundError):
            TrtYOLO("yolov4-tiny-416", category_num=2, weights=os.path.join(d, "missing.weights"))
    rgb = synth_frames(1, 416, 416, seed=BASE_SEED + 9)[0]
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    boxes, scores, classes = trt.detect(bgr, conf_th=0.3)
    dets = trt.infer(torch.from_numpy(rgb).to(dev)[None])[0].cpu().numpy()
    eb, es, ec = OT.postprocess_yolo([dets], 416, 416, 0.3, 0.5, (416, 416))
    eb[:, [0, 2]] = np.clip(eb[:, [0, 2]], 0, 415)
    eb[:, [1, 3]] = np.clip(eb[:, [1, 3]], 0, 415)
    assert len(boxes) > 0
    assert np.array_equal(boxes, eb) and np.array_equal(scores, es) and np.array_equal(classes, ec)
    with pytest.raises(ValueError):
        trt.detect(bgr[:200])
