"""CPU: the oracle (CPU restatement of the reference path) against the golden
vectors the reference itself produced (tests/golden/make_golden.py), and the
preprocess restatement against Pillow."""
import json
import os

import numpy as np
import torch

from conftest import GOLDEN, cfg_text

MODELS = ["squeeze-ernet", "squeeze-redconv", "ernet"]


def test_classifier_oracle_matches_reference_goldens(cls_golden, cls_weights):
    from oracle import classifier as OC
    from oracle import preprocess as P
    for name in MODELS:
        crops = cls_golden[f"{name}/crops"]
        x = torch.from_numpy(np.stack([P.to_tensor_normalize(c) for c in crops]))
        logits, probs, blocks = OC.forward(name, cls_weights[name], x)
        ref = cls_golden[f"{name}/logits"]
        assert np.allclose(logits.numpy(), ref, rtol=1e-5, atol=1e-5 * np.abs(ref).max()), name
        assert np.array_equal(logits.argmax(1).numpy(), cls_golden[f"{name}/argmax"])
        assert np.allclose(probs.numpy(), cls_golden[f"{name}/probs"], atol=1e-6)
        g = torch.Generator().manual_seed(1234)
        s = 240 if name == "ernet" else 140
        xr = torch.randn(3, 3, s, s, generator=g)
        lr, _, _ = OC.forward(name, cls_weights[name], xr)
        rr = cls_golden[f"{name}/rand_logits"]
        assert np.allclose(lr.numpy(), rr, rtol=1e-5, atol=1e-5 * np.abs(rr).max()), name


def test_model_summary_shapes(cls_weights):
    """model_summary/*.txt known answers: parameter totals."""
    from rtdm.synth import classifier_param_shapes
    with open(os.path.join(GOLDEN, "shapes.json")) as f:
        shapes = json.load(f)
    for name in MODELS:
        n_model = sum(int(np.prod(s)) for k, s in classifier_param_shapes(name).items()
                      if not k.endswith("running_mean") and not k.endswith("running_var"))
        assert n_model == shapes[name]["params"], name
        assert set(cls_weights[name]) == set(classifier_param_shapes(name))
        for k, s in classifier_param_shapes(name).items():
            assert tuple(cls_weights[name][k].shape) == tuple(s)


def test_darknet_oracle_matches_reference_goldens(det_golden):
    from oracle.darknet import DarknetRef
    from rtdm.synth import BASE_SEED, load_calibration, synth_darknet_weights, synth_frames
    import hashlib
    from rtdm.synth import synth_acff_params
    for case in ("yolov4-tiny-aider-416@256", "yolov4-tiny-aider-416@608", "yolov3-tiny-aider-416@416",
                 "yolov4-tiny-swish@416", "yolov4-tiny-3l-512x512@512", "yolov3-acffx@416"):
        cfg, size = case.split("@")
        size = int(size)
        text = cfg_text(cfg)
        stream = synth_darknet_weights(text, calib=load_calibration(cfg))
        assert hashlib.sha256(stream.tobytes()).hexdigest() == str(det_golden[f"{case}/stream_sha"])
        n = int(det_golden[f"{case}/io_shape"][0])
        frames = synth_frames(n, size, size, seed=BASE_SEED + 700)
        assert hashlib.sha256(frames.tobytes()).hexdigest() == str(det_golden[f"{case}/frames_sha"])
        acff = synth_acff_params(text, calib=load_calibration(cfg))  # YOLO-ACFF blocks, if any
        io = DarknetRef(text, stream, acff).forward(
            torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).numpy()
        assert np.array_equal(io[:, ::53], det_golden[f"{case}/io_rows"]), case
        if f"{case}/io" in det_golden:
            assert np.array_equal(io, det_golden[f"{case}/io"])


def test_darknet_oracle_matches_reference_goldens_cond():
    """The well-conditioned weight set (rtdm.synth COND, the set SURVEY §8d's fp16 / int8 bars
    are asserted on): the oracle io and NMS survivors against the reference Darknet's on the
    same weights (det_golden_cond.npz, all 8 cases, 2 frames each)."""
    import hashlib
    from conftest import load_npz
    from oracle import nms as ON
    from oracle.darknet import DarknetRef
    from rtdm.synth import BASE_SEED, load_calibration, synth_acff_params, synth_darknet_weights, synth_frames
    g = load_npz("det_golden_cond.npz")
    cases = sorted({k.split("/")[0] for k in g})
    assert len(cases) == 8, cases
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for case in cases:
        cfg, size = case.split("@")
        size = int(size)
        text = cfg_text(cfg)
        cal = load_calibration(cfg, "cond")
        stream = synth_darknet_weights(text, calib=cal, preset="cond")
        assert hashlib.sha256(stream.tobytes()).hexdigest() == str(g[f"{case}/stream_sha"]), case
        n = int(g[f"{case}/io_shape"][0])
        frames = synth_frames(n, size, size, seed=BASE_SEED + 700)
        io = DarknetRef(text, stream, synth_acff_params(text, calib=cal, preset="cond")).forward(
            torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).numpy()
        assert np.array_equal(io[:, ::53], g[f"{case}/io_rows"]), case
        if f"{case}/io" in g:
            assert np.array_equal(io, g[f"{case}/io"])
        out = ON.non_max_suppression(io, 0.3, 0.4)
        for b in range(n):
            ref = g[f"{case}/nms0.3_0.4/{b}"]
            got = np.zeros((0, 6), np.float32) if out[b] is None else out[b]
            assert np.array_equal(got, ref), (case, b)


def test_nms_oracle_matches_reference_goldens(det_golden):
    """The reference non_max_suppression wrapper (filters, multi-label expansion,
    class offsets, output rows) with the oracle torchvision kernel stubbed in."""
    from oracle import nms as ON
    key = "yolov4-tiny-aider-416@256"
    io = det_golden[f"{key}/io"]
    for conf, iou in ((0.3, 0.4), (0.01, 0.6)):
        out, idx = ON.non_max_suppression(io, conf, iou, return_index=True)
        for b in range(io.shape[0]):
            ref = det_golden[f"{key}/nms{conf}_{iou}/{b}"]
            got = np.zeros((0, 6), np.float32) if out[b] is None else out[b]
            assert np.array_equal(got, ref), (conf, b)
            assert np.array_equal(np.zeros((0, 2)) if idx[b] is None else idx[b],
                                  det_golden[f"{key}/nms{conf}_{iou}/{b}/idx"])
    for case in ("yolov4-tiny-aider-416@608", "yolov3-tiny-aider-416@416"):
        pass  # full-size io is not stored; covered by the GPU tests


def test_nms_kernel_properties():
    from oracle import nms as ON
    rng = np.random.default_rng(0)
    boxes = rng.uniform(0, 100, (200, 2)).astype(np.float32)
    boxes = np.concatenate([boxes, boxes + rng.uniform(1, 30, (200, 2)).astype(np.float32)], 1)
    scores = rng.uniform(0, 1, 200).astype(np.float32)
    keep = ON.nms_kernel(boxes, scores, 0.5)
    assert np.all(np.diff(scores[keep]) <= 0)  # descending
    keep_all = ON.nms_kernel(boxes, scores, 1.0)  # IoU > 1 never: everything kept
    assert len(keep_all) == 200
    assert len(ON.nms_kernel(boxes[:0], scores[:0], 0.5)) == 0
    # idempotence: NMS of the survivors keeps them all
    k2 = ON.nms_kernel(boxes[keep], scores[keep], 0.5)
    assert len(k2) == len(keep)


def test_preprocess_restatement_matches_pillow(cls_golden):
    from oracle import preprocess as P
    from rtdm.synth import synth_frames
    imgs = list(synth_frames(2, 608, 608, seed=5)) + list(synth_frames(1, 300, 451, seed=7)) + [cls_golden["src0"]]
    for img in imgs:
        for s in (140, 240):
            size = int(s * 1.14)
            if min(img.shape[:2]) < size:
                continue
            assert np.array_equal(P.resize_shorter(img, size), P.pil_resize_shorter(img, size))
    # the stored crops are exactly resize + crop of the stored sources? (real images not stored whole)
    c = cls_golden["squeeze-ernet/crops"]
    assert c.dtype == np.uint8 and c.shape[1:] == (140, 140, 3)


def test_trt_decode_oracle_pinned_by_reference_io(det_golden):
    """CalDetection restatement vs the reference YOLOLayer golden io through the
    identities that hold at scale_x_y = 1: det_conf = io[4], class_conf = max io[5:]
    (first maximum), w = io[2] / W, x = io[0] / W - w / 2 (yolo_layer.cu:203-249 vs
    models.py:252-258)."""
    from oracle.darknet import DarknetRef
    from oracle import trt_yolo as OT
    from rtdm.synth import load_calibration, synth_darknet_weights
    case = "yolov4-tiny-aider-416@256"
    text = cfg_text("yolov4-tiny-aider-416")
    ref = DarknetRef(text, synth_darknet_weights(text, calib=load_calibration("yolov4-tiny-aider-416")))
    frames = det_golden[f"{case}/frames"]
    raw = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0, raw=True).numpy()
    io = det_golden[f"{case}/io"]
    assert raw.shape == io.shape
    det = OT.cal_detection_rows(raw, ref.heads, 256, 256)
    W = 256.0
    assert np.allclose(det[..., 4], io[..., 4], rtol=2e-6, atol=1e-7)
    assert np.allclose(det[..., 6], io[..., 5:].max(-1), rtol=2e-6, atol=1e-7)
    amb = np.sort(io[..., 5:], -1)
    clear = amb[..., -1] - amb[..., -2] > 1e-6
    assert np.array_equal(det[..., 5][clear], io[..., 5:].argmax(-1)[clear].astype(np.float32))
    assert np.allclose(det[..., 2], io[..., 2] / W, rtol=1e-5, atol=1e-7)
    assert np.allclose(det[..., 3], io[..., 3] / W, rtol=1e-5, atol=1e-7)
    assert np.allclose(det[..., 0], io[..., 0] / W - det[..., 2] / 2, rtol=1e-5, atol=2e-6)
    assert np.allclose(det[..., 1], io[..., 1] / W - det[..., 3] / 2, rtol=1e-5, atol=2e-6)


def test_trt_postprocess_product_matches_oracle():
    """Host post-processing of rtdm.trt_yolo (vectorised) vs the loop restatement of
    _postprocess_yolo / _nms_boxes on seeded Detection records (no score ties)."""
    from oracle import trt_yolo as OT
    from rtdm.trt_yolo import postprocess_yolo
    rng = np.random.default_rng(11)
    for letter_box, (ih, iw) in ((False, (416, 416)), (True, (300, 500)), (True, (500, 300))):
        n = 600
        d = np.zeros((n, 7), np.float32)
        d[:, 0:2] = rng.uniform(-0.05, 0.95, (n, 2))
        d[:, 2:4] = rng.uniform(0.01, 0.3, (n, 2))
        d[:, 4] = rng.uniform(0, 1, n)
        d[:, 5] = rng.integers(0, 3, n)
        d[:, 6] = rng.uniform(0.2, 1, n)
        s = d[:, 4] * d[:, 6]
        assert len(np.unique(s)) == n
        outs = [d[:250], d[250:]]
        got = postprocess_yolo(outs, iw, ih, 0.3, 0.5, (416, 416), letter_box)
        exp = OT.postprocess_yolo(outs, iw, ih, 0.3, 0.5, (416, 416), letter_box)
        assert len(got[0]) == len(exp[0]) > 10
        for g, e in zip(got, exp):
            assert np.array_equal(g, e)
    empty = postprocess_yolo([np.zeros((5, 7), np.float32)], 416, 416, 0.3, 0.5, (416, 416))
    assert empty[0].shape == (0, 4)


def test_survivor_band_rule():
    """oracle.nms.survivors_equal_outside_band (SURVEY §8d's end-to-end fp16 rule): equal io
    -> no difference; a candidate moved across the conf threshold by < the band is excused,
    by more is not; a swap of two overlapping candidates' scores by < the band is excused
    (and what it suppresses follows), a swap by more is not."""
    from oracle import nms as ON
    io = np.zeros((1, 6, 7), np.float32)
    # two overlapping boxes (IoU 0.81), one far box, one box near conf 0.3, two others off
    io[0, :, 0:4] = [[100, 100, 40, 40], [102, 102, 40, 40], [300, 300, 30, 30], [200, 50, 20, 20],
                     [50, 300, 20, 20], [400, 400, 20, 20]]
    io[0, :, 4] = [0.9, 0.85, 0.8, 0.3004, 0.1, 0.1]
    io[0, :, 5] = [1.0, 1.0, 1.0, 1.0, 1.0, 1.0]
    io[0, :, 6] = 0.0
    n_ref, n_got, n_exc, bad = ON.survivors_equal_outside_band(io, io.copy(), 0.3, 0.4)
    assert (n_ref, n_got, n_exc, bad) == (3, 3, 0, [])
    near = io.copy()
    near[0, 3, 4] = 0.2996  # crosses 0.3 by 4e-4 (inside 1e-3): excused
    n_ref, n_got, n_exc, bad = ON.survivors_equal_outside_band(io, near, 0.3, 0.4)
    assert n_ref == 3 and n_got == 2 and n_exc == 1 and bad == []
    far = io.copy()
    far[0, 2, 4] = 0.29  # a clear survivor dropped: not excused
    assert ON.survivors_equal_outside_band(io, far, 0.3, 0.4)[3] == [(0, 2, 0)]
    tie = io.copy()
    tie[0, 0, 4], tie[0, 1, 4] = 0.8500, 0.8504  # overlapping pair, scores within 1e-3 in ref
    swapped = tie.copy()
    swapped[0, 0, 4], swapped[0, 1, 4] = 0.8504, 0.8500
    assert ON.survivors_equal_outside_band(tie, swapped, 0.3, 0.4)[3] == []
    wide = io.copy()
    wide[0, 0, 4], wide[0, 1, 4] = 0.85, 0.9  # the same swap by 5e-2: not excused
    assert len(ON.survivors_equal_outside_band(io, wide, 0.3, 0.4)[3]) == 2
