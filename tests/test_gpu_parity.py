"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Tolerances:
  fp32  class id exact; logits <= 1e-4 * max|logit| per row; NMS survivors exact
        when fed the same io.  io of the shallow tiny nets (16-21 convs): x,y <=
        1e-3 px, w,h <= 1e-3 px + 1e-4 relative (exp() of the head logit amplifies
        the ~1e-5 relative accumulation-order difference), probabilities <= 1e-5;
        the deep residual nets (75-76 convs): w,h 1e-3 relative, probabilities 1e-4.
  fp16  class id exact where the top-2 logit gap >= 0.5; logits <= 2e-2*max|logit|.
        io, tiny nets: x,y <= 0.5 px, w,h <= 0.5 px + 3e-2 relative, probabilities
        <= 2e-2; deep nets: x,y <= 2 px, w,h 0.2 relative, probabilities 5e-2.  These
        are set from measurement, not widened to pass: the oracle's fp16-storage model
        (every activation and weight rounded to fp16, fp32 arithmetic) deviates from the
        fp32 oracle by xy 0.11 px / wh 1.8 % / p 5.3e-3 on v4-tiny@608 and by xy 1.2-1.4 px
        / wh 14-17 % / p 3-4e-2 on the deep nets, and the HIP fp16 io stays below that
        model's deviation (test_gpu_pipeline.py::test_fp16_io_within_storage_floor checks
        every io row against it); SURVEY §8d's 0.5 px box bar is below the fp16-storage
        floor once exp() decodes w,h.
  Detections (every golden case): the reference's NMS survivors at conf 0.3 /
        IoU 0.4 are matched (same class, IoU >= 0.9) at >= 99% (fp32) / >= 90% (fp16;
        deep nets: within 5 points of the fp16-storage model's own match rate),
        candidates within 1e-2 of the conf threshold excluded.
"""
import numpy as np
import pytest
import torch

from conftest import cfg_text

pytestmark = pytest.mark.gpu

MODELS = ["squeeze-ernet", "squeeze-redconv", "ernet"]
SIZE = {"squeeze-ernet": 140, "squeeze-redconv": 140, "ernet": 240}


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _model(name, sd, half=False):
    from rtdm.classifier import build_model
    m = build_model(name)
    m.load_state_dict(sd)
    if half:
        m.half()
    return m


# ------------------------------------------------------------- preprocess --
def test_preprocess_bit_exact_vs_pillow(dev, cls_golden):
    from oracle import preprocess as P
    from rtdm.preprocess import preprocess_frames
    from rtdm.synth import synth_frames
    frames = [synth_frames(3, 608, 608, seed=5), synth_frames(2, 224, 224, seed=6), synth_frames(2, 300, 451, seed=7),
              cls_golden["src0"][None]]
    for f in frames:
        for s in (140, 240):
            if min(f.shape[1:3]) < int(s * 1.14):
                continue
            got = preprocess_frames(torch.from_numpy(f).to(dev), s).cpu().numpy()
            for i in range(f.shape[0]):
                rs = P.pil_resize_shorter(f[i], int(s * 1.14))
                want = P.to_tensor_normalize(P.center_crop(rs, s))
                assert np.array_equal(got[i], want), (f.shape, s, i, np.abs(got[i] - want).max())


# ------------------------------------------------------------- classifier --
@pytest.mark.parametrize("name", MODELS)
def test_classifier_fp32_golden(dev, name, cls_golden, cls_weights):
    from oracle import preprocess as P
    m = _model(name, cls_weights[name])
    crops = cls_golden[f"{name}/crops"]
    x = torch.from_numpy(np.stack([P.to_tensor_normalize(c) for c in crops])).to(dev)
    probs = m(x).cpu().numpy()
    logits = m.logits.cpu().numpy()
    ref = cls_golden[f"{name}/logits"]
    tol = 1e-4 * np.abs(ref).max(1, keepdims=True)
    assert np.all(np.abs(logits - ref) <= tol), np.abs(logits - ref).max()
    assert np.array_equal(logits.argmax(1), cls_golden[f"{name}/argmax"])
    assert np.allclose(probs, cls_golden[f"{name}/probs"], atol=1e-5)


@pytest.mark.parametrize("name", MODELS)
def test_classifier_fp32_random_inputs(dev, name, cls_golden, cls_weights):
    m = _model(name, cls_weights[name])
    s = SIZE[name]
    g = torch.Generator().manual_seed(1234)
    xr = torch.randn(3, 3, s, s, generator=g)
    m(xr.to(dev))
    logits = m.logits.cpu().numpy()
    ref = cls_golden[f"{name}/rand_logits"]
    tol = 1e-4 * np.abs(ref).max(1, keepdims=True)
    assert np.all(np.abs(logits - ref) <= tol), np.abs(logits - ref).max()


@pytest.mark.parametrize("name", MODELS)
def test_classifier_fp16(dev, name, cls_golden, cls_weights):
    from oracle import preprocess as P
    m = _model(name, cls_weights[name], half=True)
    crops = cls_golden[f"{name}/crops"]
    x = torch.from_numpy(np.stack([P.to_tensor_normalize(c) for c in crops])).to(dev)
    m(x)
    logits = m.logits.cpu().numpy()
    ref = cls_golden[f"{name}/logits"]
    gap = cls_golden[f"{name}/top2gap"]
    assert np.all(np.abs(logits - ref) <= 2e-2 * np.abs(ref).max(1, keepdims=True)), np.abs(logits - ref).max()
    sure = gap >= 0.5
    assert np.array_equal(logits.argmax(1)[sure], cls_golden[f"{name}/argmax"][sure])
    # fp16 input tensor (the reference's --trt --quant fp16 .half() path)
    m(x.half())
    assert np.all(np.abs(m.logits.cpu().numpy() - ref) <= 2e-2 * np.abs(ref).max(1, keepdims=True))


@pytest.mark.parametrize("name", MODELS)
@pytest.mark.parametrize("half", [False, True])
def test_classifier_frames_vs_oracle(dev, name, half, cls_weights):
    """uint8 frames -> fused transform + model, against oracle transform + oracle model."""
    from oracle import classifier as OC
    from oracle import preprocess as P
    from rtdm.synth import synth_frames
    m = _model(name, cls_weights[name], half=half)
    frames = synth_frames(5, 608, 608, seed=99)
    m.classify_frames(torch.from_numpy(frames).to(dev))
    logits = m.logits.cpu().numpy()
    s = SIZE[name]
    x = torch.from_numpy(np.stack([P.cli_transform(f, s) for f in frames]))
    ref, _, _ = OC.forward(name, cls_weights[name], x)
    ref = ref.numpy()
    tol = (2e-2 if half else 1e-4) * np.abs(ref).max(1, keepdims=True)
    assert np.all(np.abs(logits - ref) <= tol), np.abs(logits - ref).max()


@pytest.mark.parametrize("name", MODELS)
def test_classifier_acff_chain_matches_per_stage(dev, name, cls_weights):
    """The one-launch small-map ACFF suffix + tail (acff_chain) against the per-stage
    kernels + tail kernel: same class ids; logits within 1e-4 * max|logit| (measured
    <= 2.6e-5 relative: the two schedules differ in a few fp16 roundings of
    intermediate maps, far inside the fp16 bar of 2e-2)."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    frames = torch.from_numpy(synth_frames(37, 608, 608, seed=5)).to(dev)
    out = {}
    try:
        L.check(L.lib().rtdm_set_tuning(b"acff_band", 0))  # the chain, not the banded stages
        for mode in (0, 1):
            L.check(L.lib().rtdm_set_tuning(b"acff_chain", mode))
            m = _model(name, cls_weights[name], half=True)
            assert ("acff_chain" in m.describe(37)) == (mode == 1)
            probs = m.classify_frames(frames)
            out[mode] = (m.logits.clone(), probs.clone())
    finally:
        L.check(L.lib().rtdm_set_tuning(b"acff_chain", 1))
        L.check(L.lib().rtdm_set_tuning(b"acff_band", 0))
    a, b = out[0][0], out[1][0]
    scale = a.abs().max(1, keepdim=True).values
    assert bool(((a - b).abs() <= 1e-4 * scale).all()), ((a - b).abs() / scale).max()
    assert torch.equal(a.argmax(1), b.argmax(1))
    assert torch.allclose(out[0][1], out[1][1], atol=1e-4)


@pytest.mark.parametrize("name", MODELS)
def test_acff_band_bit_identical_to_chain(dev, name, cls_weights):
    """acff_band (opt-in: the small-map stages one launch each over output row bands, the
    tail fused into the last; ernet.py:25-45, acff.py:37-59) against acff_chain (one
    workgroup per image, the default).  On the chain's own stages (acff_band 2) the two run the same operations in the
    same order: logits and probabilities bit-identical, at b37 (ragged) and per frame.  With
    the banded pooled stage before them as well (acff_band 1: acff3 leaves
    acff_persist, whose 1x1 runs in another K order) the logits stay within 1e-3 of
    max|logit| (the fp16 bar is 2e-2) with the same class ids, and every frame's row is
    bit-identical to the frame run alone."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    frames = torch.from_numpy(synth_frames(37, 608, 608, seed=11)).to(dev)
    out = {}
    try:
        for band in (0, 2, 1):
            L.check(L.lib().rtdm_set_tuning(b"acff_band", band))
            m = _model(name, cls_weights[name], half=True)
            desc = m.describe(37)
            assert ("acff_band" in desc) == (band > 0), desc
            probs = m.classify_frames(frames)
            out[band] = (m.logits.clone(), probs.clone())
            if band == 1:
                for i in (0, 17, 36):
                    m.classify_frames(frames[i:i + 1].contiguous())
                    assert torch.equal(m.logits[0], out[1][0][i]), i
    finally:
        L.check(L.lib().rtdm_set_tuning(b"acff_band", 0))
    assert torch.equal(out[0][0], out[2][0]) and torch.equal(out[0][1], out[2][1])
    a, b = out[0][0], out[1][0]
    scale = a.abs().max(1, keepdim=True).values
    assert bool(((a - b).abs() <= 1e-3 * scale).all()), ((a - b).abs() / scale).max()
    assert torch.equal(a.argmax(1), b.argmax(1))


def test_redconv_config2_b32(dev, cls_weights):
    """BASELINE config 2 as bench.py --cfg none runs it: Squeeze-ErNET-RedConv fp16 on a
    batch of 32 224x224 uint8 sources through the device CLI transform (159 resize, 140
    crop, aider.py:412-431).  Against the oracle (transform + model): logits <= 2e-2 *
    max|logit|, class id exact where the top-2 gap >= 0.5; b1 rows bit-identical to the
    b32 rows (batch-invariant kernels); the classification-only pipeline under graph replay
    bit-identical to eager."""
    from oracle import classifier as OC
    from oracle import preprocess as P
    from rtdm.pipeline import TwoStagePipeline
    from rtdm.synth import BASE_SEED, synth_frames
    frames = synth_frames(32, 224, 224, seed=BASE_SEED + 224)
    x = torch.from_numpy(frames).to(dev)
    m = _model("squeeze-redconv", cls_weights["squeeze-redconv"], half=True)
    m.classify_frames(x)
    got = m.logits.cpu().numpy()
    ref = OC.forward("squeeze-redconv", cls_weights["squeeze-redconv"],
                     torch.from_numpy(np.stack([P.cli_transform(f, 140) for f in frames])))[0].numpy()
    assert np.all(np.abs(got - ref) <= 2e-2 * np.abs(ref).max(1, keepdims=True)), np.abs(got - ref).max()
    srt = np.sort(ref, 1)
    sure = srt[:, -1] - srt[:, -2] >= 0.5
    assert sure.sum() >= 8 and np.array_equal(got.argmax(1)[sure], ref.argmax(1)[sure])
    for i in (0, 13, 31):
        m.classify_frames(x[i:i + 1].contiguous())
        assert torch.equal(m.logits.cpu()[0], torch.from_numpy(got[i])), i
    pe = TwoStagePipeline(m, None)
    pg = TwoStagePipeline(m, None, graphs=True)
    e = pe(x)["logits"].cpu().clone()
    for _ in range(2):
        g = pg(x)["logits"].cpu().clone()
    assert torch.equal(e, g) and torch.equal(e, torch.from_numpy(got))


def test_classifier_batch_edges(dev, cls_weights):
    """n = 0, 1 and a batch larger than the first handle capacity."""
    m = _model("squeeze-ernet", cls_weights["squeeze-ernet"])
    x = torch.randn(0, 3, 140, 140, device=dev)
    assert m(x).shape == (0, 5)
    from oracle import classifier as OC
    xs = torch.randn(70, 3, 140, 140)
    p = m(xs.to(dev)).cpu()
    ref, _, _ = OC.forward("squeeze-ernet", cls_weights["squeeze-ernet"], xs)
    assert torch.equal(p.argmax(1), torch.softmax(ref, 1).argmax(1))
    with pytest.raises(ValueError):
        m(torch.randn(1, 3, 224, 224, device=dev))


# --------------------------------------------------------------- detector --
def _darknet(cfg, size, half=False, preset="he"):
    from rtdm.darknet import Darknet
    from rtdm.synth import inline_acff, load_calibration, synth_acff_params, synth_darknet_weights
    text = cfg_text(cfg)
    m = Darknet(text, (size, size))
    calib = load_calibration(cfg, preset)
    # YOLO-ACFF cfgs: the [acff] blocks' state-dict parameters go inline (others: no-op)
    stream = inline_acff(text, synth_darknet_weights(text, calib=calib, preset=preset),
                         synth_acff_params(text, calib=calib, preset=preset))
    m.load_weight_stream(stream)
    if half:
        m.half()
    return m, text, stream


def _check_io(io, ref, half, deep=False):
    if deep:
        atol, rtol, p_tol = (2.0, 0.2, 5e-2) if half else (1e-3, 1e-3, 1e-4)
    else:
        atol, rtol, p_tol = (0.5, 3e-2, 2e-2) if half else (1e-3, 1e-4, 1e-5)
    d = np.abs(io - ref)
    assert np.all(d[..., :2] <= atol), d[..., :2].max()
    bad = d[..., 2:4] > atol + rtol * np.abs(ref[..., 2:4])
    assert not bad.any(), (d[..., 2:4].max(), (d[..., 2:4] / np.maximum(np.abs(ref[..., 2:4]), 1e-6)).max())
    assert np.all(d[..., 4:] <= p_tol), d[..., 4:].max()


@pytest.mark.parametrize("half", [False, True])
def test_detector_golden_small(dev, det_golden, half):
    from rtdm.synth import synth_frames
    key = "yolov4-tiny-aider-416@256"
    m, _, stream = _darknet("yolov4-tiny-aider-416", 256, half)
    assert stream.size == int(det_golden[f"{key}/stream_n"])
    frames = det_golden[f"{key}/frames"]
    x = torch.from_numpy(frames).to(dev)
    io, _ = m(x)
    _check_io(io.cpu().numpy(), det_golden[f"{key}/io"], half)
    # the NCHW fp32 drop-in input gives the same io
    xn = (torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).to(dev)
    io2, _ = m(xn)
    _check_io(io2.cpu().numpy(), det_golden[f"{key}/io"], half)
    del synth_frames


@pytest.mark.parametrize("case", ["yolov4-tiny-aider-416@608", "yolov3-aider-416@416", "yolov3-spp-aider@608",
                                  "yolov3-tiny-aider-416@416", "yolov4-tiny-swish@416",
                                  "yolov4-tiny-3l-512x512@512", "yolov3-acffx@416"])
@pytest.mark.parametrize("half", [False, True])
def test_detector_golden_full(dev, det_golden, case, half):
    from rtdm.synth import BASE_SEED, load_calibration, synth_darknet_weights, synth_frames
    cfg, size = case.split("@")
    size = int(size)
    m, _, stream = _darknet(cfg, size, half)
    frames = synth_frames(1, size, size, seed=BASE_SEED + 700)
    io, _ = m(torch.from_numpy(frames).to(dev))
    io = io.cpu().numpy()
    assert list(io.shape) == list(det_golden[f"{case}/io_shape"])
    deep = not cfg.startswith("yolov4-tiny") and not cfg.startswith("yolov3-tiny")
    if cfg == "yolov3-acffx":
        # fp32 reaches the heads at ~1.5e-3 relative (per-layer test below).  Measured fp32:
        # xy 0.017 px, wh 0.7 %, p 2.8e-3.  fp16 end to end is not comparable on these
        # synthetic weights (the oracle's own fp16-storage model drifts ~1.2x per layer): the
        # fp16 path is checked teacher-forced, layer by layer and at io, in
        # test_yolo_acff_layers_vs_oracle.
        if half:
            assert np.isfinite(io).all()
            return
        d = np.abs(io[:, ::53] - det_golden[f"{case}/io_rows"])
        ref = det_golden[f"{case}/io_rows"]
        assert d[..., :2].max() <= 0.05 and d[..., 4:].max() <= 5e-3, (d[..., :2].max(), d[..., 4:].max())
        assert (d[..., 2:4] <= 1e-3 + 2e-2 * np.abs(ref[..., 2:4])).all()
        return
    _check_io(io[:, ::53], det_golden[f"{case}/io_rows"], half, deep)
    # detections: reference survivors matched by ours.  fp16: at least 90 %, or, where the
    # fp16-storage model of the oracle itself (oracle.darknet f16_storage) matches less --
    # the deep synthetic-weight nets: yolov3-spp@608 115/143, yolov3-aider@416 81/88,
    # measured in this container -- no more than 5 points below that model's own rate
    from rtdm.nms import non_max_suppression
    got = non_max_suppression(torch.from_numpy(io).cuda(), 0.3, 0.4)
    emu = None
    if half and deep:
        from oracle import nms as ON
        from oracle.darknet import DarknetRef
        from rtdm.synth import synth_acff_params
        cal = load_calibration(cfg)
        text = cfg_text(cfg)
        dref = DarknetRef(text, synth_darknet_weights(text, calib=cal), synth_acff_params(text, calib=cal))
        xin = torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0
        emu = ON.non_max_suppression(dref.forward(xin, f16_storage=True).numpy(), 0.3, 0.4)
    for b in range(io.shape[0]):
        ref = det_golden[f"{case}/nms0.3_0.4/{b}"]
        ref = ref[ref[:, 4] > 0.31]
        if len(ref) == 0:
            continue

        def rate(rows):
            g = np.zeros((0, 6), np.float32) if rows is None else rows
            m = 0
            for r in ref:
                same = g[g[:, 5] == r[5]]
                if len(same) and _iou(r[:4], same[:, :4]).max() >= 0.9:
                    m += 1
            return m / len(ref)
        got_rate = rate(None if got[b] is None else got[b].cpu().numpy())
        if not half:
            bar = 0.99
        elif emu is None:
            bar = 0.9
        else:
            bar = min(0.9, rate(emu[b]) - 0.05)
        print(case, "half" if half else "fp32", "detection match", round(got_rate, 3), "bar", round(bar, 3))
        assert got_rate >= bar, (case, got_rate, bar)


COND_CASES = ["yolov4-tiny-aider-416@608", "yolov3-aider-416@416", "yolov3-spp-aider@608", "yolov3-tiny-aider-416@416",
              "yolov4-tiny-swish@416", "yolov4-tiny-3l-512x512@512", "yolov3-acffx@416"]


@pytest.mark.parametrize("case", COND_CASES)
def test_detector_cond_weights_survey_bars(dev, case):
    """SURVEY §8d's detector bars on the well-conditioned synthetic weights (rtdm.synth
    COND; the reference ships no detector weights; its per-cfg knobs, CFG_COND, were chosen
    so that the fp16-storage floor meets the 0.5 px bar):
      fp32: io x,y <= 1e-3 px, w,h <= 1e-3 px + 1e-5 relative, probabilities <= 1e-4 —
            SURVEY's bars as written, for every cfg including the 75+-layer ones (measured
            r05ab: xy <= 1.2e-4 px, w,h inside 1e-3 px, p <= 1e-5); NMS survivors identical;
      fp16: every io box coordinate within 0.5 px of the fp32 oracle (x, y, w and h), and
            the NMS survivor sets (conf 0.3 / IoU 0.4) equal after excluding the candidates
            within 1e-3 of the thresholds (oracle.nms.survivors_equal_outside_band).
    4 frames per cfg (8 for the 608 detector of record); the oracle runs fp32 on the host
    and is itself pinned to the reference Darknet on these weights by
    test_oracle_golden.py::test_darknet_oracle_matches_reference_goldens_cond."""
    from oracle import nms as ON
    from oracle.darknet import DarknetRef
    from conftest import load_npz
    from rtdm.synth import BASE_SEED, load_calibration, synth_acff_params, synth_darknet_weights, synth_frames
    cfg, size = case.split("@")
    size = int(size)
    nf = 8 if case == "yolov4-tiny-aider-416@608" else 4
    frames = synth_frames(nf, size, size, seed=BASE_SEED + 700)
    text = cfg_text(cfg)
    cal = load_calibration(cfg, "cond")
    torch.set_num_threads(16)
    ref = DarknetRef(text, synth_darknet_weights(text, calib=cal, preset="cond"),
                     synth_acff_params(text, calib=cal, preset="cond"))
    io32 = ref.forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0).numpy()
    g = load_npz("det_golden_cond.npz")
    # the oracle on this host vs the reference's rows (bit-exact in the build container;
    # another CPU's conv kernels round differently in the last bits)
    dg = np.abs(io32[:2, ::53] - g[f"{case}/io_rows"])
    assert dg[..., :4].max() <= 1e-3 + 1e-4 * np.abs(g[f"{case}/io_rows"][..., :4]).max() and dg[..., 4:].max() <= 1e-4
    x = torch.from_numpy(frames).to(dev)
    m32, _, _ = _darknet(cfg, size, False, "cond")
    io = m32(x)[0].cpu().numpy()
    d = np.abs(io - io32)
    whx = (d[..., 2:4] - 1e-3) / np.maximum(np.abs(io32[..., 2:4]), 1e-30)
    print(case, "fp32 max |d|: xy", d[..., :2].max(), "wh", d[..., 2:4].max(), "wh rel excess", whx.max(),
          "p", d[..., 4:].max())
    xy_t, wh_r, p_t = 1e-3, 1e-5, 1e-4
    assert d[..., :2].max() <= xy_t, d[..., :2].max()
    assert (d[..., 2:4] <= 1e-3 + wh_r * np.abs(io32[..., 2:4])).all(), d[..., 2:4].max()
    assert d[..., 4:].max() <= p_t, d[..., 4:].max()
    nr, ng, ne, bad = ON.survivors_equal_outside_band(io32, io, 0.3, 0.4, 1e-5)
    assert not bad and nr == ng, ("fp32 survivors", nr, ng, bad[:5])
    m16, _, _ = _darknet(cfg, size, True, "cond")
    io = m16(x)[0].cpu().numpy()
    d = np.abs(io - io32)
    print(case, "fp16 max |d| px: xy", d[..., :2].max(), "wh", d[..., 2:4].max(), "p", d[..., 4:].max())
    assert d[..., :4].max() <= 0.5, (d[..., :2].max(), d[..., 2:4].max())
    nr, ng, ne, bad = ON.survivors_equal_outside_band(io32, io, 0.3, 0.4)
    print(case, f"fp16 survivors ref {nr} hip {ng}, differences inside the 1e-3 band {ne}")
    assert not bad, bad[:10]
    assert nr > 0


@pytest.mark.parametrize("cfg,size", [("yolov4-tiny-aider-416", 608), ("yolov4-tiny-aider-416", 256),
                                      ("yolov4-tiny-swish", 256)])
def test_detector_fused_head_matches_unfused(dev, cfg, size):
    """conv -> 1x1 head -> [yolo] fused into one conv_pipe_f16 launch gives the same
    io bits as the separate head conv (same fp16 activations, same MFMA K order)."""
    from rtdm import _lib as L
    from rtdm.synth import synth_frames
    x = torch.from_numpy(synth_frames(3, size, size, seed=11)).to(dev)
    outs = {}
    try:
        for fuse in (0, 1):
            L.check(L.lib().rtdm_set_tuning(b"fuse_head", fuse))
            m, _, _ = _darknet(cfg, size, True)
            io, _ = m(x)
            assert ("head1x1" in m.describe()) == bool(fuse)
            outs[fuse] = io.cpu()
    finally:
        L.check(L.lib().rtdm_set_tuning(b"fuse_head", 0))
    assert torch.equal(outs[0], outs[1])


def _iou(a, b):
    iw = np.clip(np.minimum(a[2], b[:, 2]) - np.maximum(a[0], b[:, 0]), 0, None)
    ih = np.clip(np.minimum(a[3], b[:, 3]) - np.maximum(a[1], b[:, 1]), 0, None)
    inter = iw * ih
    return inter / ((a[2] - a[0]) * (a[3] - a[1]) + (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]) - inter)


def _layer_outputs(m, n_layers, n):
    """{layer: NCHW fp32 output} of the last forward for every layer that has one.  Only two
    refusals are skipped, each by its own status and message: a layer the plan never
    materialises (its map lives only inside a fused launch: rtdm_detector_layer_output refuses
    the shape query) and a map the last detect fused away at run time -- which must be exactly
    the 1x1 reduce of each planned conv3_c32r / conv3_c64r pair (step names "conv3_c32r",
    "conv3_c64r").  Anything else
    (capacity, bad layer, a new refusal) fails the test."""
    import ctypes
    from rtdm import _lib as L
    h = m._handle
    runtime_fused = set()
    for i in range(L.lib().rtdm_detector_num_steps(h)):
        nm, layer = ctypes.create_string_buffer(64), ctypes.c_int()
        L.check(L.lib().rtdm_detector_step_info(h, i, nm, 64, ctypes.byref(layer), None, None))
        if nm.value in (b"conv3_c32r", b"conv3_c64r"):
            runtime_fused.add(layer.value)
    out, skipped = {}, set()
    for i in range(n_layers):
        c = ctypes.c_int()
        st = L.lib().rtdm_detector_layer_output(h, i, n, None, 0, ctypes.byref(c), None, None, None)
        if st != 0:
            assert st == L.RTDM_E_UNSUPPORTED and b"not materialised" in L.lib().rtdm_last_error(), (i, st)
            continue
        try:
            out[i] = m.layer_output(i, n).cpu()
        except L.RtdmError as e:
            assert e.status == L.RTDM_E_UNSUPPORTED and "fused away in the last detect" in str(e), (i, e)
            skipped.add(i)
    assert skipped == runtime_fused, (skipped, runtime_fused)
    return out


@pytest.mark.parametrize("half", [False, True])
def test_detector_layers_vs_oracle(dev, half):
    """Every materialised layer output of yolov3-aider (shortcuts, routes, upsample) vs the oracle."""
    from oracle.darknet import DarknetRef
    from rtdm.synth import synth_frames
    m, text, stream = _darknet("yolov3-aider-416", 160, half)
    frames = synth_frames(2, 160, 160, seed=3)
    m(torch.from_numpy(frames).to(dev))
    ref_io, outs = DarknetRef(text, stream).forward(
        torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0, keep_layers=True)
    checked = 0
    hip = _layer_outputs(m, len(outs), 2)
    for i, o in enumerate(outs):
        if not isinstance(o, torch.Tensor) or i not in hip:
            continue
        got = hip[i]
        scale = o.abs().max().item() + 1e-6
        err = (got - o).abs().max().item()
        assert err <= (5e-2 if half else 1e-4) * scale + (5e-2 if half else 1e-4), (i, err, scale)
        checked += 1
    assert checked >= 20


@pytest.mark.parametrize("half", [False, True])
def test_yolo_acff_layers_vs_oracle(dev, half):
    """YOLO-ACFF (yolov3-acffx.cfg: [acff] blocks, unfused shortcuts, route resize) layer by
    layer against the oracle.
    fp32: the oracle run end to end; every materialised layer within 5e-3 of its max
    (measured growth 5e-7 -> 1.5e-3 from the stem to the heads).
    fp16: teacher forced -- the oracle computes each layer from the HIP path's own fp16
    outputs of the layers it reads (DarknetRef.forward(override=...)), so each layer's
    error is its own: every materialised layer within 5e-3 of its max, and io within the
    tiny nets' fp16 bars.  End to end, fp16 on these synthetic BatchNorm-calibrated weights
    is not comparable with fp32: the oracle's own fp16-storage model drifts by ~1.2x per
    layer (rms 1.5e-3 at L0, 0.5 by the last head; mean-field BN nets are chaotic at
    init), so a cumulative bar would test the weights, not the kernels."""
    from oracle.darknet import DarknetRef
    from rtdm.synth import load_calibration, synth_acff_params, synth_darknet_weights, synth_frames
    m, text, _ = _darknet("yolov3-acffx", 416, half)
    frames = synth_frames(2, 416, 416, seed=3)
    io, _ = m(torch.from_numpy(frames).to(dev))
    io = io.cpu().numpy()
    cal = load_calibration("yolov3-acffx")
    ref = DarknetRef(text, synth_darknet_weights(text, calib=cal), synth_acff_params(text, calib=cal))
    xin = torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0
    hip = _layer_outputs(m, len(ref.mdefs), 2)
    # a layer the route resize (models.py:364-375) replaced reads back resized: not comparable
    ref.forward(xin, override={})
    hip = {i: t for i, t in hip.items() if tuple(t.shape) == tuple(ref.computed[i].shape)}
    if half:
        ref_io, _ = ref.forward(xin, keep_layers=True, override=hip)
        outs = [ref.computed.get(i) for i in range(len(ref.mdefs))]
        bar = 5e-3  # measured worst 9.9e-4 (57 layers)
    else:
        ref_io, outs = ref.forward(xin, keep_layers=True)
        bar = 5e-3
    checked, worst = 0, 0.0
    for i, got in hip.items():
        o = outs[i]
        if not isinstance(o, torch.Tensor):
            continue
        rel = (got - o).abs().max().item() / (o.abs().max().item() + 1e-6)
        worst = max(worst, rel)
        assert rel <= bar, (i, ref.mdefs[i]["type"], rel)
        checked += 1
    assert checked >= 50, checked
    print("acffx", "fp16 teacher-forced" if half else "fp32", "layers", checked, "worst rel", worst)
    if half:
        _check_io(io, ref_io.numpy(), True)


_ACFF_MINI = """[net]
width=64
height=64
channels=3

[convolutional]
batch_normalize=1
filters=8
size=3
stride=1
pad=1
activation=leaky

[acff]
filters=16
size=3

[route]
layers=-1,-2

[convolutional]
batch_normalize=1
filters=24
size=1
stride=1
pad=1
activation=leaky

[convolutional]
batch_normalize=1
filters=24
size=3
stride=1
pad=1
activation=leaky

[shortcut]
from=-3
activation=linear

[convolutional]
size=1
stride=1
pad=1
filters=14
activation=linear

[yolo]
mask=0,1
anchors=10,14, 23,27
classes=2
num=2

[route]
layers=-4

[convolutional]
size=1
stride=1
pad=1
filters=14
activation=linear

[yolo]
mask=0,1
anchors=10,14, 23,27
classes=2
num=2
"""


@pytest.mark.parametrize("half", [False, True])
def test_acff_route_resize_shortcut_small(dev, half):
    """A 64x64 net with one [acff] block (62x62 output), a route of mismatched widths (the
    ACFF map nearest-resized to 64, models.py:364-375) and a shortcut whose pre-add conv
    output is routed again (unfused ST_ADD), against the oracle: shallow, so the fp32/fp16
    bars of the tiny detectors apply."""
    from oracle.darknet import DarknetRef
    from rtdm.darknet import Darknet
    from rtdm.synth import inline_acff, synth_acff_params, synth_darknet_weights, synth_frames
    conv = synth_darknet_weights(_ACFF_MINI, seed=5)
    acff = synth_acff_params(_ACFF_MINI, seed=6)
    m = Darknet(_ACFF_MINI, (64, 64))
    m.load_weight_stream(inline_acff(_ACFF_MINI, conv, acff))
    if half:
        m.half()
    desc = m.describe()
    assert "resize nearest" in desc and "shortcut add" in desc and "acff dw3x3" in desc, desc
    frames = synth_frames(3, 64, 64, seed=21)
    io, _ = m(torch.from_numpy(frames).to(dev))
    ref = DarknetRef(_ACFF_MINI, conv, acff).forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0)
    assert io.shape == ref.shape
    _check_io(io.cpu().numpy(), ref.numpy(), half)


@pytest.mark.parametrize("half", [False, True])
def test_shortcut_channel_mismatch(dev, half):
    """[shortcut] between maps of different channel counts (weightedFeatureFusion dc > 0 and
    dc < 0, models.py:146-154) on the unfused add path, against the oracle's slicing."""
    from test_abi import _SHORTCUT_MISMATCH as cfg
    from oracle.darknet import DarknetRef
    from rtdm.darknet import Darknet
    from rtdm.synth import synth_darknet_weights, synth_frames
    w = synth_darknet_weights(cfg, seed=7)
    m = Darknet(cfg, (32, 32))
    m.load_weight_stream(w)
    if half:
        m.half()
    frames = synth_frames(3, 32, 32, seed=4)
    io, _ = m(torch.from_numpy(frames).to(dev))
    ref = DarknetRef(cfg, w).forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0)
    assert io.shape == ref.shape
    _check_io(io.cpu().numpy(), ref.numpy(), half)


# -------------------------------------------------------------------- NMS --
def _nms_compare(io, conf, iou, multi_label=True, agnostic=False, classes=None):
    from oracle import nms as ON
    from rtdm.nms import nms_batched
    n, a, no = io.shape
    max_det = a * (no - 5)
    det, idx, count = nms_batched(torch.from_numpy(io).cuda(), conf, iou, multi_label, classes, agnostic, max_det)
    det, idx, count = det.cpu().numpy(), idx.cpu().numpy(), count.cpu().numpy()
    ref, ref_idx = ON.non_max_suppression(io, conf, iou, multi_label, classes, agnostic, return_index=True)
    for b in range(n):
        r = np.zeros((0, 6), np.float32) if ref[b] is None else ref[b]
        assert count[b] == len(r), (b, count[b], len(r))
        assert np.array_equal(det[b, :count[b]], r)
        ri = np.zeros((0, 2)) if ref_idx[b] is None else ref_idx[b]
        assert np.array_equal(idx[b, :count[b]], ri)
    return count


def test_nms_golden_io(dev, det_golden):
    """NMS kernel fed the reference io: bit-exact survivors vs the reference non_max_suppression."""
    key = "yolov4-tiny-aider-416@256"
    io = det_golden[f"{key}/io"]
    from rtdm.nms import non_max_suppression
    for conf, iou in ((0.3, 0.4), (0.01, 0.6)):
        got = non_max_suppression(torch.from_numpy(io).cuda(), conf, iou)
        for b in range(io.shape[0]):
            ref = det_golden[f"{key}/nms{conf}_{iou}/{b}"]
            g = np.zeros((0, 6), np.float32) if got[b] is None else got[b].cpu().numpy()
            assert g.shape == ref.shape, (conf, b, g.shape, ref.shape)
            assert np.array_equal(g, ref)
        _nms_compare(io, conf, iou)


@pytest.mark.parametrize("split", [1, 0])
def test_nms_modes_and_edges(dev, split):
    from rtdm import _lib as L
    L.check(L.lib().rtdm_set_tuning(b"nms_split", split))
    try:
        _nms_modes_case()
    finally:
        L.check(L.lib().rtdm_set_tuning(b"nms_split", 1))


def _nms_modes_case():
    rng = np.random.default_rng(0)
    n, a, nc = 3, 3000, 3
    io = np.zeros((n, a, 5 + nc), np.float32)
    io[..., 0:2] = rng.uniform(0, 400, (n, a, 2))
    io[..., 2:4] = rng.uniform(1, 80, (n, a, 2))
    io[..., 4:] = rng.uniform(0, 1, (n, a, 1 + nc))
    io[0, 5, 2] = np.inf  # filtered by w < 4096
    io[1, 7, 0] = np.nan  # nan box -> filtered (finite check / comparisons)
    io[2] = 0  # nothing passes -> None
    for conf, iou in ((0.3, 0.4), (0.05, 0.5), (0.7, 0.9)):
        _nms_compare(io, conf, iou)
        _nms_compare(io, conf, iou, multi_label=False)
        _nms_compare(io, conf, iou, agnostic=True)
        _nms_compare(io, conf, iou, classes=[0, 2])


@pytest.mark.parametrize("split", [1, 0])
def test_nms_candidate_counts_sort_sizes(dev, split):
    """Per-image candidate counts around every power of two of the LDS path's sort (npow 1 ..
    4096: lane-shuffle stages j < 64, LDS stages j >= 64, 1 .. 4 keys per thread) and around
    the IoU-bitmask capacities (512 in LDS, 2048 in the workspace), one image each, scores
    with ties broken by the anchor index: survivors bit-exact against the oracle, with the
    <= 512-candidate images split over three launches (nms_split 1, the default: bitmask on
    (word, row block) blocks) and in one launch per image (0)."""
    from rtdm import _lib as L
    L.check(L.lib().rtdm_set_tuning(b"nms_split", split))
    try:
        _nms_counts_case()
    finally:
        L.check(L.lib().rtdm_set_tuning(b"nms_split", 1))


def _nms_counts_case():
    counts = [0, 1, 2, 3, 31, 33, 63, 64, 65, 127, 129, 255, 257, 511, 512, 513, 1023, 1025,
              2047, 2048, 2049, 4095, 4096]
    rng = np.random.default_rng(5)
    a = 4200
    io = np.zeros((len(counts), a, 6), np.float32)
    for b, c in enumerate(counts):
        io[b, :, 0:2] = rng.uniform(0, 900, (a, 2))
        io[b, :, 2:4] = rng.uniform(3, 40, (a, 2))
        io[b, :c, 4] = rng.choice(np.linspace(0.5, 1.0, 64, dtype=np.float32), c)  # score ties
        io[b, :c, 5] = 1.0
    got = _nms_compare(io, 0.3, 0.45)
    assert got[-1] > 1000


def test_nms_large_candidate_set(dev):
    """> 4096 candidates per image exercises the global-memory path."""
    rng = np.random.default_rng(1)
    io = np.zeros((2, 20000, 7), np.float32)
    io[..., 0:2] = rng.uniform(0, 600, (2, 20000, 2))
    io[..., 2:4] = rng.uniform(3, 60, (2, 20000, 2))
    io[..., 4:] = rng.uniform(0.2, 1, (2, 20000, 3))
    c = _nms_compare(io, 0.05, 0.5)
    assert c.min() > 100


# ---------------------------------------------------------------- pipeline --
def test_two_stage_pipeline(dev, cls_weights):
    from oracle import classifier as OC
    from oracle import preprocess as P
    from oracle.darknet import DarknetRef
    from oracle import nms as ON
    from rtdm.classifier import build_model
    from rtdm.pipeline import TwoStagePipeline
    from rtdm.synth import synth_frames
    cls = build_model("squeeze-ernet")
    cls.load_state_dict(cls_weights["squeeze-ernet"])
    det, text, stream = _darknet("yolov4-tiny-aider-416", 320)
    pipe = TwoStagePipeline(cls, det, 0.3, 0.4, max_det=300)
    frames = synth_frames(4, 320, 320, seed=42)
    out = pipe(torch.from_numpy(frames).to(dev))
    torch.cuda.synchronize()
    x = torch.from_numpy(np.stack([P.cli_transform(f, 140) for f in frames]))
    ref_logits, _, _ = OC.forward("squeeze-ernet", cls_weights["squeeze-ernet"], x)
    assert torch.equal(out["logits"].cpu().argmax(1), ref_logits.argmax(1))
    io_ref = DarknetRef(text, stream).forward(torch.from_numpy(frames).permute(0, 3, 1, 2).float() / 255.0)
    _check_io(out["io"].cpu().numpy(), io_ref.numpy(), False)
    # NMS on the device io is bit-exact with the oracle NMS on the same io
    ref = ON.non_max_suppression(out["io"].cpu().numpy(), 0.3, 0.4)
    cnt = out["count"].cpu().numpy()
    for b in range(4):
        r = np.zeros((0, 6), np.float32) if ref[b] is None else ref[b]
        assert cnt[b] == len(r)
        assert np.array_equal(out["det"][b, :min(cnt[b], 300)].cpu().numpy(), r[:300])
